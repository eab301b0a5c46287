set -o pipefail
# round 6, session 3: W = 8 per-rank build share with the build's phase split
O=gpurun_out/r6_3
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 bench/pagerank_share.py --ranks 0 > $O/share.log 2>&1 || exit $?
