set -o pipefail
# round 6, session 22: K1 per-wave timeline at the 8-GPU share and at the headline size
O=gpurun_out/r6_22
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python3 bench/k1_timeline.py 1250000 10000000 > $O/timeline.log 2>&1 || exit $?
