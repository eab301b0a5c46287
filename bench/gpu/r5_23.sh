set -o pipefail
# round 5, session 23: finer build phase split (entry placement / tile selection / work split)
O=gpurun_out/r5_23
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness > $O/pr.log 2>&1 || exit $?
DALGO_BUILD_SYNC=1 timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness > $O/prs.log 2>&1 || exit $?
