set -o pipefail
# round 5, session 63: bucket degree kernel with 4 independent loads per thread in flight
O=gpurun_out/r5_63
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_build.py tests/test_gpu_algos.py -m gpu -x -q -k "run_sort or native or cell or degree or rank_by or pagerank or blocked or pb_" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/pagerank_bench.py > $O/pr.log 2>&1 || exit $?
DALGO_BUILD_SYNC=1 timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness > $O/prs.log 2>&1 || exit $?
