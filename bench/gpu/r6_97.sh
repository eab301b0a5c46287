set -o pipefail
# round 6, session 97: cell-count pass with 4 entries per thread (loads first)
O=gpurun_out/r6_97
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_build.py tests/test_gpu_algos.py -k "graph or pagerank or pb_ or native or blocked" -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/pagerank_bench.py > $O/pr_w.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness > $O/pr_1.log 2>&1 || exit $?
