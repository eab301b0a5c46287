set -o pipefail
# round 6, session 50: PageRank model init with fewer kernels, srcl memset only past E
O=gpurun_out/r6_50
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_build.py tests/test_gpu_algos.py -k "pagerank or native or build or rank"  -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/pagerank_bench.py > $O/pr.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/pagerank_share.py --ranks 0 > $O/share.log 2>&1 || exit $?
