set -o pipefail
# round 6, session 88: graph / PageRank / multi-rank GPU tests after the world-scaled work items
O=gpurun_out/r6_88
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_graph_build.py tests/test_gpu_multirank.py tests/test_gpu_algos.py -k "graph or pagerank or pb_ or native or blocked or multirank or rank" -m gpu -x -q --timeout 280 --timeout-method thread > $O/tests.log 2>&1 || exit $?
