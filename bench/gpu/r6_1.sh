set -o pipefail
# round 6, session 1: relabel race fix (bucket starts from a separate launch), scale-20
# relabel test, independent build witness in the PageRank job
O=gpurun_out/r6_1
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_build.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/pagerank_bench.py > $O/pr.log 2>&1 || exit $?
