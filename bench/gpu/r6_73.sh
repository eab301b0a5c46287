set -o pipefail
# round 6, session 73: K4b split-bin combine, 64 destinations x 4 piece lanes per block
O=gpurun_out/r6_73
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_build.py tests/test_gpu_algos.py -k "graph or pagerank or pb_ or native or blocked" -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/pagerank_bench.py > $O/pr.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/pagerank_bench.py > $O/pr2.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o pr -- python3 $GRAFT_REPO_ROOT/bench/pagerank_bench.py > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit $?
