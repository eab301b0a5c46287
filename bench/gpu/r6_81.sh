set -o pipefail
# round 6, session 81: K4b phase-2 work items default 768 on one rank -- tests and the job
O=gpurun_out/r6_81
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_build.py tests/test_gpu_algos.py -k "graph or pagerank or pb_ or native or blocked" -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/pagerank_bench.py > $O/pr.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/pagerank_bench.py > $O/pr2.log 2>&1 || exit $?
