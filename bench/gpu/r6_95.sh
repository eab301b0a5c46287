set -o pipefail
# round 6, session 95: run-sort tile (run starts per block of gb_run_tile): 4096 (r6_95) or 1024 (r6_95b) instead of 2048
O=gpurun_out/r6_95
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_build.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/pagerank_bench.py > $O/pr_w.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness > $O/pr_1.log 2>&1 || exit $?
