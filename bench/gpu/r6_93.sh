set -o pipefail
# round 6, session 93: entry-cells pass with 4 (r6_93) or 8 (r6_93b) entries per thread and batched dependent loads
O=gpurun_out/r6_93
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_build.py tests/test_gpu_algos.py -k "graph or pagerank or pb_ or native or blocked" -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/pagerank_bench.py > $O/pr_w.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness > $O/pr_$i.log 2>&1 || exit $?
done
