set -o pipefail
# round 5, session 15: device-chosen dense / pruned filtered K2; cell-matrix run tables
O=gpurun_out/r5_15
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_algos.py tests/test_gpu_graph_build.py -m gpu -x -q -k "kmeans or graph or native or cell or degree or rank_by" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for n in 1 4; do
  timeout -k 10 200 python3 bench/kmeans_bench.py --noise $n > $O/km_n$n.log 2>&1 || exit $?
done
timeout -k 10 200 python3 bench/pagerank_bench.py > $O/pr.log 2>&1 || exit $?
DALGO_BUILD_SYNC=1 timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness > $O/prs.log 2>&1 || exit $?
