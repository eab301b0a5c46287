set -o pipefail
# round 6, session 5: drift-aware candidate lists (k-means) -- tests, then the job at
# several dense thresholds, separated and overlapping blobs; also the r6_4 graph items
O=gpurun_out/r6_5
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_algos.py -m gpu -x -v -k "kmeans" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_build.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gtests.log 2>&1 || exit $?
for f in 0.4 0.75 0.9 1.01; do
  DALGO_KM_DENSE_FRACTION=$f timeout -k 10 200 python3 bench/kmeans_bench.py > $O/km_sep_$f.log 2>&1 || exit $?
  DALGO_KM_DENSE_FRACTION=$f timeout -k 10 200 python3 bench/kmeans_bench.py --noise 4 > $O/km_ovl_$f.log 2>&1 || exit $?
done
timeout -k 10 200 python3 bench/kmeans_bench.py --no-drift > $O/km_sep_nodrift.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/pagerank_share.py --ranks 0 > $O/share.log 2>&1 || exit $?
