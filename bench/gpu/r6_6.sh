set -o pipefail
# round 6, session 6: drift threshold capped at a quantile of the centre shifts -- sweep
O=gpurun_out/r6_6
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_algos.py -m gpu -x -q -k "kmeans and (cand or drift or bound or dense or nbrs)" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for q in 0.5 0.75 0.9; do
  for f in 0.4 0.75; do
    DALGO_KM_DRIFT_Q=$q DALGO_KM_DENSE_FRACTION=$f timeout -k 10 200 python3 bench/kmeans_bench.py > $O/km_sep_${q}_$f.log 2>&1 || exit $?
    DALGO_KM_DRIFT_Q=$q DALGO_KM_DENSE_FRACTION=$f timeout -k 10 200 python3 bench/kmeans_bench.py --noise 4 > $O/km_ovl_${q}_$f.log 2>&1 || exit $?
  done
done
timeout -k 10 300 python3 bench/pagerank_share.py --ranks 0 > $O/share.log 2>&1 || exit $?
