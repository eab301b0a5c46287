set -o pipefail
# round 6, session 8: drift + ball with the dropped centres split by speed for the new l
O=gpurun_out/r6_8
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_algos.py -m gpu -x -q -k "kmeans and (cand or drift or dense)" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for q in 0.75 0.9 1.0; do
  for f in 0.4 0.75 1.01; do
    DALGO_KM_DRIFT_BALL=1 DALGO_KM_DRIFT_Q=$q DALGO_KM_DENSE_FRACTION=$f timeout -k 10 200 python3 bench/kmeans_bench.py > $O/km_sep_${q}_$f.log 2>&1 || exit $?
    DALGO_KM_DRIFT_BALL=1 DALGO_KM_DRIFT_Q=$q DALGO_KM_DENSE_FRACTION=$f timeout -k 10 200 python3 bench/kmeans_bench.py --noise 4 > $O/km_ovl_${q}_$f.log 2>&1 || exit $?
  done
done
