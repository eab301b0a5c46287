set -o pipefail
# round 6, session 67: drift-cap quantile with the 16x16x32 candidate K2
O=gpurun_out/r6_67
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for q in 0.8 0.9 0.95 1.0; do
  DALGO_KM_DRIFT_Q=$q timeout -k 10 200 python3 bench/kmeans_bench.py --noise 4 --no-witness > $O/ovl_q$q.log 2>&1 || exit $?
  DALGO_KM_DRIFT_Q=$q timeout -k 10 200 python3 bench/kmeans_bench.py --no-witness > $O/sep_q$q.log 2>&1 || exit $?
done
