set -o pipefail
# round 6, session 100: drift-pruned candidate lists with / without the Exponion-ball drop
O=gpurun_out/r6_100
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for b in 0 1 0 1; do
  DALGO_KM_DRIFT_BALL=$b timeout -k 10 200 python3 bench/kmeans_bench.py --noise 4 --no-witness > $O/ovl_b${b}_$RANDOM.log 2>&1 || exit $?
  DALGO_KM_DRIFT_BALL=$b timeout -k 10 200 python3 bench/kmeans_bench.py --no-witness > $O/sep_b${b}_$RANDOM.log 2>&1 || exit $?
done
