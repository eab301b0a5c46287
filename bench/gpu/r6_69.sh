set -o pipefail
# round 6, session 69: top-2 full pass (exact l) so that the first filtered iteration can
# run the candidate K2 with drift pruning
O=gpurun_out/r6_69
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for m in device auto; do
  DALGO_KM_FULL_TOP2=1 timeout -k 10 200 python3 bench/kmeans_bench.py --dense $m --no-witness > $O/sep_t2_$m.log 2>&1 || exit $?
  DALGO_KM_FULL_TOP2=1 timeout -k 10 200 python3 bench/kmeans_bench.py --noise 4 --dense $m --no-witness > $O/ovl_t2_$m.log 2>&1 || exit $?
done
timeout -k 10 200 python3 bench/kmeans_bench.py --no-witness > $O/sep_base.log 2>&1
