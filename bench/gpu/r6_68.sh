set -o pipefail
# round 6, session 68: the K2 form of the first filtered iteration (dense vs device-decided)
O=gpurun_out/r6_68
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for m in device auto; do
  timeout -k 10 200 python3 bench/kmeans_bench.py --dense $m --no-witness > $O/sep_$m.log 2>&1 || exit $?
  timeout -k 10 200 python3 bench/kmeans_bench.py --noise 4 --dense $m --no-witness > $O/ovl_$m.log 2>&1 || exit $?
done
DALGO_KM_DENSE_FRACTION=1.01 timeout -k 10 200 python3 bench/kmeans_bench.py --dense device --no-witness > $O/sep_never.log 2>&1
