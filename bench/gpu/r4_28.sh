set -o pipefail
O=gpurun_out/r4_28
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 python bench/kmeans_bench.py --no-witness > $O/km_new$r.log 2>&1 || exit 1
  DALGO_EXT_LIB=$PWD/dalgo/_xp_prev.so timeout -k 10 300 python bench/kmeans_bench.py --no-witness > $O/km_prev$r.log 2>&1 || exit 1
done
