set -o pipefail
O=gpurun_out/r4_19
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for v in timing timing_reg; do
  DALGO_EXT_LIB=$PWD/dalgo/_xp_$v.so timeout -k 10 300 python bench/probes/km_tile_timing.py --rows 100000000 > $O/${v}_100m.log 2>&1 || exit 1
done
for r in 1 2; do
  timeout -k 10 300 python bench/kmeans_bench.py --no-witness > $O/km_new$r.log 2>&1 || exit 1
  DALGO_EXT_LIB=$PWD/dalgo/_xp_reg.so timeout -k 10 300 python bench/kmeans_bench.py --no-witness > $O/km_reg$r.log 2>&1 || exit 1
done
