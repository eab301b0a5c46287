set -o pipefail
O=gpurun_out/r4_20
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for v in timing timing_reg; do
  DALGO_EXT_LIB=$PWD/dalgo/_xp_$v.so timeout -k 10 300 python bench/probes/km_tile_timing.py --rows 100000000 > $O/${v}_100m.log 2>&1 || exit 1
done
