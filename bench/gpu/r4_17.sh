set -o pipefail
O=gpurun_out/r4_17
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for v in timing tnostore tcontig; do
  DALGO_EXT_LIB=$PWD/dalgo/_xp_$v.so timeout -k 10 300 python bench/probes/km_tile_timing.py > $O/$v.log 2>&1 || exit 1
done
