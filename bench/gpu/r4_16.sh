set -o pipefail
O=gpurun_out/r4_16
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python bench/probes/km_k2_ab.py > $O/ab.log 2>&1 && \
DALGO_EXT_LIB=$PWD/dalgo/_xp_posstore.so timeout -k 10 300 python bench/probes/km_k2_ab.py > $O/ab_pos.log 2>&1 && \
DALGO_EXT_LIB=$PWD/dalgo/_xp_timing.so timeout -k 10 300 python bench/probes/km_tile_timing.py > $O/timing.log 2>&1
