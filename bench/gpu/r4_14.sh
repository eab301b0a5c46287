set -o pipefail
O=gpurun_out/r4_14
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python bench/probes/km_k2_ab.py > $O/ab_base.log 2>&1 && \
DALGO_EXT_LIB=$PWD/dalgo/_xp_nostore.so timeout -k 10 300 python bench/probes/km_k2_ab.py > $O/ab_nostore.log 2>&1 && \
DALGO_EXT_LIB=$PWD/dalgo/_xp_one.so timeout -k 10 300 python bench/probes/km_k2_ab.py > $O/ab_one.log 2>&1 && \
DALGO_EXT_LIB=$PWD/dalgo/_xp_onenostore.so timeout -k 10 300 python bench/probes/km_k2_ab.py > $O/ab_onenostore.log 2>&1
