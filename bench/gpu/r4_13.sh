set -o pipefail
O=gpurun_out/r4_13
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 300 python bench/kmeans_bench.py --no-witness > $O/km_ext.log 2>&1 && \
DALGO_EXT_LIB=$PWD/dalgo/_ab_noext.so timeout -k 10 300 python bench/kmeans_bench.py --no-witness > $O/km_noext.log 2>&1 && \
timeout -k 10 300 python bench/kmeans_bench.py --no-witness > $O/km_ext2.log 2>&1 && \
DALGO_EXT_LIB=$PWD/dalgo/_ab_noext.so timeout -k 10 300 python bench/kmeans_bench.py --no-witness > $O/km_noext2.log 2>&1
