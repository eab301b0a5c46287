set -o pipefail
O=gpurun_out/r3kmove
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_algos.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "kmeans" > $O/pytest_km.log 2>&1 && \
timeout -k 10 300 python bench/kmeans_bench.py > $O/km_default.log 2>&1 && \
DALGO_KM_INC_MAX=0.3 timeout -k 10 300 python bench/kmeans_bench.py > $O/km_inc30.log 2>&1 && \
DALGO_KM_MOVE_SORTED_MIN=1000000000 timeout -k 10 300 python bench/kmeans_bench.py > $O/km_atomic.log 2>&1
