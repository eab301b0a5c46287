set -o pipefail
mkdir -p gpurun_out/r3k
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_algos.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "kmeans" > gpurun_out/r3k/pytest_km.log 2>&1 && \
timeout -k 10 300 python bench/kmeans_bench.py > gpurun_out/r3k/kmeans_bounds.log 2>&1 && \
DALGO_KM_BOUNDS=0 timeout -k 10 300 python bench/kmeans_bench.py > gpurun_out/r3k/kmeans_nobounds.log 2>&1
