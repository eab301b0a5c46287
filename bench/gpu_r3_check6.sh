set -o pipefail
mkdir -p gpurun_out/r3g
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_algos.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "centre_stationary or kmeans" > gpurun_out/r3g/pytest_cs.log 2>&1 && \
timeout -k 10 300 python bench/kmeans_bench.py > gpurun_out/r3g/kmeans_cs.log 2>&1 && \
DALGO_KM_VARIANT=52 timeout -k 10 300 python bench/kmeans_bench.py > gpurun_out/r3g/kmeans_52.log 2>&1
