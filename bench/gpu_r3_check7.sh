set -o pipefail
mkdir -p gpurun_out/r3i
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_algos.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "centre_stationary" > gpurun_out/r3i/pytest_cs.log 2>&1 && \
timeout -k 10 300 python bench/kmeans_bench.py > gpurun_out/r3i/kmeans_cs.log 2>&1 && \
bash bench/gpu_r3_pmc_km.sh
