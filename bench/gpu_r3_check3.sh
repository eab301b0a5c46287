set -o pipefail
mkdir -p gpurun_out/r3c
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_algos.py tests/test_gpu_random.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "kmeans or philox" > gpurun_out/r3c/pytest_km.log 2>&1 && \
timeout -k 10 300 python bench/kmeans_bench.py > gpurun_out/r3c/kmeans.log 2>&1 && \
DALGO_KM_INC_MAX=0 timeout -k 10 300 python bench/kmeans_bench.py > gpurun_out/r3c/kmeans_full.log 2>&1 && \
timeout -k 10 300 python bench/pagerank_bench.py > gpurun_out/r3c/pagerank.log 2>&1 && \
bash bench/pmc_pagerank.sh > gpurun_out/r3c/pmc_pr.log 2>&1
