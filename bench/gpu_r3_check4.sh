set -o pipefail
mkdir -p gpurun_out/r3d
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_algos.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "pagerank or kmeans_incremental" > gpurun_out/r3d/pytest.log 2>&1 && \
timeout -k 10 300 python bench/pagerank_bench.py --spmv xcd > gpurun_out/r3d/pagerank_xcd.log 2>&1 && \
timeout -k 10 300 python bench/pagerank_bench.py --spmv pull > gpurun_out/r3d/pagerank_pull.log 2>&1 && \
timeout -k 10 300 python bench/kmeans_bench.py > gpurun_out/r3d/kmeans.log 2>&1
