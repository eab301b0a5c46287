set -o pipefail
mkdir -p gpurun_out/r3m
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_algos.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "pagerank or pr_spmv" > gpurun_out/r3m/pytest.log 2>&1 && \
timeout -k 10 300 python bench/pagerank_bench.py > gpurun_out/r3m/pr_pipe.log 2>&1 && \
DALGO_PR_PIPE=0 timeout -k 10 300 python bench/pagerank_bench.py > gpurun_out/r3m/pr_nopipe.log 2>&1
