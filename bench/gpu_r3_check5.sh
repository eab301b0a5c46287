set -o pipefail
mkdir -p gpurun_out/r3f
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_algos.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "pagerank or pr_spmv" > gpurun_out/r3f/pytest.log 2>&1 && \
for h in 8192 16384 32768; do DALGO_PR_HOT=$h timeout -k 10 300 python bench/pagerank_bench.py > gpurun_out/r3f/pr_hot$h.log 2>&1 || exit 1; done
