set -o pipefail
mkdir -p gpurun_out/r3a
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_gpu_algos.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "sparse_closure or transitive" > gpurun_out/r3a/pytest_closure.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3a/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3a/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3a/bench.log 2>&1 && \
timeout -k 10 300 python bench/closure_bench.py --torch-ref > gpurun_out/r3a/closure.log 2>&1
