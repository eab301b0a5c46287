set -o pipefail
mkdir -p gpurun_out/r3full
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3full/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3full/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3full/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 --rows 1250000 > gpurun_out/r3full/bench_share8.log 2>&1
