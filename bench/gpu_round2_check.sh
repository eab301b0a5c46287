set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -3 gpurun_out/pytest_gpu.log && \
timeout -k 10 300 python bench.py > gpurun_out/bench1.log 2>&1 && tail -1 gpurun_out/bench1.log && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -2 gpurun_out/smoke.log
