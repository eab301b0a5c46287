set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -3 gpurun_out/pytest_gpu.log && \
timeout -k 10 300 python bench.py > gpurun_out/bench1.log 2>&1 && tail -1 gpurun_out/bench1.log
