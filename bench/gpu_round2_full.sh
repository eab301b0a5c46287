# Round-2 verification on one MI355X: GPU tests, smoke, headline bench, kernel profiles.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -2 gpurun_out/pytest_gpu.log && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log && \
timeout -k 10 300 python bench.py > gpurun_out/bench1.log 2>&1 && tail -1 gpurun_out/bench1.log && \
timeout -k 10 600 bash bench/profile_all.sh && echo profiles-ok
