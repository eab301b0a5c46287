# full GPU suite, smoke, headline bench at 1 GPU, the 8-GPU per-rank share with the
# launch-form calibration, and a kernel-trace profile of the headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1 && tail -2 gpurun_out/final/pytest_gpu.log && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 && tail -1 gpurun_out/final/smoke.log && \
timeout -k 10 200 python bench.py > gpurun_out/final/bench_10m.log 2>&1 && tail -1 gpurun_out/final/bench_10m.log && \
timeout -k 10 200 python bench.py --rows 1250000 --steps 400 --warmup 50 --cal-steps 100 > gpurun_out/final/bench_1p25m.log 2>&1 && tail -1 gpurun_out/final/bench_1p25m.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/final/prof -o ssgd --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/final/prof.log 2>&1 && echo prof-ok
