# launch-form calibration check on one MI355X: 2-rank rehearsal test, then bench.py at
# the 1-GPU config and at the 8-GPU per-rank share (1.25M rows)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cal
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread -k "calibration or eight_ranks or fused_xgmi" > gpurun_out/cal/pytest.log 2>&1 && tail -3 gpurun_out/cal/pytest.log && \
timeout -k 10 300 python bench.py > gpurun_out/cal/bench_10m.log 2>&1 && tail -1 gpurun_out/cal/bench_10m.log && \
timeout -k 10 300 python bench.py --rows 1250000 --steps 400 --warmup 50 --cal-steps 100 > gpurun_out/cal/bench_1p25m.log 2>&1 && tail -1 gpurun_out/cal/bench_1p25m.log
