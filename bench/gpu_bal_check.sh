# count-balanced K1 ranges: numerics, then bench A/B (DALGO_LR_BALANCE=0/1) at the 1-GPU
# config and the 8-GPU per-rank share, plus the K1 timeline at 1.25M rows
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bal
timeout -k 10 400 python -u -m pytest tests/test_gpu_lr.py -x -v --timeout 200 --timeout-method thread > gpurun_out/bal/pytest_lr.log 2>&1 && tail -3 gpurun_out/bal/pytest_lr.log && \
for r in 1 2; do for b in 0 1; do
  DALGO_LR_BALANCE=$b timeout -k 10 200 python bench.py --rows 1250000 --steps 400 --warmup 50 --cal-steps 100 > gpurun_out/bal/b125_${b}_$r.log 2>&1 || exit 1
  DALGO_LR_BALANCE=$b timeout -k 10 200 python bench.py --steps 100 --warmup 10 > gpurun_out/bal/b10m_${b}_$r.log 2>&1 || exit 1
done; done && \
for f in gpurun_out/bal/b*.log; do echo $f; python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,1), 'us', d['config']['launch'], {k: round(v*1e3,1) for k,v in d.get('launch_calibration_ms_per_step',{}).items()})"; done
