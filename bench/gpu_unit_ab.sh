# K1 work-unit size when sampling (DALGO_LR_UNIT_SHIFT): timeline + bench at the 8-GPU
# per-rank share (1.25M rows) and the 1-GPU config (10M rows)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/unit
timeout -k 10 300 python -u -m pytest tests/test_gpu_lr.py -x -q --timeout 200 --timeout-method thread > gpurun_out/unit/pytest_lr.log 2>&1 && tail -1 gpurun_out/unit/pytest_lr.log || exit 1
for s in 6 4 5 3; do
  DALGO_LR_UNIT_SHIFT=$s timeout -k 10 200 python bench/k1_timeline.py 1250000 10000000 --fine 8 > gpurun_out/unit/tl_$s.log 2>&1 || exit 1
done
for r in 1 2; do for s in 6 4 5; do
  DALGO_LR_UNIT_SHIFT=$s timeout -k 10 200 python bench.py --rows 1250000 --steps 400 --warmup 50 --cal-steps 100 > gpurun_out/unit/b125_${s}_$r.log 2>&1 || exit 1
  DALGO_LR_UNIT_SHIFT=$s timeout -k 10 200 python bench.py --steps 100 --warmup 10 > gpurun_out/unit/b10m_${s}_$r.log 2>&1 || exit 1
done; done
for f in gpurun_out/unit/b*.log; do echo $f $(python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,1), d['config']['launch'])"); done
for f in gpurun_out/unit/tl_*.log; do echo $f; python -c "
import json
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); print(d['rows'], 'intra', d['intra_block_spread_p50'], 'done p50', d['block_done_p50'], 'max', d['block_done_max'], 'end', d['end_max'], 'refill', d['refill_p50'])
"; done
