# K1 fine-claim threshold (DALGO_LR_FINE, 256-row groups left when claims drop to single
# 64-row units): bench at 1.25M and 10M rows, interleaved repeats
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fine
for r in 1 2; do for f in 8 2 4 12 16; do
  DALGO_LR_FINE=$f timeout -k 10 200 python bench.py --rows 1250000 --steps 400 --warmup 50 --cal-steps 100 > gpurun_out/fine/b125_${f}_$r.log 2>&1 || exit 1
  DALGO_LR_FINE=$f timeout -k 10 200 python bench.py --steps 100 --warmup 10 > gpurun_out/fine/b10m_${f}_$r.log 2>&1 || exit 1
done; done
for f in gpurun_out/fine/b*.log; do echo $f $(python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,1), d['config']['launch'])"); done
