# K1 trace-free LEAN build (new, in-tree) vs LEAN with trace points (abtest/old.so):
# bench steps at 1.25M and 10M rows, three interleaved repeats
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/l2
timeout -k 10 300 python -u -m pytest tests/test_gpu_lr.py -x -q --timeout 200 --timeout-method thread > gpurun_out/l2/pytest_lr.log 2>&1 && tail -1 gpurun_out/l2/pytest_lr.log || exit 1
for r in 1 2 3; do for v in new old; do
  if [ $v = old ]; then export DALGO_EXT_LIB=$PWD/abtest/old.so; else unset DALGO_EXT_LIB; fi
  timeout -k 10 200 python bench.py --rows 1250000 --steps 400 --warmup 50 --cal-steps 100 > gpurun_out/l2/b125_${v}_$r.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 > gpurun_out/l2/b10m_${v}_$r.log 2>&1 || exit 1
done; done
unset DALGO_EXT_LIB
for f in gpurun_out/l2/b*.log; do echo $f $(python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,1), d['config']['launch'])"); done
