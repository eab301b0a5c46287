# K1 variant 8 built without the cross-block pool code (new, in-tree) vs with it
# (abtest/old.so): start-up timeline and bench steps, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/np
timeout -k 10 300 python -u -m pytest tests/test_gpu_lr.py -x -q --timeout 200 --timeout-method thread > gpurun_out/np/pytest_lr.log 2>&1 && tail -1 gpurun_out/np/pytest_lr.log || exit 1
for r in 1 2; do for v in new old; do
  if [ $v = old ]; then export DALGO_EXT_LIB=$PWD/abtest/old.so; else unset DALGO_EXT_LIB; fi
  timeout -k 10 200 python bench/k1_timeline.py 1250000 10000000 --fine 8 > gpurun_out/np/tl_${v}_$r.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --rows 1250000 --steps 400 --warmup 50 --cal-steps 100 > gpurun_out/np/b125_${v}_$r.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 > gpurun_out/np/b10m_${v}_$r.log 2>&1 || exit 1
done; done
unset DALGO_EXT_LIB
for f in gpurun_out/np/b*.log; do echo $f $(python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,1), d['config']['launch'])"); done
for f in gpurun_out/np/tl_*.log; do echo $f; python -c "
import json
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); print(d['rows'], 'bar', d['barrier_p50'], 'refill', d['refill_p50'], 'first', d['first_issue_p50'], 'done p50', d['block_done_p50'], 'max', d['block_done_max'], 'end', d['end_max'])
"; done
