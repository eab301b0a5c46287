#!/bin/bash
# K1 cross-block pool fractions A/B in one GPU call (results under gpurun_out/pool/).
set -e
mkdir -p gpurun_out/pool
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lr.py > gpurun_out/pool/t.log 2>&1
for pf in 0 0.05 0.1 0.2; do
  DALGO_LR_POOL=$pf timeout -k 10 100 python bench/k1_timeline.py 1250000 10000000 --fine 8 > gpurun_out/pool/tl_$pf.log 2>&1
  DALGO_LR_POOL=$pf timeout -k 10 100 python bench.py --rows 1250000 --steps 300 --warmup 30 > gpurun_out/pool/b125_$pf.log 2>&1
  DALGO_LR_POOL=$pf timeout -k 10 100 python bench.py --steps 50 --warmup 10 > gpurun_out/pool/b10m_$pf.log 2>&1
done
