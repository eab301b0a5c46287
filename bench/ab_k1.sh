#!/bin/bash
# A/B of two extension builds in ONE GPU call (box-to-box variance is larger than the
# effects measured): the in-tree build ("new") against abtest/old.so ("old", built from
# the baseline revision with `python -m dalgo._build` and copied there), loaded through
# DALGO_EXT_LIB. Results under gpurun_out/ab/.
set -e
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lr.py > gpurun_out/ab/t.log 2>&1
for v in new old; do
  if [ $v = old ]; then export DALGO_EXT_LIB=$PWD/abtest/old.so; fi
  timeout -k 10 100 python bench/k1_timeline.py 20000 1250000 --fine 8 > gpurun_out/ab/tl_s_$v.log 2>&1
  timeout -k 10 100 python bench/k1_timeline.py 125000 1000000 --frac 1.0 --fine 8 > gpurun_out/ab/tl_f_$v.log 2>&1
  timeout -k 10 100 python bench.py --algo gd --rows 1250000 --steps 100 --warmup 10 > gpurun_out/ab/gd125_$v.log 2>&1
  timeout -k 10 100 python bench.py --rows 1250000 --steps 300 --warmup 30 > gpurun_out/ab/ssgd125_$v.log 2>&1
done
