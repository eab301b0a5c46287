set -o pipefail
# round 6, session 43: the cross-block row pool in the one-kernel (fused one-step) form
O=gpurun_out/r6_43
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_lr.py -m gpu -x -q -k "persistent or fused_tail" --timeout 100 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for rep in 1 2; do
  for pf in 0 0.1 0.15 0.2; do
    DALGO_LR_POOL1=$pf DALGO_ONE_KERNEL=1 timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --secondary off --no-eval --launch env > $O/one_p${pf}_r$rep.log 2>&1 || exit $?
  done
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --secondary off --no-eval --launch env > $O/perstep_r$rep.log 2>&1 || exit $?
done
for pf in 0 0.15; do
  DALGO_LR_POOL1=$pf DALGO_ONE_KERNEL=1 timeout -k 10 120 python3 bench.py --rows 1250000 --steps 200 --warmup 20 --secondary off --no-eval --launch env > $O/one_1250000_p$pf.log 2>&1 || exit $?
done
