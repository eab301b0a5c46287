set -o pipefail
# round 6, session 36: persistent K1, block-level claims of cross-block pool chunks
O=gpurun_out/r6_36
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_lr.py -m gpu -x -q -k persistent --timeout 100 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for pf in 0 0.1 0.2 0.3; do
  for sh in 9 10; do
    DALGO_LR_POOL=$pf DALGO_LR_POOL_SHIFT=$sh DALGO_PERSISTENT=1 timeout -k 10 120 python3 bench.py --rows 1250000 --steps 400 --warmup 50 --secondary off --no-eval --launch env > $O/pers_1250000_p${pf}_s$sh.log 2>&1 || exit $?
  done
done
for pf in 0 0.1 0.2; do
  DALGO_LR_POOL=$pf DALGO_PERSISTENT=1 timeout -k 10 120 python3 bench.py --rows 10000000 --steps 200 --warmup 30 --secondary off --no-eval --launch env > $O/pers_10000000_p$pf.log 2>&1 || exit $?
done
