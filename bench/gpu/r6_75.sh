set -o pipefail
# round 6, session 75: row-pool chunk size at the 8-GPU per-rank share (1.25M rows)
O=gpurun_out/r6_75
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp DALGO_LR_POOL_MIN_ROWS=0
for pf in 0 0.15 0.3; do
  for sh in 6 7 8 9; do
    [ "$pf" = 0 ] && [ "$sh" != 9 ] && continue
    DALGO_LR_POOL=$pf DALGO_LR_POOL_SHIFT=$sh DALGO_PERSISTENT=1 timeout -k 10 120 python3 bench.py --rows 1250000 --steps 400 --warmup 50 --secondary off --no-eval --launch env > $O/pers_p${pf}_s$sh.log 2>&1 || exit $?
    DALGO_LR_POOL1=$pf DALGO_LR_POOL_SHIFT=$sh DALGO_ONE_KERNEL=1 timeout -k 10 120 python3 bench.py --rows 1250000 --steps 400 --warmup 50 --secondary off --no-eval --launch env > $O/one_p${pf}_s$sh.log 2>&1 || exit $?
  done
done
