set -o pipefail
# round 6, session 37: headline size (10M x 1024): one-kernel vs persistent with / without the pool
O=gpurun_out/r6_37
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for rep in 1 2; do
  DALGO_ONE_KERNEL=1 timeout -k 10 120 python3 bench.py --steps 300 --warmup 30 --secondary off --no-eval --launch env > $O/one_r$rep.log 2>&1 || exit $?
  for pf in 0 0.05 0.1 0.15 0.2; do
    DALGO_LR_POOL=$pf DALGO_PERSISTENT=1 timeout -k 10 120 python3 bench.py --steps 300 --warmup 30 --secondary off --no-eval --launch env > $O/pers_p${pf}_r$rep.log 2>&1 || exit $?
  done
done
