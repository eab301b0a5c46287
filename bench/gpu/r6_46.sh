set -o pipefail
# round 6, session 46: one-kernel row pool -- fraction x chunk size sweep at the headline size
O=gpurun_out/r6_46
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp DALGO_ONE_KERNEL=1
for rep in 1 2 3; do
  for pf in 0.05 0.1; do
    for sh in 8 9 10; do
      DALGO_LR_POOL1=$pf DALGO_LR_POOL_SHIFT=$sh timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --secondary off --no-eval --launch env > $O/one_p${pf}_s${sh}_r$rep.log 2>&1 || exit $?
    done
  done
done
