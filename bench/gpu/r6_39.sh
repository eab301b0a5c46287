set -o pipefail
# round 6, session 39: persistent K1 (with / without the pool) at 20 vs 300 timed steps; the auto race
O=gpurun_out/r6_39
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for st in 20 300; do
  DALGO_ONE_KERNEL=1 timeout -k 10 120 python3 bench.py --steps $st --warmup 5 --secondary off --no-eval --launch env > $O/one_s$st.log 2>&1 || exit $?
  for pf in 0 0.15; do
    DALGO_LR_POOL=$pf DALGO_PERSISTENT=1 timeout -k 10 120 python3 bench.py --steps $st --warmup 5 --secondary off --no-eval --launch env > $O/pers_p${pf}_s$st.log 2>&1 || exit $?
  done
done
timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --secondary off --no-eval > $O/auto.log 2>&1 || exit $?
timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --secondary off --no-eval --cal-steps 100 > $O/auto_cal100.log 2>&1 || exit $?
