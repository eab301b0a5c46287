set -o pipefail
# round 6, session 40: persistent K1 launch cost: cooperative vs plain launch (20 / 300 steps)
O=gpurun_out/r6_40
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for st in 20 300; do
  DALGO_ONE_KERNEL=1 timeout -k 10 120 python3 bench.py --steps $st --warmup 5 --secondary off --no-eval --launch env > $O/one_s$st.log 2>&1 || exit $?
  for co in 1 0; do
    DALGO_PERSIST_COOP=$co DALGO_PERSISTENT=1 timeout -k 10 120 python3 bench.py --steps $st --warmup 5 --secondary off --no-eval --launch env > $O/pers_c${co}_s$st.log 2>&1 || exit $?
  done
done
