set -o pipefail
# round 6, session 42: persistent K1 ms/step against the number of steps in the launch
O=gpurun_out/r6_42
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp DALGO_PERSISTENT=1
for st in 5 10 20 40 80 160; do
  timeout -k 10 120 python3 bench.py --steps $st --warmup 5 --secondary off --no-eval --launch env > $O/pers_s$st.log 2>&1 || exit $?
done
for st in 20 160; do
  DALGO_ONE_KERNEL=1 DALGO_PERSISTENT=0 timeout -k 10 120 python3 bench.py --steps $st --warmup 5 --secondary off --no-eval --launch env > $O/one_s$st.log 2>&1 || exit $?
done
