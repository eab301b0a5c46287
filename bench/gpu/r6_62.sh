set -o pipefail
# round 6, session 62: persistent K1 early-step slowness -- long warm-up before a 20-step timed launch
O=gpurun_out/r6_62
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for w in 5 200; do
  DALGO_PERSISTENT=1 timeout -k 10 120 python3 bench.py --steps 20 --warmup $w --secondary off --no-eval --launch env > $O/pers_w$w.log 2>&1 || exit $?
  DALGO_ONE_KERNEL=1 timeout -k 10 120 python3 bench.py --steps 20 --warmup $w --secondary off --no-eval --launch env > $O/one_w$w.log 2>&1 || exit $?
done
