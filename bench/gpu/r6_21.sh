set -o pipefail
# round 6, session 21: persistent K1 with two row batches in flight across the step release
O=gpurun_out/r6_21
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_lr.py -m gpu -x -q --timeout 100 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for r in 1250000 10000000; do
  DALGO_PERSISTENT=1 timeout -k 10 120 python3 bench.py --rows $r --steps 400 --warmup 50 --secondary off --no-eval --launch env > $O/pers_$r.log 2>&1 || exit $?
  DALGO_ONE_KERNEL=1 timeout -k 10 120 python3 bench.py --rows $r --steps 400 --warmup 50 --secondary off --no-eval --launch env > $O/one_$r.log 2>&1 || exit $?
done
timeout -k 10 120 python3 bench.py --rows 1250000 --steps 400 --warmup 50 --secondary off > $O/auto_1250000.log 2>&1 || exit $?
