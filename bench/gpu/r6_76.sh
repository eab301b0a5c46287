set -o pipefail
# round 6, session 76: row pool with 8 sub-range counters (one per XCD) -- chunk size at the
# 8-GPU share and at the headline size
O=gpurun_out/r6_76
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_lr.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for cfg in "0 9" "0.15 7" "0.15 8" "0.15 9" "0.3 8"; do
  set -- $cfg
  DALGO_LR_POOL_MIN_ROWS=0 DALGO_LR_POOL=$1 DALGO_LR_POOL_SHIFT=$2 DALGO_PERSISTENT=1 timeout -k 10 120 python3 bench.py --rows 1250000 --steps 400 --warmup 50 --secondary off --no-eval --launch env > $O/pers125_p$1_s$2.log 2>&1 || exit $?
  DALGO_LR_POOL_MIN_ROWS=0 DALGO_LR_POOL1=$1 DALGO_LR_POOL_SHIFT=$2 DALGO_ONE_KERNEL=1 timeout -k 10 120 python3 bench.py --rows 1250000 --steps 400 --warmup 50 --secondary off --no-eval --launch env > $O/one125_p$1_s$2.log 2>&1 || exit $?
done
for cfg in "0.15 9" "0.15 8" "0.15 7"; do
  set -- $cfg
  DALGO_LR_POOL=$1 DALGO_LR_POOL_SHIFT=$2 DALGO_PERSISTENT=1 timeout -k 10 120 python3 bench.py --steps 200 --warmup 30 --secondary off --no-eval --launch env > $O/pers10M_p$1_s$2.log 2>&1 || exit $?
  DALGO_LR_POOL1=0.1 DALGO_LR_POOL_SHIFT=$2 DALGO_ONE_KERNEL=1 timeout -k 10 120 python3 bench.py --steps 200 --warmup 30 --secondary off --no-eval --launch env > $O/one10M_p0.1_s$2.log 2>&1 || exit $?
done
