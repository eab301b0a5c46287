set -o pipefail
# round 6, session 45: bench.py default (launch race) with the one-kernel / persistent row pools
O=gpurun_out/r6_45
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_lr.py -m gpu -x -q --timeout 100 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for rep in 1 2 3; do
  timeout -k 10 120 python3 bench.py --secondary off > $O/auto_r$rep.log 2>&1 || exit $?
  DALGO_LR_POOL1=0 DALGO_LR_POOL=0 timeout -k 10 120 python3 bench.py --secondary off > $O/auto_nopool_r$rep.log 2>&1 || exit $?
done
