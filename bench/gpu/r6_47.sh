set -o pipefail
# round 6, session 47: the row pool in plain gradient launches (per-step SSGD, BMUF / EASGD at W = 1)
O=gpurun_out/r6_47
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_lr.py -m gpu -x -q --timeout 100 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for rep in 1 2; do
  timeout -k 10 200 python3 bench.py > $O/auto_r$rep.log 2>&1 || exit $?
done
DALGO_LR_POOL1=0 DALGO_LR_POOL=0 timeout -k 10 200 python3 bench.py > $O/auto_nopool.log 2>&1 || exit $?
