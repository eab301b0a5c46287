set -o pipefail
# round 6, session 78: the 16x16x32 candidate K2 as 8-wave blocks (3 point groups per wave,
# 4 waves per SIMD, 37 spilled VGPRs) -- same 384-row tiles
O=gpurun_out/r6_78
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_algos.py -k "kmeans" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/kmeans_bench.py --no-witness > $O/sep.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/kmeans_bench.py --noise 4 --no-witness > $O/ovl.log 2>&1 || exit $?
