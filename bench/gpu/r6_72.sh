set -o pipefail
# round 6, session 72: device counters re-armed after a failed launch
O=gpurun_out/r6_72
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_lr.py tests/test_gpu_k11.py -v -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1
