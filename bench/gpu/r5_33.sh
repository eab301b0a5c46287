set -o pipefail
# round 5, session 33: device-side dense / pruned K2 choice test
O=gpurun_out/r5_33
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_algos.py -m gpu -x -v -k "dense_choice" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
