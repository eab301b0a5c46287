set -o pipefail
# round 6, session 56: the row pool forced into the fused xGMI (K11) paths, ranks sharing one GPU
O=gpurun_out/r6_56
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp DALGO_GPU_SHARED_TESTS=1 DALGO_LR_POOL_MIN_ROWS=0
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_multirank.py -m gpu_shared -x -v -k "fused_xgmi or launch_calibration" --timeout 300 --timeout-method thread > $O/shared.log 2>&1 || exit $?
