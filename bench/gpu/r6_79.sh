set -o pipefail
# round 6, session 79: the opt-in shared-GPU multi-rank set (K11 / persistent / fallback
# rehearsals, ranks sharing one GPU) after the device-counter re-arm change
O=gpurun_out/r6_79
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp DALGO_GPU_SHARED_TESTS=1
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_multirank.py -m gpu_shared -v --timeout 300 --timeout-method thread > $O/shared.log 2>&1 || exit $?
