set -o pipefail
# round 6, session 60: the 8-rank shared-GPU bench rehearsal with reduced secondary sizes
O=gpurun_out/r6_60
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp DALGO_GPU_SHARED_TESTS=1
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_multirank.py -m gpu_shared -x -v -s -k "eight_ranks" --timeout 450 --timeout-method thread > $O/shared.log 2>&1 || exit $?
