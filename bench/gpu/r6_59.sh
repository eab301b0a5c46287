set -o pipefail
# round 6, session 59: the launch-calibration rehearsal after the "graph" label fix
O=gpurun_out/r6_59
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp DALGO_GPU_SHARED_TESTS=1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_multirank.py -m gpu_shared -x -v -k "launch_calibration or auto_selects or eight_ranks" --timeout 300 --timeout-method thread > $O/shared.log 2>&1 || exit $?
