set -o pipefail
# round 6, session 15: radix sort v3 (early aggregates, 16-wide look-back)
O=gpurun_out/r6_15
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_radix_sort.py -m gpu -x -q --timeout 100 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/probes/sort_bench.py > $O/sort_native.log 2>&1 || exit $?
