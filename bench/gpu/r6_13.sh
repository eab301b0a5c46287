set -o pipefail
# round 6, session 13: radix sort v2 (plain LDS histogram, pipelined ranking)
O=gpurun_out/r6_13
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_radix_sort.py -m gpu -x -q --timeout 100 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/probes/sort_bench.py > $O/sort_native.log 2>&1 || exit $?
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o sort -- python3 $GRAFT_REPO_ROOT/bench/probes/sort_bench.py > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit $?
