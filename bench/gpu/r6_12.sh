set -o pipefail
# round 6, session 12: kernel split of the native radix sort
O=gpurun_out/r6_12
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o sort -- python3 $GRAFT_REPO_ROOT/bench/probes/sort_bench.py > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit $?
