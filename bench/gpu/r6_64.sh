set -o pipefail
# round 6, session 64: kernel statistics of the full bench.py run (headline + BASELINE configs #3-#5)
O=gpurun_out/r6_64
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py > $GRAFT_REPO_ROOT/$O/bench.log 2>&1 || exit $?
