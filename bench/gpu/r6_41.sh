set -o pipefail
# round 6, session 41: kernel trace of a 20-step persistent timed region (plain launch)
O=gpurun_out/r6_41
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp DALGO_PERSIST_COOP=0 DALGO_PERSISTENT=1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$O/prof -o pers -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --secondary off --no-eval --launch env > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit $?
