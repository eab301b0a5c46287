set -o pipefail
# round 6, session 27: kernel split of the source-bucketed shuffle at the W=8 share
O=gpurun_out/r6_27
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o share -- python3 $GRAFT_REPO_ROOT/bench/pagerank_share.py --ranks 0 --reps 1 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit $?
