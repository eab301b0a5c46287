set -o pipefail
# round 6, session 23: kernel split of the W=8 per-rank build share
O=gpurun_out/r6_23
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o share -- python3 $GRAFT_REPO_ROOT/bench/pagerank_share.py --ranks 0 --reps 1 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit $?
