set -o pipefail
# round 6, session 48: kernel timeline of the one-rank PageRank job (host gaps inside the build)
O=gpurun_out/r6_48
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$O/prof -o pr -- python3 $GRAFT_REPO_ROOT/bench/pagerank_bench.py > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit $?
