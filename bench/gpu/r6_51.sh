set -o pipefail
# round 6, session 51: kernel timeline of the k-means job (overlapping blobs)
O=gpurun_out/r6_51
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$O/prof -o km -- python3 $GRAFT_REPO_ROOT/bench/kmeans_bench.py --noise 4 --no-witness > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit $?
