set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3s2proj8
mkdir -p $O
export PYTHONPATH=$GRAFT_REPO_ROOT TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_p8 -o p8 -- python3 $GRAFT_REPO_ROOT/bench/scaling_projection.py --only pagerank --worlds 8 > $O/proj8.log 2>&1 && \
python3 $GRAFT_REPO_ROOT/bench/summarize_db.py /tmp/prof_p8/p8_results.db 25 > $O/stats.md
