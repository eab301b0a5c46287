set -o pipefail
# kernel profiles of the k-means and PageRank benches (summaries written on the box)
O=$GRAFT_REPO_ROOT/gpurun_out/r3s2prof
mkdir -p $O
export PYTHONPATH=$GRAFT_REPO_ROOT TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_km -o km -- python3 $GRAFT_REPO_ROOT/bench/kmeans_bench.py > $O/prof_km.log 2>&1 && \
python3 $GRAFT_REPO_ROOT/bench/summarize_db.py /tmp/prof_km/km_results.db 30 > $O/stats_km.md && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_pr -o pr -- python3 $GRAFT_REPO_ROOT/bench/pagerank_bench.py > $O/prof_pr.log 2>&1 && \
python3 $GRAFT_REPO_ROOT/bench/summarize_db.py /tmp/prof_pr/pr_results.db 30 > $O/stats_pr.md
