set -o pipefail
# round 5, session 42: kernel timeline of the current native PageRank build
O=gpurun_out/r5_42
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pk42 -o pr -- python3 $R/bench/pagerank_bench.py --no-witness --pool-gb 0 > $R/$O/pr_prof.log 2>&1 && \
python3 $R/bench/summarize_db.py /tmp/pk42/pr_results.db 50 > $R/$O/pr_stats.md && \
python3 $R/bench/timeline_db.py /tmp/pk42/pr_results.db --min-us 0 > $R/$O/pr_timeline.md
