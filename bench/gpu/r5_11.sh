set -o pipefail
# round 5, session 11: kernel timeline of the native PageRank build (host gaps vs kernels)
O=gpurun_out/r5_11
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pk11 -o pr -- python3 $R/bench/pagerank_bench.py --no-witness --pool-gb 0 > $R/$O/pr_prof.log 2>&1 && \
python3 $R/bench/summarize_db.py /tmp/pk11/pr_results.db 50 > $R/$O/pr_stats.md && \
python3 $R/bench/timeline_db.py /tmp/pk11/pr_results.db --min-us 0 > $R/$O/pr_timeline.md
