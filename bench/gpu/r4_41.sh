set -o pipefail
# final kernel traces: k-means job (16x16 full pass) and PageRank
O=gpurun_out/r4_41
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pk41 -o km -- python3 $R/bench/kmeans_bench.py --no-witness > $R/$O/km_prof.log 2>&1 && \
python3 $R/bench/timeline_db.py /tmp/pk41/km_results.db --min-us 20 > $R/$O/km_timeline.md && \
python3 $R/bench/summarize_db.py /tmp/pk41/km_results.db 30 > $R/$O/km_stats.md && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pk41 -o pr -- python3 $R/bench/pagerank_bench.py > $R/$O/pr_prof.log 2>&1 && \
python3 $R/bench/summarize_db.py /tmp/pk41/pr_results.db 40 > $R/$O/pr_stats.md
