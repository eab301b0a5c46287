set -o pipefail
# k-means job kernel trace with the round-4 K2 changes
O=gpurun_out/r4_31
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pk31 -o km -- python3 $R/bench/kmeans_bench.py --no-witness > $R/$O/km_prof.log 2>&1 && \
python3 $R/bench/timeline_db.py /tmp/pk31/km_results.db --min-us 20 > $R/$O/timeline.md && \
python3 $R/bench/summarize_db.py /tmp/pk31/km_results.db 30 > $R/$O/stats.md
