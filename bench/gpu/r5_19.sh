set -o pipefail
# round 5, session 19: kernel timeline of the k-means job (iteration 1 split)
O=gpurun_out/r5_19
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/km19 -o km -- python3 $R/bench/kmeans_bench.py --no-witness > $R/$O/km_prof.log 2>&1 && \
python3 $R/bench/summarize_db.py /tmp/km19/km_results.db 30 > $R/$O/km_stats.md && \
python3 $R/bench/timeline_db.py /tmp/km19/km_results.db --min-us 0 > $R/$O/km_timeline.md
