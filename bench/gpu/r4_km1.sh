set -o pipefail
# round 4: where does k-means iteration 1 go? kernel timelines of the reference-shaped
# 5-iteration job (no untimed model warmup), bounds on and off
O=gpurun_out/r4km1
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
cd /tmp && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/pk1 -o km -- python3 $R/bench/kmeans_bench.py --warmup 0 --steps 5 > $R/$O/km_b1.log 2>&1 && \
python3 $R/bench/timeline_db.py /tmp/pk1/km_results.db --min-us 100 > $R/$O/timeline_b1.md && \
python3 $R/bench/summarize_db.py /tmp/pk1/km_results.db 30 > $R/$O/stats_b1.md && \
DALGO_KM_BOUNDS=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/pk0 -o km -- python3 $R/bench/kmeans_bench.py --warmup 0 --steps 5 > $R/$O/km_b0.log 2>&1 && \
python3 $R/bench/timeline_db.py /tmp/pk0/km_results.db --min-us 100 > $R/$O/timeline_b0.md && \
cd $R && timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
