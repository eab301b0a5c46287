set -o pipefail
# SSGD per-rank step at the W = 8 share (1.25M x 1024 bf16 rows): kernel trace per form
O=gpurun_out/r4_5
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
cd /tmp && \
DALGO_ONE_KERNEL=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/pk5 -o s -- python3 $R/bench.py --rows 1250000 --steps 200 --warmup 20 --no-eval --launch env > $R/$O/prof.log 2>&1 && \
python3 $R/bench/timeline_db.py /tmp/pk5/s_results.db --min-us 0 > $R/$O/timeline.md && \
python3 $R/bench/summarize_db.py /tmp/pk5/s_results.db 20 > $R/$O/stats.md && \
DALGO_ONE_KERNEL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/pk6 -o s -- python3 $R/bench.py --rows 1250000 --steps 200 --warmup 20 --no-eval --launch env > $R/$O/prof1.log 2>&1 && \
python3 $R/bench/timeline_db.py /tmp/pk6/s_results.db --min-us 0 > $R/$O/timeline1.md && \
python3 $R/bench/summarize_db.py /tmp/pk6/s_results.db 20 > $R/$O/stats1.md
