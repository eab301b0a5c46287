set -o pipefail
O=gpurun_out/r4_22
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pk22 -o p -- python3 $R/bench/pagerank_bench.py > $R/$O/prof.log 2>&1 && \
python3 $R/bench/summarize_db.py /tmp/pk22/p_results.db 40 > $R/$O/stats.md
