set -o pipefail
# round 5, session 18: driver-shaped bench.py run (headline + secondary configs); kernel
# stats of the k-means job (dense / pruned filtered K2 chosen on the device)
O=gpurun_out/r5_18
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
timeout -k 10 560 python3 bench.py > $O/bench.log 2>&1 || exit $?
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/km18 -o km -- python3 $R/bench/kmeans_bench.py --noise 4 --no-witness > $R/$O/km_prof.log 2>&1 && \
python3 $R/bench/summarize_db.py /tmp/km18/km_results.db 30 > $R/$O/km_n4_stats.md
