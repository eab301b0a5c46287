set -o pipefail
# round 5, session 2: software-pipelined 16x16 K2 full pass -- numerics, k-means job, kernel trace
O=gpurun_out/r5_2
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_algos.py -m gpu -q -k kmeans --timeout 120 --timeout-method thread > $O/km_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $O/km_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python3 bench/kmeans_bench.py > $O/km.log 2>&1 && \
timeout -k 10 200 python3 bench/kmeans_bench.py --noise 4 > $O/km_n4.log 2>&1 && \
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pk52 -o km -- python3 $R/bench/kmeans_bench.py --no-witness > $R/$O/km_prof.log 2>&1 && \
python3 $R/bench/summarize_db.py /tmp/pk52/km_results.db 30 > $R/$O/km_stats.md && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pk52 -o pr -- python3 $R/bench/pagerank_bench.py --no-witness > $R/$O/pr_prof.log 2>&1 && \
python3 $R/bench/summarize_db.py /tmp/pk52/pr_results.db 40 > $R/$O/pr_stats.md
