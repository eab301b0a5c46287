set -o pipefail
# round 5, session 5: near/far candidate tiles (k-means job), pruned ALS / closure
# variants, kernel trace of the native PageRank build
O=gpurun_out/r5_5
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_algos.py -m gpu -q -k "kmeans or als or tc_step or closure" --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $O/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python3 bench/kmeans_bench.py > $O/km.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/kmeans_bench.py --noise 4 > $O/km_n4.log 2>&1 || exit $?
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pk55 -o pr -- python3 $R/bench/pagerank_bench.py --no-witness > $R/$O/pr_prof.log 2>&1 && \
python3 $R/bench/summarize_db.py /tmp/pk55/pr_results.db 40 > $R/$O/pr_stats.md && \
python3 $R/bench/timeline_db.py /tmp/pk55/pr_results.db --min-us 200 > $R/$O/pr_timeline.md
