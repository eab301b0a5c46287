set -o pipefail
# round 5, session 7: K2 barrier before the last sub-tile (A/B), K4b phase-1 stores 8 -> 4
# per step (A/B), native graph build with sort-based degrees and fused dedup, traces
O=gpurun_out/r5_7
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_algos.py tests/test_gpu_graph_build.py -m gpu -q -k "kmeans or native or degree or pagerank or pb_ or als or tc_step" --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $O/tests.log
[ $rc -le 1 ] || exit $rc
for v in in-tree prev in-tree prev; do
  if [ $v = in-tree ]; then L=""; else L=$PWD/dalgo/_xp_$v.so; fi
  DALGO_EXT_LIB=$L timeout -k 10 120 python3 bench/probes/k2_full.py >> $O/ab.log 2>&1 || exit $?
done
for v in in-tree pbprev in-tree pbprev; do
  if [ $v = in-tree ]; then L=""; else L=$PWD/dalgo/_xp_$v.so; fi
  DALGO_EXT_LIB=$L timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness --steps 20 > $O/pr_$v.log 2>&1 || exit $?
  grep -h '"job_ms"' $O/pr_$v.log >> $O/pr_ab.log
done
timeout -k 10 200 python3 bench/kmeans_bench.py > $O/km.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/pagerank_bench.py > $O/pr.log 2>&1 || exit $?
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pk57 -o pr -- python3 $R/bench/pagerank_bench.py --no-witness > $R/$O/pr_prof.log 2>&1 && \
python3 $R/bench/summarize_db.py /tmp/pk57/pr_results.db 40 > $R/$O/pr_stats.md && \
python3 $R/bench/timeline_db.py /tmp/pk57/pr_results.db --min-us 200 > $R/$O/pr_timeline.md
