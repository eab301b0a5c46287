set -o pipefail
# round 5, session 8: K4b phase 1 (4 stores per step + packed scan) A/B, native build
# phase split, PageRank kernel trace, GPU suite
O=gpurun_out/r5_8
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_algos.py tests/test_gpu_graph_build.py -m gpu -q -k "native or degree or pagerank or pb_" --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $O/tests.log
[ $rc -le 1 ] || exit $rc
for v in in-tree pbprev in-tree pbprev; do
  if [ $v = in-tree ]; then L=""; else L=$PWD/dalgo/_xp_$v.so; fi
  DALGO_EXT_LIB=$L timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness --steps 20 > $O/pr_$v.log 2>&1 || exit $?
  grep -h '"job_ms"' $O/pr_$v.log >> $O/pr_ab.log
done
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pk58 -o pr -- python3 $R/bench/pagerank_bench.py --no-witness > $R/$O/pr_prof.log 2>&1 && \
python3 $R/bench/summarize_db.py /tmp/pk58/pr_results.db 40 > $R/$O/pr_stats.md && \
python3 $R/bench/timeline_db.py /tmp/pk58/pr_results.db --min-us 200 > $R/$O/pr_timeline.md && \
cd $R && timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_all.log 2>&1
