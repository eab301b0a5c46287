set -o pipefail
# K4b phase-1 timing probes (DALGO_PB_PROBE: 1 = no stores, 2 = no LDS c reads)
O=$GRAFT_REPO_ROOT/gpurun_out/r3s2pb3
mkdir -p $O
export PYTHONPATH=$GRAFT_REPO_ROOT TMPDIR=/tmp
cd /tmp
for p in 0 1 2; do
  DALGO_PB_PROBE=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_$p -o pb -- python3 $GRAFT_REPO_ROOT/bench/pagerank_bench.py --steps 3 > $O/prof_$p.log 2>&1 || exit 1
  python3 $GRAFT_REPO_ROOT/bench/summarize_db.py /tmp/prof_$p/pb_results.db 30 > $O/stats_$p.md || exit 1
done
