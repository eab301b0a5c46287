set -o pipefail
# round 5, session 50: run-sort tile kernel: run starts and lengths from a ballot bitmap of the
# equal-key flags (PMC r5_49: VALU-bound); census, split-sort timing, job, kernel stats
O=gpurun_out/r5_50
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_build.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/probes/run_sort_probe.py > $O/probe.log 2>&1 || exit $?
DALGO_BUILD_SYNC=1 timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness > $O/prs.log 2>&1 || exit $?
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pk50 -o pr -- python3 $R/bench/probes/run_sort_probe.py > $R/$O/probe_prof.log 2>&1 && \
python3 $R/bench/summarize_db.py /tmp/pk50/pr_results.db 40 > $R/$O/probe_stats.md
