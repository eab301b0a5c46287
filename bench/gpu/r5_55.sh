set -o pipefail
# round 5, session 55: long-run kernel with a padded histogram (33-word rows: conflict-free
# scan reads); graph-build tests, probe twice, PageRank job
O=gpurun_out/r5_55
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_build.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/probes/run_sort_probe.py --no-census > $O/probe.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/pagerank_bench.py > $O/pr.log 2>&1 || exit $?
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pk55 -o pr -- python3 $R/bench/probes/run_sort_probe.py --no-census > $R/$O/probe_prof.log 2>&1 && \
python3 $R/bench/summarize_db.py /tmp/pk55/pr_results.db 40 > $R/$O/probe_stats.md
