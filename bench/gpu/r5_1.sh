set -o pipefail
# round 5, session 1: GPU suite, smoke, bench.py with the secondary configs, PageRank
# preprocessing kernel trace
O=gpurun_out/r5_1
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $O/gpu_tests.log
# a failed assertion (rc 1) leaves the GPU usable; a timeout / abort / crash ends the call
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 560 python3 bench.py > $O/bench.log 2>&1 && \
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pk51 -o pr -- python3 $R/bench/pagerank_bench.py --no-witness > $R/$O/pr_prof.log 2>&1 && \
python3 $R/bench/summarize_db.py /tmp/pk51/pr_results.db 40 > $R/$O/pr_stats.md
