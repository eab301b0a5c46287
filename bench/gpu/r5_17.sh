set -o pipefail
# round 5, session 17: full GPU suite after the previous-cluster fallback fix; PageRank job
O=gpurun_out/r5_17
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_all.log 2>&1
rc=$?
echo "gpu suite rc=$rc" >> $O/gpu_all.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python3 bench/pagerank_bench.py > $O/pr.log 2>&1 || exit $?
DALGO_BUILD_SYNC=1 timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness > $O/prs.log 2>&1 || exit $?
