set -o pipefail
# round 5, session 44: three-tier run sort (thread / wave / block), run-length census of the
# scale-26 keys, split-sort timing, PageRank job
O=gpurun_out/r5_44
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_build.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/probes/run_sort_probe.py > $O/probe.log 2>&1 || exit $?
DALGO_BUILD_SYNC=1 timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness > $O/prs.log 2>&1 || exit $?
