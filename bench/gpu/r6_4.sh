set -o pipefail
# round 6, session 4: native ghost-list extraction + dealing kernel; W = 8 share again
O=gpurun_out/r6_4
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_build.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_multirank.py -m gpu -x -q -k "pagerank_native_build_ranks" --timeout 280 --timeout-method thread > $O/mr.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/pagerank_share.py --ranks 0 > $O/share.log 2>&1 || exit $?
