set -o pipefail
# round 6, session 26: source-bucketed shuffle for the sharded PageRank build
O=gpurun_out/r6_26
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_build.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_multirank.py -m gpu -x -q -k "pagerank_native_build_ranks or secondary_two" --timeout 300 --timeout-method thread > $O/mr.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/pagerank_share.py --ranks 0,7 > $O/share.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/pagerank_share.py --ranks 0 --direct > $O/share_direct.log 2>&1 || exit $?
