set -o pipefail
# round 6, session 2: world-1 K11 tests, owner partition, sharded PageRank build rehearsals
# (2 / 3 gloo ranks), bench.py secondaries at 2 ranks, per-algorithm witness tolerances,
# W = 8 per-rank build share
O=gpurun_out/r6_2
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_k11.py tests/test_gpu_graph_build.py -m gpu -x -v -k "k11 or owner" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_multirank.py -m gpu -x -v -k "pagerank_native_build_ranks" --timeout 280 --timeout-method thread > $O/mr.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/pagerank_share.py > $O/share.log 2>&1 || exit $?
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_multirank.py -m gpu -x -v -k "secondary" --timeout 380 --timeout-method thread > $O/mr2.log 2>&1 || exit $?
