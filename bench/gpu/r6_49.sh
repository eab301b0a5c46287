set -o pipefail
# round 6, session 49: decode offsets scanned as two rows (torch outer-dim scan was 2.6 ms)
O=gpurun_out/r6_49
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_build.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/pagerank_bench.py > $O/pr.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/pagerank_share.py --ranks 0 > $O/share.log 2>&1 || exit $?
