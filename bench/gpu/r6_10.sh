set -o pipefail
# round 6, session 10: byte-map remote-source marks (sharded build), k-means defaults
O=gpurun_out/r6_10
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_build.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_multirank.py -m gpu -x -q -k "pagerank_native_build_ranks" --timeout 280 --timeout-method thread > $O/mr.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/pagerank_share.py --ranks 0 > $O/share.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/kmeans_bench.py > $O/km_sep.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/kmeans_bench.py --noise 4 > $O/km_ovl.log 2>&1 || exit $?
