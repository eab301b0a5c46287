set -o pipefail
# round 5, session 9: allocator pool before the PageRank / k-means clocks, W = 1 deal fast
# path; then bench.py end to end (headline + secondary configs)
O=gpurun_out/r5_9
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python3 bench/pagerank_bench.py > $O/pr.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/kmeans_bench.py > $O/km.log 2>&1 || exit $?
timeout -k 10 580 python3 bench.py > $O/bench.log 2>&1
