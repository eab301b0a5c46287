set -o pipefail
# round 6, session 71: PageRank job with and without the degree relabel (current pipeline);
# entry-value / dloc buffers cleared only past the entries
O=gpurun_out/r6_71
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_graph_build.py tests/test_gpu_algos.py -k "graph or pagerank or pb_ or native or blocked" -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/pagerank_bench.py > $O/pr.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/pagerank_bench.py --no-reorder > $O/pr_noreorder.log 2>&1 || exit $?
