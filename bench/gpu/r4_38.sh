set -o pipefail
# final state: full GPU tier + smoke + headline bench + PageRank and k-means benches
O=gpurun_out/r4_38
mkdir -p $O
export PYTHONPATH=$PWD
( time timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider --durations=25 ) > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 python bench/pagerank_bench.py > $O/pagerank.log 2>&1 && \
timeout -k 10 300 python bench/kmeans_bench.py > $O/kmeans.log 2>&1
