set -o pipefail
# round-3 session-2 closing validation: GPU tier (default set), smoke, headline bench (1 GPU
# and the 8-GPU per-rank share), k-means, PageRank (K4b + pull), closure, misc
O=gpurun_out/r3s2final2
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 --rows 1250000 > $O/bench_share8.log 2>&1 && \
timeout -k 10 300 python bench/kmeans_bench.py > $O/kmeans.log 2>&1 && \
timeout -k 10 300 python bench/pagerank_bench.py > $O/pagerank.log 2>&1 && \
timeout -k 10 300 python bench/pagerank_bench.py --spmv pull > $O/pagerank_pull.log 2>&1 && \
timeout -k 10 300 python bench/closure_bench.py > $O/closure.log 2>&1 && \
timeout -k 10 300 python bench/misc_bench.py > $O/misc.log 2>&1
