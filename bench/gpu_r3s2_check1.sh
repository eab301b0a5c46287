set -o pipefail
# round-3 session-2 first check: new K4b kernels first (numerics), then the GPU tier
# (default set), smoke, headline bench, k-means, PageRank pull vs K4b at scale 26
O=gpurun_out/r3s2c1
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_algos.py -k "pb_spmv or blocked" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_pb.log 2>&1 && \
timeout -k 10 300 python bench/pagerank_bench.py --spmv blocked > $O/pagerank_blocked.log 2>&1 && \
timeout -k 10 300 python bench/pagerank_bench.py > $O/pagerank_pull.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 && \
timeout -k 10 300 python bench/kmeans_bench.py > $O/kmeans.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_pb -o pb -- python3 $GRAFT_REPO_ROOT/bench/pagerank_bench.py --spmv blocked --steps 5 > $GRAFT_REPO_ROOT/$O/prof_pb.log 2>&1
