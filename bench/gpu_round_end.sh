# round-end re-check on one MI355X: GPU suite, smoke, headline + LR-family benches,
# k-means / PageRank / misc benches (all on the current tree)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/end
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/end/pytest_gpu.log 2>&1 && tail -1 gpurun_out/end/pytest_gpu.log && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/end/smoke.log 2>&1 && tail -1 gpurun_out/end/smoke.log && \
timeout -k 10 200 python bench.py > gpurun_out/end/bench_ssgd.log 2>&1 && \
timeout -k 10 200 python bench.py --algo bmuf --steps 20 --warmup 3 > gpurun_out/end/bench_bmuf.log 2>&1 && \
timeout -k 10 200 python bench.py --algo easgd --steps 50 --warmup 5 > gpurun_out/end/bench_easgd.log 2>&1 && \
timeout -k 10 200 python bench.py --algo gd --steps 20 --warmup 3 > gpurun_out/end/bench_gd.log 2>&1 && \
timeout -k 10 300 python bench/kmeans_bench.py > gpurun_out/end/kmeans.log 2>&1 && \
timeout -k 10 300 python bench/pagerank_bench.py --steps 5 > gpurun_out/end/pagerank.log 2>&1 && \
for f in gpurun_out/end/bench_*.log gpurun_out/end/kmeans.log gpurun_out/end/pagerank.log; do echo $f; tail -1 $f | cut -c1-400; done
