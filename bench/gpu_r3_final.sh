set -o pipefail
# round-3 closing validation: GPU test tier (default set, no gpu_shared), smoke, the
# headline bench at 1 GPU and at the 8-GPU per-rank share, and the secondary benches
O=gpurun_out/r3final
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 --rows 1250000 > $O/bench_share8.log 2>&1 && \
timeout -k 10 300 python bench/kmeans_bench.py > $O/kmeans.log 2>&1 && \
timeout -k 10 300 python bench/pagerank_bench.py --spmv xcd > $O/pagerank_xcd.log 2>&1 && \
timeout -k 10 300 python bench/closure_bench.py > $O/closure.log 2>&1 && \
timeout -k 10 300 python bench/misc_bench.py > $O/misc.log 2>&1
