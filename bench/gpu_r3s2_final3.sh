set -o pipefail
# round-3 session-2 last validation: GPU tier, smoke, SSGD / BMUF / EASGD benches, k-means,
# PageRank K4b (+ kernel profile summarised on the box)
O=gpurun_out/r3s2final3
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --algo bmuf > $O/bench_bmuf.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --algo easgd > $O/bench_easgd.log 2>&1 && \
timeout -k 10 300 python bench/kmeans_bench.py > $O/kmeans.log 2>&1 && \
timeout -k 10 300 python bench/pagerank_bench.py > $O/pagerank.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_pr -o pr -- python3 $R/bench/pagerank_bench.py > $R/$O/prof_pr.log 2>&1 && \
python3 $R/bench/summarize_db.py /tmp/prof_pr/pr_results.db 30 > $R/$O/stats_pr.md
