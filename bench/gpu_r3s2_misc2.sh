set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r3s2misc2
mkdir -p $O
export PYTHONPATH=$GRAFT_REPO_ROOT TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --algo bmuf > $O/bench_bmuf.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --algo easgd > $O/bench_easgd.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_pr -o pr -- python3 $GRAFT_REPO_ROOT/bench/pagerank_bench.py > $O/prof_pr.log 2>&1 && \
python3 $GRAFT_REPO_ROOT/bench/summarize_db.py /tmp/prof_pr/pr_results.db 30 > $O/stats_pr.md
