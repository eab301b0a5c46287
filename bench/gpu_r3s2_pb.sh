set -o pipefail
# K4b (two-level propagation-blocked SpMV): numerics, then scale-26 bench variants + kernel profile
O=gpurun_out/r3s2pb${PB_TAG:-}
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_algos.py -k "pb_spmv or blocked or pagerank" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_pb.log 2>&1 && \
timeout -k 10 300 python bench/pagerank_bench.py > $O/pagerank_blocked.log 2>&1 && \
DALGO_PR_FUSE=0 timeout -k 10 300 python bench/pagerank_bench.py > $O/pagerank_blocked_nofuse.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_pb -o pb -- python3 $GRAFT_REPO_ROOT/bench/pagerank_bench.py --steps 5 > $GRAFT_REPO_ROOT/$O/prof_pb.log 2>&1 && python3 $GRAFT_REPO_ROOT/bench/summarize_db.py /tmp/prof_pb/pb_results.db 30 > $GRAFT_REPO_ROOT/$O/stats.md
