set -o pipefail
# K4b (two-level propagation-blocked SpMV): numerics, then scale-26 bench + kernel profile
O=gpurun_out/r3s2pb${PB_TAG:-}
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_algos.py -k "pb_spmv or blocked" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_pb.log 2>&1 && \
timeout -k 10 300 python bench/pagerank_bench.py --spmv blocked > $O/pagerank_blocked.log 2>&1 && \
timeout -k 10 300 python bench/pagerank_bench.py --spmv blocked --chunk 524288 > $O/pagerank_blocked_c512k.log 2>&1 && \
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_pb -o pb -- python3 $GRAFT_REPO_ROOT/bench/pagerank_bench.py --spmv blocked --steps 5 > $GRAFT_REPO_ROOT/$O/prof_pb.log 2>&1
