set -o pipefail
O=gpurun_out/r3s2t2
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_algos.py -k "pb_spmv or blocked or pagerank" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_pb.log 2>&1 && \
timeout -k 10 300 python bench/pagerank_bench.py > $O/pagerank.log 2>&1 && \
timeout -k 10 300 python bench/pagerank_bench.py --semantics standard > $O/pagerank_standard.log 2>&1 && \
timeout -k 10 600 python bench/scaling_projection.py --only pagerank > $O/proj_pagerank.log 2>&1
