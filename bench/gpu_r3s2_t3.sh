set -o pipefail
O=gpurun_out/r3s2t3
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_algos.py tests/test_gpu_multirank.py -k "pb_spmv or blocked or pagerank" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_pb.log 2>&1 && \
timeout -k 10 300 python bench/pagerank_bench.py > $O/pagerank.log 2>&1 && \
timeout -k 10 300 python bench/pagerank_bench.py --gpus 2 --backend gloo --scale 22 > $O/pagerank_2rank_gloo.log 2>&1
