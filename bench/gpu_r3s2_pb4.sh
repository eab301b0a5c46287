set -o pipefail
# K4b XCD chunk-group A/B (DALGO_PB_XCDG) + numerics
O=gpurun_out/r3s2pb4
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_algos.py -k "pb_spmv or blocked or pagerank" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_pb.log 2>&1 || exit 1
for g in 0 8 32 1; do
  DALGO_PB_XCDG=$g timeout -k 10 300 python bench/pagerank_bench.py > $O/pagerank_xcdg$g.log 2>&1 || exit 1
done
