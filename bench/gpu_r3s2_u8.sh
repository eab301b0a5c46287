set -o pipefail
O=gpurun_out/r3s2u8
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for u in 0 1 0 1; do
  DALGO_PB_U8=$u timeout -k 10 300 python bench/pagerank_bench.py --steps 20 >> $O/pr_u8_$u.log 2>&1 || exit 1
done
DALGO_PB_U8=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_algos.py -k "pb_spmv" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_u8.log 2>&1
