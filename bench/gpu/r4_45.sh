set -o pipefail
O=gpurun_out/r4_45
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_algos.py -k "kmeans or sort or accumulate" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 && \
timeout -k 10 300 python bench/kmeans_bench.py > $O/km_new0.log 2>&1 && \
for r in 1 2; do
  timeout -k 10 300 python bench/kmeans_bench.py --no-witness > $O/km_new$r.log 2>&1 || exit 1
  DALGO_EXT_LIB=$PWD/dalgo/_xp_head2.so timeout -k 10 300 python bench/kmeans_bench.py --no-witness > $O/km_old$r.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o km -- python bench/kmeans_bench.py --no-witness > $O/prof.log 2>&1
