set -o pipefail
O=gpurun_out/r4_9
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_gpu_algos.py -k "kmeans" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 && \
timeout -k 10 300 python bench/kmeans_bench.py > $O/km.log 2>&1 && \
timeout -k 10 300 python bench/kmeans_bench.py --no-witness > $O/km2.log 2>&1 && \
for A in bmuf easgd ma gd; do
  timeout -k 10 400 python bench.py --algo $A --steps 20 --warmup 5 > $O/bench_$A.log 2>&1 || exit 1
done
