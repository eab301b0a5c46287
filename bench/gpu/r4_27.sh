set -o pipefail
O=gpurun_out/r4_27
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_algos.py -k "kmeans" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 && \
timeout -k 10 300 python bench/kmeans_bench.py > $O/km1.log 2>&1 && \
timeout -k 10 300 python bench/kmeans_bench.py --no-witness > $O/km2.log 2>&1
