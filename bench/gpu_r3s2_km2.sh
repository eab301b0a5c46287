set -o pipefail
O=gpurun_out/r3s2km2
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -k "kmeans or km_" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_km.log 2>&1 || exit 1
timeout -k 10 300 python bench/kmeans_bench.py > $O/kmeans.log 2>&1
