set -o pipefail
mkdir -p gpurun_out/r3w
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python bench/kmeans_bench.py > gpurun_out/r3w/kmeans.log 2>&1
