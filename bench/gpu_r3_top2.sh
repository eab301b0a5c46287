set -o pipefail
mkdir -p gpurun_out/r3n
export PYTHONPATH=$PWD TMPDIR=/tmp
for c in 0 1 2; do DALGO_KM_TOP2_CFG=$c timeout -k 10 300 python bench/kmeans_bench.py > gpurun_out/r3n/top2_$c.log 2>&1 || exit 1; done
