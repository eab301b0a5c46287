set -o pipefail
mkdir -p gpurun_out/r4_10
export PYTHONPATH=$PWD
timeout -k 10 200 python bench/probes/k1_blocks.py --rows 1250000 > gpurun_out/r4_10/k1_125.log 2>&1 && \
timeout -k 10 200 python bench/probes/k1_blocks.py --rows 10000000 --iters 100 > gpurun_out/r4_10/k1_10m.log 2>&1
