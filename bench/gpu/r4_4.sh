set -o pipefail
mkdir -p gpurun_out/r4_4
export PYTHONPATH=$PWD
timeout -k 10 300 python bench/probes/km_k2_ab.py --rows 50000000 --at 2 > gpurun_out/r4_4/ab2.log 2>&1 && \
timeout -k 10 300 python bench/probes/km_k2_ab.py --rows 50000000 --at 3 > gpurun_out/r4_4/ab3.log 2>&1
