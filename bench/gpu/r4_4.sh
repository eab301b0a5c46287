set -o pipefail
mkdir -p gpurun_out/r4_4
export PYTHONPATH=$PWD
timeout -k 10 300 python bench/probes/km_cand_stats.py --rows 20000000 > gpurun_out/r4_4/cand_stats.log 2>&1
