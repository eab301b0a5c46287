set -o pipefail
mkdir -p gpurun_out/r4_10
export PYTHONPATH=$PWD
timeout -k 10 200 python bench/probes/k1_blocks.py --rows 2500000 --iters 300 --tbs 192,256,512 --fgs 8 --reps 3 > gpurun_out/r4_10/k1_2m5.log 2>&1 && \
timeout -k 10 200 python bench/probes/k1_blocks.py --rows 5000000 --iters 300 --tbs 192,256,512 --fgs 8 --reps 3 > gpurun_out/r4_10/k1_5m.log 2>&1 && \
timeout -k 10 200 python bench/probes/k1_blocks.py --rows 1250000 --iters 500 --tbs 192,224,256 --fgs 8 --reps 3 > gpurun_out/r4_10/k1_1m25.log 2>&1
