set -o pipefail
mkdir -p gpurun_out/r4_10
export PYTHONPATH=$PWD
timeout -k 10 300 python bench/probes/k1_blocks.py --rows 10000000 --iters 200 --tbs 128,160,192,224,256,448,512,768 --fgs 8 --reps 3 > gpurun_out/r4_10/k1_10m_sweep.log 2>&1
