set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/r3e
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-include-regex "pr_spmv|pr_update" -d gpurun_out/r3e/pmc_x3 -o run --output-format csv -- python3 bench/pagerank_bench.py --scale 26 --steps 3 --warmup 1 --spmv xcd > gpurun_out/r3e/x3.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE --kernel-include-regex "pr_spmv|pr_update" -d gpurun_out/r3e/pmc_x4 -o run --output-format csv -- python3 bench/pagerank_bench.py --scale 26 --steps 3 --warmup 1 --spmv xcd > gpurun_out/r3e/x4.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "pr_spmv|pr_update" -d gpurun_out/r3e/pmc_x1 -o run --output-format csv -- python3 bench/pagerank_bench.py --scale 26 --steps 3 --warmup 1 --spmv xcd > gpurun_out/r3e/x1.log 2>&1
