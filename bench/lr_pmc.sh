#!/bin/bash
# PMC counters for the fused LR gradient kernel (separate passes; kernel-trace only).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
CMD="python3 bench/lr_kernel_sweep.py --variants 2,3 --blocks 256 --rounds 1 --reps 3"
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" \
           "TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/lr_pmc_$i -o run --output-format csv -- $CMD > gpurun_out/lr_pmc_$i.log 2>&1 || echo "pass $i failed"
done
