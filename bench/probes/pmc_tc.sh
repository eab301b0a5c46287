#!/bin/bash
# PMC passes (kernel-trace only, one counter set per run) for the K9 closure step variants.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
SETS=("SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"
      "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
      "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE")
for v in 1 3; do
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "tc_step" \
      -d gpurun_out/pmc_tc${v}_$i -o run --output-format csv -- python3 bench/probes/tc_only.py --variant $v \
      > gpurun_out/pmc_tc${v}_$i.log 2>&1 || { echo "pmc tc$v pass $i failed (rc=$?)"; exit 1; }
  done
done
echo pmc-done
