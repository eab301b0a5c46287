#!/bin/bash
# PMC passes (kernel-trace only) for k-means assign variants, one rocprofv3 run per
# counter set. Usage (GPU box): bash bench/pmc_km_variants.sh 5,14 -> gpurun_out/pmc_kmv_<set>/
#   then python3 bench/summarize_pmc.py gpurun_out
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
VARS=${1:-5,14}
SETS=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
      "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
      "SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_MFMA SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE")
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "kmeans_assign" \
    -d gpurun_out/pmc_kmv_$i -o run --output-format csv -- \
    python3 bench/kmeans_assign_sweep.py --rows 20000000 --variants $VARS --rounds 1 \
    > gpurun_out/pmc_kmv_$i.log 2>&1 || { echo "pmc pass $i failed (rc=$?)"; exit 1; }
done
