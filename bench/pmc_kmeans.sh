#!/bin/bash
# PMC passes (kernel-trace + one counter set each) for the k-means assign variants.
# Usage (GPU box): bash bench/pmc_kmeans.sh "5 11" -> gpurun_out/pmc_km_v<variant>_<pass>/
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
VARIANTS=${1:-"5 11"}
SETS=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
      "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC"
      "SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_MFMA SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE")
for v in $VARIANTS; do
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "assign" \
      -d gpurun_out/pmc_km_v${v}_$i -o run --output-format csv -- \
      python3 bench/kmeans_assign_sweep.py --rows 20000000 --variants $v --rounds 1 \
      > gpurun_out/pmc_km_v${v}_$i.log 2>&1 || { echo "pmc v$v pass $i failed (rc=$?)"; exit 1; }
  done
done
