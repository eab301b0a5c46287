#!/bin/bash
# PMC counters (separate passes, kernel-trace only; never combined with other traces) for
# the hot kernels: K1 (LR gradient), K2/K3 (k-means), K9 (closure) + K6 (Monte Carlo).
# Usage (GPU box): bash bench/pmc_all.sh  -> gpurun_out/pmc_<workload>_<pass>/ ; then
#   python3 bench/summarize_pmc.py gpurun_out   (markdown table per kernel)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
SETS=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
      "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
      "SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_MFMA SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"
      "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum")
WL=("lr:bench.py --steps 20 --warmup 5 --no-eval --launch env"
    "kmeans:bench/kmeans_bench.py --rows 20000000 --iters 3 --no-witness"
    "misc:bench/misc_bench.py --mc-samples 2000000000 --als 20000,10000,32")
for w in "${WL[@]}"; do
  name=${w%%:*}; cmd=${w#*:}
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    timeout -k 10 180 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "dalgo::" \
      -d gpurun_out/pmc_${name}_$i -o run --output-format csv -- python3 $cmd \
      > gpurun_out/pmc_${name}_$i.log 2>&1 || { echo "pmc $name pass $i failed (rc=$?)"; exit 1; }
  done
done
