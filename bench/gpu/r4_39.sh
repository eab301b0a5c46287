#!/bin/bash
# PMC passes (kernel-trace only, one counter set per run) for the round-4 kernels:
# k-means K2 (plain first pass + candidate-pruned filtered form) and K4b.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp PYTHONPATH=$PWD
mkdir -p gpurun_out/r4_39
SETS=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
      "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
      "SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_MFMA SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE")
WL=("kmeans:bench/kmeans_bench.py --rows 20000000 --iters 5 --no-witness"
    "pagerank:bench/pagerank_bench.py --scale 26 --steps 5 --no-witness")
for w in "${WL[@]}"; do
  name=${w%%:*}; cmd=${w#*:}
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "kmeans_assign_pipe|kmeans_assign16|pb_gather|pb_accum" \
      -d gpurun_out/r4_39/pmc_${name}_$i -o run --output-format csv -- python3 $cmd \
      > gpurun_out/r4_39/pmc_${name}_$i.log 2>&1 || { echo "pmc $name pass $i failed (rc=$?)"; exit 1; }
  done
done
python3 bench/summarize_pmc.py gpurun_out > gpurun_out/r4_39/pmc_r4.md
