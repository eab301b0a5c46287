#!/bin/bash
# PMC passes (kernel-trace only, one counter set per run) for the PageRank K4 pull SpMV
# at R-MAT scale 26 (1.07B edges, the BASELINE PageRank config on one GPU).
# Usage (GPU box): bash bench/pmc_pagerank.sh -> gpurun_out/pmc_pr_<i>/ ; then
#   python3 bench/summarize_pmc.py gpurun_out --prefix pmc_pr   (markdown per kernel)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
SCALE=${SCALE:-26}
SETS=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
      "SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
      "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
      "TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE")
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "pr_spmv|pr_update" \
    -d gpurun_out/pmc_pr_$i -o run --output-format csv -- python3 bench/pagerank_bench.py \
    --scale $SCALE --steps 3 --warmup 1 > gpurun_out/pmc_pr_$i.log 2>&1
  rc=$?
  echo "pmc pagerank pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
