#!/bin/bash
# PMC passes (kernel-trace + one counter set each) for the K3 accumulate kernels
# (hist / scan / chunked scatter / segsum). Usage (GPU box): bash bench/pmc_kmeans_k3.sh
# -> gpurun_out/pmc_k3_<pass>/ ; summarise with bench/summarize_pmc.py or read the CSVs.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
SETS=("SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
      "WRITE_SIZE"
      "FETCH_SIZE")
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "scatter|hist|scan|segsum" \
    -d gpurun_out/pmc_k3_$i -o run --output-format csv -- \
    python3 bench/kmeans_bench.py --rows 20000000 --iters 3 --no-witness \
    > gpurun_out/pmc_k3_$i.log 2>&1 || { echo "pmc pass $i failed (rc=$?)"; exit 1; }
done
echo pmc_k3 done
