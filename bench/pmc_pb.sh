#!/bin/bash
# PMC passes for the K4b propagation-blocked SpMV (pb_gather / pb_accum) at scale 26,
# plus the LDS atomic throughput probe. Usage (GPU box): bash bench/pmc_pb.sh
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/pmc_pb
mkdir -p $O
timeout -k 10 60 ./bench/probes/lds_atomic_probe > $O/lds_atomic_probe.log 2>&1 || exit 1
SETS=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"
      "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU"
      "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum"
      "TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE GRBM_COUNT")
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "pb_" \
    -d $O/p$i -o run --output-format csv -- python3 bench/pagerank_bench.py \
    --spmv blocked --steps 2 --warmup 1 > $O/p$i.log 2>&1
  rc=$?
  echo "pmc pb pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
