set -o pipefail
# round 6, session 77: PMC of the k-means job kernels with the 16x16x32 candidate K2 (CND16),
# separated blobs (noise 1: iterations 3-5 on the candidate form)
O=gpurun_out/r6_77
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
SETS=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
      "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
      "SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_MFMA SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"
      "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum")
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "kmeans|km_" \
    -d $O/pmc_km_$i -o run --output-format csv -- python3 bench/probes/km_phase_split.py --noise 1 \
    > $O/pmc_km_$i.log 2>&1 || exit $?
done
