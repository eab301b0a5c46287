set -o pipefail
# round 6, session 34: PMC of the native radix sort's kernels (count / scatter)
O=gpurun_out/r6_34
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp DALGO_SORT=native
SETS=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
      "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
      "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum")
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "rs_" \
    -d $O/pmc_rs_$i -o run --output-format csv -- python3 bench/probes/sort_bench.py \
    > $O/pmc_rs_$i.log 2>&1 || exit $?
done
