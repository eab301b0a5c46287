set -o pipefail
# round 5, session 35: PMC passes (kernel-trace only, one counter set per run): k-means
# full-pass and dense filtered K2 (overlapping blobs, 20M rows); PageRank build kernels and
# K4b at scale 26
O=gpurun_out/r5_35
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
SETS=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
      "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
      "SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_MFMA SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"
      "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE")
WL=("kmeans|assign16|bench/kmeans_bench.py --rows 20000000 --noise 4 --no-witness"
    "pagerank|gb_|pb_gather|pb_accum|bench/pagerank_bench.py --steps 2 --no-witness")
for w in "${WL[@]}"; do
  name=${w%%|*}; rest=${w#*|}; cmd=${rest##*|}; regex=${rest%|*}
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    cd /tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "$regex" \
      -d /tmp/pmc35/pmc_${name}_$i -o run --output-format csv -- python3 $R/$cmd > $R/$O/pmc_${name}_$i.log 2>&1 || exit $?
    cd $R
  done
done
python3 bench/summarize_pmc.py /tmp/pmc35 > $O/pmc.md
mkdir -p $O/csv && for d in /tmp/pmc35/pmc_*; do cp $d/run_counter_collection.csv $O/csv/$(basename $d).csv; done
