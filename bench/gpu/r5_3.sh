set -o pipefail
# round 5, session 3: K2 full pass A/B (HEAD form, pipelined argmin with and without the
# pinned interleave) and PMC of the pipelined form
O=gpurun_out/r5_3
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
for v in in-tree old nopin in-tree old; do
  if [ $v = in-tree ]; then L=""; else L=$PWD/dalgo/_xp_$v.so; fi
  DALGO_EXT_LIB=$L timeout -k 10 120 python3 bench/probes/k2_full.py >> $O/ab.log 2>&1 || exit $?
done
SETS=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
      "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE")
cd /tmp
for v in in-tree old; do
  if [ $v = in-tree ]; then L=""; else L=$R/dalgo/_xp_$v.so; fi
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    DALGO_EXT_LIB=$L timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "assign16" \
      -d /tmp/pmc_${v}_${i} -o run --output-format csv -- python3 $R/bench/probes/k2_full.py --reps 2 > $R/$O/pmc_${v}_$i.log 2>&1 || exit $?
    cp /tmp/pmc_${v}_${i}/*counter_collection.csv $R/$O/pmc_${v}_$i.csv 2>/dev/null || find /tmp/pmc_${v}_${i} -name "*.csv" -exec cp {} $R/$O/ \;
  done
done
