set -o pipefail
# round 5, session 49: PMC of the run-sort tile kernel (probe at scale 26; kernel-trace
# passes, one counter set each)
O=gpurun_out/r5_49
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
SETS=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
      "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT")
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  cd /tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $set --kernel-include-regex "gb_run" \
    -d /tmp/pmc49/pmc_run_$i -o run --output-format csv -- python3 $R/bench/probes/run_sort_probe.py > $R/$O/pmc_run_$i.log 2>&1 || exit $?
  cd $R
done
python3 bench/summarize_pmc.py /tmp/pmc49 > $O/pmc.md
mkdir -p $O/csv && for d in /tmp/pmc49/pmc_*; do cp $d/run_counter_collection.csv $O/csv/$(basename $d).csv; done
