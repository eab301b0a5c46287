set -o pipefail
# round 5, session 4: 16x16 K2 prologue (dot2 norms, no sign flip, SGPR DMA addressing):
# k-means numerics, A/B vs the previous commit, PMC
O=gpurun_out/r5_4
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_algos.py tests/test_gpu_graph_build.py -m gpu -q -k "kmeans or native or degree" --timeout 120 --timeout-method thread > $O/km_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $O/km_tests.log
[ $rc -le 1 ] || exit $rc
for v in in-tree prev in-tree prev; do
  if [ $v = in-tree ]; then L=""; else L=$PWD/dalgo/_xp_$v.so; fi
  DALGO_EXT_LIB=$L timeout -k 10 120 python3 bench/probes/k2_full.py >> $O/ab.log 2>&1 || exit $?
done
timeout -k 10 200 python3 bench/kmeans_bench.py > $O/km.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/pagerank_bench.py > $O/pr.log 2>&1 || exit $?
SETS=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE")
cd /tmp
i=1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc ${SETS[0]} --kernel-include-regex "assign16" \
  -d /tmp/pmc_new -o run --output-format csv -- python3 $R/bench/probes/k2_full.py --reps 2 > $R/$O/pmc_new.log 2>&1 || exit $?
find /tmp/pmc_new -name "*counter_collection.csv" -exec cp {} $R/$O/pmc_new.csv \;
