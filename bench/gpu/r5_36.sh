set -o pipefail
# round 5, session 36: K4b phase 2 with 64-consecutive entries per atomic instruction
# (strided per-thread entries) vs groups of 4 consecutive entries per thread; A/B/A/B
O=gpurun_out/r5_36
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for v in in-tree strided in-tree strided; do
  L=""; [ $v = strided ] && L=$PWD/dalgo/_xp_strided.so
  DALGO_EXT_LIB=$L timeout -k 10 200 python3 bench/pagerank_bench.py --steps 20 > $O/pr_$v.log 2>&1 || exit $?
  cat $O/pr_$v.log >> $O/pr_ab.log
done
