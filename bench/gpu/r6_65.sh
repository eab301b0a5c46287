set -o pipefail
# round 6, session 65: K4b destination bin width 8192 vs 16384 (LDS: 2 vs 1 accumulating blocks per CU)
O=gpurun_out/r6_65
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for rep in 1 2; do
  for bw in 16384 8192; do
    timeout -k 10 300 python3 bench/pagerank_bench.py --bin-width $bw > $O/pr_bw${bw}_r$rep.log 2>&1 || exit $?
  done
done
