set -o pipefail
# round 6, session 89: K4b bin width 8192 vs 16384 again, with the nent/768 work items
O=gpurun_out/r6_89
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for bw in 16384 8192 16384 8192 16384 8192; do
  timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness --bin-width $bw > $O/pr_bw${bw}_$RANDOM.log 2>&1 || exit $?
done
