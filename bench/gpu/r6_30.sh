set -o pipefail
# round 6, session 30: XCD-aware one-rank key pass, grid sweep (W=1 PageRank build phases)
O=gpurun_out/r6_30
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for g in 16384 2048 4096 8192; do
  DALGO_GB_KEYS_BLOCKS=$g timeout -k 10 300 python3 bench/pagerank_bench.py > $O/pr_g$g.log 2>&1 || exit $?
done
