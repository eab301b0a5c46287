set -o pipefail
# round 6, session 83: K4b phase-1 wave tiles per work unit (tile length = unit / tiles)
O=gpurun_out/r6_83
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for t in 16 8 32 24 16 8 32 24 16 8 32 24; do
  DALGO_PB_TILES=$t timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness > $O/pr_tiles${t}_$RANDOM.log 2>&1 || exit $?
done
