set -o pipefail
# round 6, session 82: K4b phase-1 work-unit size (E / units edges per unit)
O=gpurun_out/r6_82
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for u in 4096 2048 8192 16384 4096 2048 8192 16384 4096 2048 8192 16384; do
  DALGO_PB_UNITS=$u timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness > $O/pr_units${u}_$RANDOM.log 2>&1 || exit $?
done
