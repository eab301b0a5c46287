set -o pipefail
# round 6, session 84: K4b phase-2 work items again, 3 runs each (run-to-run spread ~2 %)
O=gpurun_out/r6_84
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for it in 768 512 1024 640 768 512 1024 640 768 512 1024 640; do
  DALGO_PB_ITEMS=$it timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness > $O/pr_items${it}_$RANDOM.log 2>&1 || exit $?
done
