set -o pipefail
# round 6, session 80: K4b phase-2 work items per iteration (hot-bin splitting: fewer,
# larger pieces = fewer 128 KB slabs to write and combine); two boxes: 2048/1024/512, then
# 1024/768/1536 (logs *_items<N>_<random>.log)
O=gpurun_out/r6_80
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for it in 2048 1024 512 2048 1024 512; do
  DALGO_PB_ITEMS=$it timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness > $O/pr_items${it}_$RANDOM.log 2>&1 || exit $?
done
