set -o pipefail
# round 6, session 86: K4b at the W = 8 per-rank share (native layout of ranks 0 and 7):
# phase-2 work items nent/2048 (the then W > 1 default) vs fewer; three calls over
# 2048/768/1024, 512/384/768 and 256/192/128 (r6_86, r6_86b, r6_86c); DALGO_PB_ITEMS_MULTI was
# the W > 1 knob then, replaced by items = DALGO_PB_ITEMS / sqrt(W) (dalgo/ops/graph.py pb_items)
O=gpurun_out/r6_86
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for it in 2048 768 1024; do
  DALGO_PB_ITEMS_MULTI=$it timeout -k 10 300 python3 bench/pagerank_share.py --reps 1 --spmv-iters 50 > $O/share_items$it.log 2>&1 || exit $?
done
