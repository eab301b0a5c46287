set -o pipefail
# round 6, session 87: K4b at the W = 2 / 4 / 8 per-rank shares with items = 768 / sqrt(W)
# (the new default) against nent / 2048 (the old one)
O=gpurun_out/r6_87
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for w in 2 4 8; do
  timeout -k 10 300 python3 bench/pagerank_share.py --world $w --ranks 0 --reps 1 --spmv-iters 50 > $O/share_w${w}_default.log 2>&1 || exit $?
  DALGO_PB_ITEMS=$((2048 * 1000 / 1000)) timeout -k 10 300 python3 -c "import sys, math; sys.argv=['x','--world','$w','--ranks','0','--reps','1','--spmv-iters','50']; import dalgo.ops.graph as G; G.pb_items=lambda world: 2048; sys.path.insert(0,'bench'); import runpy; runpy.run_path('bench/pagerank_share.py', run_name='__main__')" > $O/share_w${w}_2048.log 2>&1 || exit $?
done
