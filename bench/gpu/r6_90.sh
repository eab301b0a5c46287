set -o pipefail
# round 6, session 90: one-kernel SSGD step, pooled fraction of the rows (3 runs each)
O=gpurun_out/r6_90
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for pf in 0.1 0.05 0.15 0.2 0.1 0.05 0.15 0.2 0.1 0.05 0.15 0.2; do
  DALGO_LR_POOL1=$pf DALGO_ONE_KERNEL=1 timeout -k 10 120 python3 bench.py --steps 200 --warmup 30 --secondary off --no-eval --launch env > $O/one_p${pf}_$RANDOM.log 2>&1 || exit $?
done
