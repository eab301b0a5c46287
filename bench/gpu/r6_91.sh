set -o pipefail
# round 6, session 91: one-kernel SSGD step, K1 workgroups per launch (3 runs each)
O=gpurun_out/r6_91
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for nb in 256 384 512 256 384 512 256 384 512; do
  DALGO_LR_BLOCKS=$nb DALGO_ONE_KERNEL=1 timeout -k 10 120 python3 bench.py --steps 200 --warmup 30 --secondary off --no-eval --launch env > $O/one_b${nb}_$RANDOM.log 2>&1 || exit $?
done
