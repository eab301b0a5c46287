set -o pipefail
# round 6, session 17: SSGD at the 8-GPU per-rank share (1.25M x 1024) -- K1 grid sweep
O=gpurun_out/r6_17
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for b in 160 192 224 240 256; do
  for a in 256; do
    DALGO_ONE_KERNEL=1 DALGO_LR_BLOCKS=$b DALGO_LR_RPB_ALIGN=$a timeout -k 10 120 python3 bench.py --rows 1250000 --steps 400 --warmup 50 --secondary off --no-eval --launch env > $O/b${b}_a$a.log 2>&1 || exit $?
  done
done
