set -o pipefail
# round 6, session 57: K1 ring depth (rows kept ahead per wave) at the 8-GPU share and the headline size
O=gpurun_out/r6_57
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for rep in 1 2; do
  for ra in 2 1; do
    DALGO_LR_RING_AHEAD=$ra DALGO_ONE_KERNEL=1 timeout -k 10 120 python3 bench.py --rows 1250000 --steps 200 --warmup 20 --secondary off --no-eval --launch env > $O/one_1250000_ra${ra}_r$rep.log 2>&1 || exit $?
    DALGO_LR_RING_AHEAD=$ra DALGO_ONE_KERNEL=1 timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --secondary off --no-eval --launch env > $O/one_10M_ra${ra}_r$rep.log 2>&1 || exit $?
  done
done
