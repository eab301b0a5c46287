set -o pipefail
# round 6, session 44: A/B of the one-kernel row pool at the headline size (alternating runs)
O=gpurun_out/r6_44
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for rep in 1 2 3 4 5; do
  for pf in 0 0.1; do
    DALGO_LR_POOL1=$pf DALGO_ONE_KERNEL=1 timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --secondary off --no-eval --launch env > $O/one_p${pf}_r$rep.log 2>&1 || exit $?
  done
done
