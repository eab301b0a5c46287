set -o pipefail
# round 6, session 63: bench.py launch race length (steps per candidate form) vs the timed result
O=gpurun_out/r6_63
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for rep in 1 2; do
  for c in 20 50 100; do
    timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --secondary off --no-eval --cal-steps $c > $O/auto_c${c}_r$rep.log 2>&1 || exit $?
  done
done
