set -o pipefail
# round 5, session 14: dense K2 with per-block moved-row lists; rocPRIM sort digit widths
O=gpurun_out/r5_14
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_algos.py -m gpu -x -q -k "kmeans" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for n in 1 4; do
  for m in auto always never; do
    timeout -k 10 200 python3 bench/kmeans_bench.py --noise $n --dense $m > $O/km_n${n}_$m.log 2>&1 || exit $?
  done
done
timeout -k 10 120 bench/probes/sort_probe 1060000000 52 > $O/sort52.log 2>&1 || exit $?
timeout -k 10 120 bench/probes/sort_probe 1060000000 40 > $O/sort40.log 2>&1 || exit $?
