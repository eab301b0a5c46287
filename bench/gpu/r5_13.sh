set -o pipefail
# round 5, session 13: dense top-2 16x16x32 K2 for filtered k-means iterations
O=gpurun_out/r5_13
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_algos.py -m gpu -x -q -k "kmeans" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for n in 1 4; do
  for m in auto never always; do
    timeout -k 10 200 python3 bench/kmeans_bench.py --noise $n --dense $m > $O/km_n${n}_$m.log 2>&1 || exit $?
  done
done
