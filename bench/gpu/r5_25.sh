set -o pipefail
# round 5, session 25: small D2H read latencies; dense K2 top-2 with one min3 per 4 keys (k-means A/B)
O=gpurun_out/r5_25
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 100 python3 bench/probes/d2h_probe.py > $O/d2h.log 2>&1 || exit $?
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_algos.py -m gpu -x -q -k "kmeans" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for n in 1 4; do
  timeout -k 10 200 python3 bench/kmeans_bench.py --noise $n > $O/km_n$n.log 2>&1 || exit $?
done
