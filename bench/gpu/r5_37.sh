set -o pipefail
# round 5, session 37: first k-means pass in 4 row parts, each part's sorted K3 on a side
# stream under the next part's K2
O=gpurun_out/r5_37
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_algos.py -m gpu -x -q -k "kmeans" --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for n in 1 4 1; do
  timeout -k 10 200 python3 bench/kmeans_bench.py --noise $n >> $O/km_n$n.log 2>&1 || exit $?
done
