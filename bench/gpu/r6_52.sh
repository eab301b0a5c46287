set -o pipefail
# round 6, session 52: candidate-pruned K2 on the 16x16x32 tiling (DALGO_KM_CAND16)
O=gpurun_out/r6_52
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_algos.py -m gpu -x -q -k "candidates or cand16" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for f in "" "--noise 4"; do
  tag=$( [ -z "$f" ] && echo sep || echo ovl )
  timeout -k 10 200 python3 bench/kmeans_bench.py $f > $O/km_${tag}_base.log 2>&1 || exit $?
  DALGO_KM_CAND16=1 timeout -k 10 200 python3 bench/kmeans_bench.py $f > $O/km_${tag}_c16.log 2>&1 || exit $?
  DALGO_KM_CAND16=1 DALGO_KM_DENSE_FRACTION=0.9 timeout -k 10 200 python3 bench/kmeans_bench.py $f > $O/km_${tag}_c16_d09.log 2>&1 || exit $?
done
