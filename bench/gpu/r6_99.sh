set -o pipefail
# round 6, session 99: dense vs candidate K2 threshold with the 16x16x32 candidate form
# (overlapping blobs: iteration 3 has 74.8 % of the rows active, just under 0.75)
O=gpurun_out/r6_99
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for f in 0.7 0.75 0.7 0.75; do
  DALGO_KM_DENSE_FRACTION=$f timeout -k 10 200 python3 bench/kmeans_bench.py --noise 4 --no-witness > $O/ovl_f${f}_$RANDOM.log 2>&1 || exit $?
done
