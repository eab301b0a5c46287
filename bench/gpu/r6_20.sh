set -o pipefail
# round 6, session 20: k-means with the drift-aware pruned K2 in every filtered iteration
O=gpurun_out/r6_20
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python3 bench/kmeans_bench.py --dense never > $O/km_sep_never.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/kmeans_bench.py --dense never --noise 4 > $O/km_ovl_never.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/kmeans_bench.py --dense always > $O/km_sep_always.log 2>&1 || exit $?
