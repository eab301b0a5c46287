set -o pipefail
# round 6, session 54: 16x16x32 candidate K2 also right after the full pass (--dense never)
O=gpurun_out/r6_54
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python3 bench/kmeans_bench.py --dense never > $O/km_sep_never.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/kmeans_bench.py --dense never --noise 4 > $O/km_ovl_never.log 2>&1 || exit $?
