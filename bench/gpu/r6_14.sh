set -o pipefail
# round 6, session 14: radix pass timing experiments (no look-back / no write)
O=gpurun_out/r6_14
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for x in 0 1 2 3; do DALGO_RS_XP=$x timeout -k 10 200 python3 bench/probes/sort_bench.py > $O/xp$x.log 2>&1 || exit $?; done
