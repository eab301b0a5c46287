set -o pipefail
# round 6, session 19: rocPRIM onesweep configurations for the build's key sorts
O=gpurun_out/r6_19
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for c in 0 1 2; do DALGO_RS_CFG=$c timeout -k 10 200 python3 bench/probes/sort_bench.py > $O/cfg$c.log 2>&1 || exit $?; done
