set -o pipefail
# round 5, session 52: split point of the key sort -- 6 radix passes over bits 4..51 (runs
# equal above bit 4: almost all of 1-2 keys) against 5 passes over bits 12..51
O=gpurun_out/r5_52
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 bench/probes/run_sort_probe.py --lo-bits 4 > $O/lo4.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/probes/run_sort_probe.py --lo-bits 12 --no-census > $O/lo12.log 2>&1 || exit $?
