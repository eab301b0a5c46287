set -o pipefail
# round 5, session 54: per-key rank tier up to 64 (tree) / 128 / 256 keys (experiment
# builds, bench/probes/build_variant.py); A/B/A on one box
O=gpurun_out/r5_54
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 bench/probes/run_sort_probe.py --no-census > $O/rank64.log 2>&1 || exit $?
for v in rank128 rank256; do
  DALGO_EXT_LIB=$PWD/bench/variants/$v.so timeout -k 10 300 python3 bench/probes/run_sort_probe.py --no-census > $O/$v.log 2>&1 || exit $?
done
timeout -k 10 300 python3 bench/probes/run_sort_probe.py --no-census > $O/rank64b.log 2>&1 || exit $?
