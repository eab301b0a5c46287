set -o pipefail
# round 5, session 51: where the run-sort tile kernel's time goes -- the same probe on
# experiment builds (bench/probes/build_variant.py): no wave tier, no class networks, no
# short-run work at all (staging + equal-key bitmap only)
O=gpurun_out/r5_51
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 bench/probes/run_sort_probe.py --no-census > $O/base.log 2>&1 || exit $?
for v in nomid noclass noshort; do
  DALGO_EXT_LIB=$PWD/bench/variants/$v.so timeout -k 10 300 python3 bench/probes/run_sort_probe.py --no-census > $O/$v.log 2>&1 || exit $?
done
