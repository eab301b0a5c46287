set -o pipefail
# round 6, session 58: incremental K3 (km_dsegsum) with 16-B per-lane row loads
O=gpurun_out/r6_58
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_algos.py -m gpu -x -q -k "kmeans" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/kmeans_bench.py > $O/km_sep.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/kmeans_bench.py --noise 4 > $O/km_ovl.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/probes/km_phase_split.py --noise 4 > $O/ovl_phases.log 2>&1 || exit $?
