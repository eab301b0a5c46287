set -o pipefail
# round 5, session 56: wave tier with a 128-key network for runs of 65-128 keys (tree) vs
# the 256-key network for all (experiment build), A/B/A; graph-build tests
O=gpurun_out/r5_56
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_build.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/probes/run_sort_probe.py --no-census > $O/w2.log 2>&1 || exit $?
DALGO_EXT_LIB=$PWD/bench/variants/wave4.so timeout -k 10 300 python3 bench/probes/run_sort_probe.py --no-census > $O/w4.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/probes/run_sort_probe.py --no-census > $O/w2b.log 2>&1 || exit $?
