set -o pipefail
# round 5, session 53: run sort with per-key ranks for runs of 2-64 keys (replaces the
# thread / class-network / wave-rank tiers); LR GPU tests with device-generated data
O=gpurun_out/r5_53
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_build.py tests/test_gpu_lr.py -m gpu -x -q --durations=8 --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/probes/run_sort_probe.py --no-census > $O/probe.log 2>&1 || exit $?
DALGO_BUILD_SYNC=1 timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness > $O/prs.log 2>&1 || exit $?
