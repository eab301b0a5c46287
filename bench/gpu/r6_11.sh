set -o pipefail
# round 6, session 11: native LSD radix sort -- correctness, then A/B against rocPRIM
O=gpurun_out/r6_11
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_radix_sort.py -m gpu -x -v --timeout 100 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/probes/sort_bench.py > $O/sort_native.log 2>&1 || exit $?
DALGO_SORT=rocprim timeout -k 10 200 python3 bench/probes/sort_bench.py > $O/sort_rocprim.log 2>&1 || exit $?
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_build.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gtests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench/pagerank_bench.py > $O/pr.log 2>&1 || exit $?
