set -o pipefail
# round 5, session 32: tile list sorted by the rocPRIM u64 sort (torch.sort cold: 32 ms); (no flag array,
# no nonzero); incremental K3 with dword row loads
O=gpurun_out/r5_32
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_graph_build.py tests/test_gpu_algos.py -m gpu -x -q -k "native or cell or degree or rank_by or pagerank or blocked or pb_ or kmeans" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/pagerank_bench.py > $O/pr.log 2>&1 || exit $?
DALGO_BUILD_SYNC=1 timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness > $O/prs.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/kmeans_bench.py > $O/km_n1.log 2>&1 || exit $?
