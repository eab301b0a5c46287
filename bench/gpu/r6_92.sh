set -o pipefail
# round 6, session 92: keys per decode block of the PageRank build (DALGO_GB_DEC_ROWS)
O=gpurun_out/r6_92
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
DALGO_GB_DEC_ROWS=32768 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_build.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_32768.log 2>&1 || exit $?
for r in 65536 32768 131072 16384; do
  DALGO_GB_DEC_ROWS=$r timeout -k 10 300 python3 bench/pagerank_bench.py > $O/pr_dec${r}_w.log 2>&1 || exit $?
done
for r in 65536 32768 131072 16384 65536 32768 131072 16384; do
  DALGO_GB_DEC_ROWS=$r timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness > $O/pr_dec${r}_$RANDOM.log 2>&1 || exit $?
done
