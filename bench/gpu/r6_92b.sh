set -o pipefail
# round 6, session 92b: decode block size, smaller values
O=gpurun_out/r6_92b
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
DALGO_GB_DEC_ROWS=4096 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_build.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_4096.log 2>&1 || exit $?
for r in 16384 8192 4096 16384 8192 4096; do
  DALGO_GB_DEC_ROWS=$r timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness > $O/pr_dec${r}_$RANDOM.log 2>&1 || exit $?
done
