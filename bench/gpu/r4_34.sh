set -o pipefail
O=gpurun_out/r4_34
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_algos.py -k "pb_ or pagerank" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 && \
for r in 1 2; do
  timeout -k 10 300 python bench/pagerank_bench.py > $O/pr_new$r.log 2>&1 || exit 1
  DALGO_EXT_LIB=$PWD/dalgo/_xp_prev.so timeout -k 10 300 python bench/pagerank_bench.py > $O/pr_prev$r.log 2>&1 || exit 1
done
