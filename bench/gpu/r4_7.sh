set -o pipefail
O=gpurun_out/r4_7
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
timeout -k 10 200 python -u -m pytest tests/test_gpu_algos.py -k "pb_ or pagerank" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 && \
timeout -k 10 300 python bench/pagerank_bench.py > $O/pr1.log 2>&1 && \
timeout -k 10 300 python bench/pagerank_bench.py > $O/pr2.log 2>&1 && \
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pk7 -o p -- python3 $R/bench/pagerank_bench.py > $R/$O/prof.log 2>&1 && \
python3 $R/bench/summarize_db.py /tmp/pk7/p_results.db 8 > $R/$O/stats.md
