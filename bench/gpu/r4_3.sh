set -o pipefail
# round 4: candidate-pruned K2 for the filtered k-means iterations
O=gpurun_out/r4_3
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
timeout -k 10 300 python -u -m pytest tests/test_gpu_algos.py -k "kmeans" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 && \
timeout -k 10 300 python bench/kmeans_bench.py > $O/km_cand.log 2>&1 && \
timeout -k 10 300 python bench/probes/km_cand_stats.py --rows 20000000 > $O/cand_stats.log 2>&1 && \
timeout -k 10 300 python bench/probes/km_cand_stats.py --rows 20000000 --no-candidates > $O/nocand_stats.log 2>&1 && \
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pk1 -o km -- python3 $R/bench/kmeans_bench.py --no-witness > $R/$O/km_prof.log 2>&1 && \
python3 $R/bench/timeline_db.py /tmp/pk1/km_results.db --min-us 20 > $R/$O/timeline.md && \
python3 $R/bench/summarize_db.py /tmp/pk1/km_results.db 30 > $R/$O/stats.md
