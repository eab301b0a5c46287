set -o pipefail
# round 4: k-means device-count iterations: GPU tests of the k-means kernels, the
# reference-shaped 5-iteration job (bounds on / off) and its kernel timeline
O=gpurun_out/r4km1
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_gpu_algos.py -k kmeans -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_km.log 2>&1 && \
timeout -k 10 300 python bench/kmeans_bench.py > $O/km_b1.log 2>&1 && \
timeout -k 10 300 python bench/kmeans_bench.py --no-bound-filter > $O/km_b0.log 2>&1 && \
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pk1 -o km -- python3 $R/bench/kmeans_bench.py --no-witness > $R/$O/km_prof.log 2>&1 && \
python3 $R/bench/timeline_db.py /tmp/pk1/km_results.db --min-us 50 > $R/$O/timeline_b1.md && \
python3 $R/bench/summarize_db.py /tmp/pk1/km_results.db 30 > $R/$O/stats_b1.md
