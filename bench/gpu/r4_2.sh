set -o pipefail
# round 4: k-means fused-epilogue iterations + pruned K1 validation
O=gpurun_out/r4_2
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_gpu_algos.py tests/test_gpu_lr.py -k "kmeans or lr or sync or rows or pagerank or pb_ or pr_" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 && \
timeout -k 10 300 python bench/kmeans_bench.py > $O/km_b1.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 && \
DALGO_GPU_SHARED_TESTS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py -k "fused_xgmi and graph or launch_calibration" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_shared.log 2>&1 && \
timeout -k 10 120 ./bench/probes/hbm_probe 16 > $O/hbm.log 2>&1 && \
timeout -k 10 300 python bench/pagerank_bench.py > $O/pagerank.log 2>&1 && \
cd /tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pk1 -o km -- python3 $R/bench/kmeans_bench.py --no-witness > $R/$O/km_prof.log 2>&1 && \
python3 $R/bench/timeline_db.py /tmp/pk1/km_results.db --min-us 50 > $R/$O/timeline_b1.md && \
python3 $R/bench/summarize_db.py /tmp/pk1/km_results.db 30 > $R/$O/stats_b1.md
