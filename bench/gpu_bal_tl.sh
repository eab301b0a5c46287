# K1 timeline with / without count-balanced ranges (1.25M and 10M rows)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/baltl
timeout -k 10 200 python bench/k1_timeline.py 1250000 10000000 --fine 8 > gpurun_out/baltl/static.log 2>&1 && \
timeout -k 10 200 python bench/k1_timeline.py 1250000 10000000 --balance --fine 8 > gpurun_out/baltl/balance.log 2>&1 && \
cat gpurun_out/baltl/static.log gpurun_out/baltl/balance.log | grep rows
