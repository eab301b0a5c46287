# PageRank overlapped ghost exchange: numerics (accumulate pass, 2-rank script), and the
# one-GPU cost of splitting the SpMV by source at each rank share (scale 26)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prov
timeout -k 10 300 python -u -m pytest tests/test_gpu_algos.py tests/test_gpu_multirank.py -x -v --timeout 200 --timeout-method thread -k "pr_spmv or pagerank or closure" > gpurun_out/prov/pytest.log 2>&1 && tail -2 gpurun_out/prov/pytest.log && \
timeout -k 10 500 python -u bench/scaling_projection.py --only pagerank > gpurun_out/prov/proj.log 2>&1 && tail -3 gpurun_out/prov/proj.log
