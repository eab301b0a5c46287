# K2 one-wave-per-SIMD variants (55-59) vs the default 52: numerics, then an interleaved sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/k2w
timeout -k 10 300 python -u -m pytest tests/test_gpu_algos.py -x -q --timeout 120 --timeout-method thread -k "pipelined and (55 or 56 or 57 or 58 or 59 or ties)" > gpurun_out/k2w/pytest.log 2>&1 && tail -2 gpurun_out/k2w/pytest.log && \
timeout -k 10 300 python -u bench/kmeans_assign_sweep.py --rows 20000000 --variants 52,55,56,57,58,59 --rounds 5 > gpurun_out/k2w/sweep20m.log 2>&1 && cat gpurun_out/k2w/sweep20m.log
