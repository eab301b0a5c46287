set -o pipefail
O=gpurun_out/r4_11
mkdir -p $O
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_gpu_lr.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench1.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench2.log 2>&1
