set -o pipefail
O=gpurun_out/r3list2
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lr.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_lr.log 2>&1 && \
timeout -k 10 300 python bench/lr_list_probe.py > $O/probe.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 --rows 1250000 > $O/bench_share8.log 2>&1 && \
DALGO_LR_LIST=0 timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 --rows 1250000 > $O/bench_share8_walk.log 2>&1 && \
DALGO_LR_LIST=0 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_walk.log 2>&1 && \
timeout -k 10 300 python bench/k1_timeline.py --list 1250000 10000000 > $O/timeline_list.log 2>&1
