set -o pipefail
O=gpurun_out/r4_46
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 python bench/kmeans_bench.py > $O/km.log 2>&1
