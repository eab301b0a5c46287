set -o pipefail
O=gpurun_out/r3s2mc
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -k "monte or mc_pi" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_mc.log 2>&1 && \
timeout -k 10 300 python bench/misc_bench.py > $O/misc.log 2>&1
