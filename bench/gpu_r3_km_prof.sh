set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/r3l
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3l/prof -o run --output-format csv -- python3 bench/kmeans_bench.py --rows 20000000 > gpurun_out/r3l/km.log 2>&1; echo rc=$?
