set -o pipefail
mkdir -p gpurun_out/r3b
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r3b/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3b/bench_prof.log 2>&1; echo "prof rc=$?"
DALGO_ROCTX=1 timeout -k 10 120 rocprofv3 --marker-trace --kernel-trace -d gpurun_out/r3b/marker -o run --output-format csv -- python3 optimization/ssgd.py --device cuda --synthetic 200000,256 --n-iterations 20 --quiet --no-plot --metrics-out gpurun_out/r3b/ssgd_metrics.jsonl > gpurun_out/r3b/marker.log 2>&1; echo "marker rc=$?"
