set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/r3j
DALGO_LAUNCH=env timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/r3j/tr_ps -o run --output-format csv -- python3 bench.py --gpus 1 --steps 100 --warmup 20 --rows 1250000 --launch env --no-eval > gpurun_out/r3j/ps.log 2>&1; echo rc=$?
DALGO_ONE_KERNEL=1 timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/r3j/tr_ok -o run --output-format csv -- python3 bench.py --gpus 1 --steps 100 --warmup 20 --rows 1250000 --launch env --no-eval > gpurun_out/r3j/ok.log 2>&1; echo rc=$?
