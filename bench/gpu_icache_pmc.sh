# K1 start-up: instruction-cache behaviour at the 8-GPU per-rank share (1.25M rows)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/icache
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/icache/avail.txt 2>&1 || true
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INST_CYCLES[A-Z_]*" gpurun_out/icache/avail.txt | sort -u > gpurun_out/icache/names.txt || true
cat gpurun_out/icache/names.txt
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --kernel-trace -d gpurun_out/icache/p1 -o k1 --output-format csv -- python3 bench.py --rows 1250000 --steps 50 --warmup 5 --launch env > gpurun_out/icache/p1.log 2>&1
echo rc=$?
