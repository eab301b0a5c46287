set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/r3h
for v in 60; do
DALGO_KM_VARIANT=$v timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES --kernel-include-regex "kmeans_assign" -d gpurun_out/r3h/pmc_$v -o run --output-format csv -- python3 bench/kmeans_bench.py --rows 20000000 --steps 2 > gpurun_out/r3h/pmc_$v.log 2>&1 || exit 1
done
