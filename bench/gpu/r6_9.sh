set -o pipefail
O=gpurun_out/r6_9
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
DALGO_KM_DRIFT_BALL=1 DALGO_KM_DRIFT_Q=0.9 timeout -k 10 300 python3 bench/probes/kmeans_bound_probe.py > $O/probe.log 2>&1 || exit $?
