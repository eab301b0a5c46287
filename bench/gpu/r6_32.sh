set -o pipefail
# round 6, session 32: k-means job phase split per iteration (separated / overlapping blobs)
O=gpurun_out/r6_32
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python3 bench/probes/km_phase_split.py > $O/sep.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/probes/km_phase_split.py --noise 4 > $O/ovl.log 2>&1 || exit $?
