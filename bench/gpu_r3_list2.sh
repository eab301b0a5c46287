set -o pipefail
O=gpurun_out/r3list
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python bench/k1_timeline.py 1250000 10000000 > $O/timeline_walk.log 2>&1 && \
timeout -k 10 300 python bench/k1_timeline.py --list 1250000 10000000 > $O/timeline_list.log 2>&1
