set -o pipefail
# round 6, session 24: split relabel (DALGO_GB_RELABEL_PASSES) in the sharded build's owner partition
O=gpurun_out/r6_24
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
DALGO_GB_RELABEL_PASSES=3 timeout -k 10 200 python3 -u -m pytest tests/test_gpu_graph_build.py -m gpu -x -q -k owner --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for p in 1 2 3 4; do
  DALGO_GB_RELABEL_PASSES=$p timeout -k 10 200 python3 bench/pagerank_share.py --ranks 0 > $O/share_p$p.log 2>&1 || exit $?
done
