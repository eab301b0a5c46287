set -o pipefail
# round 6, session 29: XCD-aware logical blocks in the owner partition
O=gpurun_out/r6_29
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graph_build.py -m gpu -x -q -k owner --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for g in 1024 2048 4096; do
  DALGO_GB_OWNER_BLOCKS=$g timeout -k 10 200 python3 bench/pagerank_share.py --ranks 0 --reps 3 > $O/share_g$g.log 2>&1 || exit $?
done
