set -o pipefail
# round 6, session 98: rehearsal of the final tree (cell-count pass batched too)
O=gpurun_out/r6_98
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q --durations=25 --timeout 280 --timeout-method thread > $O/gpu_all.log 2>&1
rc=$?
echo "gpu suite rc=$rc" >> $O/gpu_all.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 560 python3 bench.py > $O/bench.log 2>&1 || exit $?
