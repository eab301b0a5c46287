set -o pipefail
# round 5, session 64: end-of-round rehearsal 5 (final tree) -- full GPU suite, smoke(), driver-shaped bench.py
O=gpurun_out/r5_64
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --durations=30 --timeout 120 --timeout-method thread > $O/gpu_all.log 2>&1
rc=$?
echo "gpu suite rc=$rc" >> $O/gpu_all.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 560 python3 bench.py > $O/bench.log 2>&1 || exit $?
