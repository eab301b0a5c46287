set -o pipefail
# round 6, session 96: final-tree check after the run-tile A/B rebuilds (smoke + GPU suite)
O=gpurun_out/r6_96
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q --timeout 280 --timeout-method thread > $O/gpu_all.log 2>&1 || exit $?
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
