set -o pipefail
# round 5, session 34: active / dense histories of small k-means runs (test coverage of both forms)
O=gpurun_out/r5_34
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python3 bench/probes/km_dense_choice.py > $O/hist.log 2>&1 || exit $?
