set -o pipefail
# round 5, session 24: vectorised decode key loads (job A/B vs r5_23); host-side cProfile of the build
O=gpurun_out/r5_24
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 200 python3 bench/pagerank_bench.py > $O/pr.log 2>&1 || exit $?
DALGO_BUILD_SYNC=1 timeout -k 10 200 python3 bench/probes/pr_build_profile.py > $O/build_cprofile.log 2>&1 || exit $?
