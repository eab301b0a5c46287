set -o pipefail
# round 5, session 27: host profile of the build after the device-side work split
O=gpurun_out/r5_27
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
DALGO_BUILD_SYNC=1 timeout -k 10 200 python3 bench/probes/pr_build_profile.py --top 60 > $O/build_cprofile.log 2>&1 || exit $?
