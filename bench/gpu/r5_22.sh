set -o pipefail
# round 5, session 22: K2 full pass with one 8-wave block per CU (half the centre-chunk
# traffic per point) vs two 4-wave blocks, A/B/A/B
O=gpurun_out/r5_22
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for v in "" "$PWD/dalgo/_xp_nw8.so" "" "$PWD/dalgo/_xp_nw8.so"; do
  DALGO_EXT_LIB=$v timeout -k 10 200 python3 bench/probes/k2_full.py >> $O/ab.log 2>&1 || exit $?
done
