set -o pipefail
# round 5, session 12: PageRank job with the scale-16 process warm-up (vs cold), pool on/off
O=gpurun_out/r5_12
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for args in "--pool-gb 0" "--pool-gb 96" "--pool-gb 0 --no-warm"; do
  tag=$(echo $args | tr -d ' -')
  timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness $args > $O/pr_$tag.log 2>&1 || exit $?
done
DALGO_BUILD_SYNC=1 timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness --pool-gb 0 > $O/prs_poolgb0.log 2>&1 || exit $?
timeout -k 10 200 python3 bench/pagerank_bench.py > $O/pr_witness.log 2>&1 || exit $?
