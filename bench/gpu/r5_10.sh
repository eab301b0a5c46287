set -o pipefail
# round 5, session 10: PageRank job -- allocator pool vs none, degree relabeling vs none,
# host-synchronised phase split
O=gpurun_out/r5_10
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for args in "--pool-gb 0" "--pool-gb 96" "--pool-gb 0 --no-reorder" "--pool-gb 0"; do
  tag=$(echo $args | tr -d ' -')
  timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness $args > $O/pr_$tag.log 2>&1 || exit $?
  DALGO_BUILD_SYNC=1 timeout -k 10 200 python3 bench/pagerank_bench.py --no-witness $args > $O/prs_$tag.log 2>&1 || exit $?
done
