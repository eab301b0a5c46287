set -o pipefail
O=gpurun_out/r3s2sweep
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for ch in 1048576 4194304 16777216 67108864; do
  timeout -k 10 300 python bench/pagerank_bench.py --chunk $ch > $O/pr_c$ch.log 2>&1 || exit 1
done
timeout -k 10 300 python bench/pagerank_bench.py --bin-width 8192 > $O/pr_bw8k.log 2>&1
