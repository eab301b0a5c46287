set -o pipefail
O=gpurun_out/r3s2bw
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for bw in 16384 8192 16384 8192; do
  timeout -k 10 300 python bench/pagerank_bench.py --steps 20 --bin-width $bw >> $O/pr_bw$bw.log 2>&1 || exit 1
done
