#!/bin/bash
# Kernel-level profiles of the headline workloads (rocprofv3 kernel trace + stats).
# Usage (on the GPU box): bash bench/profile_all.sh  -> gpurun_out/prof_*/
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for w in "ssgd:bench.py --steps 20 --warmup 5" \
         "kmeans:bench/kmeans_bench.py --rows 20000000 --steps 3" \
         "ssgd_small:bench.py --steps 200 --warmup 20 --rows 1250000" \
         "pagerank:bench/pagerank_bench.py --steps 5" \
         "misc:bench/misc_bench.py"; do
  name=${w%%:*}; cmd=${w#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$name -o run --output-format csv -- python3 $cmd > gpurun_out/prof_$name.log 2>&1
done
