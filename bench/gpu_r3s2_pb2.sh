set -o pipefail
# K4b chunk-size sweep + PMC of the current kernels
O=gpurun_out/r3s2pb2
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp
for ch in 262144 1048576 2097152; do
  timeout -k 10 300 python bench/pagerank_bench.py --spmv blocked --chunk $ch > $O/pagerank_blocked_c$ch.log 2>&1 || exit 1
done
bash bench/pmc_pb.sh
