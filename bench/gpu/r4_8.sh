set -o pipefail
# local-SGD family on the headline config: exact device counts + held-out witness
O=gpurun_out/r4_8
mkdir -p $O
export PYTHONPATH=$PWD
for A in bmuf easgd ma gd; do
  timeout -k 10 400 python bench.py --algo $A --steps 20 --warmup 5 > $O/bench_$A.log 2>&1 || exit 1
done
