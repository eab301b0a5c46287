set -o pipefail
# round 6, session 61: bench.py at 8 gloo ranks sharing one GPU, output streamed to a file
O=gpurun_out/r6_61
mkdir -p $O
export PYTHONPATH=$PWD TMPDIR=/tmp DALGO_ALLOW_SHARED_SPIN=1
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 8 --backend gloo --rows 400000 --steps 5 --warmup 2 --secondary off > $O/b8_nosec.log 2>&1 || exit $?
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr 127.0.0.1 --master-port 29562 bench.py --gpus 8 --backend gloo --rows 400000 --steps 5 --warmup 2 --secondary-steps 5 --secondary-warmup 2 --km-rows 2000000 --pr-scale 16 --km-pool-gb 8 --pr-pool-gb 8 > $O/b8_sec.log 2>&1 || exit $?
