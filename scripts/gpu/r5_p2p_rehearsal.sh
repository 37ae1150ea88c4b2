# bench.py at world 2 and 4 on ONE GPU (ranks share cuda:0, gloo group for the library path):
# exercises the count-table all-reduce picker and the peer-mapped kernel on the NB side stream
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
AVENIR_COMM_BACKEND=rccl-emul timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 2 --rows-per-gpu 67108864 > gpurun_out/r5/rehearsal_w2.log 2>&1 &&
AVENIR_COMM_BACKEND=rccl-emul timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 4 --steps 10 --warmup 2 --rows-per-gpu 67108864 > gpurun_out/r5/rehearsal_w4.log 2>&1
