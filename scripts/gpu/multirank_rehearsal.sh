# bench.py at world 2 and 4 on ONE GPU (ranks share cuda:0; RCCL code paths over a gloo group),
# then the 1-GPU bench under rocprofv3 kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AVENIR_COMM_BACKEND=rccl-emul timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 2 --rows-per-gpu 268435456 > gpurun_out/rehearsal_w2.log 2>&1 &&
AVENIR_COMM_BACKEND=rccl-emul timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 4 --steps 10 --warmup 2 --rows-per-gpu 268435456 > gpurun_out/rehearsal_w4.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/bprof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 > gpurun_out/bench_prof.log 2>&1
