#!/bin/bash
# Multi-rank rehearsal of the headline bench on a ONE-GPU box: N ranks share the GPU and talk over
# gloo (GPU tensors staged through host memory, parallel/comm.py).  Exercises the sharded sweep
# (C1 all-gather, C5 decision broadcast, C4 checkpoint moves) with the real HIP kernels; RCCL itself
# only runs on a multi-GPU node.   usage: bash scripts/rehearse_multirank.sh [N]
set -e
N=${1:-2}
mkdir -p gpurun_out
MOPT_COMM_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node "$N" --master-addr 127.0.0.1 --master-port 29511 \
    bench.py --gpus "$N" --steps 64 --warmup 16 > gpurun_out/rehearse_$N.log 2>&1
tail -1 gpurun_out/rehearse_$N.log
