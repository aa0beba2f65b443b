#!/bin/bash
# Rehearse the multi-rank DDP path on a 1-GPU box: 2 ranks share device 0 with gloo as the
# gradient transport (RCCL refuses two ranks on one device).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLMPI_GLOO_DEVICE=cuda
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 \
  bench.py --gpus 2 --steps 4 --warmup 2 --batch 64 --backend gloo > gpurun_out/bench2.log 2>&1; echo "bench2 rc=$?"
DLMPI_DESYNC_CHECK=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 3 --warmup 1 --batch 32 --backend gloo --config unet512 > gpurun_out/bench2u.log 2>&1; echo "bench2u rc=$?"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 \
  tests/ddp_gpu_rehearsal.py > gpurun_out/ddp2.log 2>&1; echo "ddp2 rc=$?"
