"""Stock PyTorch-ROCm baseline for the headline config (the "reference on MI355X" bar of
BASELINE.md): the same torchvision-identical ResNet-50 parameters run through eager torch.nn
(MIOpen convs, channels_last, torch.autocast bf16), torch DDP over the nccl(=RCCL) backend,
torch.optim.SGD(momentum=0.9, weight_decay=1e-5) -- i.e. what /root/reference/pytorch/resnet/main.py
does, at bs=256/GPU on 224x224 synthetic data.

python benchmarks/torch_baseline.py [--steps K] [--warmup W] [--batch B]   (torchrun for N > 1)
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--no_channels_last", action="store_true")
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    import torch.nn as nn

    from deeplearning_mpi_amd.models import ARCHS

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    lrank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(lrank)
    dev = torch.device("cuda", lrank)
    if world > 1:
        dist.init_process_group("nccl")
    torch.backends.cudnn.benchmark = True
    model = ARCHS[args.arch](num_classes=1000).to(dev)

    class Eager(nn.Module):
        def __init__(self, m):
            super().__init__()
            self.m = m

        def forward(self, x):
            return self.m.forward_torch(x)

    net = Eager(model)
    if not args.no_channels_last:
        net = net.to(memory_format=torch.channels_last)
    if world > 1:
        net = nn.parallel.DistributedDataParallel(net, device_ids=[lrank])
    opt = torch.optim.SGD(net.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-5)
    crit = nn.CrossEntropyLoss()
    x = torch.randn(args.batch, 3, 224, 224, device=dev)
    if not args.no_channels_last:
        x = x.to(memory_format=torch.channels_last)
    y = torch.randint(1000, (args.batch,), device=dev)

    def step():
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = net(x)
            loss = crit(out, y)
        loss.backward()
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if rank == 0:
        print(json.dumps({"metric": "images/sec stock PyTorch DDP (MIOpen, autocast bf16, channels_last)",
                          "value": round(args.batch * world * args.steps / dt, 2), "n_gpus": world,
                          "ms_per_step": round(dt / args.steps * 1000, 3), "arch": args.arch,
                          "per_gpu_batch": args.batch, "loss": round(float(loss.item()), 4)}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
