"""Headline benchmark: ResNet-50 DDP training throughput, images/sec for the whole job.

Config (BASELINE.json): ResNet-50, bs=256 per GPU, 3x224x224 synthetic ImageNet-shaped data,
random-init weights, bf16 compute (fp32 master weights, fp32 gradient all-reduce), SGD momentum
0.9 / wd 1e-5 (the reference optimizer, /root/reference/pytorch/resnet/main.py:114), one process
per GPU over RCCL.  Every timed step is a full training step: forward, loss, backward with
bucketed gradient all-reduce, optimizer update.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W]
        (N > 1: launched by torch.distributed.run / torchrun or mpirun, one rank per GPU)
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

BASELINE_VALUE = None   # the reference publishes no number


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--bucket_mb", type=float, default=None)
    ap.add_argument("--profile_steps", type=int, default=0, help="print a per-phase breakdown")
    args = ap.parse_args()

    import torch

    import deeplearning_mpi_amd as dl
    from deeplearning_mpi_amd.data import device_batch
    from deeplearning_mpi_amd.models import ARCHS
    from deeplearning_mpi_amd.ops import CrossEntropyLoss
    from deeplearning_mpi_amd.optim import SGD

    comm = dl.init_distributed("rccl")
    world = comm.world_size
    dev = comm.device
    torch.manual_seed(0)
    model = ARCHS[args.arch](num_classes=args.classes).to(dev)
    ddp = dl.DistributedDataParallel(model, bucket_cap_mb=args.bucket_mb)
    opt = SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-5)
    crit = CrossEntropyLoss()
    x, y = device_batch("classification", args.batch, dev, (3, args.image, args.image), args.classes,
                        seed=1234 + comm.rank)

    def step():
        opt.zero_grad()
        loss = crit(ddp(x), y)
        loss.backward()
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    comm.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    tmax = torch.tensor([dt], dtype=torch.float64, device=dev)
    comm.allreduce(tmax, "max")
    dt = float(tmax.item())
    lossv = float(loss.item())
    global_batch = args.batch * world
    ips = global_batch * args.steps / dt
    if comm.rank == 0:
        print(json.dumps({
            "metric": "images/sec (whole node) ResNet-50 DDP bs=256/GPU",
            "value": round(ips, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1000, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(ips / BASELINE_VALUE, 4) if BASELINE_VALUE else None),
            "dtype": "bf16",
            "data": "synthetic (random 3x224x224 images / labels generated on device, random-init weights)",
            "config": {"model": args.arch, "global_batch": global_batch, "seq_len": None,
                       "image": args.image, "per_gpu_batch": args.batch,
                       "parallelism": f"dp{world}", "optimizer": "SGD(momentum=0.9, wd=1e-5)",
                       "final_loss": round(lossv, 4)},
        }), flush=True)
    dl.destroy_distributed()


if __name__ == "__main__":
    main()
