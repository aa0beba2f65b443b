"""Stock PyTorch-ROCm baseline for the bench.py configs (the "reference on MI355X" bar of
BASELINE.md): the same parameters run through eager torch.nn (MIOpen convs, channels_last,
torch.autocast bf16), torch DDP over the nccl(=RCCL) backend, and the reference optimizers --
torch.optim.SGD(momentum=0.9, weight_decay=1e-5) for ResNet (/root/reference/pytorch/resnet/main.py:114),
torch.optim.Adam + BCEWithLogits + clip_grad_norm_(1.0) for UNet (/root/reference/pytorch/unet/train.py:160-194).

python benchmarks/torch_baseline.py [--config resnet50|resnet152|resnet18_cifar|unet512|unet1024]
                                    [--steps K] [--warmup W] [--batch B]      (torchrun for N > 1)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from bench import PRESETS

    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="resnet50", choices=sorted(PRESETS))
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--no_channels_last", action="store_true")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"],
                    help="bf16: torch.autocast (default); fp32: plain fp32, as the reference trains "
                         "(/root/reference/pytorch/resnet/main.py:123-132, no autocast)")
    args = ap.parse_args()
    cfg = dict(PRESETS[args.config])
    if args.batch:
        cfg["batch"] = args.batch
    import torch
    import torch.distributed as dist
    import torch.nn as nn
    import torch.nn.functional as F

    from deeplearning_mpi_amd.models import ARCHS, UNet

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    lrank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(lrank)
    dev = torch.device("cuda", lrank)
    if world > 1:
        dist.init_process_group("nccl")
    # MIOpen exhaustive find (benchmark=True) on the UNet's 512^2 / 1024^2 shapes runs for many
    # minutes; the classification nets use it (as the reference's main.py:31 does)
    torch.backends.cudnn.benchmark = cfg["task"] == "cls"
    torch.manual_seed(0)
    seg = cfg["task"] == "seg"
    model = (UNet(out_classes=1, in_channels=cfg["cin"]) if seg else ARCHS[cfg["arch"]](num_classes=cfg["classes"]))
    model = model.to(dev)

    class Eager(nn.Module):
        def __init__(self, m):
            super().__init__()
            self.m = m

        def forward(self, x):
            return self.m.forward_torch(x)

    net = Eager(model)
    cl = not args.no_channels_last
    if cl:
        net = net.to(memory_format=torch.channels_last)
    if world > 1:
        net = nn.parallel.DistributedDataParallel(net, device_ids=[lrank])
    B, S, C = cfg["batch"], cfg["image"], cfg["cin"]
    # the same fixed device batch as bench.py (device_batch, seed 1234 + rank), so the two final
    # losses are comparable
    from deeplearning_mpi_amd.data import device_batch

    x, y = device_batch("segmentation" if seg else "classification", B, dev, (C, S, S), cfg["classes"],
                        seed=1234 + rank)
    if cl:
        x = x.to(memory_format=torch.channels_last)
    if seg:
        opt = torch.optim.Adam(net.parameters(), lr=1e-4)
    else:
        opt = torch.optim.SGD(net.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-5)

    def step():
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=args.precision == "bf16"):
            out = net(x)
        if seg:
            loss = F.binary_cross_entropy_with_logits(out.float().squeeze(1), y)
            loss.backward()
            torch.nn.utils.clip_grad_norm_(net.parameters(), 1.0)
        else:
            loss = F.cross_entropy(out.float(), y)
            loss.backward()
        opt.step()
        return loss

    for i in range(args.warmup):
        step()
        torch.cuda.synchronize()
        print(f"warmup step {i} done", file=sys.stderr, flush=True)
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
        mode = "autocast bf16" if args.precision == "bf16" else "fp32"
        print(json.dumps({"metric": f"stock PyTorch DDP (MIOpen, {mode}, channels_last): " + cfg["metric"],
                          "value": round(B * world * args.steps / dt, 2), "n_gpus": world,
                          "ms_per_step": round(dt / args.steps * 1000, 3), "config": args.config,
                          "per_gpu_batch": B, "precision": args.precision,
                          "loss": round(float(loss.item()), 4)}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
