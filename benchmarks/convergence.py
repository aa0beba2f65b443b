"""Training-curve parity: the native engine (bf16 gfx950 kernels, fp32 master weights) against stock
PyTorch (eager torch.nn / MIOpen, fp32) on the same model, initial weights, data order and optimizer.

A learnable synthetic task stands in for the datasets (no downloads here):
  * classification -- 10 classes, each a fixed random 3x32x32 template plus per-sample noise;
    ResNet-18 (the reference's CIFAR model, /root/reference/pytorch/resnet/main.py:36-54) with the
    reference optimizer SGD(lr, momentum 0.9, weight decay 1e-5);
  * segmentation -- binary masks of random discs over noisy images; the reference UNet with Adam +
    BCEWithLogits + clip_grad_norm_(1.0) (/root/reference/pytorch/unet/train.py:160-194).
Prints one JSON line per run with the loss every `--log_every` steps and the held-out accuracy /
Dice at the end, for both implementations.

python benchmarks/convergence.py [--task cls|seg] [--steps 300] [--batch 128]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def cls_data(n, g, templates, noise=1.0):
    y = torch.randint(0, templates.shape[0], (n,), generator=g, device=templates.device)
    x = templates[y] + noise * torch.randn((n,) + tuple(templates.shape[1:]), generator=g, device=templates.device)
    return x, y


def seg_data(n, size, g, dev):
    yy, xx = torch.meshgrid(torch.arange(size, device=dev), torch.arange(size, device=dev), indexing="ij")
    cy = torch.rand(n, 1, 1, generator=g, device=dev) * size
    cx = torch.rand(n, 1, 1, generator=g, device=dev) * size
    r = (0.15 + 0.2 * torch.rand(n, 1, 1, generator=g, device=dev)) * size
    m = (((yy - cy) ** 2 + (xx - cx) ** 2) < r ** 2).float()
    x = m.unsqueeze(1).repeat(1, 3, 1, 1) * 0.8 + 0.6 * torch.randn(n, 3, size, size, generator=g, device=dev)
    return x, m


def run(args, native):
    from deeplearning_mpi_amd.models import UNet, resnet18
    from deeplearning_mpi_amd.ops import BCEWithLogitsLoss, CrossEntropyLoss, dice_per_sample
    from deeplearning_mpi_amd.optim import SGD, Adam, clip_grad_norm_

    dev = torch.device("cuda")
    torch.manual_seed(args.seed)
    if args.task == "cls":
        model = resnet18(num_classes=10).to(dev)
    else:
        model = UNet(out_classes=1).to(dev)
    if native:
        fwd = model
        if args.task == "cls":
            opt = SGD(model.parameters(), lr=args.lr, momentum=0.9, weight_decay=1e-5)
            crit = CrossEntropyLoss()
        else:
            opt = Adam(model.parameters(), lr=args.lr)
            crit = BCEWithLogitsLoss()
    else:
        fwd = model.forward_torch
        if args.task == "cls":
            opt = torch.optim.SGD(model.parameters(), lr=args.lr, momentum=0.9, weight_decay=1e-5)
            crit = torch.nn.CrossEntropyLoss()
        else:
            opt = torch.optim.Adam(model.parameters(), lr=args.lr)
            crit = torch.nn.BCEWithLogitsLoss()
    g = torch.Generator(device=dev).manual_seed(1000 + args.seed)
    templates = torch.randn(10, 3, 32, 32, generator=g, device=dev) if args.task == "cls" else None
    losses = []
    model.train()
    t0 = time.perf_counter()
    for step in range(args.steps):
        if args.task == "cls":
            x, y = cls_data(args.batch, g, templates, args.noise)
        else:
            x, y = seg_data(args.batch, args.size, g, dev)
        opt.zero_grad()
        out = fwd(x)
        loss = crit(out, y) if args.task == "cls" else crit(out.squeeze(1), y)
        loss.backward()
        if args.task == "seg":
            if native:
                clip_grad_norm_(model.parameters(), 1.0, optimizer=opt)
            else:
                torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        if step % args.log_every == 0 or step == args.steps - 1:
            losses.append((step, round(float(loss.detach()), 5)))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    model.eval()
    ge = torch.Generator(device=dev).manual_seed(777)
    with torch.no_grad():
        if args.task == "cls":
            x, y = cls_data(1024, ge, templates, args.noise)
            out = fwd(x)
            metric = ("accuracy", (out.argmax(1) == y).float().mean().item())
        else:
            x, y = seg_data(16, args.size, ge, dev)
            out = fwd(x)
            metric = ("dice", dice_per_sample(out.float(), y).mean().item())
    return {"impl": "native-bf16" if native else "torch-fp32", "task": args.task, "steps": args.steps,
            "batch": args.batch, "loss": losses, metric[0]: round(metric[1], 4), "seconds": round(dt, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--task", default="cls", choices=["cls", "seg"])
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--log_every", type=int, default=25)
    ap.add_argument("--noise", type=float, default=6.0, help="classification: per-sample noise / template scale")
    args = ap.parse_args()
    if args.batch is None:
        args.batch = 128 if args.task == "cls" else 8
    if args.lr is None:
        args.lr = 0.05 if args.task == "cls" else 1e-3
    for native in (True, False):
        print(json.dumps(run(args, native)), flush=True)


if __name__ == "__main__":
    main()
