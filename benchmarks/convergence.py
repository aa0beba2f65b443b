"""Training-curve parity: the native engine (bf16 gfx950 kernels, fp32 master weights) against stock
PyTorch (eager torch.nn / MIOpen, fp32) on the same model, initial weights, data order and optimizer.

A learnable synthetic task stands in for the datasets (no downloads here):
  * classification -- 10 classes, each a fixed random 3x32x32 template plus per-sample noise;
    ResNet-18 (the reference's CIFAR model, /root/reference/pytorch/resnet/main.py:36-54) with the
    reference optimizer SGD(lr, momentum 0.9, weight decay 1e-5);
  * segmentation -- binary masks of random discs over noisy images; the reference UNet with Adam +
    BCEWithLogits + clip_grad_norm_(1.0) (/root/reference/pytorch/unet/train.py:160-194).
Prints one JSON line per run with the loss every `--log_every` steps and the held-out accuracy /
Dice at the end, for every implementation of ``--impls``: native (the engine), autocast (stock
PyTorch, torch.autocast bf16, channels_last -- the same compute precision) and fp32 (stock PyTorch
fp32); ``--torch_seeds`` repeats the autocast run with other seeds (other initial weights and data
stream) to show the SGD noise the native-vs-autocast gap is to be read against.

python benchmarks/convergence.py [--task cls|seg] [--arch resnet18|resnet50] [--size 32] [--steps 300]
       [--batch 128] [--impls native,autocast,fp32] [--torch_seeds 1]
Bench shapes (round 6): --task cls --arch resnet50 --size 224 --batch 256; --task seg --size 512 --batch 16.
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


def run(args, impl, seed):
    from deeplearning_mpi_amd.models import ARCHS, UNet
    from deeplearning_mpi_amd.ops import BCEWithLogitsLoss, CrossEntropyLoss, dice_per_sample
    from deeplearning_mpi_amd.optim import SGD, Adam, clip_grad_norm_

    native = impl == "native"
    amp = impl == "autocast"
    dev = torch.device("cuda")
    torch.manual_seed(seed)
    if args.task == "cls":
        model = ARCHS[args.arch](num_classes=10).to(dev)
    else:
        model = UNet(out_classes=1).to(dev)
    if not native:
        model = model.to(memory_format=torch.channels_last)
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
    g = torch.Generator(device=dev).manual_seed(1000 + seed)
    # the task (class templates) is fixed by --seed; the seed of the run moves init and data order
    gt = torch.Generator(device=dev).manual_seed(1000 + args.seed)
    templates = torch.randn(10, 3, args.size, args.size, generator=gt, device=dev) if args.task == "cls" else None

    def fwd_(x):
        if native:
            return fwd(x)
        x = x.to(memory_format=torch.channels_last)
        if amp:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                return fwd(x).float()
        return fwd(x)
    losses = []
    model.train()
    t0 = time.perf_counter()
    base_lr = args.lr
    for step in range(args.steps):
        if args.warmup_steps:   # linear learning-rate warm-up (both implementations alike)
            for grp in opt.param_groups:
                grp["lr"] = base_lr * min(1.0, (step + 1) / args.warmup_steps)
        _STATE["where"] = f"{impl} seed {seed} step {step}"
        if args.task == "cls":
            x, y = cls_data(args.batch, g, templates, args.noise)
        else:
            x, y = seg_data(args.batch, args.size, g, dev)
        opt.zero_grad()
        out = fwd_(x)
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
            print(f"[convergence] {impl} seed {seed} step {step} loss {losses[-1][1]}", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    model.eval()
    ge = torch.Generator(device=dev).manual_seed(777)
    with torch.no_grad():
        if args.task == "cls":
            hits = 0
            for _ in range(4):   # 1,024 held-out samples in 4 batches
                x, y = cls_data(256, ge, templates, args.noise)
                hits += (fwd_(x).argmax(1) == y).sum().item()
            metric = ("accuracy", hits / 1024)
        else:
            x, y = seg_data(16, args.size, ge, dev)
            out = fwd_(x)
            metric = ("dice", dice_per_sample(out.float(), y).mean().item())
    name = {"native": "native-bf16", "autocast": "torch-autocast-bf16", "fp32": "torch-fp32"}[impl]
    return {"impl": name, "seed": seed, "task": args.task, "arch": args.arch if args.task == "cls" else "unet",
            "size": args.size, "steps": args.steps, "batch": args.batch, "lr": args.lr, "loss": losses,
            metric[0]: round(metric[1], 4), "seconds": round(dt, 1)}


_STATE = {"where": "start"}


def _heartbeat():
    # stock PyTorch's first convolutions search MIOpen algorithms for minutes: a line every 30 s keeps a
    # silence watchdog from taking that for a hang
    while True:
        time.sleep(30)
        print(f"[convergence] alive: {_STATE['where']}", file=sys.stderr, flush=True)


def main():
    import threading

    threading.Thread(target=_heartbeat, daemon=True).start()
    ap = argparse.ArgumentParser()
    ap.add_argument("--task", default="cls", choices=["cls", "seg"])
    ap.add_argument("--arch", default="resnet18", help="classification model (resnet18 / resnet50 / ...)")
    ap.add_argument("--impls", default="native,fp32", help="native / autocast / fp32, comma-separated")
    ap.add_argument("--torch_seeds", type=int, default=0, help="extra autocast runs with seeds seed+1 ..")
    ap.add_argument("--warmup_steps", type=int, default=0, help="linear learning-rate warm-up steps")
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--size", type=int, default=None, help="image size (default 32 cls / 64 seg)")
    ap.add_argument("--lr", type=float, default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--log_every", type=int, default=25)
    ap.add_argument("--noise", type=float, default=6.0, help="classification: per-sample noise / template scale")
    args = ap.parse_args()
    if args.batch is None:
        args.batch = 128 if args.task == "cls" else 8
    if args.lr is None:
        args.lr = 0.05 if args.task == "cls" else 1e-3
    if args.size is None:
        args.size = 32 if args.task == "cls" else 64
    for impl in args.impls.split(","):
        print(json.dumps(run(args, impl, args.seed)), flush=True)
    for k in range(1, args.torch_seeds + 1):
        print(json.dumps(run(args, "autocast", args.seed + k)), flush=True)


if __name__ == "__main__":
    main()
