"""UNet data-parallel segmentation training (the reference's pytorch/unet/train.py).

Same flags/defaults (--num_epochs 100, --batch_size 16, --learning_rate 1e-4, --random_seed 42,
--model_dir saved_models, --model_filename model.pth, --resume), same log file
(logs/training_log_YYYYmmdd_HHMMSS.log: header, "Started training at", per-epoch
"Epoch e | Loss: x | Duration: s", every 10 epochs "Epoch e | Dice Score: x", final block) and the
same Adam + BCEWithLogits + clip_grad_norm_(1.0) step (/root/reference/pytorch/unet/train.py:143-244).

Deliberate fixes: the NaN/Inf skip is collective (decided from the
all-reduced gradient norm on the device, identical on every rank -> no deadlock, no host sync);
the log and checkpoints are written by global rank 0 only; evaluation uses the unwrapped module.
Additions: --synthetic, --image_size, --in_channels, --data_dir, --scale, --up_sample_mode,
--backend, --device, --max_norm, --steps_per_epoch, --workers.
"""
from __future__ import annotations

import argparse
import os
import sys
import random
import time
from datetime import datetime

import numpy as np
import torch
from torch.utils.data import DataLoader
from tqdm import tqdm

from .. import parallel
from ..data import CarvanaDataset, DeviceBatches, DeviceCachedDataset, DistributedSampler, SyntheticMasks
from ..models import UNet
from ..ops import BCEWithLogitsLoss, backward, dice_per_sample
from ..optim import Adam, clip_grad_norm_
from ..utils.graphs import CapturedStep
from ..utils.checkpoint import load_checkpoint, resume_state, save_checkpoint, set_rng_state
from .classification import use_graph


def build_argparser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    p.add_argument("--num_epochs", type=int, default=100, help="Number of training epochs.")
    p.add_argument("--batch_size", type=int, default=16, help="Batch size per process.")
    p.add_argument("--learning_rate", type=float, default=0.0001, help="Learning rate.")
    p.add_argument("--random_seed", type=int, default=42, help="Seed for reproducibility.")
    p.add_argument("--model_dir", type=str, default="saved_models", help="Directory to save model.")
    p.add_argument("--model_filename", type=str, default="model.pth", help="Model filename.")
    p.add_argument("--resume", action="store_true", help="Resume from a checkpoint.")
    p.add_argument("--synthetic", action="store_true")
    p.add_argument("--synthetic_size", type=int, default=64)
    p.add_argument("--image_size", type=int, default=512)
    p.add_argument("--in_channels", type=int, default=3)
    p.add_argument("--data_dir", default="data")
    p.add_argument("--scale", type=float, default=0.2)
    p.add_argument("--up_sample_mode", default="conv_transpose", choices=["conv_transpose", "bilinear"])
    p.add_argument("--backend", default="nccl")
    p.add_argument("--device", default="auto")
    p.add_argument("--max_norm", type=float, default=1.0)
    p.add_argument("--steps_per_epoch", type=int, default=0)
    p.add_argument("--workers", type=int, default=max(1, (os.cpu_count() or 2) // 2))
    p.add_argument("--data_on_device", default="auto", choices=["auto", "0", "1"],
                   help="decode the dataset once and keep it in GPU memory; batches are device-side gathers "
                        "(auto: on for GPU runs when it needs < 1/4 of the GPU memory)")
    p.add_argument("--log_dir", default="logs")
    p.add_argument("--eval_every", type=int, default=10)
    p.add_argument("--bucket_mb", type=float, default=None)
    p.add_argument("--precision", default="bf16", choices=["bf16", "fp32"],
                   help="bf16: native gfx950 kernels on bf16 activations; fp32: the same kernels on fp32 "
                        "activations and weights (fp32 MFMA)")
    p.add_argument("--graph", nargs="?", const="1", default="auto", choices=["auto", "0", "1"],
                   help="replay each full-size training step from a captured hipGraph (ragged last batches run "
                        "eagerly); auto = on for launch-bound GPU training")
    p.add_argument("--benchmark_steps", type=int, default=0,
                   help="time this many steps on a synthetic device batch, print images/sec and exit")
    return p


def set_random_seeds(seed):
    """Seeds + the reference's cuDNN flags (C16: resnet/main.py:26-33, unet/train.py:35-41).  The
    flags only affect stock torch ops; the engine's own kernels are deterministic by construction
    (fixed-order reductions, no float atomics; the bilinear up-sampling backward is a gather)."""
    torch.manual_seed(seed)
    np.random.seed(seed)
    random.seed(seed)
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = True


def create_log_file(log_dir="logs") -> str:
    return os.path.join(log_dir, f"training_log_{datetime.now().strftime('%Y%m%d_%H%M%S')}.log")


class RankLog:
    def __init__(self, path, rank):
        self.path, self.rank = path, rank
        if rank == 0 and path:
            os.makedirs(os.path.dirname(path) or ".", exist_ok=True)

    def __call__(self, msg):
        if self.rank == 0 and self.path:
            with open(self.path, "a") as f:
                f.write(msg + "\n")


@torch.no_grad()
def evaluate_model(model, device, test_loader) -> float:
    model.eval()
    scores = []
    for batch in test_loader:
        images = batch["image"].to(device, dtype=torch.float32)
        masks = batch["mask"].to(device, dtype=torch.float32)
        scores.append(dice_per_sample(model(images), masks))
    model.train()
    if not scores:
        return 0.0
    return torch.cat(scores).mean().item()


def build_data_loaders(args, device):
    if args.synthetic:
        ds = SyntheticMasks(args.synthetic_size, (args.in_channels, args.image_size, args.image_size),
                            seed=args.random_seed)
    else:
        ds = CarvanaDataset(images_dir=os.path.join(args.data_dir, "images"),
                            mask_dir=os.path.join(args.data_dir, "masks"), scale=args.scale)
    train_size = int(0.8 * len(ds))
    test_size = len(ds) - train_size
    # same split on every rank (seeded generator rather than the global RNG)
    train_ds, test_ds = torch.utils.data.random_split(ds, [train_size, test_size],
                                                      generator=torch.Generator().manual_seed(args.random_seed))
    if _use_device_data(args, device, ds):
        # the reference dataset is deterministic (no augmentation): decode / resize once, keep the
        # tensors in HBM, and serve every batch as an index gather on the device
        train_c, test_c = DeviceCachedDataset(train_ds, device), DeviceCachedDataset(test_ds, device)
        sampler = DistributedSampler(train_c)
        return DeviceBatches(train_c, args.batch_size, sampler), DeviceBatches(test_c, args.batch_size), sampler
    kw = dict(batch_size=args.batch_size, num_workers=args.workers, pin_memory=device.type == "cuda")
    sampler = DistributedSampler(train_ds)
    # evaluation runs on rank 0 only: its loader gets a private generator so it never advances the
    # global host RNG that every rank restores on --resume
    return (DataLoader(train_ds, sampler=sampler, **kw),
            DataLoader(test_ds, shuffle=False, generator=torch.Generator().manual_seed(args.random_seed), **kw),
            sampler)


def _use_device_data(args, device, ds) -> bool:
    """--data_on_device auto: on for GPU runs whose decoded dataset needs < 1/4 of the GPU memory."""
    if args.data_on_device != "auto":
        return args.data_on_device == "1"
    if device.type != "cuda":
        return False
    s = ds[0]
    per = sum(torch.as_tensor(v).numel() * 4 for v in s.values())
    return per * len(ds) < torch.cuda.get_device_properties(device).total_memory // 4


def benchmark(args, train_step, captured, x, y, comm, device) -> dict:
    """--benchmark_steps: synthetic device batch, 3 warm-up steps, timed steps, images/sec."""
    g = torch.Generator(device=device).manual_seed(1234 + comm.rank)
    x.copy_(torch.randn(x.shape, generator=g, device=device))
    y.copy_((torch.rand(y.shape, generator=g, device=device) > 0.5).float())
    step = captured if captured is not None else (lambda: train_step(x, y))
    for _ in range(3):
        step()
    comm.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.benchmark_steps):
        loss = step()
    comm.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ips = args.batch_size * comm.world_size * args.benchmark_steps / dt
    if comm.rank == 0:
        print(f"benchmark: UNet {args.in_channels}x{args.image_size}^2 bs={args.batch_size}/rank x {comm.world_size} "
              f"ranks, {args.benchmark_steps} steps: {ips:.2f} images/sec ({dt / args.benchmark_steps * 1e3:.1f} "
              f"ms/step), loss {float(loss.detach()):.4f}")
    parallel.destroy_distributed()
    return {"images_per_sec": ips}


def run(args) -> dict:
    comm = parallel.init_distributed(args.backend)
    rank, world, local_rank = comm.rank, comm.world_size, comm.local_rank
    device = comm.device if args.device == "auto" else torch.device(args.device)
    set_random_seeds(args.random_seed)
    log = RankLog(create_log_file(args.log_dir), rank)
    gpu = torch.cuda.get_device_name(device) if device.type == "cuda" else "cpu"
    log(f"Batch size: {args.batch_size}")
    log(f"Number of workers: {os.cpu_count()}")
    log(f"Learning rate: {args.learning_rate}")
    log(f"Number of epochs: {args.num_epochs}")
    log(f"World size: {world}, Local rank: {local_rank}, GPU: {gpu}")

    train_loader, test_loader, sampler = build_data_loaders(args, device)
    model = UNet(out_classes=1, up_sample_mode=args.up_sample_mode, in_channels=args.in_channels).to(device)
    model.precision = args.precision
    ddp = parallel.DistributedDataParallel(model, bucket_cap_mb=args.bucket_mb)
    model_filepath = os.path.join(args.model_dir, args.model_filename)
    optimizer = Adam(model.parameters(), lr=args.learning_rate)
    criterion = BCEWithLogitsLoss()
    start_epoch = 0
    if args.resume:
        # weights (reference layout) + the sidecar: Adam moments and step, next epoch, RNG states
        meta = load_checkpoint(ddp, model_filepath, map_location=device, optimizer=optimizer)
        start_epoch = int(meta.get("next_epoch", 0))
        set_rng_state(meta.get("rng"))
    args.graph = use_graph(args, device, pixels=args.batch_size * args.image_size * args.image_size,
                           comm_backend=getattr(comm, "backend", "single"))

    def train_step(images, masks):
        pred = ddp(images).squeeze(1)
        loss = criterion(pred, masks)
        optimizer.zero_grad()
        backward(loss)
        # collective NaN/Inf guard: a non-finite all-reduced grad norm skips the step on all ranks
        clip_grad_norm_(model.parameters(), max_norm=args.max_norm, optimizer=optimizer)
        optimizer.step()
        return loss

    S = args.image_size
    x_static = torch.zeros(args.batch_size, args.in_channels, S, S, device=device)
    y_static = torch.zeros(args.batch_size, S, S, device=device)
    captured = None
    if args.graph and device.type == "cuda":
        captured = CapturedStep(lambda: train_step(x_static, y_static), warmup=2, inputs=(x_static, y_static),
                                comm=comm)
    if args.benchmark_steps:
        return benchmark(args, train_step, captured, x_static, y_static, comm, device)
    history = {"loss": [], "dice": []}
    if rank == 0:
        print(f"Logging training progress to: {log.path}")
    log(f"Started training at {datetime.now()}")
    try:
        for epoch in range(start_epoch, args.num_epochs):
            sampler.set_epoch(epoch)
            t0 = time.time()
            ddp.train()
            loss_sum = torch.zeros((), device=device)
            nb = 0
            bar = tqdm(train_loader, desc=f"Epoch {epoch + 1}/{args.num_epochs}", unit="batch",
                       disable=rank != 0 or not sys.stderr.isatty())   # no per-step host sync for a loss postfix
            for batch in bar:
                images = batch["image"].to(device, dtype=torch.float32, non_blocking=True)
                masks = batch["mask"].to(device, dtype=torch.float32, non_blocking=True)
                if captured is not None and images.shape == x_static.shape:
                    captured.set_inputs(images, masks)
                    loss = captured()
                else:
                    loss = train_step(images, masks)
                loss_sum += torch.nan_to_num(loss.detach(), nan=0.0, posinf=0.0, neginf=0.0)
                nb += 1
                if args.steps_per_epoch and nb >= args.steps_per_epoch:
                    break
            avg_loss = (loss_sum / max(1, nb)).item()
            history["loss"].append(avg_loss)
            print(f"Epoch {epoch + 1} finished with loss: {avg_loss:.4f}")
            log(f"Epoch {epoch + 1} | Loss: {avg_loss:.4f} | Duration: {time.time() - t0:.2f}s")
            if (epoch + 1) % args.eval_every == 0 and rank == 0:
                state = resume_state(epoch + 1)   # epoch-boundary RNG states, taken before evaluating
                dice = evaluate_model(model, device, test_loader)
                save_checkpoint(ddp, model_filepath, optimizer=optimizer, extra=state, rank=rank)
                print("-" * 75)
                print(f"Epoch {epoch + 1} Dice Score: {dice:.4f}")
                print("-" * 75)
                log(f"Epoch {epoch + 1} | Dice Score: {dice:.4f}")
                history["dice"].append(dice)
        if rank == 0:
            print("\n" + "=" * 80 + "\nTRAINING COMPLETED - FINAL EVALUATION\n" + "=" * 80)
            state = resume_state(args.num_epochs)
            final = evaluate_model(model, device, test_loader)
            save_checkpoint(ddp, model_filepath, optimizer=optimizer, extra=state, rank=rank)
            print(f"FINAL DICE COEFFICIENT: {final:.4f}\n" + "=" * 80 + "\n")
            log("=" * 80)
            log("FINAL TRAINING RESULTS")
            log("=" * 80)
            log(f"TRAINING COMPLETED | Final Dice Coefficient: {final:.4f} | Training finished at: {datetime.now()}")
            log(f"Total training epochs: {args.num_epochs}")
            log(f"Final learning rate: {args.learning_rate}")
            log(f"Model saved to: {model_filepath}")
            log("=" * 80)
            history["final_dice"] = final
    finally:
        parallel.destroy_distributed()
    return history


def main(argv=None):
    return run(build_argparser().parse_args(argv))
