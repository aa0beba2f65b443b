"""ResNet data-parallel classification training (the reference's pytorch/resnet/{main,resnet}.py).

Flags keep the reference names and defaults: --num_epochs, --batch_size (per
process), --learning_rate, --random_seed, --model_dir, --model_filename, --resume.  Non-breaking
additions: --arch, --num_classes, --synthetic, --data_root, --image_size, --backend, --device,
--bucket_mb, --workers, --eval_every, --steps_per_epoch, --precision, --graph, --data_on_device,
--benchmark_steps.

Deliberate fixes of reference quirks: the sampler's epoch is advanced every epoch;
evaluation runs on the unwrapped module (no stray rank-0-only collective, K8) with a non-augmenting
test transform; checkpoints are written by GLOBAL rank 0 only; the per-step loss stays on the
device (one host sync per epoch instead of one per step).
"""
from __future__ import annotations

import argparse
import os
import random
import time

import numpy as np
import torch
from torch.utils.data import DataLoader

from .. import parallel
from ..data import CIFAR10, CifarTransform, DeviceBatches, DeviceImageDataset, DistributedSampler, SyntheticImages
from ..models import ARCHS
from ..ops import CrossEntropyLoss, backward, top1_correct
from ..optim import SGD
from ..utils.checkpoint import load_checkpoint, resume_state, save_checkpoint, set_rng_state
from ..utils.graphs import CapturedStep


def build_argparser(variant: str = "main") -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    p.add_argument("--num_epochs", type=int, help="Number of training epochs.", default=100)
    p.add_argument("--batch_size", type=int, help="Training batch size for one process.",
                   default=128 if variant == "main" else 32)
    p.add_argument("--learning_rate", type=float, help="Learning rate.", default=0.1)
    p.add_argument("--random_seed", type=int, help="Random seed.", default=0)
    p.add_argument("--model_dir", type=str, help="Directory for saving models.", default="saved_models")
    p.add_argument("--model_filename", type=str, help="Model filename.", default="resnet_distributed.pth")
    p.add_argument("--resume", action="store_true", help="Resume training from saved checkpoint.")
    # additions
    p.add_argument("--arch", default="resnet18", choices=sorted(ARCHS))
    p.add_argument("--num_classes", type=int, default=10)
    p.add_argument("--synthetic", action="store_true", help="random data instead of CIFAR-10")
    p.add_argument("--synthetic_size", type=int, default=1024, help="images per epoch (synthetic)")
    p.add_argument("--data_root", default="./data")
    p.add_argument("--image_size", type=int, default=32)
    p.add_argument("--backend", default="nccl", help="nccl|rccl (GPU, RCCL) or gloo (CPU)")
    p.add_argument("--device", default="auto", help="auto | cpu | cuda")
    p.add_argument("--bucket_mb", type=float, default=None)
    p.add_argument("--workers", type=int, default=8 if variant != "main" else 15)
    p.add_argument("--eval_every", type=int, default=10)
    p.add_argument("--test_batch_size", type=int, default=None if variant == "main" else 128)
    p.add_argument("--steps_per_epoch", type=int, default=0, help="cap steps per epoch (0 = full epoch)")
    p.add_argument("--eval_before_train", action="store_true", default=variant != "main",
                   help="resnet.py variant: evaluate/save before training on eval epochs")
    p.add_argument("--precision", default="bf16", choices=["bf16", "fp32"],
                   help="bf16: native gfx950 kernels on bf16 activations; fp32: the same kernels on fp32 "
                        "activations and weights (fp32 MFMA)")
    p.add_argument("--graph", nargs="?", const="1", default="auto", choices=["auto", "0", "1"],
                   help="replay each full-size training step from a captured hipGraph (ragged last batches run "
                        "eagerly); auto = on for launch-bound GPU training")
    p.add_argument("--data_on_device", default="auto", choices=["auto", "0", "1"],
                   help="keep CIFAR-10 resident in GPU memory and build each augmented batch with one kernel "
                        "(data/device.py); auto = on for GPU training on real data")
    p.add_argument("--benchmark_steps", type=int, default=0,
                   help="time this many steps on a synthetic device batch, print images/sec and exit")
    return p


def use_graph(args, device, pixels=None, comm_backend="single") -> bool:
    """--graph auto: capture the step when it is launch-bound -- native bf16 kernels on a GPU and a
    step smaller than the auxiliary-stream threshold (N*H*W < DLMPI_AUX_MIN_PIXELS, default 1M:
    the reference's ResNet-18 on CIFAR, 46k -> 85k img/s).  Larger steps run their weight-gradient
    and residual-branch streams concurrently, which a replayed graph loses (measured: ResNet-50
    bs 256 -7 %, ResNet-152 -13 %, UNet 512 -2 %, profiles/r2_graph_ab).  Auto mode also requires a
    capturable data plane: RCCL (device collectives on the comm stream) or a single rank -- gloo's
    host-staged collectives (the DLMPI_GLOO_DEVICE=cuda rehearsal) cannot live inside a hipGraph."""
    if args.graph in (True, "1"):
        return device.type == "cuda"
    if args.graph in (False, "0"):
        return False
    if device.type != "cuda" or comm_backend not in ("rccl", "single"):
        return False
    if pixels is None:
        side = args.image_size if getattr(args, "synthetic", False) else 32
        pixels = args.batch_size * side * side
    return pixels < int(os.environ.get("DLMPI_AUX_MIN_PIXELS", str(1 << 20)))


def set_random_seeds(seed: int):
    """Seeds + the reference's cuDNN flags (C16: resnet/main.py:26-33, unet/train.py:35-41).  The
    flags only affect stock torch ops; the engine's own kernels are deterministic by construction
    (fixed-order reductions, no float atomics; the bilinear up-sampling backward is a gather)."""
    torch.manual_seed(seed)
    np.random.seed(seed)
    random.seed(seed)
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = True


@torch.no_grad()
def evaluate(model, device, test_loader) -> float:
    model.eval()
    correct = torch.zeros(1, dtype=torch.int64, device=device)
    total = 0
    for images, labels in test_loader:
        images, labels = images.to(device, non_blocking=True), labels.to(device, non_blocking=True)
        correct += top1_correct(model(images), labels).to(torch.int64)
        total += labels.size(0)
    model.train()
    return correct.item() / max(1, total)


def run(args) -> dict:
    comm = parallel.init_distributed(args.backend)
    rank, world, local_rank = comm.rank, comm.world_size, comm.local_rank
    device = comm.device if args.device == "auto" else torch.device(args.device)
    set_random_seeds(args.random_seed)
    model = ARCHS[args.arch](num_classes=args.num_classes).to(device)
    model.precision = args.precision
    ddp = parallel.DistributedDataParallel(model, bucket_cap_mb=args.bucket_mb)
    model_filepath = os.path.join(args.model_dir, args.model_filename)
    args.graph = use_graph(args, device, comm_backend=getattr(comm, "backend", "single"))

    # the training step reads its batch from fixed tensors so that it can be captured (--graph)
    x_static = torch.empty((args.batch_size, 3, args.image_size, args.image_size) if args.synthetic else
                           (args.batch_size, 3, 32, 32), device=device)
    y_static = torch.zeros(args.batch_size, dtype=torch.int64, device=device)
    on_device = (args.data_on_device == "1" or
                 (args.data_on_device == "auto" and device.type == "cuda" and not args.synthetic))
    test_bs = args.test_batch_size or args.batch_size
    if args.synthetic:
        shape = (3, args.image_size, args.image_size)
        train_set = SyntheticImages(args.synthetic_size, shape, args.num_classes, seed=1)
        test_set = SyntheticImages(max(64, args.synthetic_size // 8), shape, args.num_classes, seed=2)
    elif on_device:
        # the whole dataset in HBM; one kernel per batch does gather + crop/flip + normalize
        train_set = DeviceImageDataset.cifar10(args.data_root, True, device, seed=args.random_seed)
        test_set = DeviceImageDataset.cifar10(args.data_root, False, device, augment=False)
    else:
        # download=False semantics: the data must already be under data_root (see download.py)
        # augmentation = f(seed, epoch, index) (data/datasets.py SampleRng): rank-, worker- and
        # resume-independent
        train_set = CIFAR10(args.data_root, train=True, transform=CifarTransform(True), seed=args.random_seed)
        test_set = CIFAR10(args.data_root, train=False, transform=CifarTransform(False))
    sampler = DistributedSampler(train_set, seed=0)
    if on_device and not args.synthetic:
        train_loader = DeviceBatches(train_set, args.batch_size, sampler,
                                     out=(x_static, y_static) if args.graph else None)
        test_loader = DeviceBatches(test_set, test_bs)
    else:
        pin = device.type == "cuda"
        # workers are re-created every epoch (reference default) so they see the dataset's epoch
        train_loader = DataLoader(train_set, batch_size=args.batch_size, sampler=sampler, num_workers=args.workers,
                                  pin_memory=pin)
        # a private generator: rank-0-only evaluation must not advance the global host RNG (its
        # state is the resume state every rank restores)
        test_loader = DataLoader(test_set, batch_size=test_bs, shuffle=False, num_workers=args.workers,
                                 pin_memory=pin, generator=torch.Generator().manual_seed(args.random_seed))
    criterion = CrossEntropyLoss()
    optimizer = SGD(model.parameters(), lr=args.learning_rate, momentum=0.9, weight_decay=1e-5)
    start_epoch = 0
    if args.resume:
        # weights (reference layout) + the sidecar: optimizer state, next epoch, RNG states
        meta = load_checkpoint(ddp, model_filepath, map_location=device, optimizer=optimizer)
        start_epoch = int(meta.get("next_epoch", 0))
        set_rng_state(meta.get("rng"))

    def train_step(x, y):
        optimizer.zero_grad()
        loss = criterion(ddp(x), y)
        backward(loss)
        optimizer.step()
        return loss

    captured = None
    if args.graph and device.type == "cuda":
        captured = CapturedStep(lambda: train_step(x_static, y_static), warmup=2, inputs=(x_static, y_static),
                                comm=comm)

    if args.benchmark_steps:
        return benchmark(args, train_step, captured, x_static, y_static, comm, device)

    history = {"loss": [], "accuracy": [], "images_per_sec": []}

    def eval_and_save(epoch, next_epoch):
        state = resume_state(next_epoch)   # RNG states of the epoch boundary, taken before evaluating
        accuracy = evaluate(model, device, test_loader)
        save_checkpoint(ddp, model_filepath, optimizer=optimizer, extra=state, rank=rank)
        print("-" * 75)
        print("Epoch: {}, Accuracy: {}".format(epoch, accuracy))
        print("-" * 75)
        history["accuracy"].append(accuracy)

    try:
        for epoch in range(start_epoch, args.num_epochs):
            sampler.set_epoch(epoch)
            if hasattr(train_set, "set_epoch"):
                train_set.set_epoch(epoch)
            if args.eval_before_train and epoch % args.eval_every == 0 and rank == 0:
                eval_and_save(epoch, epoch)
            print("Local Rank: {}, Epoch: {}, Training ...".format(local_rank, epoch))
            ddp.train()
            loss_sum = torch.zeros((), device=device)
            nb = 0
            t0 = time.perf_counter()
            for inputs, labels in train_loader:
                inputs = inputs.to(device, non_blocking=True)
                labels = labels.to(device, non_blocking=True)
                if captured is not None and inputs.shape[0] == args.batch_size:
                    captured.set_inputs(inputs, labels)
                    loss = captured()
                else:   # eager step (also the ragged last batch of a graph run)
                    loss = train_step(inputs, labels)
                loss_sum += loss.detach()
                nb += 1
                if args.steps_per_epoch and nb >= args.steps_per_epoch:
                    break
            mean_loss = (loss_sum / max(1, nb)).item()
            dt = time.perf_counter() - t0
            history["loss"].append(mean_loss)
            history["images_per_sec"].append(nb * args.batch_size * world / dt)
            print("Local Rank: {}, Epoch: {}, Loss: {}".format(local_rank, epoch, mean_loss))
            if rank == 0:
                print(f"Epoch {epoch} throughput: {history['images_per_sec'][-1]:.1f} images/sec ({nb} steps)")
            if not args.eval_before_train and epoch % args.eval_every == 0 and rank == 0:
                eval_and_save(epoch, epoch + 1)
            print(f"Epoch {epoch} completed")
    finally:
        parallel.destroy_distributed()
    return history


def benchmark(args, train_step, captured, x, y, comm, device) -> dict:
    """--benchmark_steps: synthetic device batch, 3 warm-up steps, timed steps, images/sec."""
    g = torch.Generator(device=device).manual_seed(1234 + comm.rank)
    x.copy_(torch.randn(x.shape, generator=g, device=device))
    y.copy_(torch.randint(args.num_classes, y.shape, generator=g, device=device))
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
        print(f"benchmark: {args.arch} bs={args.batch_size}/rank x {comm.world_size} ranks, "
              f"{args.benchmark_steps} steps: {ips:.1f} images/sec ({dt / args.benchmark_steps * 1e3:.2f} ms/step), "
              f"loss {float(loss.detach()):.4f}")
    parallel.destroy_distributed()
    return {"images_per_sec": ips}


def main(variant="main", argv=None):
    args = build_argparser(variant).parse_args(argv)
    return run(args)
