"""Multi-rank DDP rehearsal on GPU compute (launched with torchrun by scripts/two_rank_one_gpu.sh;
not collected by pytest).  With DLMPI_GLOO_DEVICE=cuda two ranks may share one GPU: the gradient
buckets travel over gloo, everything else (engine, arena, reducer, bucket launch order, K3/K4/K5
collectives) is the production path.  Checks, per model: DDP gradient == mean over ranks of the
local (no_sync) gradients, and parameters stay identical across ranks after optimizer steps."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import deeplearning_mpi_amd as dl  # noqa: E402
from deeplearning_mpi_amd.models import UNet, resnet18  # noqa: E402
from deeplearning_mpi_amd.ops import bce_with_logits, cross_entropy  # noqa: E402
from deeplearning_mpi_amd.optim import SGD  # noqa: E402


def check(name, make, batch, loss_fn, comm):
    torch.manual_seed(comm.rank)              # different init per rank: K4 must broadcast rank 0's
    model = make().to(comm.device)
    ddp = dl.DistributedDataParallel(model, bucket_cap_mb=1.0, first_bucket_cap_mb=0.25)
    g = torch.Generator(device=comm.device).manual_seed(100 + comm.rank)
    x, y = batch(g)
    a = model.arena
    a.zero_grad()
    with ddp.no_sync():
        loss_fn(ddp(x), y).backward()
    local = a.grad.clone()
    want = local.clone()
    comm.allreduce(want, "sum")
    want /= comm.world_size
    a.zero_grad()
    loss_fn(ddp(x), y).backward()
    torch.cuda.synchronize()
    got = a.grad.clone()
    err = ((got - want).norm() / want.norm()).item()
    # BN statistics are per-rank (as in torch DDP); the two forwards see identical inputs and
    # buffers (K5 broadcast) so the only difference is the reduction itself
    ok = err < 1e-5
    opt = SGD(model.parameters(), lr=0.01, momentum=0.9)
    for _ in range(2):
        opt.zero_grad()
        loss_fn(ddp(x), y).backward()
        opt.step()
    flat = a.flat.clone()
    ref = flat.clone()
    comm.broadcast(ref, 0)
    same = torch.equal(flat, ref)
    print(f"rank {comm.rank} {name}: grad rel err {err:.2e} ({'OK' if ok else 'FAIL'}), params identical: {same}",
          flush=True)
    return ok and same


def main():
    comm = dl.init_distributed("gloo" if os.environ.get("DLMPI_GLOO_DEVICE") == "cuda" else "rccl")
    assert comm.device.type == "cuda", comm.device
    ok = check("resnet18", lambda: resnet18(num_classes=10),
               lambda g: (torch.randn(16, 3, 32, 32, device=comm.device, generator=g),
                          torch.randint(10, (16,), device=comm.device, generator=g)),
               lambda o, t: cross_entropy(o, t), comm)
    ok &= check("unet", lambda: UNet(out_classes=1),
                lambda g: (torch.randn(2, 3, 64, 64, device=comm.device, generator=g),
                           (torch.rand(2, 64, 64, device=comm.device, generator=g) > 0.5).float()),
                lambda o, t: bce_with_logits(o.squeeze(1), t), comm)
    dl.destroy_distributed()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
