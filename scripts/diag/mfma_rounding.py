"""Rounding bias of the fp32 accumulation in our GEMMs vs hipBLASLt / MIOpen: all-positive operands,
mean signed relative error against fp64 (round-to-nearest: ~0; truncation: about -K*eps/4)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from deeplearning_mpi_amd.ops.act import Act  # noqa: E402
from deeplearning_mpi_amd.ops.backend import NativeBackend  # noqa: E402

dev = "cuda"
torch.manual_seed(0)
M, C, K = 4096, 1024, 256
for dt in (torch.float32, torch.bfloat16):
    nb = NativeBackend(dev, dt)
    x = torch.rand(M, C, device=dev).to(dt)
    w = torch.rand(K, 1, 1, C, device=dev).to(dt)
    y = Act.empty(1, 64, 64, K, dt, dev)
    nb.conv_fwd(Act(x, 1, 64, 64, C), w, K, 1, 1, 1, 0, y)
    ref = x.double() @ w.view(K, C).double().t()
    r = (y.buf.double() - ref) / ref
    lib = (x.float() @ w.view(K, C).float().t()).double()
    rl = (lib - ref) / ref
    print(f"{dt}: ours mean rel err {r.mean().item():+.2e} (|max| {r.abs().max().item():.2e}); "
          f"torch.mm fp32 {rl.mean().item():+.2e} (|max| {rl.abs().max().item():.2e}); K*eps/4 = {C * 2**-24 / 2:.2e}")
