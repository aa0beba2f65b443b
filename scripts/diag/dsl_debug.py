"""Per-parameter gradient comparison: FUSE_APPLY on vs off on a small ResNet-50 step (GPU)."""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from deeplearning_mpi_amd.models import engine, resnet50  # noqa: E402
from deeplearning_mpi_amd.ops import cross_entropy  # noqa: E402

DEV = "cuda"
torch.manual_seed(0)
m1 = resnet50(num_classes=10).to(DEV)
m2 = copy.deepcopy(m1)
g = torch.Generator(device=DEV).manual_seed(11)
x = torch.randn(16, 3, 96, 96, device=DEV, generator=g)
y = torch.randint(10, (16,), device=DEV, generator=g)
res = {}
for m, on in ((m1, True), (m2, False)):
    engine.FUSE_APPLY = on
    m.arena.zero_grad()
    loss = cross_entropy(m(x), y)
    loss.backward()
    torch.cuda.synchronize()
    res[on] = (loss.item(), {n: p.grad.clone() for n, p in m.named_parameters()}, m.arena.grad.clone())
print("loss", res[True][0], res[False][0])
rows = []
for n, g1 in res[True][1].items():
    g0 = res[False][1][n]
    d = ((g1 - g0).norm() / g0.norm().clamp_min(1e-12)).item()
    rows.append((d, n))
for d, n in sorted(rows, reverse=True)[:25]:
    print(f"{d:10.3e} {n}")
a, b = res[True][2], res[False][2]
print("arena rel", ((a - b).norm() / b.norm()).item())
