"""Sensitivity of a random-init bf16 ResNet-50 step to fp32 summation order alone: the same model and
batch, all fusions off, once with the streaming 1x1 forward kernel (one BN partial row per block)
and once with the general kernel (one row per tile) -- bit-identical conv outputs, statistics that
differ only in fp32 order.  Prints loss and gradient differences (GPU)."""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from deeplearning_mpi_amd.models import engine, resnet50  # noqa: E402
from deeplearning_mpi_amd.ops import cross_entropy  # noqa: E402
from deeplearning_mpi_amd.ops.backend import NativeBackend  # noqa: E402

DEV = "cuda"
torch.manual_seed(0)
m1 = resnet50(num_classes=10).to(DEV)
m2 = copy.deepcopy(m1)
g = torch.Generator(device=DEV).manual_seed(11)
x = torch.randn(16, 3, 96, 96, device=DEV, generator=g)
y = torch.randint(10, (16,), device=DEV, generator=g)
engine.FUSE_APPLY = False
nb = NativeBackend(DEV)
out = []
for m, st in ((m1, 1), (m2, 0)):
    nb.C.set_conv_stream(st)
    m.arena.zero_grad()
    loss = cross_entropy(m(x), y)
    loss.backward()
    torch.cuda.synchronize()
    out.append((loss.item(), m.arena.grad.clone()))
nb.C.set_conv_stream(-1)
print("loss", out[0][0], out[1][0], "grad rel", ((out[0][1] - out[1][1]).norm() / out[1][1].norm()).item())
