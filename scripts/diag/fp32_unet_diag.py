"""Per-parameter gradient error of the native fp32 UNet and of the fp32 reference engine vs the
fp64 reference engine (one training step from one init)."""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from deeplearning_mpi_amd.models import UNet  # noqa: E402
from deeplearning_mpi_amd.ops import bce_with_logits  # noqa: E402

DEV = "cuda"
mode = sys.argv[1] if len(sys.argv) > 1 else "conv_transpose"
g = torch.Generator(device=DEV).manual_seed(5)
x = torch.randn(2, 3, 64, 64, device=DEV, generator=g)
y = (torch.rand(2, 64, 64, device=DEV, generator=g) > 0.5).float()
torch.manual_seed(0)
m0 = UNet(out_classes=1, up_sample_mode=mode).to(DEV)
res, outs = [], []
for prec, dt in (("fp32", torch.float32), ("ref", torch.float32), ("ref", torch.float64)):
    m = copy.deepcopy(m0).to(dt)
    m.precision = prec
    m.train()
    o = m(x.to(dt))
    loss = bce_with_logits(o.squeeze(1), y.to(dt))
    loss.backward()
    torch.cuda.synchronize()
    print(prec, dt, type(m._be).__name__, getattr(m._be, "dt", None), "loss", repr(loss.item()), loss.dtype,
          "param dtype", next(m.parameters()).dtype)
    outs.append(o.detach().double())
    res.append({n: p.grad.double().clone() for n, p in m.named_parameters()})


def e(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


print("logits err native %.2e torch32 %.2e" % (e(outs[0], outs[2]), e(outs[1], outs[2])))
print(f"{'param':55s} native  torch32  nat-vs-t32  |g64|")
for n in res[0]:
    a, t, b = res[0][n], res[1][n], res[2][n]
    print(f"{n:55s} {e(a, b):.2e} {e(t, b):.2e} {e(a, t):.2e} {b.norm().item():.3e}")
