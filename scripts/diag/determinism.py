"""Run-to-run determinism of UNet training (3 SGD steps) under the default schedule and with the
deferred BN passes: identical losses / parameters expected."""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import deeplearning_mpi_amd.models.engine as E  # noqa: E402
from deeplearning_mpi_amd.models import UNet  # noqa: E402
from deeplearning_mpi_amd.ops import bce_with_logits  # noqa: E402
from deeplearning_mpi_amd.optim import SGD  # noqa: E402

DEV = "cuda"
g = torch.Generator(device=DEV).manual_seed(11)
x = torch.randn(2, 3, 64, 64, device=DEV, generator=g)
y = (torch.rand(2, 64, 64, device=DEV, generator=g) > 0.5).float()
torch.manual_seed(0)
m0 = UNet(out_classes=1).to(DEV)


def run(flag, aux):
    E.DEFER_BN_FWD = E.DEFER_BN_BWD = flag
    m = copy.deepcopy(m0)
    m.engine_setup(DEV)
    m._be.aux_min_pixels = 0 if aux else 1 << 40
    opt = SGD(m.parameters(), lr=0.05, momentum=0.9)
    ls = []
    for _ in range(3):
        opt.zero_grad()
        loss = bce_with_logits(m(x).squeeze(1), y)
        loss.backward()
        ls.append(float(loss))
        grads = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        opt.step()
    torch.cuda.synchronize()
    return ls, grads


base = run(False, True)
for tag, flag, aux in (("same", False, True), ("deferred", True, True), ("noaux", False, False),
                       ("deferred-noaux", True, False)):
    ls, gr = run(flag, aux)
    diff = [n for n in gr if not torch.equal(gr[n], base[1][n])]
    print(f"{tag:15s} losses {'==' if ls == base[0] else '!='} {ls} ; grads differing (last step): {len(diff)} {diff[:4]}")
