"""ResNet-50 bs-256 11-step loss trajectories (tests/test_benchscale_gpu.py's setup) of the native
engine under kernel-choice variants, to tell a numerics change from trajectory chaos.

usage: python scripts/diag/benchscale_variants.py [variant ...]
variants: prod | noautotune | nodefer | nostream | nohalo | nopipe
"""
import sys

import torch

from deeplearning_mpi_amd.data import device_batch
from deeplearning_mpi_amd.models import resnet50
from deeplearning_mpi_amd.ops import cross_entropy
from deeplearning_mpi_amd.optim import SGD

DEV = "cuda"


def run(variant):
    torch.manual_seed(0)
    m = resnet50(num_classes=1000).to(DEV)
    m.engine_setup(DEV)
    C = m._be.C
    C.set_conv_autotune(0 if variant == "noautotune" else -1)
    C.set_conv_stream(0 if variant == "nostream" else -1)
    C.set_conv_halo(0 if variant == "nohalo" else -1)
    C.set_conv_pipe(0 if variant == "nopipe" else -1)
    if variant == "nodefer":
        m._be.wgrad_defer = None
    x, y = device_batch("classification", 256, torch.device(DEV), (3, 224, 224), 1000, seed=1234)
    opt = SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-5)
    lo = []
    for _ in range(11):
        opt.zero_grad()
        loss = cross_entropy(m(x), y)
        loss.backward()
        opt.step()
        lo.append(round(float(loss.detach()), 4))
    for f in (C.set_conv_autotune, C.set_conv_stream, C.set_conv_halo, C.set_conv_pipe):
        f(-1)
    print(variant, lo, flush=True)


if __name__ == "__main__":
    for v in sys.argv[1:] or ["prod"]:
        run(v)
