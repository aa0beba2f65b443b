"""Diagnose the split recast under hipGraph capture: one ResNet-50 (8 x 64^2) captured SGD step with
the split recast on (argv[1] == "1") or off, with faulthandler on."""
import faulthandler
import sys

import torch

faulthandler.enable(all_threads=True)
sys.path.insert(0, ".")
from deeplearning_mpi_amd.models import resnet50
from deeplearning_mpi_amd.ops import cross_entropy
from deeplearning_mpi_amd.optim import SGD
from deeplearning_mpi_amd.utils.graphs import CapturedStep

split = sys.argv[1] == "1"
torch.manual_seed(0)
m = resnet50(num_classes=10).cuda().train()
x = torch.randn(8, 3, 64, 64, device="cuda")
y = torch.randint(0, 10, (8,), device="cuda")
m.engine_setup(x.device)
m._be.aux_min_pixels = 0
if not split:
    m._arena._cast_split = None
opt = SGD(m.parameters(), lr=0.1, momentum=0.9)


def step():
    opt.zero_grad()
    loss = cross_entropy(m(x), y)
    loss.backward()
    opt.step()
    return loss


st = CapturedStep(step, warmup=1, inputs=(x, y))
for i in range(3):
    print("step", i, float(st()), "graph", st.graph is not None, "err", st.capture_error, flush=True)
torch.cuda.synchronize()
print("ok split", split, "split_casts", m._arena.split_casts, flush=True)
