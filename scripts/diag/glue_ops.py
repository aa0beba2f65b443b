"""List the torch (aten) ops that launch device work inside one eager training step of the native
engine, with their Python call sites: every GPU kernel of the step should be ours."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from deeplearning_mpi_amd.models import ARCHS  # noqa: E402
from deeplearning_mpi_amd.ops import backward, cross_entropy  # noqa: E402
from deeplearning_mpi_amd.optim import SGD  # noqa: E402

arch = sys.argv[1] if len(sys.argv) > 1 else "resnet18"
prec = sys.argv[2] if len(sys.argv) > 2 else "fp32"
dev = "cuda"
m = ARCHS[arch](num_classes=10).to(dev)
m.precision = prec
opt = SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-4)
x = torch.randn(128, 3, 32, 32, device=dev)
y = torch.randint(10, (128,), device=dev)


def step():
    opt.zero_grad()
    loss = cross_entropy(m(x), y)
    backward(loss)
    opt.step()


for _ in range(3):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
    step()
    torch.cuda.synchronize()
IGN = {"aten::empty", "aten::view", "aten::as_strided", "aten::slice", "aten::select", "aten::reshape",
       "aten::permute", "aten::detach", "aten::alias", "aten::t", "aten::transpose", "aten::expand",
       "aten::unsqueeze", "aten::squeeze", "aten::empty_strided", "aten::_reshape_alias", "aten::lift_fresh",
       "aten::resolve_conj", "aten::resolve_neg", "aten::result_type", "aten::empty_like", "aten::item",
       "aten::_local_scalar_dense", "aten::is_nonzero", "aten::record_stream", "aten::set_", "aten::narrow",
       "aten::unbind", "aten::split", "aten::chunk", "aten::numel", "aten::size", "aten::stride", "aten::dim"}
seen = {}
for ev in prof.events():
    if not ev.name.startswith("aten::") or ev.name in IGN:
        continue
    st = [f for f in (ev.stack or []) if "deeplearning_mpi_amd" in f or "glue_ops" in f]
    key = (ev.name, st[0] if st else "?")
    seen[key] = seen.get(key, 0) + 1
for (name, site), n in sorted(seen.items(), key=lambda t: -t[1]):
    print(f"{n:4d}  {name:28s} {site}")


# call sites of the remaining device-work torch calls (TorchFunctionMode sees every torch API call)
import traceback  # noqa: E402

from torch.overrides import TorchFunctionMode  # noqa: E402

WATCH = ("zeros", "zero_", "fill_", "add_", "copy_", "index", "cat", "stack", "ones_like", "clone", "to", "mul_",
         "sum", "zeros_like")


class Log(TorchFunctionMode):
    def __torch_function__(self, func, types, args=(), kwargs=None):
        name = getattr(func, "__name__", str(func))
        if name in WATCH:
            st = [f for f in traceback.extract_stack()[:-1] if "deeplearning_mpi_amd" in f.filename or
                  "glue_ops" in f.filename]
            site = f"{st[-1].filename.split('repo/')[-1]}:{st[-1].lineno}" if st else "?"
            print(f"  call {name:10s} {site}")
        return func(*args, **(kwargs or {}))


with Log():
    step()
torch.cuda.synchronize()
