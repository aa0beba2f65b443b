"""In-model check of every fused conv1 (conv prologue 3): compare the native fused call against the
unfused pair on the same inputs inside a ResNet-50 forward (GPU)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from deeplearning_mpi_amd.models import resnet50  # noqa: E402
from deeplearning_mpi_amd.ops import cross_entropy  # noqa: E402
from deeplearning_mpi_amd.ops.act import Act  # noqa: E402
from deeplearning_mpi_amd.ops.backend import NativeBackend  # noqa: E402

DEV = "cuda"
orig = NativeBackend.conv_fwd_bn_apply
k = [0]


def check(self, xp, w, K, z, bias, stats, *fin):
    k[0] += 1
    # reference on copies first (the fused call overwrites y / mbits / running stats)
    y2 = Act(torch.empty_like(xp.y.buf), xp.y.N, xp.y.H, xp.y.W, xp.y.C, xp.y.off)
    mb2 = torch.empty_like(xp.mbits)
    self.bn_apply(xp.z, xp.scale, xp.shift, xp.res, xp.relu, y2, mbits=mb2)
    z2 = Act(torch.empty_like(z.buf), z.N, z.H, z.W, z.C, z.off)
    st2 = torch.zeros_like(stats)
    fin2 = list(fin)
    fin2[3] = fin[3].clone() if fin[3] is not None else None
    fin2[4] = fin[4].clone() if fin[4] is not None else None
    fin2[7:11] = [torch.empty_like(t) for t in fin[7:11]]
    self.conv_fwd_bn(y2, w, K, 1, 1, 1, 0, z2, bias, st2, *fin2)
    r = orig(self, xp, w, K, z, bias, stats, *fin)
    torch.cuda.synchronize()
    dy = (xp.y.buf.float() - y2.buf.float()).abs().max().item()
    dm = (xp.mbits != mb2).sum().item()
    dz = (z.buf.float() - z2.buf.float()).abs().max().item()
    print(f"call {k[0]}: x {tuple(xp.z.buf.shape)} ld {xp.z.ld} off {xp.z.off} res ld {getattr(xp.res, 'ld', None)} "
          f"y ld {xp.y.ld} z {tuple(z.buf.shape)} ld {z.ld} off {z.off}  |dy| {dy:.3g} mbits {dm} |dz| {dz:.3g} "
          f"scale {(fin[7] - fin2[7]).abs().max().item():.3g}", flush=True)
    return r


NativeBackend.conv_fwd_bn_apply = check
torch.manual_seed(0)
m = resnet50(num_classes=10).to(DEV)
g = torch.Generator(device=DEV).manual_seed(11)
x = torch.randn(16, 3, 96, 96, device=DEV, generator=g)
y = torch.randint(10, (16,), device=DEV, generator=g)
loss = cross_entropy(m(x), y)
print("loss", loss.item())
