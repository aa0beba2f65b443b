"""Which statistics columns of the streaming dgrad (z2 case, 512 -> 512) disagree with fp64 sums."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from deeplearning_mpi_amd.models.engine import BwdFuse  # noqa: E402
from deeplearning_mpi_amd.ops.act import Act  # noqa: E402
from deeplearning_mpi_amd.ops.backend import NativeBackend  # noqa: E402

DEV = "cuda"
nb = NativeBackend(DEV)
for (N, H, W, K, C, z2on, bits) in [(2, 14, 14, 512, 512, True, True), (2, 14, 14, 512, 512, False, True),
                                     (2, 14, 14, 512, 512, True, False), (8, 14, 14, 512, 128, True, True)]:
    g = torch.Generator(device=DEV).manual_seed(7)
    rows = N * H * W
    dy = Act(torch.randn(rows, K, device=DEV, generator=g).to(torch.bfloat16), N, H, W, K)
    wT = (torch.randn(C, 1, 1, K, device=DEV, generator=g) / K ** 0.5).to(torch.bfloat16)
    res = Act(torch.randn(rows, C, device=DEV, generator=g).to(torch.bfloat16), N, H, W, C)
    z = Act(torch.randn(rows, C, device=DEV, generator=g).to(torch.bfloat16), N, H, W, C)
    z2 = Act(torch.randn(rows, C, device=DEV, generator=g).to(torch.bfloat16), N, H, W, C) if z2on else None
    if bits:
        yv = torch.randn(rows, C, device=DEV, generator=g)
        pos = (yv > 0).view(-1, C // 8, 8).to(torch.uint8)
        mb = (pos * (2 ** torch.arange(8, device=DEV, dtype=torch.uint8))).sum(-1).to(torch.uint8).contiguous()
        fuse = BwdFuse(None, z, z2, mbits=mb)
    else:
        fuse = BwdFuse(None, z, z2, torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV))
    nb.C.set_dgrad_stream(1)
    dx = Act.empty(N, H, W, C, torch.bfloat16, DEV)
    p = nb.conv_dgrad(dy, wT, C, 1, 1, 1, 0, dx, res=res if bits else None, fuse=fuse)
    torch.cuda.synchronize()
    print("ran", nb.C.dgrad_stream_last(), "shape", (N, H, W, K, C), "z2", z2on, "bits", bits, "G", p.shape[0])
    v = dx.buf.double()
    refs = [v.sum(0), (v * z.buf.double()).sum(0)] + ([(v * z2.buf.double()).sum(0)] if z2on else [])
    s = p.double().sum(0)
    for k, r in enumerate(refs):
        err = (s[k] - r).abs()
        bad = (err > 1e-4 * r.abs().max()).nonzero().flatten().tolist()
        print(f"  stat {k}: max rel err {(err.max() / r.abs().max()).item():.3g}, bad cols {len(bad)}: {bad[:24]}")
        if bad:
            c = bad[0]
            print("   col", c, "got", s[k][c].item(), "ref", r[c].item(), "rows", [p[gg, k, c].item() for gg in range(min(4, p.shape[0]))])
nb.C.set_dgrad_stream(-1)
