"""1x1 convolution with <= 4 output channels (the UNet head, csrc/kernels/head.hip): the streaming
dot-product kernel against an fp32 reference of the same op, with channel-slice inputs, fp32 and bf16
outputs, bias and ragged row counts; the dispatch takes it (head1x1_last) and the GEMM path (forced off)
agrees to fp32 summation-order noise; and a UNet forward runs it for its head."""
import pytest
import torch

from deeplearning_mpi_amd.ops.act import Act
from deeplearning_mpi_amd.ops.backend import NativeBackend

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize("C,kv,ld,off,out_f32,M", [
    (64, 1, 64, 0, True, 16 * 96 * 96),     # UNet head width
    (64, 1, 192, 128, True, 5 * 7 * 11),    # channel slice of a wider buffer, ragged rows
    (32, 3, 32, 0, False, 1000),
    (128, 2, 128, 0, True, 4099),
    (512, 4, 512, 0, False, 777),
    (16, 1, 16, 0, True, 3),
])
def test_head1x1_matches_fp32(C, kv, ld, off, out_f32, M):
    be = NativeBackend(DEV)
    g = torch.Generator(device=DEV).manual_seed(C * 7 + kv)
    xb = torch.randn(M, ld, device=DEV, generator=g).to(torch.bfloat16)
    x = Act(xb, M, 1, 1, C, off)
    Kp = 8
    w = (torch.randn(Kp, C, device=DEV, generator=g) / C ** 0.5).to(torch.bfloat16)
    bias = torch.randn(Kp, device=DEV, generator=g)
    yt = torch.full((M, kv), float("nan"), device=DEV, dtype=torch.float32 if out_f32 else torch.bfloat16)
    y = Act(yt, M, 1, 1, kv)
    be.conv_fwd(x, w, Kp, 1, 1, 1, 0, y, bias=bias, kvalid=kv)
    torch.cuda.synchronize()
    assert be.C.head1x1_last() == 1
    ref = xb[:, off:off + C].float() @ w[:kv].float().t() + bias[:kv]
    tol = 1e-5 if out_f32 else 8e-3
    assert _rel(yt.float(), ref) < tol
    # the GEMM path of the same call agrees
    y2t = torch.full_like(yt, float("nan"))
    be.C.set_head1x1(0)
    try:
        be.conv_fwd(x, w, Kp, 1, 1, 1, 0, Act(y2t, M, 1, 1, kv), bias=bias, kvalid=kv)
        torch.cuda.synchronize()
        assert be.C.head1x1_last() == 0
    finally:
        be.C.set_head1x1(1)
    assert _rel(y2t.float(), yt.float()) < tol


def test_unet_forward_runs_head_kernel():
    from deeplearning_mpi_amd.models import UNet

    torch.manual_seed(0)
    m = UNet(out_classes=1).to(DEV)
    x = torch.randn(2, 3, 64, 64, device=DEV)
    out = m(x)
    torch.cuda.synchronize()
    assert m._be.C.head1x1_last() == 1
    assert out.shape == (2, 1, 64, 64) and torch.isfinite(out).all()
