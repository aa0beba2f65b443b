"""Streaming 1x1 data gradient (csrc/kernels/conv1x1_dgrad_stream.hip) against the general
implicit-GEMM kernel: persistent blocks with resident weights that prefetch the next tile's A and
its epilogue operands (residual gradient, BN input z, ReLU mask bits) under the current tile's
epilogue.  dx must be bit-identical (same MFMA dot products, same fp32 epilogue order, one bf16
rounding), the BN-backward partials equal up to fp32 summation order, masked lanes exactly zero,
and a dx written into the left half of a [rows][2C] buffer (the dual data-gradient layout) must
leave the right half untouched."""
import pytest
import torch

from deeplearning_mpi_amd.models.engine import BwdFuse
from deeplearning_mpi_amd.ops.act import Act
from deeplearning_mpi_amd.ops.backend import NativeBackend

pytestmark = pytest.mark.gpu
DEV = "cuda"

SHAPES = [
    # N, H, W, K (dy channels = GEMM reduction), C (dx channels)
    (4, 14, 14, 128, 256),     # 784 rows: 12.25 tiles of 64 (ragged last tile)
    (2, 7, 9, 256, 512),       # 126 rows: tiles of 32, ragged
    (3, 5, 7, 128, 128),       # 105 rows, one 128-channel column
    (8, 28, 28, 256, 512),
    (32, 56, 56, 128, 256),    # layer-1 scale (100k rows, every block walks many tiles)
    (4, 14, 14, 512, 64),      # long reduction into 64-channel tiles
    (2, 28, 28, 512, 128),
    (2, 14, 14, 512, 512),     # layer-3.0 conv1 dual / layer-4 conv1 widths
]


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def _run(nb, mode_on, dy, wT, C, res, fuse, out_layout, bias):
    N, H, W = dy.N, dy.H, dy.W
    nb.C.set_dgrad_stream(mode_on)
    if out_layout == "dual":
        buf = torch.full((N * H * W, 2 * C), 7.0, device=DEV).to(torch.bfloat16)
        dx = Act(buf, N, H, W, C, 0)
    else:
        dx = Act.empty(N, H, W, C, torch.bfloat16, DEV)
    part = nb.conv_dgrad(dy, wT, C, 1, 1, 1, 0, dx, res=res, fuse=fuse, bias=bias)
    torch.cuda.synchronize()
    ran = nb.C.dgrad_stream_last()
    nb.C.set_dgrad_stream(-1)
    return dx, part, ran


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("mode", ["bits", "bits_z2", "from_z", "from_z2", "res_only", "plain"])
def test_dgrad_stream_matches_general_kernel(shape, mode):
    N, H, W, K, C = shape
    nb = NativeBackend(DEV)
    g = torch.Generator(device=DEV).manual_seed(N * 1000 + K + C)
    rows = N * H * W
    dy = Act(torch.randn(rows, K, device=DEV, generator=g).to(torch.bfloat16), N, H, W, K)
    wT = (torch.randn(C, 1, 1, K, device=DEV, generator=g) / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn(C, device=DEV, generator=g) * 0.1 if mode in ("bits", "bits_z2", "res_only") else None
    res = None
    if mode in ("bits", "bits_z2", "res_only"):
        res = Act(torch.randn(rows, C, device=DEV, generator=g).to(torch.bfloat16), N, H, W, C)
    fuse = None
    z = z2 = None
    if mode.endswith("z2"):
        z2 = Act(torch.randn(rows, C, device=DEV, generator=g).to(torch.bfloat16), N, H, W, C)
    if mode.startswith("bits"):
        z = Act(torch.randn(rows, C, device=DEV, generator=g).to(torch.bfloat16), N, H, W, C)
        y = torch.randn(rows, C, device=DEV, generator=g)
        pos = (y > 0).view(-1, C // 8, 8).to(torch.uint8)
        mb = (pos * (2 ** torch.arange(8, device=DEV, dtype=torch.uint8))).sum(-1).to(torch.uint8).contiguous()
        fuse = BwdFuse(None, z, z2, mbits=mb)
        keep = y > 0
    elif mode.startswith("from_z"):
        z = Act(torch.randn(rows, C, device=DEV, generator=g).to(torch.bfloat16), N, H, W, C)
        sc, sh = torch.rand(C, device=DEV, generator=g) + 0.5, torch.randn(C, device=DEV, generator=g) * 0.5
        fuse = BwdFuse(None, z, z2, sc, sh)
        keep = torch.addcmul(sh, z.buf.float(), sc) > 0
    for layout in ("dense", "dual"):
        # mode 2: also the opt-in variants (K = 512 with a residual / mask bits / z2 on 32 x 64 tiles)
        dx1, p1, ran1 = _run(nb, 2, dy, wT, C, res, fuse, layout, bias)
        dx0, p0, ran0 = _run(nb, 0, dy, wT, C, res, fuse, layout, bias)
        assert ran1 == 1 and ran0 == 0
        if K <= 256:
            assert torch.equal(dx1.buf, dx0.buf), (layout, _rel(dx1.buf, dx0.buf))
        else:   # the general kernel may split the 8 K-steps of a small grid (split-K): another fp32 order
            assert _rel(dx1.buf, dx0.buf) < 1e-2, (layout, _rel(dx1.buf, dx0.buf))
        if layout == "dual":
            assert bool((dx1.buf[:, C:].float() == 7.0).all())
        d = dx1.buf[:, :C]
        if fuse is None:
            assert p1 is None and p0 is None
            continue
        assert (d[~keep] == 0).all()
        ns = 3 if z2 is not None else 2
        assert p1.shape[1:] == p0.shape[1:] == (ns, C)
        v = d.double()
        ref = [v.sum(0), (v * z.buf.double()).sum(0)] + ([(v * z2.buf.double()).sum(0)] if z2 is not None else [])
        s1, s0 = p1.double().sum(0), p0.double().sum(0)
        v0 = dx0.buf[:, :C].double()   # K > 256: the general kernel's own dx (another fp32 order)
        ref0 = [v0.sum(0), (v0 * z.buf.double()).sum(0)] + ([(v0 * z2.buf.double()).sum(0)] if z2 is not None else [])
        for k, (r, r0) in enumerate(zip(ref, ref0)):
            scale = r.abs().max().clamp_min(1e-3)
            assert ((s1[k] - r).abs().max() / scale).item() < 1e-4, (k, layout)
            assert ((s0[k] - r0).abs().max() / scale).item() < 1e-4, (k, layout)


def test_dgrad_stream_dual_bottleneck_bit_identical():
    """The production ResNet-50 step path with the dual layout on every eligible 1x1: the streaming
    data gradient on vs off gives the same loss and gradients equal up to the fp32 summation order
    of the fused BN partials (which feeds every BN backward upstream of it)."""
    import copy

    from deeplearning_mpi_amd.models import engine, resnet50
    from deeplearning_mpi_amd.ops import cross_entropy

    torch.manual_seed(0)
    m1 = resnet50(num_classes=10).to(DEV)
    m2 = copy.deepcopy(m1)
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(16, 3, 112, 112, device=DEV, generator=g)
    y = torch.randint(10, (16,), device=DEV, generator=g)
    nb = NativeBackend(DEV)
    losses = []
    old = engine.DUAL_MIN_ROWS
    engine.DUAL_MIN_ROWS = 0   # the dual layout on every eligible 1x1 (K = 2 x 64 / 2 x 128)
    try:
        for m, on in ((m1, 1), (m2, 0)):
            nb.C.set_dgrad_stream(on)
            m.arena.zero_grad()
            loss = cross_entropy(m(x), y)
            loss.backward()
            losses.append(loss.detach())
        torch.cuda.synchronize()
    finally:
        nb.C.set_dgrad_stream(-1)
        engine.DUAL_MIN_ROWS = old
    assert torch.equal(losses[0], losses[1])
    g1, g2 = m1.arena.grad, m2.arena.grad
    assert torch.isfinite(g1).all()
    assert ((g1 - g2).norm() / g2.norm()).item() < 3e-2
