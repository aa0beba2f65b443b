"""Numerics of every gfx950 HIP kernel against the fp32 torch reference backend (same op
semantics, same bf16-rounded inputs).  Shapes follow SURVEY.md §2.5 (ResNet stem / 3x3 / 1x1 /
strided / downsample, UNet concat widths, linear heads, odd tile remainders)."""
import pytest
import torch

from deeplearning_mpi_amd.ops.act import Act, Deferred, pad8
from deeplearning_mpi_amd.models.engine import BwdFuse
from deeplearning_mpi_amd.ops.backend import NativeBackend, RefBackend

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _be():
    return NativeBackend(DEV), RefBackend(DEV)


def _act(N, H, W, C, ld=None, off=0, scale=1.0):
    ld = ld or C
    buf = (torch.randn(N * H * W, ld, device=DEV) * scale).to(torch.bfloat16)
    a = Act(buf, N, H, W, C, off)
    r = Act(buf.float(), N, H, W, C, off)
    return a, r


def _empty(N, H, W, C, dtype=torch.bfloat16, ld=None):
    return Act.empty(N, H, W, C, dtype, DEV, ld)


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


CONV_SHAPES = [
    # N, H, W, Cin, Cout, R, stride, pad
    (2, 32, 32, 3, 64, 7, 2, 3),       # ResNet stem (Cin padded to 8)
    (2, 14, 14, 64, 64, 3, 1, 1),
    (2, 14, 14, 128, 128, 3, 2, 1),
    (3, 7, 7, 256, 64, 1, 1, 0),       # M = 147: tile remainders
    (2, 8, 8, 64, 256, 1, 1, 0),
    (2, 14, 14, 256, 512, 1, 2, 0),    # downsample 1x1 stride 2
    (1, 16, 24, 192, 64, 3, 1, 1),     # UNet decoder level-1 concat width
    (2, 15, 20, 512, 1024, 3, 1, 1),   # UNet bottleneck at the reference 240x320 scale
    (2, 4, 4, 512, 512, 3, 1, 1),      # tiny grid, 72 K-steps: in-launch split-K (8 slices)
    (4, 4, 4, 256, 256, 3, 2, 1),      # split-K with stride-2 data-gradient phases
]


@pytest.mark.parametrize("shape", CONV_SHAPES)
def test_conv_fwd(shape):
    nb, rb = _be()
    N, H, W, Cin, K, R, s, p = shape
    Cp, Kp = pad8(Cin), pad8(K)
    x, xr = _act(N, H, W, Cp)
    w = (torch.randn(Kp, R, R, Cp, device=DEV) / (R * R * Cin) ** 0.5).to(torch.bfloat16)
    bias = torch.randn(Kp, device=DEV)
    P, Q = (H + 2 * p - R) // s + 1, (W + 2 * p - R) // s + 1
    res, resr = _act(N, P, Q, Kp)
    y = _empty(N, P, Q, Kp)
    yr = _empty(N, P, Q, Kp, torch.float32)
    mt = nb.conv_mtiles(N, H, W, Cp, Kp, R, R, s, p)
    st = torch.zeros(mt, 2, Kp, device=DEV)
    str_ = torch.zeros(1, 2, Kp, device=DEV)
    nb.conv_fwd(x, w, Kp, R, R, s, p, y, bias=bias, stats=st)
    rb.conv_fwd(xr, w.float(), Kp, R, R, s, p, yr, bias=bias, stats=str_)
    torch.cuda.synchronize()
    assert _rel(y.buf, yr.buf) < 1e-2
    assert _rel(st.sum(0)[0], str_[0, 0]) < 2e-2
    assert _rel(st.sum(0)[1], str_[0, 1]) < 2e-2
    # fused residual + relu + affine
    sc, sh = torch.rand(Kp, device=DEV) + 0.5, torch.randn(Kp, device=DEV)
    nb.conv_fwd(x, w, Kp, R, R, s, p, y, res=res, scale=sc, shift=sh, relu=True)
    rb.conv_fwd(xr, w.float(), Kp, R, R, s, p, yr, res=resr, scale=sc, shift=sh, relu=True)
    assert _rel(y.buf, yr.buf) < 1e-2


@pytest.mark.parametrize("shape", CONV_SHAPES[1:])
def test_conv_dgrad(shape):
    nb, rb = _be()
    N, H, W, Cin, K, R, s, p = shape
    Cp, Kp = pad8(Cin), pad8(K)
    P, Q = (H + 2 * p - R) // s + 1, (W + 2 * p - R) // s + 1
    dy, dyr = _act(N, P, Q, Kp)
    wT = (torch.randn(Cp, R, R, Kp, device=DEV) / (R * R * K) ** 0.5).to(torch.bfloat16)
    res, resr = _act(N, H, W, Cp)
    dx = _empty(N, H, W, Cp)
    dxr = _empty(N, H, W, Cp, torch.float32)
    nb.conv_dgrad(dy, wT, Cp, R, R, s, p, dx, res=res)
    rb.conv_dgrad(dyr, wT.float(), Cp, R, R, s, p, dxr, res=resr)
    torch.cuda.synchronize()
    assert _rel(dx.buf, dxr.buf) < 1e-2


@pytest.mark.parametrize("shape", [(2, 20, 20, 64, 128, 3, 1, 1), (3, 9, 11, 256, 256, 1, 1, 0),
                                   (2, 16, 16, 128, 384, 3, 2, 1), (2, 18, 18, 256, 320, 3, 1, 1),
                                   (2, 17, 19, 64, 64, 3, 1, 1), (2, 16, 16, 32, 64, 3, 1, 1)])
@pytest.mark.parametrize("bn", [0, 64, 256])
def test_conv_fwd_256_row_tile(shape, bn):
    """The 256x128 single-stage tile and the 256x256 tile (the pipelined 8-wave kernel) forced on small
    shapes, incl. BN statistics partials and row/column remainders."""
    nb, rb = _be()
    N, H, W, Cin, K, R, s, p = shape
    if (bn == 64) != (K == 64) or (bn == 256 and Cin < 64):
        pytest.skip("tile does not apply")
    Cp, Kp = pad8(Cin), pad8(K)
    P, Q = (H + 2 * p - R) // s + 1, (W + 2 * p - R) // s + 1
    x, xr = _act(N, H, W, Cp)
    w = (torch.randn(Kp, R, R, Cp, device=DEV) / (R * R * Cin) ** 0.5).to(torch.bfloat16)
    y = _empty(N, P, Q, Kp)
    yr = _empty(N, P, Q, Kp, torch.float32)
    mt = (N * P * Q + 255) // 256
    st = torch.empty(mt, 2, Kp, device=DEV)
    rows = nb.C.conv2d_fwd(x.buf, N, H, W, Cp, Cp, 0, w, Kp, R, R, s, p, y.buf, Kp, 0, None, None, 0, 0, None, None,
                           False, st, 256, 0, bn)
    assert rows == mt
    str_ = torch.empty(1, 2, Kp, device=DEV)
    rb.conv_fwd(xr, w.float(), Kp, R, R, s, p, yr, stats=str_)
    torch.cuda.synchronize()
    assert _rel(y.buf, yr.buf) < 1e-2
    assert _rel(st.sum(0), str_.sum(0)) < 2e-2


@pytest.mark.parametrize("shape", [(2, 20, 20, 64, 256, 1, 1, 0), (3, 9, 11, 128, 512, 1, 1, 0),
                                   (2, 16, 16, 256, 256, 3, 2, 1), (2, 17, 19, 64, 768, 3, 1, 1)])
def test_conv_fwd_128x256_wide_tile(shape):
    """The 128x256 tile (the pipelined 8-wave kernel, conv_pipe_kernel) forced on small shapes: forward
    with BN partials, row remainders, 3x3 / strided taps, and the residual + affine + ReLU epilogue."""
    nb, rb = _be()
    N, H, W, Cin, K, R, s, p = shape
    Cp, Kp = pad8(Cin), pad8(K)
    P, Q = (H + 2 * p - R) // s + 1, (W + 2 * p - R) // s + 1
    x, xr = _act(N, H, W, Cp)
    w = (torch.randn(Kp, R, R, Cp, device=DEV) / (R * R * Cin) ** 0.5).to(torch.bfloat16)
    res, resr = _act(N, P, Q, Kp)
    y = _empty(N, P, Q, Kp)
    yr = _empty(N, P, Q, Kp, torch.float32)
    mt = (N * P * Q + 127) // 128
    st = torch.empty(mt, 2, Kp, device=DEV)
    rows = nb.C.conv2d_fwd(x.buf, N, H, W, Cp, Cp, 0, w, Kp, R, R, s, p, y.buf, Kp, 0, None, None, 0, 0, None, None,
                           False, st, 128, 0, 256)
    assert rows == mt
    str_ = torch.empty(1, 2, Kp, device=DEV)
    rb.conv_fwd(xr, w.float(), Kp, R, R, s, p, yr, stats=str_)
    torch.cuda.synchronize()
    assert _rel(y.buf, yr.buf) < 1e-2
    assert _rel(st.sum(0), str_.sum(0)) < 2e-2
    # residual + affine + relu epilogue through the same tile
    sc, sh = torch.rand(Kp, device=DEV) + 0.5, torch.randn(Kp, device=DEV)
    nb.C.conv2d_fwd(x.buf, N, H, W, Cp, Cp, 0, w, Kp, R, R, s, p, y.buf, Kp, 0, None, res.buf, Kp, 0, sc, sh,
                    True, None, 128, 0, 256)
    rb.conv_fwd(xr, w.float(), Kp, R, R, s, p, yr, res=resr, scale=sc, shift=sh, relu=True)
    torch.cuda.synchronize()
    assert _rel(y.buf, yr.buf) < 1e-2


def test_wide_tile_bit_identical_to_128x128():
    """At a bench shape (ResNet-50 layer-1 expand, 16 images) the 128x256 tile and the default
    128x128 tile give bit-identical outputs (same per-element K order) and equal BN partial sums
    up to fp32 summation order."""
    nb, rb = _be()
    N, H, W, C, K = 16, 56, 56, 64, 256
    x, xr = _act(N, H, W, C)
    w = (torch.randn(K, 1, 1, C, device=DEV) / C ** 0.5).to(torch.bfloat16)
    ys, sts = [], []
    for bn in (256, 128):
        y = _empty(N, H, W, K)
        st = torch.empty((N * H * W + 127) // 128, 2, K, device=DEV)
        nb.C.conv2d_fwd(x.buf, N, H, W, C, C, 0, w, K, 1, 1, 1, 0, y.buf, K, 0, None, None, 0, 0, None, None,
                        False, st, 128, 0, bn)
        ys.append(y.buf)
        sts.append(st)
    torch.cuda.synchronize()
    assert torch.equal(ys[0], ys[1])
    assert torch.allclose(sts[0].double().sum(0), sts[1].double().sum(0), rtol=1e-5, atol=1e-2)


PIPE_SHAPES = [(2, 14, 14, 256, 256, 3, 1, 1), (3, 7, 7, 512, 512, 3, 1, 1), (2, 16, 16, 128, 256, 3, 2, 1),
               (4, 14, 14, 1024, 256, 1, 1, 0), (2, 28, 28, 128, 128, 3, 1, 1), (1, 32, 32, 64, 64, 3, 1, 1),
               (2, 9, 11, 192, 320, 3, 1, 1), (2, 14, 14, 512, 1024, 1, 2, 0)]


@pytest.mark.parametrize("shape", PIPE_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_pipelined_conv_bit_identical_to_single_stage(shape):
    """The pipelined 8-wave kernel (LDS ring, counted vmcnt, one barrier per K-step) forced on against
    the single-stage gather kernel: forward with BN partials and the data gradient (incl. stride-2
    sub-pixel phases, ragged M / Kout tails) -- same K order, so bit-identical outputs; statistics
    column sums equal to fp32 rounding; bit-reproducible from run to run."""
    nb, _ = _be()
    N, H, W, Cin, K, R, s, p = shape
    Cp, Kp = pad8(Cin), pad8(K)
    P, Q = (H + 2 * p - R) // s + 1, (W + 2 * p - R) // s + 1
    torch.manual_seed(3)
    x, _ = _act(N, H, W, Cp)
    w = (torch.randn(Kp, R, R, Cp, device=DEV) / (R * R * Cin) ** 0.5).to(torch.bfloat16)
    dy, _ = _act(N, P, Q, Kp)
    wT = w.permute(3, 1, 2, 0).contiguous()
    out = {}
    C = nb.C
    try:
        C.set_conv_halo(0)
        C.set_conv3_stream(0)
        C.set_conv_stream(0)
        C.set_dgrad_stream(0)
        C.set_conv_autotune(0)
        C.set_conv_splitk(1)   # the single-stage kernel would split small grids' K (another order)
        for mode in (0, 1, 1):
            C.set_conv_pipe(mode)
            y = _empty(N, P, Q, Kp)
            st = torch.zeros(nb.conv_mtiles(N, H, W, Cp, Kp, R, R, s, p), 2, Kp, device=DEV)
            nb.conv_fwd(x, w, Kp, R, R, s, p, y, stats=st)
            dx = _empty(N, H, W, Cp)
            nb.conv_dgrad(dy, wT, Cp, R, R, s, p, dx)
            torch.cuda.synchronize()
            out.setdefault(mode, []).append((y.buf.clone(), st.double().sum(0), dx.buf.clone()))
    finally:
        for f in (C.set_conv_pipe, C.set_conv_halo, C.set_conv_stream, C.set_dgrad_stream, C.set_conv_autotune,
                  C.set_conv3_stream):
            f(-1)
        C.set_conv_splitk(0)
    base, p1, p2 = out[0][0], out[1][0], out[1][1]
    assert torch.equal(p1[0], p2[0]) and torch.equal(p1[1], p2[1]) and torch.equal(p1[2], p2[2])
    assert torch.equal(p1[0], base[0]), "forward differs from the single-stage kernel"
    assert torch.equal(p1[2], base[2]), "data gradient differs from the single-stage kernel"
    assert _rel(p1[1], base[1]) < 1e-5


@pytest.mark.parametrize("shape", [CONV_SHAPES[1], CONV_SHAPES[2], CONV_SHAPES[3], CONV_SHAPES[5]])
@pytest.mark.parametrize("mode", ["mask", "two", "from_z", "bits"])
def test_conv_dgrad_fused_bn_backward(shape, mode):
    """dgrad epilogue: + residual, ReLU mask of the consumer, BN-backward partials
    {sum dx, sum dx*z [, sum dx*z2]} (multi-phase tile numbering for stride 2), then the
    finalize/apply path that consumes them."""
    nb, rb = _be()
    N, H, W, Cin, K, R, s, p = shape
    Cp, Kp = pad8(Cin), pad8(K)
    P, Q = (H + 2 * p - R) // s + 1, (W + 2 * p - R) // s + 1
    dy, dyr = _act(N, P, Q, Kp)
    wT = (torch.randn(Cp, R, R, Kp, device=DEV) / (R * R * K) ** 0.5).to(torch.bfloat16)
    res, resr = _act(N, H, W, Cp)
    m, mr = _act(N, H, W, Cp)
    z, zr = _act(N, H, W, Cp)
    two = mode == "two"
    z2, z2r = _act(N, H, W, Cp) if two else (None, None)
    sc = sh = None
    mb = None
    if mode == "from_z":   # mask recomputed from the BN input: z*scale + shift > 0
        sc, sh = torch.rand(Cp, device=DEV) + 0.5, torch.randn(Cp, device=DEV) * 0.5
        m = mr = None
    if mode == "bits":     # mask bits of y as written by the forward BN-apply
        pos = (m.buf.float() > 0).view(-1, Cp // 8, 8).to(torch.uint8)
        mb = (pos * (2 ** torch.arange(8, device=DEV, dtype=torch.uint8))).sum(-1).to(torch.uint8).contiguous()
    dx = _empty(N, H, W, Cp)
    dxr = _empty(N, H, W, Cp, torch.float32)
    part = nb.conv_dgrad(dy, wT, Cp, R, R, s, p, dx, res=res,
                         fuse=BwdFuse(None if mb is not None else m, z, z2, sc, sh, mb))
    rb.conv_dgrad(dyr, wT.float(), Cp, R, R, s, p, dxr, res=resr, fuse=BwdFuse(mr, zr, z2r, sc, sh))
    torch.cuda.synchronize()
    assert part.shape[1] == (3 if two else 2) and part.shape[2] == Cp
    assert _rel(dx.buf, dxr.buf) < 1e-2
    keep = (m.buf > 0) if m is not None else (z.buf.float() * sc + sh > 0)
    assert (dx.buf[~keep] == 0).all()   # masked lanes are exactly zero
    # partials are sums of the stored bf16 gradient: compare against the same sums in fp64
    v = dx.buf.double()
    ref = [v.sum(0), (v * z.buf.double()).sum(0)] + ([(v * z2.buf.double()).sum(0)] if two else [])
    got = part.double().sum(0)
    for k, r in enumerate(ref):
        assert ((got[k] - r).abs().max() / r.abs().max()).item() < 1e-4, k
    # consumer side: finalize from the fused partials == unfused reduction of the masked grad
    C = Cp
    mean, invstd = torch.randn(C, device=DEV) * 0.1, torch.rand(C, device=DEV) + 0.5
    gamma = torch.rand(C, device=DEV) + 0.5
    dg1, db1, dg2, db2 = (torch.zeros(C, device=DEV) for _ in range(4))
    o1, o2 = _empty(N, H, W, C), _empty(N, H, W, C)
    nb.bn_bwd(dx, None, z, mean, invstd, gamma, dg1, db1, o1, pre=part, k2=1)
    nb.bn_bwd(dx, None, z, mean, invstd, gamma, dg2, db2, o2)
    torch.cuda.synchronize()
    assert _rel(db1, db2) < 1e-4 and _rel(dg1, dg2) < 1e-3
    assert _rel(o1.buf, o2.buf) < 1e-2


@pytest.mark.parametrize("shape", CONV_SHAPES)
def test_conv_wgrad(shape):
    nb, rb = _be()
    N, H, W, Cin, K, R, s, p = shape
    Cp, Kp = pad8(Cin), pad8(K)
    P, Q = (H + 2 * p - R) // s + 1, (W + 2 * p - R) // s + 1
    x, xr = _act(N, H, W, Cp)
    dy, dyr = _act(N, P, Q, Kp)
    g = torch.randn(K * R * R * Cin, device=DEV)
    gr = g.clone()
    nb.conv_wgrad(dy, x, R, R, s, p, g, Cin, K)
    rb.conv_wgrad(dyr, xr, R, R, s, p, gr, Cin, K)
    torch.cuda.synchronize()
    assert _rel(g, gr) < 5e-3


def test_wgrad_reduce_batched_bit_identical():
    """Deferred weight-gradient split reductions (set_wgrad_defer, the engine backward's mode): 19
    gradients of mixed kinds (gather / 1x1 direct / 3x3 spatial-tile kernels; two-stage and
    direct reductions; channel un-padding) queued and launched as batched kernels -- the queue
    flushes at 16 entries, when a gradient is accumulated twice, and when deferral ends -- give
    bit-identical gradients to the immediate two-launch reductions, in a handful of launches."""
    nb, _ = _be()
    C = nb.C
    torch.manual_seed(3)
    jobs = []
    shapes = CONV_SHAPES + [(64, 14, 14, 256, 128, 3, 1, 1), (8, 28, 28, 64, 64, 1, 1, 0), (2, 56, 56, 64, 64, 1, 1, 0)]
    for sh in shapes + shapes[:6]:
        N, H, W, Cin, K, R, s, p = sh
        Cp, Kp = pad8(Cin), pad8(K)
        P, Q = (H + 2 * p - R) // s + 1, (W + 2 * p - R) // s + 1
        jobs.append((_act(N, H, W, Cp)[0], _act(N, P, Q, Kp)[0], R, s, p, Cin, K))
    jobs = jobs[:19]
    g0 = [torch.randn(K * R * R * Cin, device=DEV) for (_, _, R, _, _, Cin, K) in jobs]

    def run(defer):
        gs = [g.clone() for g in g0]
        n0 = C.wgrad_reduce_launches()
        C.set_wgrad_defer(defer)
        try:
            for i, (x, dy, R, s, p, Cin, K) in enumerate(jobs):
                nb.conv_wgrad(dy, x, R, R, s, p, gs[i], Cin, K)
                if i == 17:   # the same gradient slot accumulated twice inside one queue
                    nb.conv_wgrad(dy, x, R, R, s, p, gs[i], Cin, K)
            if defer:
                assert C.wgrad_pending() > 0
        finally:
            C.set_wgrad_defer(False)
        assert C.wgrad_pending() == 0
        torch.cuda.synchronize()
        return gs, C.wgrad_reduce_launches() - n0

    imm, n_imm = run(False)
    dfr, n_dfr = run(True)
    for i, (a, b) in enumerate(zip(imm, dfr)):
        assert torch.equal(a, b), i
    assert n_dfr <= 6 < n_imm, (n_dfr, n_imm)   # 3 flushes of at most 2 launches


HALO_SHAPES = [
    # N, H, W, Cin, Cout, x channel stride / offset (a concat slice)
    (2, 16, 16, 64, 64, None, 0),        # 8 x 16 tiles
    (2, 14, 14, 256, 256, None, 0),      # 9 x 14 tiles (ResNet layer 3)
    (3, 7, 7, 512, 512, None, 0),        # 18 x 7 tiles, ragged rows (ResNet layer 4)
    (1, 28, 30, 128, 128, None, 0),
    (2, 9, 37, 64, 192, 192, 64),        # 192 outputs: a 64-wide last tile column; x a channel slice
    (4, 56, 56, 64, 64, None, 0),        # ResNet layer 1
    (2, 4, 4, 512, 512, None, 0),        # tiny grid: split-K over chunk-major K-steps
]


@pytest.mark.parametrize("shape", HALO_SHAPES, ids=lambda s: "x".join(str(v) for v in s[:5]))
def test_conv3x3_halo_tiles(shape):
    """3x3 / stride-1 / pad-1 forward (with BN statistics) and data gradient (with the fused
    BN-backward epilogue, mask from z) by 2-D halo tiles vs the im2col gather path and the fp32
    reference: same bf16 products, fp32 sums in another order (chunk-major K)."""
    nb, rb = _be()
    N, H, W, Cin, K, ldx, xoff = shape
    x, xr = _act(N, H, W, Cin, ld=ldx, off=xoff)
    w = (torch.randn(K, 3, 3, Cin, device=DEV) / (9 * Cin) ** 0.5).to(torch.bfloat16)
    wT = w.permute(3, 1, 2, 0).contiguous()
    dy, dyr = _act(N, H, W, K)
    z, _ = _act(N, H, W, Cin)
    sc, sh = torch.rand(Cin, device=DEV) + 0.5, torch.randn(Cin, device=DEV) * 0.5
    out = {}
    nb.C.set_conv3_stream(0)   # 64 -> 64: the halo kernel itself, not the streaming 3x3 kernel
    for mode in (2, 0):   # 2: halo tiles on any grid (the default keeps them to >= 28 x 28)
        nb.C.set_conv_halo(mode)
        y = _empty(N, H, W, K)
        mt = nb.conv_mtiles(N, H, W, Cin, K, 3, 3, 1, 1)
        st = torch.zeros(mt, 2, K, device=DEV)
        rows = nb.conv_fwd(x, w, K, 3, 3, 1, 1, y, stats=st)
        assert rows <= mt and nb.C.conv_halo_last() == (mode == 2)
        dx = _empty(N, H, W, Cin)
        part = nb.conv_dgrad(dy, wT, Cin, 3, 3, 1, 1, dx, fuse=BwdFuse(None, z, None, sc, sh))
        assert nb.C.conv_halo_last() == (mode == 2)
        torch.cuda.synchronize()
        out[mode] = (y.buf.clone(), st.double().sum(0), dx.buf.clone(), part.double().sum(0), mt)
    nb.C.set_conv_halo(-1)
    nb.C.set_conv3_stream(-1)
    yr = _empty(N, H, W, K, torch.float32)
    rb.conv_fwd(xr, w.float(), K, 3, 3, 1, 1, yr)
    dxr = _empty(N, H, W, Cin, torch.float32)
    rb.conv_dgrad(dyr, wT.float(), Cin, 3, 3, 1, 1, dxr)
    torch.cuda.synchronize()
    h, g = out[2], out[0]
    assert _rel(h[0], yr.buf) < 1e-2 and _rel(h[0], g[0]) < 1e-2
    assert _rel(h[1], g[1]) < 5e-4   # sums of bf16 outputs that may round the other way
    keep = (z.buf.float() * sc + sh) > 0
    assert _rel(h[2], torch.where(keep, dxr.buf, torch.zeros_like(dxr.buf))) < 1e-2
    assert _rel(h[2], g[2]) < 1e-2
    assert _rel(h[3], g[3]) < 1e-3


HALO_PIPE_SHAPES = [
    # N, H, W, Cin, Cout, x channel stride / offset: shapes on 256 x 128 halo tiles (Cout >= 256)
    (2, 16, 16, 64, 256, None, 0),        # one 64-channel chunk: 9 K-steps (odd)
    (2, 14, 14, 256, 256, None, 0),       # ResNet layer 3, 4 chunks
    (1, 28, 30, 128, 384, None, 0),       # ragged tiles, 3 output tile columns
    (2, 9, 37, 64, 256, 192, 64),         # x a channel slice of a concat buffer
    (1, 32, 32, 512, 512, None, 0),       # UNet bottleneck-like, 8 chunks; dgrad on 256 x 128 too
    (2, 4, 4, 512, 512, None, 0),         # tiny grid: split-K keeps the single-stage kernel
]


@pytest.mark.parametrize("shape", HALO_PIPE_SHAPES, ids=lambda s: "x".join(str(v) for v in s[:5]))
def test_halo_pipe_bit_identical(shape):
    """conv_halo_pipe_kernel (the 256 x 128 halo tile with a double-buffered weight tile) against the
    single-stage halo kernel: same K order and epilogue, so forward output + BN statistics and the data
    gradient + fused BN-backward partials are bit-identical."""
    nb, _ = _be()
    N, H, W, Cin, K, ldx, xoff = shape
    x, _ = _act(N, H, W, Cin, ld=ldx, off=xoff)
    w = (torch.randn(K, 3, 3, Cin, device=DEV) / (9 * Cin) ** 0.5).to(torch.bfloat16)
    wT = w.permute(3, 1, 2, 0).contiguous()
    dy, _ = _act(N, H, W, K)
    z, _ = _act(N, H, W, Cin)
    sc, sh = torch.rand(Cin, device=DEV) + 0.5, torch.randn(Cin, device=DEV) * 0.5
    out = {}
    nb.C.set_conv_halo(2)   # halo tiles on any grid
    try:
        for on in (1, 0):
            nb.C.set_halo_pipe(on)
            y = _empty(N, H, W, K)
            mt = nb.conv_mtiles(N, H, W, Cin, K, 3, 3, 1, 1)
            st = torch.zeros(mt, 2, K, device=DEV)
            nb.conv_fwd(x, w, K, 3, 3, 1, 1, y, stats=st)
            assert nb.C.conv_halo_last()
            dx = _empty(N, H, W, Cin)
            part = nb.conv_dgrad(dy, wT, Cin, 3, 3, 1, 1, dx, fuse=BwdFuse(None, z, None, sc, sh))
            torch.cuda.synchronize()
            out[on] = (y.buf.clone(), st.clone(), dx.buf.clone(), part.clone())
    finally:
        nb.C.set_halo_pipe(1)
        nb.C.set_conv_halo(-1)
    for a, b in zip(out[1], out[0]):
        assert torch.equal(a, b)


CONV3_STREAM_SHAPES = [
    # N, H, W, x channel stride / offset, y channel stride / offset
    (2, 16, 16, None, 0, None, 0),      # one 8 x 16 tile per 8 rows
    (3, 56, 56, None, 0, None, 0),      # ResNet layer 1 (14-wide tiles)
    (2, 37, 23, 192, 64, 128, 64),      # ragged tiles; x and y channel slices (UNet concat buffers)
    (1, 9, 5, None, 0, None, 0),        # fewer tiles than blocks
]


@pytest.mark.parametrize("shape", CONV3_STREAM_SHAPES, ids=lambda s: "x".join(str(v) for v in s[:3]))
def test_conv3x3_stream_64(shape):
    """Streaming 64 -> 64 3x3 kernel (conv3x3_stream.hip): forward with bias + BN statistics, data
    gradient with the fused BN-backward epilogue (mask from z) and plain, against the fp32 reference
    and the halo kernel (same K order and epilogue arithmetic; one-ulp bf16 differences in a few
    elements from the swapped MFMA operands)."""
    nb, rb = _be()
    N, H, W, ldx, xoff, ldy, yoff = shape
    C = K = 64
    x, xr = _act(N, H, W, C, ld=ldx, off=xoff)
    w = (torch.randn(K, 3, 3, C, device=DEV) / (9 * C) ** 0.5).to(torch.bfloat16)
    wT = w.permute(3, 1, 2, 0).contiguous()
    bias = torch.randn(K, device=DEV) * 0.1
    dy, dyr = _act(N, H, W, K)
    z, _ = _act(N, H, W, C)
    sc, sh = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.5
    out = {}
    for mode in (1, 0):   # 1: streaming kernel; 0: the halo kernel (on any grid)
        nb.C.set_conv3_stream(mode)
        nb.C.set_conv_halo(2)
        y = Act(torch.zeros(N * H * W, ldy or K, dtype=torch.bfloat16, device=DEV), N, H, W, K, yoff)
        mt = nb.conv_mtiles(N, H, W, C, K, 3, 3, 1, 1)
        st = torch.zeros(mt, 2, K, device=DEV)
        rows = nb.conv_fwd(x, w, K, 3, 3, 1, 1, y, bias=bias, stats=st)
        assert rows <= mt and nb.C.conv3_stream_last() == mode
        dx = _empty(N, H, W, C)
        part = nb.conv_dgrad(dy, wT, C, 3, 3, 1, 1, dx, fuse=BwdFuse(None, z, None, sc, sh))
        assert nb.C.conv3_stream_last() == mode
        dx2 = _empty(N, H, W, C)
        nb.conv_dgrad(dy, wT, C, 3, 3, 1, 1, dx2)
        assert nb.C.conv3_stream_last() == mode
        torch.cuda.synchronize()
        out[mode] = (y.buf.clone(), st.double().sum(0), dx.buf.clone(), part.double().sum(0), dx2.buf.clone())
    nb.C.set_conv3_stream(-1)
    nb.C.set_conv_halo(-1)
    s_, h_ = out[1], out[0]
    yr = _empty(N, H, W, K, torch.float32)
    rb.conv_fwd(xr, w.float(), K, 3, 3, 1, 1, yr, bias=bias)
    assert _rel(s_[0][:, yoff:yoff + K], yr.buf) < 1e-2
    dxr = _empty(N, H, W, C, torch.float32)
    rb.conv_dgrad(dyr, wT.float(), C, 3, 3, 1, 1, dxr)
    assert _rel(s_[4], dxr.buf) < 1e-2
    keep = (z.buf.float() * sc + sh) > 0
    assert _rel(s_[2], torch.where(keep, dxr.buf, torch.zeros_like(dxr.buf))) < 1e-2
    # same K order, operands swapped (D^T fragments): the fp32 sums round the other way in a few
    # elements -- one bf16 ulp, well under 0.5 % of them
    for a, b in ((s_[0], h_[0]), (s_[2], h_[2]), (s_[4], h_[4])):
        assert int((a != b).sum()) <= max(8, a.numel() // 200) and _rel(a, b) < 8e-3
    assert _rel(s_[1], h_[1]) < 2e-3 and _rel(s_[3], h_[3]) < 2e-3


WGRAD3_SHAPES = [
    # N, H, W, Cin (real), Ko, x channel stride / offset, dy channel stride / offset
    (2, 16, 16, 64, 64, None, 0, None, 0),        # 64 x 64 tiles, 2 x 2 pixel blocks per image
    (2, 13, 11, 128, 64, None, 0, None, 0),       # 64 x 128 tiles; ragged 8 x 8 blocks at both edges
    (3, 9, 20, 64, 128, 192, 64, None, 0),        # 128 x 64 tiles; x a channel slice of a concat buffer
    (2, 7, 7, 256, 256, None, 0, 512, 256),       # dy a channel slice; 7 x 7 = one ragged block
    (1, 40, 24, 60, 128, None, 0, None, 0),       # Cin padded 60 -> 64: un-padded gradient columns
    (64, 14, 14, 256, 128, None, 0, None, 0),     # many pixel splits
]


@pytest.mark.parametrize("shape", WGRAD3_SHAPES, ids=lambda s: "x".join(str(v) for v in s[:5]))
def test_wgrad3x3_spatial_tiles(shape):
    """3x3 / stride-1 / pad-1 weight gradient by 8 x 8 pixel blocks with a staged halo
    (conv_wgrad3.hip) against the fp32 reference, and against the general gather kernel (same bf16
    products, fp32 sums in another order); accumulates into a non-zero gradient slot like the arena."""
    nb, rb = _be()
    N, H, W, Cin, K, ldx, xoff, ldy, dyoff = shape
    Cp = pad8(Cin)
    x, xr = _act(N, H, W, Cp, ld=ldx, off=xoff)
    dy, dyr = _act(N, H, W, K, ld=ldy, off=dyoff)
    g0 = torch.randn(K * 9 * Cin, device=DEV)
    out = {}
    for mode in (1, 0):
        nb.C.set_wgrad3(mode)
        g = g0.clone()
        nb.conv_wgrad(dy, x, 3, 3, 1, 1, g, Cin, K)
        torch.cuda.synchronize()
        assert nb.C.wgrad3_last() == mode
        out[mode] = g
    nb.C.set_wgrad3(-1)
    gr = g0.clone()
    rb.conv_wgrad(dyr, xr, 3, 3, 1, 1, gr, Cin, K)
    torch.cuda.synchronize()
    assert _rel(out[1], gr) < 5e-3
    assert _rel(out[1], out[0]) < 1e-4


def test_linear_heads():
    nb, rb = _be()
    for (N, Cin, K) in [(8, 2048, 1000), (16, 512, 10)]:
        Kp = pad8(K)
        x, xr = _act(N, 1, 1, Cin)
        w = (torch.randn(Kp, 1, 1, Cin, device=DEV) / Cin ** 0.5).to(torch.bfloat16)
        w[K:] = 0
        bias = torch.randn(Kp, device=DEV)
        out = torch.empty(N, K, device=DEV)
        outr = torch.empty(N, K, device=DEV)
        nb.conv_fwd(x, w, Kp, 1, 1, 1, 0, Act(out, N, 1, 1, K), bias=bias, kvalid=K if K < Kp else 0)
        rb.conv_fwd(xr, w.float(), Kp, 1, 1, 1, 0, Act(outr, N, 1, 1, K), bias=bias)
        torch.cuda.synchronize()
        assert _rel(out, outr) < 1e-2


def test_unet_head_1ch():
    nb, rb = _be()
    N, H, W = 2, 16, 16
    x, xr = _act(N, H, W, 64)
    w = (torch.randn(8, 1, 1, 64, device=DEV) / 8).to(torch.bfloat16)
    w[1:] = 0
    bias = torch.zeros(8, device=DEV)
    bias[0] = 0.3
    o = torch.empty(N * H * W, 1, device=DEV)
    orf = torch.empty(N * H * W, 1, device=DEV)
    nb.conv_fwd(x, w, 8, 1, 1, 1, 0, Act(o, N, H, W, 1), bias=bias, kvalid=1)
    rb.conv_fwd(xr, w.float(), 8, 1, 1, 1, 0, Act(orf, N, H, W, 1), bias=bias)
    assert _rel(o, orf) < 1e-2


@pytest.mark.parametrize("stream", [1, 0], ids=["stream", "igemm"])
@pytest.mark.parametrize("N,H,W,Ci,Co", [(2, 8, 12, 256, 256), (2, 4, 4, 1024, 512),   # 2nd: split-K
                                         (2, 8, 12, 128, 128), (3, 5, 7, 256, 256), (2, 6, 8, 64, 64)])
def test_convT(N, H, W, Ci, Co, stream):
    """ConvTranspose2d(2, 2) into a channel slice of a concat buffer: the streaming 1x1 kernel over
    4 Cout columns (C 64 / 128 / 256 where an N-tile fits one sub-pixel block) and the 4-phase
    implicit GEMM, against the fp32 reference; the rest of the buffer is untouched."""
    nb, rb = _be()
    x, xr = _act(N, H, W, Ci)
    wf = (torch.randn(Co, 2, 2, Ci, device=DEV) / Ci ** 0.5).to(torch.bfloat16)
    bias = torch.randn(Co, device=DEV)
    cat = _empty(N, 2 * H, 2 * W, Co + 128)
    cat.buf.fill_(7.0)
    catr = _empty(N, 2 * H, 2 * W, Co + 128, torch.float32)
    nb.C.set_convT_stream(stream)
    try:
        nb.convT_fwd(x, wf, Co, cat.slice(0, Co), bias)
        torch.cuda.synchronize()
        assert nb.C.convT_stream_last() == int(stream and Ci in (128, 256))
    finally:
        nb.C.set_convT_stream(1)
    rb.convT_fwd(xr, wf.float(), Co, catr.slice(0, Co), bias)
    torch.cuda.synchronize()
    assert _rel(cat.nhwc()[..., :Co], catr.nhwc()[..., :Co]) < 1e-2
    assert bool((cat.buf[:, Co:] == 7.0).all())


def test_bn_family():
    nb, rb = _be()
    N, H, W, C = 4, 14, 14, 256
    x, xr = _act(N, H, W, C)
    res, resr = _act(N, H, W, C)
    st, _ = nb.bn_stats(x)
    str_, _ = rb.bn_stats(xr)
    assert _rel(st.sum(0), str_.sum(0)) < 1e-4
    gamma, beta = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
    outs = []
    for be, s in ((nb, st), (rb, str_)):
        rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        v = torch.empty(4, C, device=DEV)
        be.bn_finalize(s, s.shape[0], C, N * H * W, gamma, beta, rm, rv, 0.1, 1e-5, v[0], v[1], v[2], v[3])
        outs.append((v, rm, rv))
    for a, b in zip(outs[0], outs[1]):
        assert _rel(a, b) < 1e-4
    v = outs[0][0]
    y = _empty(N, H, W, C)
    yr = _empty(N, H, W, C, torch.float32)
    bits = torch.empty(N * H * W, C // 8, dtype=torch.uint8, device=DEV)
    nb.bn_apply(x, v[0], v[1], res, True, y, mbits=bits)
    rb.bn_apply(xr, v[0], v[1], resr, True, yr)
    assert _rel(y.buf, yr.buf) < 1e-2
    unpacked = RefBackend._unpack_bits(bits, y).reshape(-1, C)
    assert torch.equal(unpacked, y.buf.float() > 0)   # bit e == (stored y > 0)
    # residual that is itself a BN output, applied on the fly (the ResNet downsample branch)
    rs, rh = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
    y2, y2r = _empty(N, H, W, C), _empty(N, H, W, C, torch.float32)
    bits2 = torch.empty_like(bits)
    nb.bn_apply(x, v[0], v[1], Deferred.bn(res, rs, rh), True, y2, mbits=bits2)
    rb.bn_apply(xr, v[0], v[1], Deferred.bn(resr, rs, rh), True, y2r)
    assert _rel(y2.buf, y2r.buf) < 1e-2
    assert torch.equal(RefBackend._unpack_bits(bits2, y2).reshape(-1, C), y2.buf.float() > 0)
    dy, dyr = _act(N, H, W, C)
    dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    dgr, dbr = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    dx, dxr = _empty(N, H, W, C), _empty(N, H, W, C, torch.float32)
    dyo, dyor = _empty(N, H, W, C), _empty(N, H, W, C, torch.float32)
    yb = Act(y.buf, N, H, W, C)
    nb.bn_bwd(dy, yb, x, v[2], v[3], gamma, dg, db, dx, dyo)
    rb.bn_bwd(dyr, Act(y.buf.float(), N, H, W, C), xr, v[2], v[3], gamma, dgr, dbr, dxr, dyor)
    torch.cuda.synchronize()
    assert _rel(dg, dgr) < 1e-3 and _rel(db, dbr) < 1e-3
    assert _rel(dx.buf, dxr.buf) < 2e-2
    assert _rel(dyo.buf, dyor.buf) < 1e-2


@pytest.mark.parametrize("T,C", [(300, 256), (600, 64), (6272, 64), (1568, 512), (40000, 64)])
def test_bn_finalize_column_paths(T, C):
    """Every finalize path (single-pass T <= 512, the sliced last-arriver kernel beyond) against
    the fp32 reference on random per-tile partials."""
    nb, rb = _be()
    torch.manual_seed(T + C)
    M = T * 128
    x = torch.randn(T, 1, C, device=DEV) * 3 + 1
    st = torch.cat([x, x * x + torch.rand(T, 1, C, device=DEV)], 1) * 128
    gamma, beta = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
    outs = []
    for be in (nb, rb):
        rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        v = torch.empty(4, C, device=DEV)
        be.bn_finalize(st, T, C, M, gamma, beta, rm, rv, 0.1, 1e-5, v[0], v[1], v[2], v[3])
        outs.append((v.clone(), rm, rv))
    torch.cuda.synchronize()
    for a, b in zip(outs[0], outs[1]):
        assert _rel(a, b) < 1e-5


def test_pools_and_layout():
    nb, rb = _be()
    x = torch.randn(2, 3, 20, 18, device=DEV)
    a = nb.nchw_to_nhwc(x, 8)
    ar = rb.nchw_to_nhwc(x, 8)
    assert _rel(a.buf, ar.buf) < 1e-2
    # 2x2 space-to-depth of the padded image (S2D stem input), odd sizes included
    for (H, W, pad) in [(20, 18, 3), (23, 17, 3), (8, 8, 1)]:
        x = torch.randn(2, 3, H, W, device=DEV)
        U, V = (H + 2 * pad + 1) // 2, (W + 2 * pad + 1) // 2
        a, ar = nb.s2d(x, pad, U, V, 4), rb.s2d(x, pad, U, V, 4)
        assert a.buf.shape == ar.buf.shape == (2 * U * V, 16)
        assert torch.equal(a.buf.float(), ar.buf.to(torch.bfloat16).float())
    for (k, s, p, H, W, C) in [(3, 2, 1, 16, 16, 64), (2, 2, 0, 16, 24, 128)]:
        xa, xr = _act(2, H, W, C)
        OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        y, yr = _empty(2, OH, OW, C), _empty(2, OH, OW, C, torch.float32)
        idx = nb.maxpool_fwd(xa, k, s, p, y)
        idxr = rb.maxpool_fwd(xr, k, s, p, yr)
        assert _rel(y.buf, yr.buf) < 1e-6
        dy, dyr = _act(2, OH, OW, C)
        add, addr = _act(2, H, W, C)
        dx, dxr = _empty(2, H, W, C), _empty(2, H, W, C, torch.float32)
        nb.maxpool_bwd(dy, idx, xa, k, s, p, dx, add=add)
        rb.maxpool_bwd(dyr, idxr, xr, k, s, p, dxr, add=addr)
        assert _rel(dx.buf, dxr.buf) < 1e-2
    xa, xr = _act(4, 7, 7, 2048)
    y, yr = _empty(4, 1, 1, 2048), _empty(4, 1, 1, 2048, torch.float32)
    nb.avgpool_fwd(xa, y)
    rb.avgpool_fwd(xr, yr)
    assert _rel(y.buf, yr.buf) < 1e-2
    dx, dxr = _empty(4, 7, 7, 2048), _empty(4, 7, 7, 2048, torch.float32)
    nb.avgpool_bwd(y, dx)
    rb.avgpool_bwd(Act(y.buf.float(), 4, 1, 1, 2048), dxr)
    assert _rel(dx.buf, dxr.buf) < 1e-2
    xa, xr = _act(2, 8, 6, 64)
    y, yr = _empty(2, 16, 12, 64), _empty(2, 16, 12, 64, torch.float32)
    nb.upsample_fwd(xa, y)
    rb.upsample_fwd(xr, yr)
    assert _rel(y.buf, yr.buf) < 1e-2
    dx, dxr = _empty(2, 8, 6, 64), _empty(2, 8, 6, 64, torch.float32)
    nb.upsample_bwd(y, dx)
    rb.upsample_bwd(Act(y.buf.float(), 2, 16, 12, 64), dxr)
    assert _rel(dx.buf, dxr.buf) < 1e-2


def test_maxpool_bwd_fused_bn_stats():
    """ResNet stem: max-pool backward + ReLU mask (from z) + BN-backward partials in one kernel."""
    nb, rb = _be()
    N, H, W, C = 2, 16, 16, 64
    z, zr = _act(N, H, W, C)
    sc, sh = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.3
    y = _empty(N, H, W, C)
    nb.bn_apply(z, sc, sh, None, True, y)
    OH = OW = 8
    p = _empty(N, OH, OW, C)
    idx = nb.maxpool_fwd(y, 3, 2, 1, p)
    # BN-apply + ReLU fused into the pool (the stem's BN output never materialised): same values
    # and the same argmax as pooling the stored bf16 output
    p2 = _empty(N, OH, OW, C)
    idx2 = nb.maxpool_fwd(z, 3, 2, 1, p2, bn=(sc, sh))
    torch.cuda.synchronize()
    assert torch.equal(p2.buf, p.buf) and torch.equal(idx2, idx)
    dy, dyr = _act(N, OH, OW, C)
    dx, dxr = _empty(N, H, W, C), _empty(N, H, W, C, torch.float32)
    part = nb.maxpool_bwd(dy, idx, y, 3, 2, 1, dx, fuse=BwdFuse(None, z, None, sc, sh))
    # reference: plain gather backward, then the mask and the sums
    plain = _empty(N, H, W, C)
    nb.maxpool_bwd(dy, idx, y, 3, 2, 1, plain)
    keep = z.buf.float() * sc + sh > 0
    want = torch.where(keep, plain.buf.float(), torch.zeros_like(plain.buf, dtype=torch.float32))
    torch.cuda.synchronize()
    assert torch.equal(dx.buf.float(), want)
    ps = part.double().sum(0)
    v = dx.buf.double()
    assert torch.allclose(ps[0], v.sum(0), rtol=1e-4, atol=1e-3)
    assert torch.allclose(ps[1], (v * z.buf.double()).sum(0), rtol=1e-4, atol=1e-3)


def test_outer_dgrad_fused_bn_matches_gemm_path():
    """UNet head (1x1 conv, one output channel): the outer-product data gradient with the BN-backward
    fusion gives the same masked dx as the GEMM kernel's fused epilogue, and the same partial sums."""
    nb, rb = _be()
    N, H, W, C, Kp = 2, 24, 20, 64, 8
    z, zr = _act(N, H, W, C)
    sc, sh = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.3
    dy, _ = _act(N, H, W, Kp)
    dy.buf[:, 1:] = 0                                    # channels >= K are padding
    wT = torch.zeros(C, 1, 1, Kp, device=DEV, dtype=torch.bfloat16)
    wT[..., 0] = (torch.randn(C, 1, 1, device=DEV) * 0.2).to(torch.bfloat16)
    fuse = BwdFuse(None, z, None, sc, sh)
    dx1, dx2 = _empty(N, H, W, C), _empty(N, H, W, C)
    p1 = nb.conv_dgrad(dy, wT, C, 1, 1, 1, 0, dx1, fuse=fuse)
    p2 = nb.outer_dgrad_bn(dy, wT.view(-1), Kp, dx2, fuse)
    torch.cuda.synchronize()
    assert torch.equal(dx1.buf, dx2.buf)
    assert torch.allclose(p1.double().sum(0), p2.double().sum(0), rtol=1e-5, atol=1e-4)
    keep = z.buf.float() * sc + sh > 0
    want = torch.where(keep, dy.buf[:, :1].float() * wT.view(C, Kp)[:, 0].float(), torch.zeros(1, device=DEV))
    assert torch.equal(dx2.buf.float(), want.to(torch.bfloat16).float())


def test_maxpool_bwd_add_fused_bn_stats():
    """UNet encoder output: pool backward + skip-concat gradient slice + ReLU mask + BN partials."""
    nb, rb = _be()
    N, H, W, C, CAT = 2, 16, 16, 64, 192
    z, zr = _act(N, H, W, C)
    sc, sh = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.3
    y = _empty(N, H, W, C)
    nb.bn_apply(z, sc, sh, None, True, y)
    p = _empty(N, H // 2, W // 2, C)
    idx = nb.maxpool_fwd(y, 2, 2, 0, p)
    dy, _ = _act(N, H // 2, W // 2, C)
    cat, _ = _act(N, H, W, CAT)
    add = cat.slice(CAT - C, C)
    dx = _empty(N, H, W, C)
    part = nb.maxpool_bwd(dy, idx, y, 2, 2, 0, dx, add=add, fuse=BwdFuse(None, z, None, sc, sh))
    plain = _empty(N, H, W, C)
    nb.maxpool_bwd(dy, idx, y, 2, 2, 0, plain, add=add)
    keep = z.buf.float() * sc + sh > 0
    torch.cuda.synchronize()
    assert torch.equal(dx.buf.float(), torch.where(keep, plain.buf.float(), torch.zeros_like(keep, dtype=torch.float32)))
    ps, v = part.double().sum(0), dx.buf.double()
    assert torch.allclose(ps[0], v.sum(0), rtol=1e-4, atol=1e-3)
    assert torch.allclose(ps[1], (v * z.buf.double()).sum(0), rtol=1e-4, atol=1e-3)


def test_conv_fwd_bnbwd():
    """ConvTranspose data-gradient (2x2/s2 conv) producing the gradient of a BN+ReLU output: masked
    store + BN-backward partials in the GEMM epilogue == plain conv, then mask, then sums."""
    nb, rb = _be()
    N, H, W, Cin, K = 2, 16, 16, 128, 64
    x, _ = _act(N, H, W, Cin)
    w = (torch.randn(K, 2, 2, Cin, device=DEV) * 0.05).to(torch.bfloat16)
    z, _ = _act(N, H // 2, W // 2, K)
    sc, sh = torch.rand(K, device=DEV) + 0.5, torch.randn(K, device=DEV) * 0.3
    y = _empty(N, H // 2, W // 2, K)
    part = nb.conv_fwd_bnbwd(x, w, K, 2, 2, 2, 0, y, BwdFuse(None, z, None, sc, sh))
    plain = _empty(N, H // 2, W // 2, K)
    nb.conv_fwd(x, w, K, 2, 2, 2, 0, plain)
    keep = z.buf.float() * sc + sh > 0
    torch.cuda.synchronize()
    assert torch.equal(y.buf.float(), torch.where(keep, plain.buf.float(), torch.zeros_like(keep, dtype=torch.float32)))
    ps, v = part.double().sum(0), y.buf.double()
    assert torch.allclose(ps[0], v.sum(0), rtol=1e-4, atol=1e-3)
    assert torch.allclose(ps[1], (v * z.buf.double()).sum(0), rtol=1e-4, atol=1e-3)


def test_losses_eval_optim():
    nb, rb = _be()
    logits = torch.randn(64, 1000, device=DEV)
    labels = torch.randint(1000, (64,), device=DEV)
    go = torch.ones(1, device=DEV)
    l1, s1 = nb.ce_fwd(logits, labels)
    l2, s2 = rb.ce_fwd(logits, labels)
    assert abs(l1.item() - l2.item()) < 1e-4
    assert _rel(nb.ce_bwd(logits, labels, s1, go), rb.ce_bwd(logits, labels, s2, go)) < 1e-4
    lg = torch.randn(2, 32, 32, device=DEV)
    t = (torch.rand(2, 32, 32, device=DEV) > 0.5).float()
    assert abs(nb.bce_fwd(lg, t).item() - rb.bce_fwd(lg, t).item()) < 1e-5
    assert _rel(nb.bce_bwd(lg, t, go), rb.bce_bwd(lg, t, go)) < 1e-4
    assert nb.argmax_correct(logits, labels).item() == rb.argmax_correct(logits, labels).item()
    assert _rel(nb.dice(lg, t), rb.dice(lg, t)) < 1e-5
    n = 100003
    for be_args in [(0.1, 0.9, 0.0, 1e-5, False), (0.05, 0.9, 0.0, 0.0, True)]:
        p, g, m = torch.randn(n, device=DEV), torch.randn(n, device=DEV), torch.randn(n, device=DEV)
        p2, g2, m2 = p.clone(), g.clone(), m.clone()
        for first in (True, False):
            nb.sgd(p, g, m, *be_args, first)
            rb.sgd(p2, g2, m2, *be_args, first)
        assert _rel(p, p2) < 1e-6 and _rel(m, m2) < 1e-6
    p, g = torch.randn(n, device=DEV), torch.randn(n, device=DEV)
    m, v = torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    p2, m2, v2 = p.clone(), m.clone(), v.clone()
    for step in (1, 2):
        nb.adam(p, g, m, v, 1e-3, 0.9, 0.999, 1e-8, 0.0, False, 1 - 0.9 ** step, 1 - 0.999 ** step)
        rb.adam(p2, g, m2, v2, 1e-3, 0.9, 0.999, 1e-8, 0.0, False, 1 - 0.9 ** step, 1 - 0.999 ** step)
    assert _rel(p, p2) < 1e-6
    nrm, coef = torch.empty(1, device=DEV), torch.empty(2, device=DEV)
    nrm2, coef2 = torch.empty(1, device=DEV), torch.empty(2, device=DEV)
    nb.grad_norm(g, 1.0, nrm, coef)
    rb.grad_norm(g, 1.0, nrm2, coef2)
    assert _rel(nrm, nrm2) < 1e-5 and _rel(coef, coef2) < 1e-5


@pytest.mark.parametrize("model", ["resnet50", "unet1"])
def test_cast_weights_all_layouts(model):
    """Multi-tensor weight re-layout + cast (cast.hip) for every entry of a real model -- 1x1,
    3x3 and 7x7 forward / data-gradient copies, transposed-conv copies, the 1-channel UNet input
    conv (merged-row transpose path) -- bit-exact against the torch reference re-layout."""
    from deeplearning_mpi_amd.models import UNet, resnet50

    torch.manual_seed(0)
    m = (resnet50(num_classes=1000) if model == "resnet50" else UNet(out_classes=1, in_channels=1)).to(DEV)
    a = m.arena
    a.refresh(force=True)
    torch.cuda.synchronize()
    got = a.compute.clone()
    want = torch.zeros_like(a.compute)
    RefBackend(DEV, torch.float32).cast_weights(a._entries, a._compute_total, want)
    assert torch.equal(got, want)


# ------------------------------------------------------------------ operand prologues (Deferred)
PRO_SHAPES = [
    # N, H, W, Cin, Cout, R, stride, pad
    (2, 14, 14, 64, 64, 3, 1, 1),
    (3, 7, 7, 256, 64, 1, 1, 0),        # row remainders
    (2, 16, 16, 128, 256, 3, 2, 1),     # stride 2: dgrad phases
    (2, 14, 14, 256, 512, 1, 2, 0),
    (1, 16, 24, 192, 64, 3, 1, 1),      # UNet concat width
    (8, 64, 64, 64, 64, 3, 1, 1),       # 256-row tiles
    (2, 4, 4, 512, 512, 3, 1, 1),       # split-K
]


def _static_kernels(on: bool):
    """Pin the plain implicit-GEMM kernel with the static tile rules (the operand-prologue kernels
    have no register epilogue, streaming or autotuned variant): for bit-identity comparisons."""
    C = NativeBackend(DEV).C
    C.set_conv_stream(0 if on else -1)
    C.set_conv_autotune(0 if on else -1)
    C.set_conv_halo(0 if on else -1)    # 3x3 halo tiles sum chunk-major (no prologue variant)
    C.set_conv3_stream(0 if on else -1)  # streaming 64 -> 64 3x3 kernel (no prologue variant)
    C.set_wgrad3(0 if on else -1)       # 3x3 spatial-tile weight gradient (no prologue variant)
    C.set_dgrad_stream(0 if on else -1)  # streaming 1x1 data gradient (no prologue variant)


def _deferred_pair(N, H, W, C):
    """(affine Deferred, its materialized Act) and (bnbwd Deferred, materialized)."""
    from deeplearning_mpi_amd.ops.act import Deferred

    nb = NativeBackend(DEV)
    z, _ = _act(N, H, W, C)
    sc, sh = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.5
    aff = Deferred.affine(z, sc, sh)
    dy, _ = _act(N, H, W, C)
    coef = torch.stack([torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.1,
                        torch.randn(C, device=DEV) * 0.1])
    bwd = Deferred.bnbwd(dy, z, coef)
    return (aff, nb.materialize(aff)), (bwd, nb.materialize(bwd))


@pytest.mark.parametrize("shape", PRO_SHAPES)
def test_conv_prologues_bit_identical_to_materialized_operands(shape):
    """Forward with a deferred BN-apply+ReLU operand, data gradient with a deferred BN-backward
    operand, weight gradient with either or both: every result bit-identical to the same kernels
    on the materialized tensors (incl. zero padding taps, row tails, stride-2 phases, split-K)."""
    nb = NativeBackend(DEV)
    _static_kernels(True)
    try:
        _prologue_case(nb, shape)
    finally:
        _static_kernels(False)


def _prologue_case(nb, shape):
    N, H, W, Cin, K, R, s, p = shape
    Cp, Kp = pad8(Cin), pad8(K)
    P, Q = (H + 2 * p - R) // s + 1, (W + 2 * p - R) // s + 1
    (aff, affm), _ = _deferred_pair(N, H, W, Cp)
    w = (torch.randn(Kp, R, R, Cp, device=DEV) / (R * R * Cin) ** 0.5).to(torch.bfloat16)
    # forward + BN stats
    ys = [_empty(N, P, Q, Kp) for _ in range(2)]
    sts = [torch.zeros(nb.conv_mtiles(N, H, W, Cp, Kp, R, R, s, p, pro=pro), 2, Kp, device=DEV) for pro in (1, 0)]
    nb.conv_fwd(aff, w, Kp, R, R, s, p, ys[0], stats=sts[0])
    nb.conv_fwd(affm, w, Kp, R, R, s, p, ys[1], stats=sts[1])
    torch.cuda.synchronize()
    assert torch.equal(ys[0].buf, ys[1].buf)
    assert torch.allclose(sts[0].sum(0), sts[1].sum(0), rtol=1e-5, atol=1e-3)
    # data gradient: dy operand deferred (BN backward of the layer above)
    _, (bwd, bwdm) = _deferred_pair(N, P, Q, Kp)
    wT = (torch.randn(Cp, R, R, Kp, device=DEV) / (R * R * K) ** 0.5).to(torch.bfloat16)
    dxs = [_empty(N, H, W, Cp) for _ in range(2)]
    nb.conv_dgrad(bwd, wT, Cp, R, R, s, p, dxs[0])
    nb.conv_dgrad(bwdm, wT, Cp, R, R, s, p, dxs[1])
    torch.cuda.synchronize()
    assert torch.equal(dxs[0].buf, dxs[1].buf)
    # weight gradient: dy deferred, x deferred, both
    for dyo, xo in ((bwd, affm), (bwdm, aff), (bwd, aff)):
        g1 = torch.zeros(K * R * R * Cin, device=DEV)
        g2 = torch.zeros_like(g1)
        nb.conv_wgrad(dyo, xo, R, R, s, p, g1, Cin, K)
        nb.conv_wgrad(bwdm, affm, R, R, s, p, g2, Cin, K)
        torch.cuda.synchronize()
        assert torch.equal(g1, g2), (type(dyo).__name__, type(xo).__name__)



# ------------------------------------------------------------------ streaming 1x1 forward
STREAM_SHAPES = [
    # N, H, W, Cin, Cout: 1x1 / stride 1 (the ResNet expand convs, small)
    (4, 14, 14, 64, 256),      # 784 rows: 6.1 tiles of 128, ragged last tile
    (2, 7, 9, 64, 128),        # 126 rows: a single partial tile
    (8, 28, 28, 128, 512),
    (4, 14, 14, 256, 1024),
    (3, 5, 7, 256, 64),        # 105 rows, one N-tile
    (32, 56, 56, 64, 256),     # bench-layer scale (100k rows, every block walks many tiles)
    (4, 28, 28, 64, 64),       # 64 -> 64 (the layer-1 block-1 conv1): 128 x 64 tiles
    (4, 28, 28, 256, 512, 2),  # stride-2 projection (gathered rows), even grid
    (3, 15, 13, 256, 128, 2),  # stride 2 over an odd grid: 8 x 7 outputs
]


@pytest.mark.parametrize("shape", STREAM_SHAPES)
@pytest.mark.parametrize("ld_out", ["dense", "dual"])
def test_stream1x1_matches_general_kernel(shape, ld_out):
    """conv1x1_stream.hip (persistent blocks, resident weights, prefetch under the epilogue, one
    statistics row per block) against the general implicit-GEMM kernel: identical outputs (same
    MFMA dot products and rounding), statistics summed over rows equal to fp32 noise, BN finalize
    over the block rows equal to the finalize over the tile rows; 'dual' writes into the right half
    of a [rows][2K] buffer (the dual data-gradient layout) and must leave the left half untouched."""
    N, H, W, Cin, K = shape[:5]
    s = shape[5] if len(shape) > 5 else 1
    P, Q = (H - 1) // s + 1, (W - 1) // s + 1
    nb = NativeBackend(DEV)
    x, _ = _act(N, H, W, Cin)
    w = (torch.randn(K, 1, 1, Cin, device=DEV) / Cin ** 0.5).to(torch.bfloat16)
    bias = torch.randn(K, device=DEV) * 0.1
    gamma, beta = torch.rand(K, device=DEV) + 0.5, torch.randn(K, device=DEV)
    out = {}
    for mode in (1, 0):
        nb.C.set_conv_stream(mode)
        mt = nb.conv_mtiles(N, H, W, Cin, K, 1, 1, s, 0)
        if ld_out == "dual":
            buf = torch.full((N * P * Q, 2 * K), 7.0, device=DEV).to(torch.bfloat16)
            y = Act(buf, N, P, Q, K, K)
        else:
            y = _empty(N, P, Q, K)
        st = torch.zeros(mt, 2, K, device=DEV)   # an autotuned tile may write fewer rows than mt
        v = torch.empty(4, K, device=DEV)
        rm, rv = torch.zeros(K, device=DEV), torch.ones(K, device=DEV)
        nb.conv_fwd_bn(x, w, K, 1, 1, s, 0, y, bias, st, N * P * Q, gamma, beta, rm, rv, 0.1, 1e-5,
                       v[0], v[1], v[2], v[3])
        torch.cuda.synchronize()
        assert nb.C.conv_stream_last() == mode   # the streaming kernel ran (mode 1) / did not (mode 0)
        out[mode] = (y.buf.clone(), st.sum(0), v.clone(), rm.clone(), rv.clone(), mt)
    nb.C.set_conv_stream(-1)
    if Cin <= 256:
        assert torch.equal(out[1][0], out[0][0])
    else:   # the general kernel may split the 8 K-steps (split-K): another fp32 summation order
        assert _rel(out[1][0], out[0][0]) < 1e-2
    if ld_out == "dual":
        assert bool((out[1][0][:, :K].float() == 7.0).all())
    tol = 1e-5 if Cin <= 256 else 2e-4   # (split-K outputs differ in the last bf16 bit)
    assert _rel(out[1][1], out[0][1]) < tol
    for a, b in zip(out[1][2:5], out[0][2:5]):
        assert _rel(a, b) < tol


WGRAD_FAST_SHAPES = [
    # N, H, W, Cin, Cout, R, stride, pad, x channel stride / offset
    (4, 14, 14, 256, 1024, 1, 1, 0, None, 0),   # direct 1x1, 128 x 128 tiles
    (2, 28, 28, 512, 128, 1, 1, 0, None, 0),
    (3, 9, 11, 64, 64, 1, 1, 0, None, 0),       # Ko = 64: 64 x 256 tiles; 297 pixels (ragged K-step)
    (2, 14, 14, 96, 96, 1, 1, 0, None, 0),      # ragged column tiles: the general staging
    (2, 13, 13, 64, 256, 1, 1, 0, 192, 64),     # x a channel slice of a concat buffer
    (2, 28, 28, 256, 512, 1, 2, 0, None, 0),    # strided 1x1 (gather): dy side only
    (2, 15, 15, 64, 128, 3, 2, 1, None, 0),     # 3x3 stride 2 (gather)
]


@pytest.mark.parametrize("shape", WGRAD_FAST_SHAPES, ids=lambda s: "x".join(str(v) for v in s[:8]))
def test_wgrad_fast_staging_bit_identical(shape):
    """conv_wgrad_kernel's scalar-base staging (full K-steps of a tile whose column pieces all exist)
    against the per-piece selected staging: the same bytes land in the same LDS slots, so the weight
    gradient is bit-identical; and it matches an fp32 reference."""
    nb, rb = _be()
    N, H, W, Cin, K, R, s, p, ldx, xoff = shape
    P = (H + 2 * p - R) // s + 1
    x, xr = _act(N, H, W, Cin, ld=ldx, off=xoff)
    dy, dyr = _act(N, P, P, K)
    out = {}
    try:
        for on in (1, 0):
            nb.C.set_wgrad_fast(on)
            g = torch.zeros(K * R * R * Cin, device=DEV)
            nb.conv_wgrad(dy, x, R, R, s, p, g, Cin, K)
            torch.cuda.synchronize()
            out[on] = g
    finally:
        nb.C.set_wgrad_fast(1)
    assert torch.equal(out[1], out[0])
    ref = torch.zeros_like(out[0])
    rb.conv_wgrad(dyr, xr, R, R, s, p, ref, Cin, K)
    assert _rel(out[1], ref) < 1e-2
