"""The fp32 precision path (``--precision fp32``): the native kernels instantiated for fp32
activations and weights (GEMMs on v_mfma_f32_16x16x4_f32, fp32 elementwise / pooling / layout
kernels) against the reference backend in float64 on the same fp32 inputs, plus one training step
of ResNet-18 (CIFAR shape) and UNet through the native fp32 engine against the fp64 reference
engine."""
import copy

import pytest
import torch

from deeplearning_mpi_amd.models.engine import BwdFuse
from deeplearning_mpi_amd.ops.act import Act, pad8
from deeplearning_mpi_amd.ops.backend import NativeBackend, RefBackend

pytestmark = pytest.mark.gpu
DEV = "cuda"
F32, F64 = torch.float32, torch.float64


def _be():
    nb = NativeBackend(DEV, F32)
    assert nb.act_dtype == F32 and nb.f32
    return nb, RefBackend(DEV, F64)


def _act(N, H, W, C, ld=None, off=0):
    ld = ld or C
    buf = torch.randn(N * H * W, ld, device=DEV)
    return Act(buf, N, H, W, C, off), Act(buf.double(), N, H, W, C, off)


def _empty(N, H, W, C, dt=F32, ld=None):
    return Act.empty(N, H, W, C, dt, DEV, ld)


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


CONV_SHAPES = [
    # N, H, W, Cin, Cout, R, stride, pad
    (2, 16, 16, 3, 64, 3, 1, 1),       # CIFAR stem (Cin padded to 8: small-channel staging)
    (2, 14, 14, 48, 40, 3, 1, 1),      # C >= 32 but not a multiple of 32: small-channel staging too
    (2, 14, 14, 64, 64, 3, 1, 1),
    (2, 14, 14, 128, 128, 3, 2, 1),
    (3, 7, 7, 256, 64, 1, 1, 0),       # tile remainders
    (2, 14, 14, 256, 512, 1, 2, 0),    # downsample 1x1 stride 2
    (1, 16, 24, 192, 64, 3, 1, 1),     # UNet decoder concat width
    (2, 4, 4, 512, 512, 3, 1, 1),      # tiny grid: in-launch split-K
]
TOL = 2e-5   # fp32 accumulation over <= 4608 products vs fp64


@pytest.mark.parametrize("shape", CONV_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_conv_fwd_dgrad_wgrad_fp32(shape):
    nb, rb = _be()
    N, H, W, Cin, K, R, s, p = shape
    Cp, Kp = pad8(Cin), pad8(K)
    P, Q = (H + 2 * p - R) // s + 1, (W + 2 * p - R) // s + 1
    x, xr = _act(N, H, W, Cp)
    w = torch.randn(Kp, R, R, Cp, device=DEV) / (R * R * Cin) ** 0.5
    bias = torch.randn(Kp, device=DEV)
    y, yr = _empty(N, P, Q, Kp), _empty(N, P, Q, Kp, F64)
    st = torch.zeros(nb.conv_mtiles(N, H, W, Cp, Kp, R, R, s, p), 2, Kp, device=DEV)
    str_ = torch.zeros(1, 2, Kp, device=DEV, dtype=F64)
    nb.conv_fwd(x, w, Kp, R, R, s, p, y, bias=bias, stats=st)
    rb.conv_fwd(xr, w.double(), Kp, R, R, s, p, yr, bias=bias.double(), stats=str_)
    torch.cuda.synchronize()
    assert _rel(y.buf, yr.buf) < TOL
    assert _rel(st.double().sum(0)[0], str_[0, 0]) < 1e-4
    assert _rel(st.double().sum(0)[1], str_[0, 1]) < 1e-4
    # fused residual + folded affine + ReLU epilogue
    res, resr = _act(N, P, Q, Kp)
    sc, sh = torch.rand(Kp, device=DEV) + 0.5, torch.randn(Kp, device=DEV)
    nb.conv_fwd(x, w, Kp, R, R, s, p, y, res=res, scale=sc, shift=sh, relu=True)
    rb.conv_fwd(xr, w.double(), Kp, R, R, s, p, yr, res=resr, scale=sc.double(), shift=sh.double(), relu=True)
    assert _rel(y.buf, yr.buf) < TOL
    # data gradient (+ residual), every sub-pixel phase of the strided case
    dy, dyr = _act(N, P, Q, Kp)
    wT = w.permute(3, 1, 2, 0).contiguous()
    dx, dxr = _empty(N, H, W, Cp), _empty(N, H, W, Cp, F64)
    res, resr = _act(N, H, W, Cp)
    nb.conv_dgrad(dy, wT, Cp, R, R, s, p, dx, res=res)
    rb.conv_dgrad(dyr, wT.double(), Cp, R, R, s, p, dxr, res=resr)
    torch.cuda.synchronize()
    assert _rel(dx.buf, dxr.buf) < TOL
    # weight gradient, accumulated into a non-zero slot like the gradient arena
    g = torch.randn(K * R * R * Cin, device=DEV)
    gr = g.double()
    nb.conv_wgrad(dy, x, R, R, s, p, g, Cin, K)
    rb.conv_wgrad(dyr, xr, R, R, s, p, gr, Cin, K)
    torch.cuda.synchronize()
    assert _rel(g, gr) < TOL


def test_convT_and_linear_fp32():
    nb, rb = _be()
    N, H, W, Ci, Co = 2, 8, 12, 256, 128
    x, xr = _act(N, H, W, Ci)
    wf = torch.randn(Co, 2, 2, Ci, device=DEV) / Ci ** 0.5
    bias = torch.randn(Co, device=DEV)
    cat, catr = _empty(N, 2 * H, 2 * W, Co + 64), _empty(N, 2 * H, 2 * W, Co + 64, F64)
    nb.convT_fwd(x, wf, Co, cat.slice(0, Co), bias)
    rb.convT_fwd(xr, wf.double(), Co, catr.slice(0, Co), bias.double())
    torch.cuda.synchronize()
    assert _rel(cat.nhwc()[..., :Co], catr.nhwc()[..., :Co]) < TOL
    Nn, Cin, K = 16, 512, 10
    Kp = pad8(K)
    x, xr = _act(Nn, 1, 1, Cin)
    w = torch.randn(Kp, 1, 1, Cin, device=DEV) / Cin ** 0.5
    w[K:] = 0
    b = torch.randn(Kp, device=DEV)
    out, outr = torch.empty(Nn, K, device=DEV), torch.empty(Nn, K, device=DEV, dtype=F64)
    nb.conv_fwd(x, w, Kp, 1, 1, 1, 0, Act(out, Nn, 1, 1, K), bias=b, kvalid=K)
    rb.conv_fwd(xr, w.double(), Kp, 1, 1, 1, 0, Act(outr, Nn, 1, 1, K), bias=b.double())
    torch.cuda.synchronize()
    assert _rel(out, outr) < TOL


def test_bn_family_fp32():
    nb, rb = _be()
    N, H, W, C = 4, 14, 14, 256
    x, xr = _act(N, H, W, C)
    res, resr = _act(N, H, W, C)
    st, _ = nb.bn_stats(x)
    str_, _ = rb.bn_stats(xr)
    assert _rel(st.double().sum(0), str_.sum(0)) < 1e-5
    gamma, beta = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
    v = torch.empty(4, C, device=DEV)
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    nb.bn_finalize(st, st.shape[0], C, N * H * W, gamma, beta, rm, rv, 0.1, 1e-5, v[0], v[1], v[2], v[3])
    vr = torch.empty(4, C, device=DEV, dtype=F64)
    rmr, rvr = torch.zeros(C, device=DEV, dtype=F64), torch.ones(C, device=DEV, dtype=F64)
    rb.bn_finalize(str_, 1, C, N * H * W, gamma.double(), beta.double(), rmr, rvr, 0.1, 1e-5, vr[0], vr[1], vr[2],
                   vr[3])
    for a, b in ((v, vr), (rm, rmr), (rv, rvr)):
        assert _rel(a, b) < 1e-5
    y, yr = _empty(N, H, W, C), _empty(N, H, W, C, F64)
    bits = torch.empty(N * H * W, C // 8, dtype=torch.uint8, device=DEV)
    nb.bn_apply(x, v[0], v[1], res, True, y, mbits=bits)
    rb.bn_apply(xr, v[0].double(), v[1].double(), resr, True, yr)
    assert _rel(y.buf, yr.buf) < 1e-6
    assert torch.equal(RefBackend._unpack_bits(bits, y).reshape(-1, C), y.buf > 0)
    dy, dyr = _act(N, H, W, C)
    dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    dgr, dbr = torch.zeros(C, device=DEV, dtype=F64), torch.zeros(C, device=DEV, dtype=F64)
    dx, dxr = _empty(N, H, W, C), _empty(N, H, W, C, F64)
    dyo, dyor = _empty(N, H, W, C), _empty(N, H, W, C, F64)
    nb.bn_bwd(dy, y, x, v[2], v[3], gamma, dg, db, dx, dyo)
    rb.bn_bwd(dyr, Act(y.buf.double(), N, H, W, C), xr, v[2].double(), v[3].double(), gamma.double(), dgr, dbr, dxr,
              dyor)
    torch.cuda.synchronize()
    assert _rel(dg, dgr) < 1e-5 and _rel(db, dbr) < 1e-5
    assert _rel(dx.buf, dxr.buf) < 1e-4
    assert torch.equal(dyo.buf.double(), dyor.buf)
    cs, csr = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV, dtype=F64)
    nb.channel_sum(x, cs)
    rb.channel_sum(xr, csr)
    assert _rel(cs, csr) < 1e-5


def test_fused_bn_backward_epilogues_fp32():
    """Dgrad epilogue with the ReLU mask from z + BN-backward partials, the max-pool backward and the
    1-channel head's outer-product data gradient with the same fusion, in fp32."""
    nb, rb = _be()
    N, H, W, C, K = 2, 16, 16, 64, 128
    z, zr = _act(N, H, W, C)
    sc, sh = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.3
    keep = z.buf * sc + sh > 0
    dy, dyr = _act(N, H, W, K)
    wT = torch.randn(C, 3, 3, K, device=DEV) / (9 * K) ** 0.5
    dx, dxr = _empty(N, H, W, C), _empty(N, H, W, C, F64)
    part = nb.conv_dgrad(dy, wT, C, 3, 3, 1, 1, dx, fuse=BwdFuse(None, z, None, sc, sh))
    pr = rb.conv_dgrad(dyr, wT.double(), C, 3, 3, 1, 1, dxr, fuse=BwdFuse(None, zr, None, sc.double(), sh.double()))
    torch.cuda.synchronize()
    assert _rel(dx.buf, dxr.buf) < TOL
    assert _rel(part.double().sum(0), pr.sum(0)) < 1e-4
    # max-pool backward (ResNet stem 3x3/s2) fused with the mask + partials
    y = _empty(N, H, W, C)
    nb.bn_apply(z, sc, sh, None, True, y)
    pooled = _empty(N, H // 2, W // 2, C)
    idx = nb.maxpool_fwd(y, 3, 2, 1, pooled)
    g, _ = _act(N, H // 2, W // 2, C)
    d1, d2 = _empty(N, H, W, C), _empty(N, H, W, C)
    p1 = nb.maxpool_bwd(g, idx, y, 3, 2, 1, d1, fuse=BwdFuse(None, z, None, sc, sh))
    nb.maxpool_bwd(g, idx, y, 3, 2, 1, d2)
    torch.cuda.synchronize()
    assert torch.equal(d1.buf, torch.where(keep, d2.buf, torch.zeros_like(d2.buf)))
    v = d1.buf.double()
    assert torch.allclose(p1.double().sum(0)[0], v.sum(0), rtol=1e-5, atol=1e-4)
    assert torch.allclose(p1.double().sum(0)[1], (v * z.buf.double()).sum(0), rtol=1e-5, atol=1e-4)
    # outer-product head gradient == the GEMM path's fused epilogue
    Kp = 8
    dyh, _ = _act(N, H, W, Kp)
    dyh.buf[:, 1:] = 0
    wh = torch.zeros(C, 1, 1, Kp, device=DEV)
    wh[..., 0] = torch.randn(C, 1, 1, device=DEV) * 0.2
    o1, o2 = _empty(N, H, W, C), _empty(N, H, W, C)
    q1 = nb.conv_dgrad(dyh, wh, C, 1, 1, 1, 0, o1, fuse=BwdFuse(None, z, None, sc, sh))
    q2 = nb.outer_dgrad_bn(dyh, wh.view(-1), Kp, o2, BwdFuse(None, z, None, sc, sh))
    torch.cuda.synchronize()
    assert torch.equal(o1.buf, o2.buf)
    assert torch.allclose(q1.double().sum(0), q2.double().sum(0), rtol=1e-5, atol=1e-4)


def test_pools_layout_upsample_fp32():
    nb, rb = _be()
    x = torch.randn(2, 3, 20, 18, device=DEV)
    a, ar = nb.nchw_to_nhwc(x, 8), rb.nchw_to_nhwc(x.double(), 8)
    assert a.buf.dtype == F32 and torch.equal(a.buf.double(), ar.buf)
    for (H, W, pad) in [(20, 18, 3), (23, 17, 3)]:
        x = torch.randn(2, 3, H, W, device=DEV)
        U, V = (H + 2 * pad + 1) // 2, (W + 2 * pad + 1) // 2
        a, ar = nb.s2d(x, pad, U, V, 4), rb.s2d(x.double(), pad, U, V, 4)
        assert torch.equal(a.buf.double(), ar.buf)
    for (k, s, p, H, W, C) in [(3, 2, 1, 16, 16, 64), (2, 2, 0, 16, 24, 128)]:
        xa, xr = _act(2, H, W, C)
        OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        y, yr = _empty(2, OH, OW, C), _empty(2, OH, OW, C, F64)
        idx = nb.maxpool_fwd(xa, k, s, p, y)
        idxr = rb.maxpool_fwd(xr, k, s, p, yr)
        assert torch.equal(y.buf.double(), yr.buf)
        dy, dyr = _act(2, OH, OW, C)
        add, addr = _act(2, H, W, C)
        dx, dxr = _empty(2, H, W, C), _empty(2, H, W, C, F64)
        nb.maxpool_bwd(dy, idx, xa, k, s, p, dx, add=add)
        rb.maxpool_bwd(dyr, idxr, xr, k, s, p, dxr, add=addr)
        assert _rel(dx.buf, dxr.buf) < 1e-6
    xa, xr = _act(4, 7, 7, 512)
    y, yr = _empty(4, 1, 1, 512), _empty(4, 1, 1, 512, F64)
    nb.avgpool_fwd(xa, y)
    rb.avgpool_fwd(xr, yr)
    assert _rel(y.buf, yr.buf) < 1e-6
    dx, dxr = _empty(4, 7, 7, 512), _empty(4, 7, 7, 512, F64)
    nb.avgpool_bwd(y, dx)
    rb.avgpool_bwd(Act(y.buf.double(), 4, 1, 1, 512), dxr)
    assert _rel(dx.buf, dxr.buf) < 1e-6
    for (H, W) in [(8, 6), (15, 20), (1, 5)]:
        xa, xr = _act(2, H, W, 64)
        y, yr = _empty(2, 2 * H, 2 * W, 64), _empty(2, 2 * H, 2 * W, 64, F64)
        nb.upsample_fwd(xa, y)
        rb.upsample_fwd(xr, yr)
        assert _rel(y.buf, yr.buf) < 1e-6
        g, gr = _act(2, 2 * H, 2 * W, 64)
        dx, dxr = _empty(2, H, W, 64), _empty(2, H, W, 64, F64)
        nb.upsample_bwd(g, dx)
        rb.upsample_bwd(gr, dxr)
        assert _rel(dx.buf, dxr.buf) < 1e-5, (H, W)


def test_bilinear_backward_is_deterministic_gather():
    """The bilinear x2 backward is a gather (no float atomics): repeated runs are bit-identical, in
    bf16 and fp32, and match autograd of the align_corners interpolation."""
    for dt in (torch.bfloat16, F32):
        nb = NativeBackend(DEV, dt)
        g = Act(torch.randn(2 * 64 * 96, 128, device=DEV).to(dt), 2, 64, 96, 128)
        outs = []
        for _ in range(3):
            dx = _empty(2, 32, 48, 128, dt)
            nb.upsample_bwd(g, dx)
            outs.append(dx.buf.clone())
        torch.cuda.synchronize()
        assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
        rb = RefBackend(DEV, F64)
        dxr = _empty(2, 32, 48, 128, F64)
        rb.upsample_bwd(Act(g.buf.double(), 2, 64, 96, 128), dxr)
        assert _rel(outs[0], dxr.buf) < (1e-2 if dt == torch.bfloat16 else 1e-5)


def test_cast_weights_fp32_copies_exact():
    """fp32 compute copies of every weight layout are exact copies of the master parameters."""
    from deeplearning_mpi_amd.models import resnet18

    torch.manual_seed(0)
    m = resnet18(num_classes=10).to(DEV)
    m.precision = "fp32"
    ar = m.engine_setup(DEV)
    assert ar.compute.dtype == F32
    want = torch.zeros_like(ar.compute)
    RefBackend(DEV, F32).cast_weights(ar._entries, ar._compute_total, want)
    torch.cuda.synchronize()
    assert torch.equal(ar.compute, want)


def _model(name):
    from deeplearning_mpi_amd.models import UNet, resnet18, resnet50
    from deeplearning_mpi_amd.ops import bce_with_logits, cross_entropy

    g = torch.Generator(device=DEV).manual_seed(5)
    if name.startswith("unet"):
        make = lambda: UNet(out_classes=1, up_sample_mode="bilinear" if "bilinear" in name else "conv_transpose")  # noqa
        x = torch.randn(2, 3, 64, 64, device=DEV, generator=g)
        y = (torch.rand(2, 64, 64, device=DEV, generator=g) > 0.5).float()
        return make, x, lambda o: bce_with_logits(o.squeeze(1), y.to(o.dtype))
    side = 32 if name == "resnet18" else 64
    make = lambda: (resnet18 if name == "resnet18" else resnet50)(num_classes=10)   # noqa: E731
    x = torch.randn(16, 3, side, side, device=DEV, generator=g)
    y = torch.randint(10, (16,), device=DEV, generator=g)
    return make, x, lambda o: cross_entropy(o, y)


@pytest.mark.parametrize("name", ["resnet18", "resnet50", "unet", "unet_bilinear"])
def test_training_step_every_op_matches_fp64(name):
    """One forward + backward of the native fp32 engine with every backend call shadowed by the
    fp64 reference on the same inputs (utils/shadow.py): all outputs within 2e-5 (max-relative; BN
    partial sums per statistic row)."""
    from deeplearning_mpi_amd.utils.shadow import ShadowBackend

    make, x, lossf = _model(name)
    torch.manual_seed(0)
    m = make().to(DEV)
    m.precision = "fp32"
    m.train()
    m.engine_setup(DEV)
    assert m._be.name == "native" and m._be.f32
    sh = ShadowBackend(m._be, RefBackend(DEV, F64), tol=2e-5)
    m._be = sh
    lossf(m(x)).backward()
    torch.cuda.synchronize()
    print({k: f"{v:.1e}" for k, v in sorted(sh.worst.items())})
    assert sh.calls > 40
    assert not sh.records, sh.records[:5]
    # the training forward runs conv + BN statistics + finalize as conv_fwd_bn (ops.cpp)
    for op in ("conv_fwd_bn", "conv_dgrad", "conv_wgrad", "bn_bwd"):
        assert op in sh.worst


@pytest.mark.parametrize("name", ["resnet18", "unet"])
def test_training_step_end_to_end_fp32_vs_fp64(name):
    """End to end, the native fp32 engine, stock torch fp32 ops (reference backend, fp32) and fp64
    agree on the loss to fp32 rounding.  Gradients are only loosely comparable: a forward value
    within rounding of a ReLU's zero lands on either side in different precisions, and one such
    flipped mask element (measured: 1 of 262k elements of the UNet decoder, |z*scale+shift| = 2e-6)
    moves every upstream gradient by ~5e-3 relative -- for stock torch fp32 as well, depending on
    which elements its rounding flips (scripts/diag/trace_compare.py finds the call)."""
    make, x, lossf = _model(name)
    torch.manual_seed(0)
    m0 = make().to(DEV)
    runs = []
    for prec, dt in (("fp32", F32), ("ref", F32), ("ref", F64)):
        m = copy.deepcopy(m0).to(dt)
        m.precision = prec
        m.train()
        loss = lossf(m(x.to(dt)))
        loss.backward()
        torch.cuda.synchronize()
        runs.append((float(loss), [p.grad.detach().double().clone() for p in m.parameters()]))
    (ln, gn), (lt, gt), (l64, g64) = runs
    assert abs(ln - l64) < 1e-5 * abs(l64) and abs(lt - l64) < 1e-5 * abs(l64)
    for a, b in zip(gn, g64):
        assert torch.isfinite(a).all()
        if b.norm() > 0:
            assert ((a - b).norm() / b.norm()).item() < 3e-2
