"""The engine's hand-written forward/backward schedules vs eager torch autograd (CPU, fp32
reference backend).  Sizes are chosen so BatchNorm is well conditioned."""
import copy

import pytest
import torch
import torch.nn.functional as F

from deeplearning_mpi_amd.models import UNet, resnet18, resnet50
from deeplearning_mpi_amd.ops import bce_with_logits, cross_entropy
from deeplearning_mpi_amd.models.engine import resolve
from deeplearning_mpi_amd.ops.act import Act


def _err(a, ref):
    return ((a.double() - ref).abs().max() / ref.abs().max().clamp_min(1e-30)).item()


def _run_pair(make, x, y, loss_e, loss_t, skip=lambda n: False):
    """The engine (reference backend in float64) against eager torch autograd in float64: with the
    rounding noise removed the hand-written schedules must reproduce autograd essentially exactly
    (fp32 comparisons are dominated by BatchNorm conditioning)."""
    torch.manual_seed(0)
    m1 = make().double()
    m3 = copy.deepcopy(m1)
    x = x.double()
    y = y.double() if y.is_floating_point() else y
    m1.train()
    m3.train()
    o1 = m1(x)
    l1 = loss_e(o1, y)
    l1.backward()
    o3 = m3.forward_torch(x)
    l3 = loss_t(o3, y)
    l3.backward()
    assert _err(o1.detach(), o3.detach()) < 1e-9
    assert abs(l1.item() - l3.item()) < 1e-9
    for (n, p1), (_, p3) in zip(m1.named_parameters(), m3.named_parameters()):
        if skip(n) or p3.grad.abs().max() == 0:
            continue
        assert _err(p1.grad, p3.grad) < 1e-6, (n, _err(p1.grad, p3.grad))
    for (n, b1), (_, b3) in zip(m1.named_buffers(), m3.named_buffers()):
        if b1.is_floating_point():
            assert _err(b1, b3) < 1e-9, n
        else:
            assert torch.equal(b1, b3), n
    m1.eval()
    m3.eval()
    with torch.no_grad():
        assert _err(m1(x), m3.forward_torch(x)) < 1e-9
    return m1


def test_resnet18_train_step_matches_torch():
    g = torch.Generator().manual_seed(1)
    x = torch.randn(16, 3, 64, 64, generator=g)
    y = torch.randint(10, (16,), generator=g)
    _run_pair(lambda: resnet18(num_classes=10), x, y, cross_entropy, F.cross_entropy)


def test_bottleneck_blocks_exact():
    torch.manual_seed(0)
    m = resnet50(num_classes=10)
    m2 = copy.deepcopy(m)
    m.train()
    m2.train()
    ar = m.engine_setup("cpu")
    be = m._be
    for bi, (blk, ref) in enumerate([(m.blocks[0], m2.layer1[0]), (m.blocks[1], m2.layer1[1]),
                                     (m.blocks[3], m2.layer2[0])]):
        N, H, W = 4, 8, 8
        Cin = ref.conv1.in_channels
        x = torch.randn(N, Cin, H, W)
        xa = Act.empty(N, H, W, Cin, torch.float32, "cpu")
        xa.nhwc().copy_(x.permute(0, 2, 3, 1))
        ar.zero_grad()
        y, st = blk.fwd(be, xa, True, True)
        y = resolve(be, y)   # a block output may be pending (engine.FUSE_APPLY: its consumer applies it)
        gy = torch.randn(N, y.C, y.H, y.W)
        dya = Act.empty(N, y.H, y.W, y.C, torch.float32, "cpu")
        dya.nhwc().copy_(gy.permute(0, 2, 3, 1))
        dx = blk.bwd(be, st, dya)
        xt = x.clone().requires_grad_(True)
        for p in ref.parameters():
            p.grad = None
        yt = ref.forward_torch(xt)
        yt.backward(gy)
        assert torch.allclose(y.nchw(), yt, atol=1e-4)
        assert torch.allclose(dx.nchw(), xt.grad, atol=1e-4, rtol=1e-3)
        mod = [m.layer1[0], m.layer1[1], m.layer2[0]][bi]
        for (n, p1), (_, p2) in zip(mod.named_parameters(), ref.named_parameters()):
            assert ((p1.grad - p2.grad).abs().max() / p2.grad.abs().max()).item() < 1e-5, n


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("mode", ["conv_transpose", "bilinear"])
def test_unet_train_step_matches_torch(mode, fused):
    """Both backward schedules: fused BN-backward epilogues, and separate bn_bwd passes (the pool-
    and head-apply deferrals must then keep the stored BN output for the ReLU mask)."""
    g = torch.Generator().manual_seed(1)
    x = torch.randn(4, 3, 64, 64, generator=g)
    y = (torch.rand(4, 64, 64, generator=g) > 0.5).float()
    skip = lambda n: n.endswith("bias") and "double_conv.double_conv" in n  # conv bias before train-BN: grad == 0

    def make():
        m = UNet(out_classes=1, up_sample_mode=mode)
        m.fuse_bn_bwd = fused
        return m

    _run_pair(make, x, y, lambda o, t: bce_with_logits(o.squeeze(1), t),
              lambda o, t: F.binary_cross_entropy_with_logits(o.squeeze(1), t), skip=skip)


def test_unet_shapes_and_multiclass():
    m = UNet(out_classes=2)
    m.eval()
    with torch.no_grad():
        y = m(torch.randn(1, 3, 32, 32))
        y2 = m.forward_torch(torch.randn(1, 3, 32, 32))
    assert y.shape == (1, 2, 32, 32) == y2.shape


def test_resnet50_fused_bn_backward_matches_torch_and_unfused():
    """BN-backward reductions fused into the dgrad epilogue (incl. the 3-statistic downsample
    variant) reproduce fp64 autograd and the unfused schedule."""
    g = torch.Generator().manual_seed(2)
    x = torch.randn(4, 3, 64, 64, generator=g)
    y = torch.randint(10, (4,), generator=g)
    m1 = _run_pair(lambda: resnet50(num_classes=10), x, y, cross_entropy, F.cross_entropy)
    assert m1.fuse_bn_bwd
    torch.manual_seed(0)
    m2 = resnet50(num_classes=10).double()
    m2.fuse_bn_bwd = False
    m2.train()
    cross_entropy(m2(x.double()), y).backward()
    for (n, p1), (_, p2) in zip(m1.named_parameters(), m2.named_parameters()):
        assert _err(p1.grad, p2.grad) < 1e-9, n


@pytest.mark.parametrize("norm_type", [1.0, 2.0, 3.0, float("inf")])
def test_clip_grad_norm_matches_torch(norm_type):
    """clip_grad_norm_ for every p against torch.nn.utils.clip_grad_norm_ (arena-backed model)."""
    from deeplearning_mpi_amd.models import resnet18
    from deeplearning_mpi_amd.ops import cross_entropy
    from deeplearning_mpi_amd.optim import clip_grad_norm_

    torch.manual_seed(0)
    m = resnet18(num_classes=10)
    loss = cross_entropy(m(torch.randn(2, 3, 32, 32)), torch.tensor([1, 7]))
    loss.backward()
    ref = [p.grad.detach().clone().requires_grad_(False) for p in m.parameters()]
    shadows = [torch.zeros_like(g, requires_grad=True) for g in ref]
    for s, g in zip(shadows, ref):
        s.grad = g.clone()
    want = torch.nn.utils.clip_grad_norm_(shadows, 0.5, norm_type=norm_type)
    got = clip_grad_norm_(m.parameters(), 0.5, norm_type=norm_type)
    torch.testing.assert_close(got.double(), want.double(), rtol=1e-4, atol=1e-6)
    for p, s in zip(m.parameters(), shadows):
        torch.testing.assert_close(p.grad, s.grad, rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("name", ["resnet18", "resnet50", "resnet152", "unet", "unet_bilinear"])
def test_flat_gradient_layout_follows_backward_ready_order(name):
    """The DDP reducer launches buckets strictly in index order, so a bucket whose last gradient
    arrives after a later bucket's would hold that later all-reduce back.  The flat layout (hence
    the bucket order) must be exactly the order in which the engine backward announces gradients
    ready -- recorded here through the reducer hook -- for every bucket split."""
    from deeplearning_mpi_amd.models import ARCHS, UNet

    torch.manual_seed(0)
    if name.startswith("unet"):
        m = UNet(out_classes=1, up_sample_mode="bilinear" if "bilinear" in name else "conv_transpose")
        x = torch.randn(1, 3, 32, 32)
    else:
        m = ARCHS[name](num_classes=10)
        x = torch.randn(2, 3, 32, 32)
    a = m.arena
    seq = []
    out = m(x)
    a.hook = seq.append
    out.float().mean().backward()
    a.hook = None
    assert seq == a.order
    for caps in ((2 << 20, 32 << 20, 4 << 20), (1 << 18, 1 << 20, 1 << 18)):
        _, pb = a.buckets(*caps)
        bseq = [pb[i] for i in seq]
        assert bseq == sorted(bseq)


@pytest.mark.parametrize("fused", [True, False])
def test_dual_dgrad_matches_torch(monkeypatch, fused):
    """1x1 data gradients over [dy | z] with weights {W*k1, W*k2} and bias W.k3 (engine.DUAL_DGRAD,
    dz only materialised for the weight gradient): the fp64 engine still reproduces autograd, and
    the dual path is taken for every eligible 1x1 conv (all but the last block's conv3, whose
    gradient comes from the average-pool backward)."""
    from deeplearning_mpi_amd.models import engine

    monkeypatch.setattr(engine, "DUAL_DGRAD", True)
    monkeypatch.setattr(engine, "DUAL_MIN_ROWS", 0)
    calls = []
    orig = engine.ConvUnit.bwd

    def counted(self, be, ctx, dy, *a, **k):
        if self.dual and ctx is not None and ctx[1] is not None and ctx[1].ld == 2 * ctx[1].C \
                and dy.buf.data_ptr() == ctx[1].buf.data_ptr():
            calls.append(self)
        return orig(self, be, ctx, dy, *a, **k)

    monkeypatch.setattr(engine.ConvUnit, "bwd", counted)
    g = torch.Generator().manual_seed(4)
    x = torch.randn(4, 3, 64, 64, generator=g)
    y = torch.randint(10, (4,), generator=g)
    def make():
        m = resnet50(num_classes=10)
        m.fuse_bn_bwd = fused   # unfused: dy still lands in the [dy | z] buffers, read with their stride
        return m

    _run_pair(make, x, y, cross_entropy, F.cross_entropy)
    assert len(calls) == 2 * 16 - 1   # dy written into the [dy | z] buffer (dual GEMM only when fused)
