"""End-to-end model numerics on the GPU.

The native engine runs bf16 activations with fp32 accumulation/master weights, like
``torch.autocast(bfloat16)``.  Both are compared with an fp64 eager-torch oracle on the same
parameters and data; the engine's deviation (logits, loss, every parameter gradient, BN buffers)
must stay within a small factor of stock autocast's own deviation -- i.e. the engine is at least
as accurate as the stock bf16 path the reference would run (BN-heavy nets amplify rounding, so
an absolute tolerance against fp32 would be meaningless)."""
import copy

import pytest
import torch
import torch.nn.functional as F

from deeplearning_mpi_amd.models import UNet, resnet18, resnet50
from deeplearning_mpi_amd.ops import bce_with_logits, cross_entropy

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _err(a, ref):
    a, ref = a.double().flatten(), ref.double().flatten()
    return ((a - ref).norm() / ref.norm().clamp_min(1e-30)).item()


def _compare(make, x, y, loss_e, loss_t, skip=lambda n: False, slack=3.0, floor=2e-2):
    torch.manual_seed(0)
    m1 = make().to(DEV)
    m2 = copy.deepcopy(m1)
    m3 = copy.deepcopy(m1).double()
    for m in (m1, m2, m3):
        m.train()
    o1 = m1(x)
    loss_e(o1, y).backward()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        o2 = m2.forward_torch(x)
    loss_t(o2.float(), y).backward()
    o3 = m3.forward_torch(x.double())
    loss_t(o3, y.double() if y.is_floating_point() else y).backward()
    torch.cuda.synchronize()
    assert _err(o1, o3) <= slack * _err(o2, o3) + 1e-2
    bad = []
    for (n, p1), (_, p2), (_, p3) in zip(m1.named_parameters(), m2.named_parameters(), m3.named_parameters()):
        if skip(n) or p3.grad.abs().max() == 0:
            continue
        e1, e2 = _err(p1.grad, p3.grad), _err(p2.grad, p3.grad)
        if e1 > slack * e2 + floor:
            bad.append((n, round(e1, 4), round(e2, 4)))
    assert not bad, bad
    for (n, b1), (_, b2), (_, b3) in zip(m1.named_buffers(), m2.named_buffers(), m3.named_buffers()):
        if b1.is_floating_point():
            assert _err(b1, b3) <= slack * _err(b2, b3) + 1e-2, n
    m1.eval()
    m3.eval()
    with torch.no_grad():
        assert _err(m1(x), m3.forward_torch(x.double())) < 5e-2


def test_resnet18_engine_vs_autocast():
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.randn(16, 3, 64, 64, device=DEV, generator=g)
    y = torch.randint(10, (16,), device=DEV, generator=g)
    _compare(lambda: resnet18(num_classes=10), x, y, cross_entropy, F.cross_entropy)


def test_resnet50_engine_vs_autocast():
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.randn(8, 3, 128, 128, device=DEV, generator=g)
    y = torch.randint(1000, (8,), device=DEV, generator=g)
    _compare(lambda: resnet50(num_classes=1000), x, y, cross_entropy, F.cross_entropy)


@pytest.mark.parametrize("mode", ["conv_transpose", "bilinear"])
def test_unet_engine_vs_autocast(mode):
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.randn(2, 3, 64, 96, device=DEV, generator=g)
    y = (torch.rand(2, 64, 96, device=DEV, generator=g) > 0.5).float()
    skip = lambda n: n.endswith("bias") and "double_conv.double_conv" in n   # conv bias before train-BN
    _compare(lambda: UNet(out_classes=1, up_sample_mode=mode), x, y,
             lambda o, t: bce_with_logits(o.squeeze(1), t),
             lambda o, t: F.binary_cross_entropy_with_logits(o.squeeze(1), t), skip=skip)


def test_unet_1ch_input_and_training_decreases_loss():
    torch.manual_seed(0)
    from deeplearning_mpi_amd.optim import Adam, clip_grad_norm_

    m = UNet(out_classes=1, in_channels=1).to(DEV)
    opt = Adam(m.parameters(), lr=1e-3)
    x = torch.randn(2, 1, 64, 64, device=DEV)
    t = (x[:, 0] > 0).float()
    losses = []
    for _ in range(8):
        out = m(x)
        assert out.shape == (2, 1, 64, 64)
        loss = bce_with_logits(out.squeeze(1), t)
        opt.zero_grad()
        loss.backward()
        clip_grad_norm_(m.parameters(), 1.0, optimizer=opt)
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0]


def test_resnet_training_decreases_loss():
    torch.manual_seed(0)
    from deeplearning_mpi_amd.optim import SGD

    m = resnet18(num_classes=10).to(DEV)
    opt = SGD(m.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-5)
    x = torch.randn(32, 3, 32, 32, device=DEV)
    y = torch.randint(10, (32,), device=DEV)
    losses = []
    for _ in range(10):
        opt.zero_grad()
        loss = cross_entropy(m(x), y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < 0.5 * losses[0]


@pytest.mark.parametrize("make,loss", [
    (lambda: resnet50(num_classes=10), "ce"),
    (lambda: UNet(out_classes=1), "bce"),
])
def test_auxiliary_streams_bitwise_equal_single_stream(make, loss):
    """Weight gradients on the side stream and the ResNet downsample branch on the branch stream
    change only WHEN kernels run, not what they compute: one training step with the auxiliary
    streams must give bit-identical gradients and BN statistics to the same step on one stream
    (a missing stream dependency would show up as a mismatch)."""
    torch.manual_seed(0)
    m1 = make().to(DEV)
    m2 = copy.deepcopy(m1)
    g = torch.Generator(device=DEV).manual_seed(5)
    if loss == "ce":
        x = torch.randn(32, 3, 64, 64, device=DEV, generator=g)
        y = torch.randint(10, (32,), device=DEV, generator=g)
        fn = lambda m: cross_entropy(m(x), y)   # noqa: E731
    else:
        x = torch.randn(2, 3, 64, 64, device=DEV, generator=g)
        y = (torch.rand(2, 64, 64, device=DEV, generator=g) > 0.5).float()
        fn = lambda m: bce_with_logits(m(x).squeeze(1), y)   # noqa: E731
    m1.engine_setup(DEV)
    m2.engine_setup(DEV)
    m1._be.aux_min_pixels = 0       # small test inputs: force the auxiliary streams on
    assert m1._be.side_stream is not None
    m2._be.side_stream = None       # everything on the current stream
    m2._be.branch_stream = None
    m2._be.chunk_serial = True      # the same image-chunked forward BN-applies (engine.PendingApply), serially
    for m in (m1, m2):
        m.arena.zero_grad()
        fn(m).backward()
    torch.cuda.synchronize()
    assert torch.equal(m1.arena.grad, m2.arena.grad)
    for (n, b1), (_, b2) in zip(m1.named_buffers(), m2.named_buffers()):
        assert torch.equal(b1, b2), n
