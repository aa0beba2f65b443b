"""End-to-end model numerics on the GPU: the native bf16 engine vs eager fp32 torch with the same
parameters (forward logits, loss, every parameter gradient by cosine similarity, BN buffers)."""
import copy

import pytest
import torch
import torch.nn.functional as F

from deeplearning_mpi_amd.models import UNet, resnet18, resnet50
from deeplearning_mpi_amd.ops import bce_with_logits, cross_entropy

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return (a @ b / (a.norm() * b.norm() + 1e-30)).item()


def _compare(make, x, y, loss_e, loss_t, skip_bias_before_bn=False, min_cos=0.99):
    torch.manual_seed(0)
    m1 = make().to(DEV)
    m2 = copy.deepcopy(m1)
    m1.train()
    m2.train()
    o1 = m1(x)
    l1 = loss_e(o1, y)
    l1.backward()
    o2 = m2.forward_torch(x)
    l2 = loss_t(o2, y)
    l2.backward()
    torch.cuda.synchronize()
    assert abs(l1.item() - l2.item()) < 2e-2 * max(1.0, abs(l2.item()))
    assert _cos(o1, o2) > 0.999
    bad = []
    for (n, p1), (_, p2) in zip(m1.named_parameters(), m2.named_parameters()):
        if skip_bias_before_bn and n.endswith("bias") and "double_conv" in n and (".0." in n or ".3." in n):
            continue   # conv bias followed by training-mode BN: exact gradient is 0
        c = _cos(p1.grad, p2.grad)
        if c < min_cos:
            bad.append((n, c))
    assert not bad, bad
    for (n, b1), (_, b2) in zip(m1.named_buffers(), m2.named_buffers()):
        if b1.is_floating_point():
            assert _cos(b1, b2) > 0.999, n
    m1.eval()
    m2.eval()
    with torch.no_grad():
        assert _cos(m1(x), m2.forward_torch(x)) > 0.999


def test_resnet18_engine_vs_torch():
    x = torch.randn(16, 3, 64, 64, device=DEV)
    y = torch.randint(10, (16,), device=DEV)
    _compare(lambda: resnet18(num_classes=10), x, y, cross_entropy, F.cross_entropy)


def test_resnet50_engine_vs_torch():
    x = torch.randn(8, 3, 128, 128, device=DEV)
    y = torch.randint(1000, (8,), device=DEV)
    _compare(lambda: resnet50(num_classes=1000), x, y, cross_entropy, F.cross_entropy, min_cos=0.97)


@pytest.mark.parametrize("mode", ["conv_transpose", "bilinear"])
def test_unet_engine_vs_torch(mode):
    x = torch.randn(2, 3, 64, 96, device=DEV)
    y = (torch.rand(2, 64, 96, device=DEV) > 0.5).float()
    _compare(lambda: UNet(out_classes=1, up_sample_mode=mode), x, y,
             lambda o, t: bce_with_logits(o.squeeze(1), t),
             lambda o, t: F.binary_cross_entropy_with_logits(o.squeeze(1), t), skip_bias_before_bn=True)


def test_unet_1ch_input():
    torch.manual_seed(0)
    m = UNet(out_classes=1, in_channels=1).to(DEV)
    x = torch.randn(2, 1, 64, 64, device=DEV)
    out = m(x)
    assert out.shape == (2, 1, 64, 64)
    bce_with_logits(out.squeeze(1), (torch.rand(2, 64, 64, device=DEV) > 0.5).float()).backward()
    assert torch.isfinite(m.arena.grad).all()
