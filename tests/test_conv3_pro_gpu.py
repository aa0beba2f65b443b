"""The BN-apply + ReLU of a 64-channel producer computed inside the streaming 64 -> 64 3x3 forward
(engine.FUSE_APPLY_3X3, conv3x3_stream.hip PRO): the kernel applies it to its staged input tiles and
stores it once.  Same arithmetic as the standalone apply pass (bn_apply_kernel's fma order) and the
same conv kernel, so a whole training step is bit-identical to the unfused schedule
(set_conv3_pro(0)); the fused launch must actually run."""
import copy

import pytest
import torch

from deeplearning_mpi_amd.models import UNet, resnet50
from deeplearning_mpi_amd.ops import bce_with_logits, cross_entropy
from deeplearning_mpi_amd.optim import SGD, Adam, clip_grad_norm_

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _steps(model, make_opt, x, y, loss_fn, fused, clip=False, steps=3, units=()):
    model.train()
    model.engine_setup(DEV)
    for u in units(model) if units else ():
        u.fuse3 = True
    C = model._be.C
    C.set_conv3_pro(1 if fused else 0)
    calls = {"n": 0}   # fused launches through the backend
    be = model._be
    f0 = be.conv3_fwd_bn_apply

    def counted(*a, **k):
        calls["n"] += 1
        return f0(*a, **k)

    be.conv3_fwd_bn_apply = counted
    try:
        opt = make_opt(model.parameters())
        losses = []
        for _ in range(steps):
            opt.zero_grad()
            loss = loss_fn(model(x), y)
            loss.backward()
            if clip:
                clip_grad_norm_(model.parameters(), 1.0, optimizer=opt)
            opt.step()
            losses.append(loss.detach().clone())
        torch.cuda.synchronize()
    finally:
        C.set_conv3_pro(1)
        del be.conv3_fwd_bn_apply
    return losses, [p.detach().clone() for p in model.parameters()] + [b.detach().clone() for b in model.buffers()], \
        calls["n"]


def test_unet_fused_3x3_apply_bit_identical():
    torch.manual_seed(0)
    m = UNet(out_classes=1, in_channels=3).to(DEV)
    m2 = copy.deepcopy(m)
    x = torch.randn(2, 3, 64, 96, device=DEV)
    y = (torch.rand(2, 64, 96, device=DEV) > 0.5).float()
    loss = lambda o, t: bce_with_logits(o.squeeze(1), t)
    opt = lambda ps: Adam(ps, lr=1e-3)
    la, pa, na = _steps(m, opt, x, y, loss, True, clip=True)
    lb, pb, nb = _steps(m2, opt, x, y, loss, False, clip=True)
    assert na >= 2 * 3   # the level-1 encoder and decoder DoubleConvs, every step
    for a, b in zip(la + pa, lb + pb):
        assert torch.equal(a, b)


def test_resnet50_default_schedule_does_not_fuse():
    torch.manual_seed(0)
    m = resnet50(num_classes=10).to(DEV)
    _, _, n = _steps(m, lambda ps: SGD(ps, lr=0.05), torch.randn(2, 3, 64, 64, device=DEV),
                     torch.randint(0, 10, (2,), device=DEV), cross_entropy, True, steps=1)
    assert n == 0


def test_resnet50_fused_3x3_apply_bit_identical():
    torch.manual_seed(0)
    m = resnet50(num_classes=10).to(DEV)
    m2 = copy.deepcopy(m)
    x = torch.randn(4, 3, 112, 112, device=DEV)
    y = torch.randint(0, 10, (4,), device=DEV)
    opt = lambda ps: SGD(ps, lr=0.05, momentum=0.9, weight_decay=1e-5)
    # ResNet keeps the unfused schedule by default; the kernel path is checked on layer 1's conv2
    units = lambda mm: [b.u[1] for b in mm.blocks[:3]]
    la, pa, na = _steps(m, opt, x, y, cross_entropy, True, units=units)
    lb, pb, nb = _steps(m2, opt, x, y, cross_entropy, False, units=units)
    assert na >= 3 * 3   # layer 1's three conv2
    for a, b in zip(la + pa, lb + pb):
        assert torch.equal(a, b)
