"""The weight recast split over two streams (utils/arena.py ``mark_cast_group``): the first layer's
compute copies on the current stream, the rest on the side stream beside the first layer's forward.
The training step must be bit-identical to the one-launch recast on the current stream, eager and
from a hipGraph replay, and the side-stream path must actually run."""
import copy

import pytest
import torch

from deeplearning_mpi_amd.models import UNet, resnet50
from deeplearning_mpi_amd.ops import bce_with_logits, cross_entropy
from deeplearning_mpi_amd.optim import SGD, Adam

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(model, opt_fn, x, y, loss_fn, split, steps=4, graph=False):
    model.train()
    model.engine_setup(x.device)
    be = model._be
    be.aux_min_pixels = 0   # auxiliary streams on at this small size (the side stream carries the recast)
    if not split:
        model._arena._cast_split = None
        model._arena.refresh(force=True)   # (one-launch descriptors built outside any capture)
    n0 = model._arena.split_casts
    opt = opt_fn(model.parameters())

    def step():
        opt.zero_grad()
        loss = loss_fn(model(x), y)
        loss.backward()
        opt.step()
        return loss

    if graph:
        from deeplearning_mpi_amd.utils.graphs import CapturedStep

        step = CapturedStep(step, warmup=2, inputs=(x, y))   # the 2nd eager step recasts, the 3rd captures
        assert steps >= 4
    losses = [step().detach().clone() for _ in range(steps)]
    torch.cuda.synchronize()
    used = model._arena.split_casts > n0
    if graph:
        assert step.graph is not None, step.capture_error   # captured and replayed
    return losses, [p.detach().clone() for p in model.parameters()], used


def _unet_pair():
    torch.manual_seed(0)
    m = UNet(out_classes=1, in_channels=3).to(DEV)
    return m, copy.deepcopy(m)


def _unet_data(n=2):
    x = torch.randn(n, 3, 64, 64, device=DEV)
    y = (torch.rand(n, 64, 64, device=DEV) > 0.5).float()
    return x, y


def _unet_loss(o, t):
    return bce_with_logits(o.squeeze(1), t)


@pytest.mark.parametrize("graph", [False, True])
def test_unet_split_recast_bit_identical(graph):
    m, m2 = _unet_pair()
    x, y = _unet_data()
    opt = lambda ps: Adam(ps, lr=1e-3)
    la, pa, used_a = _run(m, opt, x, y, _unet_loss, True, graph=graph)
    lb, pb, used_b = _run(m2, opt, x, y, _unet_loss, False, graph=graph)
    assert used_a and not used_b
    for a, b in zip(la, lb):
        assert torch.equal(a, b)
    for a, b in zip(pa, pb):
        assert torch.equal(a, b)


def test_split_recast_eval_after_update_sees_new_weights():
    """An eval forward right after an optimizer step (no training forward in between) recasts on the
    split path and must match a fresh one-launch recast of the same masters."""
    m, _ = _unet_pair()
    x, y = _unet_data()
    _run(m, lambda ps: Adam(ps, lr=1e-3), x, y, _unet_loss, True, steps=2)
    m.eval()
    with torch.no_grad():
        a = m(x).clone()
        m._arena._cast_split = None
        m._arena.refresh(force=True)
        b = m(x).clone()
    torch.cuda.synchronize()
    assert torch.equal(a, b)


def test_resnet_recast_not_split():
    """ResNet marks no first layer (the overlap measured slower there): every recast is one launch."""
    torch.manual_seed(0)
    m = resnet50(num_classes=10).to(DEV)
    x = torch.randn(4, 3, 64, 64, device=DEV)
    y = torch.randint(0, 10, (4,), device=DEV)
    _, _, used = _run(m, lambda ps: SGD(ps, lr=0.1, momentum=0.9), x, y, cross_entropy, True, steps=2)
    assert not used and m._arena._cast_split is None
