"""Deferred, batched weight-gradient split reductions (ops.cpp wgrad_reduce_or_defer, the engine
backward's mode) at model level: one training step's parameter gradients are bit-identical to the
step with every reduction launched right after its weight-gradient GEMM (two launches each), and the
step issues a handful of reduction launches instead of one or two per convolution."""
import pytest
import torch

from deeplearning_mpi_amd.models import resnet18, resnet50, UNet
from deeplearning_mpi_amd.ops import cross_entropy

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(name):
    g = torch.Generator().manual_seed(5)
    if name == "resnet50":
        x = torch.randn(8, 3, 96, 96, generator=g)
        return (lambda: resnet50(num_classes=100)), x, torch.randint(0, 100, (8,), generator=g)
    if name == "resnet18":
        x = torch.randn(32, 3, 32, 32, generator=g)
        return (lambda: resnet18(num_classes=10)), x, torch.randint(0, 10, (32,), generator=g)
    x = torch.randn(2, 3, 64, 64, generator=g)
    return (lambda: UNet(out_classes=1)), x, None


@pytest.mark.parametrize("name", ["resnet50", "resnet18", "unet"])
def test_deferred_wgrad_reductions_bit_identical(name):
    make, x, y = _model(name)
    x = x.to(DEV)
    y = y.to(DEV) if y is not None else None
    torch.manual_seed(0)
    m0 = make().to(DEV)
    state = {k: v.clone() for k, v in m0.state_dict().items()}
    grads, launches = {}, {}
    for defer in (True, False):
        m = make().to(DEV)
        m.load_state_dict(state)
        m.train()
        m.engine_setup(DEV)
        C = m._be.C
        C.set_conv_autotune(0)   # the same tiles in both runs
        if not defer:
            m._be.wgrad_defer = None   # the engine then launches each reduction immediately
        n0 = C.wgrad_reduce_launches()
        out = m(x)
        loss = cross_entropy(out, y) if y is not None else out.float().square().mean()
        loss.backward()
        torch.cuda.synchronize()
        launches[defer] = C.wgrad_reduce_launches() - n0
        assert C.wgrad_pending() == 0
        grads[defer] = [p.grad.detach().clone() for p in m.parameters()]
        C.set_conv_autotune(-1)
    for i, (a, b) in enumerate(zip(grads[True], grads[False])):
        assert torch.equal(a, b), (name, i, (a - b).abs().max().item())
    assert launches[True] < launches[False], launches
    if name == "resnet50":
        assert launches[True] <= 10, launches
