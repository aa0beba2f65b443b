"""Dual 1x1 data gradient on the GPU (models/engine.py DUAL_DGRAD): the data gradient of a 1x1
stride-1 conv behind a training BatchNorm reduces over [dy | z] with weights {W*k1, W*k2} and an
fp32 bias W.k3 instead of over the materialised dz = k1*dy + k2*z + k3.

* ``dual_dgrad_weights`` kernel vs torch (exact: one rounding of the same fp32 product; the bias
  within fp32 summation-order noise);
* the whole production path at a ResNet-50 layer-1 shape vs an fp32 reference of dz . W;
* ResNet-50 training step with the dual path forced on every eligible conv: as close to the fp64
  oracle as stock bf16 autocast (tests/test_models_gpu.py criterion), forward bit-identical to
  the dual-off engine."""
import copy

import pytest
import torch

from deeplearning_mpi_amd.models import resnet50
from deeplearning_mpi_amd.ops import cross_entropy
from deeplearning_mpi_amd.ops.act import Act

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _be():
    from deeplearning_mpi_amd.ops.backend import NativeBackend

    return NativeBackend(torch.device(DEV))


@pytest.mark.parametrize("C,K", [(64, 256), (256, 64), (128, 512), (24, 40)])
def test_dual_weights_kernel(C, K):
    be = _be()
    g = torch.Generator(device=DEV).manual_seed(C + K)
    w = torch.randn(C, K, device=DEV, generator=g).to(torch.bfloat16)
    coef = torch.randn(3, K, device=DEV, generator=g)
    w2, b = be.dual_weights(w, C, K, coef)
    torch.cuda.synchronize()
    wf = w.float()
    assert torch.equal(w2[:, :K], (wf * coef[0]).to(torch.bfloat16))
    assert torch.equal(w2[:, K:], (wf * coef[1]).to(torch.bfloat16))
    ref = (wf.double() * coef[2].double()).sum(1)
    assert torch.allclose(b.double(), ref, rtol=1e-5, atol=1e-5 * ref.abs().max().item())


def test_dual_dgrad_layer1_shape():
    """dx = [dy | z] . {W k1, W k2} + W.k3 through the production dgrad dispatch (ResNet-50 layer-1
    conv3, 256 -> 64 channels at 56x56, 32 images) vs fp32 dz . W."""
    be = _be()
    N, H, W, K, C = 32, 56, 56, 256, 64
    g = torch.Generator(device=DEV).manual_seed(7)
    buf = torch.randn(N * H * W, 2 * K, device=DEV, generator=g).to(torch.bfloat16)
    buf[:, K:] += 1.5   # BN inputs with a nonzero mean
    coef = torch.randn(3, K, device=DEV, generator=g) * 0.1
    wT = (torch.randn(C, K, device=DEV, generator=g) * 0.05).to(torch.bfloat16)
    w2, b = be.dual_weights(wT, C, K, coef)
    dx = Act.empty(N, H, W, C, torch.bfloat16, DEV)
    be.conv_dgrad(Act(buf, N, H, W, 2 * K), w2, C, 1, 1, 1, 0, dx, bias=b)
    torch.cuda.synchronize()
    dy, z = buf[:, :K].float(), buf[:, K:].float()
    dz = coef[0] * dy + coef[1] * z + coef[2]
    ref = dz @ wT.float().t()
    err = ((dx.buf.float() - ref).norm() / ref.norm()).item()
    assert err < 1.5e-2, err


def test_resnet50_dual_step_vs_oracle(monkeypatch):
    from deeplearning_mpi_amd.models import engine

    from test_models_gpu import _compare

    monkeypatch.setattr(engine, "DUAL_DGRAD", True)
    monkeypatch.setattr(engine, "DUAL_MIN_ROWS", 0)
    g = torch.Generator(device=DEV).manual_seed(3)
    x = torch.randn(8, 3, 128, 128, device=DEV, generator=g)
    y = torch.randint(10, (8,), device=DEV, generator=g)
    _compare(lambda: resnet50(num_classes=10), x, y, cross_entropy, torch.nn.functional.cross_entropy)


def test_resnet50_dual_forward_identical_and_grads_close(monkeypatch):
    from deeplearning_mpi_amd.models import engine

    torch.manual_seed(0)
    m1 = resnet50(num_classes=10).to(DEV)
    m2 = copy.deepcopy(m1)
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(16, 3, 96, 96, device=DEV, generator=g)
    y = torch.randint(10, (16,), device=DEV, generator=g)
    losses = []
    for m, on in ((m1, True), (m2, False)):
        monkeypatch.setattr(engine, "DUAL_DGRAD", on)
        monkeypatch.setattr(engine, "DUAL_MIN_ROWS", 0)
        m.arena.zero_grad()
        loss = cross_entropy(m(x), y)
        loss.backward()
        losses.append(loss.detach())
    torch.cuda.synchronize()
    assert torch.equal(losses[0], losses[1])
    g1, g2 = m1.arena.grad, m2.arena.grad
    assert ((g1 - g2).norm() / g2.norm()).item() < 3e-2
