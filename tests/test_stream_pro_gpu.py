"""Deferred BN-apply + ReLU rebuilt in the streaming 1x1 forward kernel's operand prologue
(conv1x1_stream.hip PRO, engine.STREAM_PRO): the bottleneck's bn2 output is never stored; conv3
computes relu(z * scale + shift) from the staged z tile.

* kernel level: conv output and BN statistics through the streaming kernel with the deferred operand
  bit-identical to the streaming kernel over the materialised BN-apply output;
* model level: a ResNet-50 training step with the deferral on vs off is bit-identical (losses and
  every gradient), because the rebuilt operand has the bits of the stored one."""
import copy

import pytest
import torch

from deeplearning_mpi_amd.models import engine, resnet50
from deeplearning_mpi_amd.ops import cross_entropy
from deeplearning_mpi_amd.ops.act import Act, Deferred
from deeplearning_mpi_amd.ops.backend import NativeBackend

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("shape", [(4, 14, 14, 64, 256), (2, 28, 28, 128, 512), (3, 7, 9, 64, 128),
                                   (16, 56, 56, 64, 256)])
def test_stream_prologue_bit_identical(shape):
    N, H, W, C, K = shape
    be = NativeBackend(torch.device(DEV))
    g = torch.Generator(device=DEV).manual_seed(C + K + H)
    M = N * H * W
    z = Act(torch.randn(M, C, device=DEV, generator=g).to(torch.bfloat16), N, H, W, C)
    sc, sh = torch.rand(C, device=DEV, generator=g) + 0.5, torch.randn(C, device=DEV, generator=g) * 0.3
    w = (torch.randn(K, 1, 1, C, device=DEV, generator=g) / C ** 0.5).to(torch.bfloat16)
    assert be.stream_pro_ok(M, C, K)
    y = Act.empty(N, H, W, C, torch.bfloat16, DEV)
    be.bn_apply(z, sc, sh, None, True, y)
    out = {}
    for deferred in (True, False):
        x = Deferred.affine(z, sc, sh) if deferred else y
        o = Act.empty(N, H, W, K, torch.bfloat16, DEV)
        mt = be.conv_mtiles(N, H, W, C, K, 1, 1, 1, 0, pro=deferred)
        st = torch.zeros(mt, 2, K, device=DEV)
        rows = be.conv_fwd(x, w, K, 1, 1, 1, 0, o, stats=st)
        torch.cuda.synchronize()
        assert be.C.conv_stream_last() == 1
        out[deferred] = (o.buf.clone(), st.clone(), rows)
    assert torch.equal(out[True][0], out[False][0])
    assert torch.equal(out[True][1], out[False][1])


def test_resnet50_step_stream_prologue_bit_identical(monkeypatch):
    torch.manual_seed(0)
    m1 = resnet50(num_classes=10).to(DEV)
    m2 = copy.deepcopy(m1)
    g = torch.Generator(device=DEV).manual_seed(5)
    # 32 x 112^2: layer1 conv3 at 28^2 x 64 -> 256 (streaming kernel, 2 columns)
    x = torch.randn(32, 3, 112, 112, device=DEV, generator=g)
    y = torch.randint(10, (32,), device=DEV, generator=g)
    res = []
    orig = NativeBackend.conv_fwd_bn
    n = [0]

    def counting(self, xx, *a, **k):
        n[0] += isinstance(xx, Deferred)
        return orig(self, xx, *a, **k)

    monkeypatch.setattr(NativeBackend, "conv_fwd_bn", counting)
    for m, on in ((m1, True), (m2, False)):
        monkeypatch.setattr(engine, "STREAM_PRO", on)
        m.arena.zero_grad()
        n[0] = 0
        loss = cross_entropy(m(x), y)
        loss.backward()
        torch.cuda.synchronize()
        res.append((loss.detach(), m.arena.grad.clone(), n[0]))
    assert res[0][2] > 0 and res[1][2] == 0, (res[0][2], res[1][2])
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])
