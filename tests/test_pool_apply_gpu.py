"""The UNet encoder skip's BN-apply fused into the 2x2 max-pool (models/unet.py FUSE_POOL_APPLY,
pool.hip maxpool_fwd_fixed_kernel with ys) and the last decoder BN-apply fused into the 1x1 head and its
weight gradient (FUSE_HEAD_APPLY): kernel level -- pooled values, indices and the stored applied input
bit-identical to bn_apply + max-pool, the head over a Deferred.affine input bit-identical to the head
over the stored apply; model level -- one UNet training step (loss, every gradient, running
statistics) bit-identical to the unfused schedule."""
import copy

import pytest
import torch

import deeplearning_mpi_amd.models.unet as unet_mod
from deeplearning_mpi_amd.models import UNet
from deeplearning_mpi_amd.ops import bce_with_logits
from deeplearning_mpi_amd.ops.act import Act, Deferred
from deeplearning_mpi_amd.ops.backend import NativeBackend

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("N,H,W,C,ld,off", [(2, 16, 24, 64, 192, 128), (3, 8, 8, 128, 128, 0)])
def test_pool_apply_kernel_bit_identical(N, H, W, C, ld, off):
    be = NativeBackend(DEV)
    g = torch.Generator(device=DEV).manual_seed(C + H)
    z = Act(torch.randn(N * H * W, C, device=DEV, generator=g).to(torch.bfloat16), N, H, W, C)
    sc = torch.rand(C, device=DEV, generator=g) + 0.5
    sh = torch.randn(C, device=DEV, generator=g) * 0.3
    # unfused: bn_apply into the concat slice, pool of the slice
    cat0 = Act(torch.zeros(N * H * W, ld, device=DEV, dtype=torch.bfloat16), N, H, W, ld).slice(off, C)
    be.bn_apply(z, sc, sh, None, True, cat0)
    down0 = Act.empty(N, H // 2, W // 2, C, torch.bfloat16, DEV)
    idx0 = be.maxpool_fwd(cat0, 2, 2, 0, down0)
    # fused
    cat1 = Act(torch.zeros(N * H * W, ld, device=DEV, dtype=torch.bfloat16), N, H, W, ld).slice(off, C)
    down1 = Act.empty(N, H // 2, W // 2, C, torch.bfloat16, DEV)
    idx1 = be.maxpool_fwd(z, 2, 2, 0, down1, bn=(sc, sh), store=cat1)
    torch.cuda.synchronize()
    assert torch.equal(cat0.buf.view(torch.int16), cat1.buf.view(torch.int16))
    assert torch.equal(down0.buf.view(torch.int16), down1.buf.view(torch.int16))
    assert torch.equal(idx0, idx1)


def test_head_over_deferred_apply_bit_identical():
    be = NativeBackend(DEV)
    N, H, W, C = 2, 32, 48, 64
    g = torch.Generator(device=DEV).manual_seed(11)
    z = Act(torch.randn(N * H * W, C, device=DEV, generator=g).to(torch.bfloat16), N, H, W, C)
    sc = torch.rand(C, device=DEV, generator=g) + 0.5
    sh = torch.randn(C, device=DEV, generator=g) * 0.3
    w = (torch.randn(8, C, device=DEV, generator=g) / 8).to(torch.bfloat16)
    b = torch.randn(8, device=DEV, generator=g)
    y0 = torch.empty(N * H * W, 1, device=DEV)
    y1 = torch.empty(N * H * W, 1, device=DEV)
    be.conv_fwd(be.materialize(Deferred.affine(z, sc, sh)), w, 8, 1, 1, 1, 0, Act(y0, N, H, W, 1), bias=b, kvalid=1)
    be.conv_fwd(Deferred.affine(z, sc, sh), w, 8, 1, 1, 1, 0, Act(y1, N, H, W, 1), bias=b, kvalid=1)
    torch.cuda.synchronize()
    assert be.C.head1x1_last() == 1
    assert torch.equal(y0, y1)


def test_unet_step_bit_identical_to_unfused(monkeypatch):
    torch.manual_seed(0)
    base = UNet(out_classes=1).to(DEV)
    x = torch.randn(2, 3, 64, 64, device=DEV)
    t = (torch.rand(2, 64, 64, device=DEV) > 0.5).float()
    res = {}
    for fuse in (True, False):
        monkeypatch.setattr(unet_mod, "FUSE_POOL_APPLY", fuse)
        monkeypatch.setattr(unet_mod, "FUSE_HEAD_APPLY", fuse)
        m = copy.deepcopy(base)
        loss = bce_with_logits(m(x).squeeze(1), t)
        loss.backward()
        torch.cuda.synchronize()
        res[fuse] = (loss.detach().clone(), [p.grad.clone() for p in m.parameters()],
                     [b.clone() for b in m.buffers()])
    assert torch.equal(res[True][0], res[False][0])
    for a, b in zip(res[True][1], res[False][1]):
        assert torch.equal(a, b)
    for a, b in zip(res[True][2], res[False][2]):
        assert torch.equal(a, b)
