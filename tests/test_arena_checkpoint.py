import copy
import os

import torch

from deeplearning_mpi_amd.models import UNet, resnet18, resnet50
from deeplearning_mpi_amd.parallel import DistributedDataParallel
from deeplearning_mpi_amd.utils import checkpoint as ck


def test_state_dict_keys_match_reference():
    m = resnet18(num_classes=10)
    ddp = DistributedDataParallel(m)
    sd = ddp.state_dict()
    assert len(sd) == 122   # SURVEY.md §5.4 (torchvision resnet18 + 10-class fc, DDP-wrapped)
    assert "module.conv1.weight" in sd and "module.layer1.0.conv1.weight" in sd and "module.fc.bias" in sd
    assert sd["module.bn1.num_batches_tracked"].dtype == torch.int64
    u = DistributedDataParallel(UNet(out_classes=1))
    sdu = u.state_dict()
    assert len(sdu) == 136
    assert "module.down_conv1.double_conv.double_conv.0.weight" in sdu and "module.conv_last.bias" in sdu


def test_param_counts():
    assert sum(p.numel() for p in resnet18(num_classes=10).parameters()) == 11181642
    assert sum(p.numel() for p in UNet(out_classes=1).parameters()) == 36963201   # SURVEY.md §2.2 C8 (train.py uses 1 class)


def test_arena_rehomes_and_buckets():
    m = resnet50(num_classes=1000)
    ref = copy.deepcopy(m)
    ar = m.engine_setup("cpu")
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        assert torch.equal(p, q), n
        assert ar.owns(p)
        assert p.grad is not None and p.grad.shape == p.shape
    bounds, pb = ar.buckets(2 * 2 ** 20, 32 * 2 ** 20)
    assert bounds[0][0] == 0 and bounds[-1][1] >= ar.total - ar.ALIGN
    for (s0, e0), (s1, e1) in zip(bounds, bounds[1:]):
        assert e0 == s1
    assert max(pb) == len(bounds) - 1
    # fc is registered last -> first in the flat buffer -> first bucket
    assert pb[ar.index[id(m.fc.weight)]] == 0
    # small tail bucket: the stem (registered first -> end of the flat buffer) goes out in a last
    # bucket of <= 4 MB instead of at the end of a 32 MB one
    b2, pb2 = ar.buckets(2 * 2 ** 20, 32 * 2 ** 20, 4 * 2 ** 20)
    assert len(b2) == len(bounds) + 1 and b2[:-2] == bounds[:-1]
    assert b2[-2][1] == b2[-1][0] and b2[-1][1] == bounds[-1][1]
    assert 0 < (b2[-1][1] - b2[-1][0]) * 4 <= 4 * 2 ** 20
    assert pb2[ar.index[id(m.conv1.weight)]] == len(b2) - 1
    for i, p in enumerate(ar.params):   # every parameter lies inside its bucket
        s, e = b2[pb2[i]]
        assert s <= ar.offsets[i] and ar.offsets[i] + p.numel() <= e


def test_compute_copy_refresh():
    m = resnet18(num_classes=10)
    ar = m.engine_setup("cpu")
    u = m.blocks[0].u[0]                   # layer1.0.conv1 (3x3, 64 -> 64)
    w = ar.get_compute(u.h_fwd).view(64, 3, 3, 64).clone()
    with torch.no_grad():
        m.layer1[0].conv1.weight.add_(1.0)
    ar.refresh()
    w2 = ar.get_compute(u.h_fwd).view(64, 3, 3, 64)
    assert torch.allclose(w2.permute(0, 3, 1, 2), m.layer1[0].conv1.weight)
    assert not torch.equal(w, w2)


def test_s2d_stem_weight_layout():
    """7x7/s2 stem as a 4x4/s1 conv over the 2x2 space-to-depth image: W2[k][a][b][slot*4 + c] =
    w[k][c][2a + vh][2b + vw] (slot = 2 vh + vw), zero past the 7x7 window and for c = 3; refreshed
    with the other compute copies."""
    m = resnet18(num_classes=10)
    ar = m.engine_setup("cpu")
    assert type(m.u_stem).__name__ == "S2DConvUnit"
    with torch.no_grad():
        m.conv1.weight.add_(0.5)
    ar.refresh()
    w = m.conv1.weight.detach()
    w2 = m.u_stem.w2.view(64, 4, 4, 4, 4)   # [k][a][b][slot][c]
    ref = torch.zeros(64, 4, 4, 4, 4)
    for vh in (0, 1):
        for vw in (0, 1):
            blk = w[:, :, vh::2, vw::2].permute(0, 2, 3, 1)   # [k][a][b][c]
            ref[:, :blk.shape[1], :blk.shape[2], vh * 2 + vw, :3] = blk
    assert torch.equal(w2, ref)


def test_checkpoint_roundtrip(tmp_path):
    torch.manual_seed(0)
    m = resnet18(num_classes=10)
    ddp = DistributedDataParallel(m)
    p = os.path.join(tmp_path, "resnet_distributed.pth")
    ck.save_checkpoint(ddp, p, extra={"epoch": 3})
    m2 = resnet18(num_classes=10)
    ddp2 = DistributedDataParallel(m2)
    meta = ck.load_checkpoint(ddp2, p)
    for (n, a), (_, b) in zip(ddp.state_dict().items(), ddp2.state_dict().items()):
        assert torch.equal(a, b), n
    assert meta.get("epoch") == 3
    # a plain (non-DDP) torchvision-style state_dict without the module. prefix also loads
    sd = {k[len("module."):]: v for k, v in ddp.state_dict().items()}
    torch.save(sd, p + ".plain")
    m3 = resnet18(num_classes=10)
    ck.load_checkpoint(m3, p + ".plain")
    assert torch.equal(m3.fc.weight, m.fc.weight)
