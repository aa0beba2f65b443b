"""Device-resident input pipeline (data/device.py, csrc/kernels/data.hip): the CPU reference of
the batch kernel against the reference CIFAR transform, sampler-order iteration, the cached
dataset, and (GPU) the HIP kernel against the reference."""
import numpy as np
import pytest
import torch

from deeplearning_mpi_amd.data import (CifarTransform, DeviceBatches, DeviceCachedDataset, DeviceImageDataset,
                                       DistributedSampler, SyntheticMasks, image_batch_reference)
from deeplearning_mpi_amd.data.datasets import CIFAR_MEAN, CIFAR_STD
from deeplearning_mpi_amd.data.device import _aug_params


class _FixedRng:
    """Feeds CifarTransform the crop offsets / flip the device pipeline drew."""

    def __init__(self, i, j, flip):
        self.i, self.j, self.flip = i, j, flip

    def integers(self, lo, hi, size):
        return np.array([self.i, self.j])

    def random(self):
        return 0.0 if self.flip else 1.0


def _data(n=40, seed=0):
    g = np.random.default_rng(seed)
    return g.integers(0, 256, size=(n, 32, 32, 3), dtype=np.uint8), g.integers(0, 10, size=n)


def test_aug_params_range_and_spread():
    idx = torch.arange(5000)
    oi, oj, fl = _aug_params(idx, seed=3, epoch=7, pad=4)
    assert int(oi.min()) == 0 and int(oi.max()) == 8 and int(oj.min()) == 0 and int(oj.max()) == 8
    assert 0.45 < fl.float().mean().item() < 0.55
    oi2, _, _ = _aug_params(idx, seed=3, epoch=8, pad=4)
    assert not torch.equal(oi, oi2)      # a new epoch draws new crops


def test_reference_batch_matches_reference_cifar_transform():
    data, labels = _data()
    idx = torch.tensor([5, 0, 39, 17, 17, 3])
    x, y = image_batch_reference(torch.from_numpy(data), torch.from_numpy(labels), idx, 4, True, 11, 2,
                                 CIFAR_MEAN, CIFAR_STD)
    oi, oj, fl = _aug_params(idx, 11, 2, 4)
    tr = CifarTransform(train=True)
    for b, d in enumerate(idx.tolist()):
        want = tr(data[d], _FixedRng(int(oi[b]), int(oj[b]), int(fl[b])))
        assert torch.allclose(x[b], want, atol=1e-6), b
        assert int(y[b]) == labels[d]
    # eval transform: no crop / flip
    x, _ = image_batch_reference(torch.from_numpy(data), torch.from_numpy(labels), idx, 4, False, 11, 2,
                                 CIFAR_MEAN, CIFAR_STD)
    assert torch.allclose(x[1], CifarTransform(train=False)(data[0], None), atol=1e-6)


@pytest.mark.parametrize("world,rank", [(1, 0), (3, 1)])
def test_device_batches_follow_distributed_sampler(world, rank):
    data, labels = _data(50)
    ds = DeviceImageDataset(data, labels, "cpu", augment=False)
    sampler = DistributedSampler(ds, num_replicas=world, rank=rank, seed=0)
    sampler.set_epoch(4)
    order = list(iter(sampler))
    got = []
    for x, y in DeviceBatches(ds, 8, sampler):
        assert x.shape[1:] == (3, 32, 32) and x.dtype == torch.float32
        got += y.tolist()
    assert got == [int(labels[i]) for i in order]


def test_device_batches_write_fixed_buffers():
    data, labels = _data(20)
    ds = DeviceImageDataset(data, labels, "cpu", augment=True, seed=1)
    xs, ys = torch.zeros(8, 3, 32, 32), torch.zeros(8, dtype=torch.int64)
    batches = list(DeviceBatches(ds, 8, out=(xs, ys)))
    assert len(batches) == 3 and batches[0][0] is xs and batches[2][0] is not xs   # ragged tail: fresh tensors
    ref, _ = image_batch_reference(ds.data, ds.labels, torch.arange(16, 20), 4, True, 1, 0, CIFAR_MEAN, CIFAR_STD)
    assert torch.equal(batches[2][0], ref)


def test_device_cached_dataset_dict_items():
    src = SyntheticMasks(12, (3, 16, 16), seed=2)
    ds = DeviceCachedDataset(src, "cpu")
    b = ds.batch(torch.tensor([3, 0, 11]))
    assert set(b) == {"image", "mask"}
    for k, i in enumerate([3, 0, 11]):
        assert torch.equal(b["image"][k], src[i]["image"]) and torch.equal(b["mask"][k], src[i]["mask"])


@pytest.mark.gpu
def test_image_batch_kernel_matches_reference():
    data, labels = _data(300, seed=5)
    for augment in (True, False):
        ds = DeviceImageDataset(data, labels, "cuda", augment=augment, seed=9)
        idx = torch.randint(0, 300, (128,), generator=torch.Generator().manual_seed(0))
        x, y = ds.batch(idx.cuda(), epoch=3)
        xr, yr = image_batch_reference(torch.from_numpy(data), torch.from_numpy(labels), idx, 4, augment, 9, 3,
                                       CIFAR_MEAN, CIFAR_STD)
        torch.cuda.synchronize()
        assert torch.allclose(x.cpu(), xr, atol=1e-6) and torch.equal(y.cpu(), yr)
