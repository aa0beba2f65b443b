"""Device-resident input pipeline.

The reference feeds its GPUs through ``torch.utils.data.DataLoader`` worker processes: per-sample
Python/PIL transforms, collation, pinned host buffers and a host->device copy every step
(/root/reference/pytorch/resnet/main.py:82-97, unet/train.py:78-101).  Its datasets are small
(CIFAR-10: 150 MB of uint8; the UNet cell images at scale 0.2: ~0.3 GB as fp32) next to 288 GB of
HBM3E per MI355X, so here the dataset is made resident on the GPU once and every batch is one
device-side gather:

* :class:`DeviceImageDataset` -- uint8 HWC images + labels in HBM; a batch is ONE HIP kernel
  (``csrc/kernels/data.hip``): gather by index + RandomCrop(32, padding=4) + RandomHorizontalFlip
  + ToTensor + Normalize (the reference CIFAR transform), written as fp32 NCHW.  The augmentation
  parameters are a hash of (seed, epoch, dataset index), so they do not depend on the batch size,
  rank count or worker count, and :func:`image_batch_reference` reproduces them exactly on the CPU.
* :class:`DeviceCachedDataset` -- any deterministic map-style dataset (the reference UNet's
  image/mask dataset has no random augmentation) materialised once on the device; batches are
  ``index_select`` gathers.
* :class:`DeviceBatches` -- iterates either in :class:`DistributedSampler` order (the epoch's index
  list goes to the device in one copy), optionally writing into fixed tensors so a captured
  hipGraph step can consume them without a copy.
"""
from __future__ import annotations

import numpy as np
import torch

from .datasets import CIFAR10, CIFAR_MEAN, CIFAR_STD

_M32 = 0xFFFFFFFF


def _fmix32(h: torch.Tensor) -> torch.Tensor:
    """murmur3 finalizer on uint32 values held in int64 (mod 2^32 arithmetic), = data.hip:fmix32."""
    h = h & _M32
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & _M32
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & _M32
    return h ^ (h >> 16)


def _aug_params(idx: torch.Tensor, seed: int, epoch: int, pad: int):
    """(crop row offset, crop col offset, flip) per sample, exactly as the HIP kernel draws them."""
    base = ((seed * 0x9E3779B1) + (epoch * 0x85EBCA77)) & _M32
    h = _fmix32((idx.to(torch.int64) & _M32) + base)
    span = 2 * pad + 1
    return h % span, (h >> 8) % span, (h >> 16) & 1


def image_batch_reference(data_hwc_u8: torch.Tensor, labels: torch.Tensor, idx: torch.Tensor, pad: int,
                          augment: bool, seed: int, epoch: int, mean, std):
    """CPU/torch reference of the device batch kernel (also the CPU execution path)."""
    idx = idx.to(torch.int64).cpu()
    imgs = data_hwc_u8[idx.to(data_hwc_u8.device)].cpu().permute(0, 3, 1, 2).float() / 255.0   # [B, C, H, W]
    B, C, H, W = imgs.shape
    if augment:
        oi, oj, flip = _aug_params(idx, seed, epoch, pad)
        padded = torch.nn.functional.pad(imgs, (pad, pad, pad, pad))
        out = torch.empty_like(imgs)
        for b in range(B):
            crop = padded[b, :, int(oi[b]):int(oi[b]) + H, int(oj[b]):int(oj[b]) + W]
            out[b] = crop.flip(-1) if int(flip[b]) else crop
        imgs = out
    m = torch.tensor(mean[:C], dtype=torch.float32).view(1, C, 1, 1)
    s = torch.tensor(std[:C], dtype=torch.float32).view(1, C, 1, 1)
    return (imgs - m) / s, labels.cpu()[idx]


class DeviceImageDataset:
    """uint8 images [N, H, W, C] + int64 labels resident on ``device``; ``batch`` assembles
    normalised (optionally crop/flip-augmented) fp32 NCHW batches with one kernel."""

    def __init__(self, images_hwc_u8, labels, device, augment=False, pad=4, mean=CIFAR_MEAN, std=CIFAR_STD, seed=0):
        self.device = torch.device(device)
        self.data = torch.as_tensor(np.ascontiguousarray(images_hwc_u8)).to(self.device)
        self.labels = torch.as_tensor(np.asarray(labels, dtype=np.int64)).to(self.device)
        assert self.data.dtype == torch.uint8 and self.data.dim() == 4 and self.data.shape[-1] <= 3
        self.N, self.H, self.W, self.C = self.data.shape
        self.augment, self.pad, self.seed = augment, pad, seed
        self.mean, self.std = list(mean)[:self.C], list(std)[:self.C]
        self._native = None
        if self.device.type == "cuda":
            from .._ext import native

            self._native = native()

    @classmethod
    def cifar10(cls, root, train, device, augment=None, seed=0):
        data, targets = CIFAR10._load(root, train)
        return cls(data, targets, device, augment=train if augment is None else augment, seed=seed)

    def __len__(self):
        return self.N

    def batch(self, idx: torch.Tensor, epoch: int = 0, out=None):
        """idx: int64 dataset indices on the device -> (x [B, C, H, W] fp32, y [B] int64)."""
        B = idx.numel()
        if out is None:
            x = torch.empty(B, self.C, self.H, self.W, dtype=torch.float32, device=self.device)
            y = torch.empty(B, dtype=torch.int64, device=self.device)
        else:
            x, y = out
        if self._native is not None:
            self._native.image_batch(self.data, self.labels, idx, self.H, self.W, self.C, self.pad, self.augment,
                                     self.seed, epoch, self.mean, self.std, x, y)
        else:
            xr, yr = image_batch_reference(self.data, self.labels, idx, self.pad, self.augment, self.seed, epoch,
                                           self.mean, self.std)
            x.copy_(xr)
            y.copy_(yr)
        return x, y


class DeviceCachedDataset:
    """A deterministic map-style dataset (items: tensors, numbers or dicts of them) stacked once
    into device tensors; ``batch`` gathers by index (dict items come back as dicts)."""

    def __init__(self, dataset, device):
        self.device = torch.device(device)
        items = [dataset[i] for i in range(len(dataset))]
        if not items:
            raise ValueError("empty dataset")
        self.keys = list(items[0].keys()) if isinstance(items[0], dict) else None
        fields = self.keys if self.keys is not None else range(len(items[0]) if isinstance(items[0], (tuple, list))
                                                               else 1)

        def get(it, k):
            if self.keys is not None:
                return it[k]
            return it[k] if isinstance(it, (tuple, list)) else it

        self.fields = [torch.stack([torch.as_tensor(get(it, k)) for it in items]).to(self.device) for k in fields]
        self.N = len(items)

    def __len__(self):
        return self.N

    def batch(self, idx: torch.Tensor, epoch: int = 0, out=None):
        vals = [f.index_select(0, idx) for f in self.fields]
        if out is not None:
            for o, v in zip(out, vals):
                o.copy_(v)
            vals = list(out)
        if self.keys is not None:
            return dict(zip(self.keys, vals))
        return vals[0] if len(vals) == 1 else tuple(vals)


class DeviceBatches:
    """Batches of a device-resident dataset in ``sampler`` order (a DistributedSampler: this rank's
    shard, shuffled by seed + epoch), or in order without a sampler.  ``out``: fixed tensors every
    full batch is written into (for a captured training step)."""

    def __init__(self, dataset, batch_size, sampler=None, drop_last=False, out=None):
        self.ds, self.bs, self.sampler, self.drop_last, self.out = dataset, batch_size, sampler, drop_last, out

    def __len__(self):
        n = len(self.sampler) if self.sampler is not None else len(self.ds)
        return n // self.bs if self.drop_last else (n + self.bs - 1) // self.bs

    def __iter__(self):
        order = list(iter(self.sampler)) if self.sampler is not None else list(range(len(self.ds)))
        epoch = getattr(self.sampler, "epoch", 0)
        idx = torch.tensor(order, dtype=torch.int64).to(self.ds.device, non_blocking=True)
        n = idx.numel()
        for s in range(0, n, self.bs):
            e = min(n, s + self.bs)
            if e - s < self.bs and self.drop_last:
                break
            full = e - s == self.bs
            yield self.ds.batch(idx[s:e], epoch, out=self.out if (full and self.out is not None) else None)
