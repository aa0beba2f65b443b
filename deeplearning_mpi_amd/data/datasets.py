"""Datasets: synthetic (benchmarks / tests), CIFAR-10 (no torchvision dependency) and the
image/mask segmentation dataset of the reference UNet.

* ``SyntheticImages`` / ``SyntheticMasks`` -- deterministic random data of a given shape; the
  benchmark path generates a batch directly on the GPU instead (``device_batch``).
* ``CIFAR10`` -- reads the official binary (``cifar-10-batches-bin``) or python
  (``cifar-10-batches-py``) releases from ``root``; the reference uses
  ``torchvision.datasets.CIFAR10(download=False)`` (/root/reference/pytorch/resnet/main.py:89-92).
  Transforms identical to the reference: RandomCrop(32, padding=4), RandomHorizontalFlip,
  ToTensor, Normalize((0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010)).
* ``SegmentationDataset`` (alias ``CarvanaDataset``) -- same semantics as
  /root/reference/pytorch/unet/data_loading.py:52-134: images/masks matched by stem, resized by
  ``scale`` (bicubic / nearest), HWC->CHW, /255 when >1, mask values mapped to indices and
  binarised (>0) to float32; returns ``{'image', 'mask'}``.
"""
from __future__ import annotations

import os
import pickle
from os import listdir
from os.path import isfile, join, splitext

import numpy as np
import torch
from torch.utils.data import Dataset

CIFAR_MEAN = (0.4914, 0.4822, 0.4465)
CIFAR_STD = (0.2023, 0.1994, 0.2010)


class SyntheticImages(Dataset):
    def __init__(self, n=1024, shape=(3, 224, 224), num_classes=1000, seed=0):
        self.n, self.shape, self.num_classes, self.seed = n, shape, num_classes, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1000003 + i)
        return torch.randn(self.shape, generator=g), int(torch.randint(self.num_classes, (1,), generator=g))


class SyntheticMasks(Dataset):
    def __init__(self, n=64, shape=(3, 512, 512), seed=0):
        self.n, self.shape, self.seed = n, shape, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1000003 + i)
        img = torch.rand(self.shape, generator=g)
        mask = (torch.rand(self.shape[1:], generator=g) > 0.5).float()
        return {"image": img, "mask": mask}


def device_batch(kind, batch, device, shape=(3, 224, 224), num_classes=1000, seed=0):
    """A synthetic batch generated directly on ``device`` (no host->device traffic)."""
    g = torch.Generator(device=device).manual_seed(seed)
    x = torch.randn((batch,) + tuple(shape), generator=g, device=device)
    if kind == "classification":
        y = torch.randint(num_classes, (batch,), generator=g, device=device)
    else:
        y = (torch.rand((batch,) + tuple(shape[1:]), generator=g, device=device) > 0.5).float()
    return x, y


# ----------------------------------------------------------------------------- CIFAR-10
class CifarTransform:
    """RandomCrop(32, 4) + RandomHorizontalFlip + ToTensor + Normalize (reference main.py:82-87)."""

    def __init__(self, train=True, mean=CIFAR_MEAN, std=CIFAR_STD):
        self.train = train
        self.mean = torch.tensor(mean).view(3, 1, 1)
        self.std = torch.tensor(std).view(3, 1, 1)

    def __call__(self, img_hwc_uint8: np.ndarray, rng: np.random.Generator):
        x = img_hwc_uint8
        if self.train:
            p = np.pad(x, ((4, 4), (4, 4), (0, 0)))
            i, j = rng.integers(0, 9, size=2)
            x = p[i:i + 32, j:j + 32]
            if rng.random() < 0.5:
                x = x[:, ::-1]
        t = torch.from_numpy(np.ascontiguousarray(x)).permute(2, 0, 1).float().div_(255.0)
        return (t - self.mean) / self.std


class CIFAR10(Dataset):
    def __init__(self, root, train=True, transform=None, seed=0):
        self.root = root
        self.train = train
        self.transform = transform
        self.data, self.targets = self._load(root, train)
        self._rng = np.random.default_rng(seed)

    @staticmethod
    def _load(root, train):
        binp = join(root, "cifar-10-batches-bin")
        pyp = join(root, "cifar-10-batches-py")
        if os.path.isdir(binp):
            files = [f"data_batch_{i}.bin" for i in range(1, 6)] if train else ["test_batch.bin"]
            raw = np.concatenate([np.fromfile(join(binp, f), dtype=np.uint8).reshape(-1, 3073) for f in files])
            labels = raw[:, 0].astype(np.int64)
            data = raw[:, 1:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1)
            return np.ascontiguousarray(data), labels
        if os.path.isdir(pyp):
            files = [f"data_batch_{i}" for i in range(1, 6)] if train else ["test_batch"]
            datas, labels = [], []
            for f in files:   # user-provided dataset files (the standard CIFAR python release)
                with open(join(pyp, f), "rb") as fh:
                    d = pickle.load(fh, encoding="latin1")
                datas.append(np.asarray(d["data"], dtype=np.uint8).reshape(-1, 3, 32, 32))
                labels.extend(d["labels"] if "labels" in d else d["fine_labels"])
            data = np.concatenate(datas).transpose(0, 2, 3, 1)
            return np.ascontiguousarray(data), np.asarray(labels, dtype=np.int64)
        raise FileNotFoundError(f"CIFAR-10 not found under {root} (expected cifar-10-batches-bin or -py)")

    def __len__(self):
        return len(self.targets)

    def __getitem__(self, i):
        img = self.data[i]
        if self.transform is not None:
            x = self.transform(img, self._rng)
        else:
            x = torch.from_numpy(img).permute(2, 0, 1).float().div_(255.0)
        return x, int(self.targets[i])


# ----------------------------------------------------------------------------- segmentation
def load_image(filename):
    from PIL import Image

    ext = splitext(filename)[1]
    if ext == ".npy":
        return Image.fromarray(np.load(filename))   # allow_pickle=False (numpy default)
    if ext in (".pt", ".pth"):
        return Image.fromarray(torch.load(filename, weights_only=True).numpy())
    return Image.open(filename)


class SegmentationDataset(Dataset):
    def __init__(self, images_dir, mask_dir, scale=1.0, mask_suffix=""):
        from pathlib import Path

        assert 0 < scale <= 1, "Scale must be between 0 and 1"
        self.images_dir, self.mask_dir = Path(images_dir), Path(mask_dir)
        self.scale, self.mask_suffix = scale, mask_suffix
        self.ids = [splitext(f)[0] for f in listdir(images_dir) if isfile(join(images_dir, f)) and not f.startswith(".")]
        if not self.ids:
            raise RuntimeError(f"No input file found in {images_dir}, make sure you put your images there")
        uniq = [self._unique(i) for i in self.ids]
        self.mask_values = list(sorted(np.unique(np.concatenate(uniq), axis=0).tolist()))

    def _mask_file(self, idx):
        files = list(self.mask_dir.glob(idx + self.mask_suffix + ".*"))
        if not files:
            raise FileNotFoundError(f"No mask file found for index '{idx}' with suffix '{self.mask_suffix}' "
                                    f"in directory '{self.mask_dir}'")
        return files[0]

    def _unique(self, idx):
        mask = np.asarray(load_image(self._mask_file(idx)))
        if mask.ndim == 2:
            return np.unique(mask)
        if mask.ndim == 3:
            return np.unique(mask.reshape(-1, mask.shape[-1]), axis=0)
        raise ValueError(f"Loaded masks should have 2 or 3 dimensions, found {mask.ndim}")

    def __len__(self):
        return len(self.ids)

    @staticmethod
    def preprocess(mask_values, pil_img, scale, is_mask):
        from PIL import Image

        w, h = pil_img.size
        nw, nh = int(scale * w), int(scale * h)
        assert nw > 0 and nh > 0, "Scale is too small, resized images would have no pixel"
        pil_img = pil_img.resize((nw, nh), resample=Image.NEAREST if is_mask else Image.BICUBIC)
        img = np.asarray(pil_img)
        if is_mask:
            mask = np.zeros((nh, nw), dtype=np.int64)
            for i, v in enumerate(mask_values):
                if img.ndim == 2:
                    mask[img == v] = i
                else:
                    mask[(img == v).all(-1)] = i
            return mask
        img = img[np.newaxis, ...] if img.ndim == 2 else img.transpose((2, 0, 1))
        if (img > 1).any():
            img = img / 255.0
        return img

    def __getitem__(self, idx):
        name = self.ids[idx]
        mask_file = list(self.mask_dir.glob(name + self.mask_suffix + ".*"))
        img_file = list(self.images_dir.glob(name + ".*"))
        assert len(img_file) == 1, f"Either no image or multiple images found for the ID {name}: {img_file}"
        assert len(mask_file) == 1, f"Either no mask or multiple masks found for the ID {name}: {mask_file}"
        mask = load_image(mask_file[0])
        img = load_image(img_file[0])
        assert img.size == mask.size, f"Image and mask {name} should be the same size"
        img = self.preprocess(self.mask_values, img, self.scale, is_mask=False)
        mask = self.preprocess(self.mask_values, mask, self.scale, is_mask=True)
        return {"image": torch.as_tensor(img.copy()).float().contiguous(),
                "mask": torch.as_tensor((mask > 0).astype(np.float32)).float().contiguous()}


class CarvanaDataset(SegmentationDataset):
    def __init__(self, images_dir, mask_dir, scale=1):
        super().__init__(images_dir, mask_dir, scale, mask_suffix="")
