"""Datasets: synthetic (benchmarks / tests), CIFAR-10 (no torchvision dependency) and the
image/mask segmentation dataset of the reference UNet.

* ``SyntheticImages`` / ``SyntheticMasks`` -- deterministic random data of a given shape; the
  benchmark path generates a batch directly on the GPU instead (``device_batch``).
* ``CIFAR10`` -- reads the official binary (``cifar-10-batches-bin``) or python
  (``cifar-10-batches-py``) releases from ``root``; the reference uses
  ``torchvision.datasets.CIFAR10(download=False)`` (/root/reference/pytorch/resnet/main.py:89-92).
  Transforms identical to the reference: RandomCrop(32, padding=4), RandomHorizontalFlip,
  ToTensor, Normalize((0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010)).
* ``SegmentationDataset`` (alias ``CarvanaDataset``) -- the training targets of
  /root/reference/pytorch/unet/data_loading.py:52-134 (see the class docstring for how they are
  produced here); returns ``{'image', 'mask'}``.
"""
from __future__ import annotations

import os
import pickle
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


_M64 = (1 << 64) - 1


class SampleRng:
    """Counter-based random stream of ONE sample: splitmix64 over (seed, epoch, index).

    The augmentation of sample ``i`` in epoch ``e`` is a pure function of (seed, e, i): it does not
    depend on which DataLoader worker or rank loads the sample, on how many samples that worker
    loaded before, or on whether the run was interrupted and resumed -- so ``--resume`` continues
    with exactly the crops and flips an uninterrupted run would have drawn,
    with no generator state to checkpoint.  Offers the two ``np.random.Generator`` calls the
    transforms use."""

    __slots__ = ("_s",)

    def __init__(self, seed: int, epoch: int, index: int):
        self._s = ((seed & 0xFFFFFFFF) * 0x9E3779B97F4A7C15 ^ (epoch & 0xFFFFFFFF) * 0xC2B2AE3D27D4EB4F
                   ^ (index & 0xFFFFFFFFFFFF) * 0x165667B19E3779F9) & _M64

    def _next(self) -> int:
        self._s = (self._s + 0x9E3779B97F4A7C15) & _M64
        z = self._s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
        return z ^ (z >> 31)

    def integers(self, low, high, size=None):
        span = int(high) - int(low)
        if size is None:
            return int(low) + self._next() % span
        return np.array([int(low) + self._next() % span for _ in range(int(np.prod(size)))]).reshape(size)

    def random(self) -> float:
        return (self._next() >> 11) * (1.0 / (1 << 53))


class CIFAR10(Dataset):
    """CIFAR-10 from the official binary / python releases.  Augmentation randomness comes from
    :class:`SampleRng` keyed by (``seed``, epoch, index); call :meth:`set_epoch` every epoch (the
    apps do it next to ``DistributedSampler.set_epoch``; DataLoader workers must not be persistent,
    so each epoch's workers start from the updated dataset object)."""

    def __init__(self, root, train=True, transform=None, seed=0):
        self.root = root
        self.train = train
        self.transform = transform
        self.data, self.targets = self._load(root, train)
        self.seed = int(seed)
        self.epoch = 0

    def set_epoch(self, epoch: int):
        self.epoch = int(epoch)

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
            x = self.transform(img, SampleRng(self.seed, self.epoch, i))
        else:
            x = torch.from_numpy(img).permute(2, 0, 1).float().div_(255.0)
        return x, int(self.targets[i])


# ----------------------------------------------------------------------------- segmentation
_ARRAY_EXT = {".npy", ".pt", ".pth"}


def read_array(path) -> np.ndarray:
    """Decode one image or mask file to a numpy array (HW or HWC).  ``.npy`` through numpy without
    pickles, ``.pt``/``.pth`` as a weights-only tensor, anything else through PIL."""
    ext = os.path.splitext(str(path))[1].lower()
    if ext == ".npy":
        return np.load(path)
    if ext in (".pt", ".pth"):
        return torch.load(path, weights_only=True).numpy()
    from PIL import Image

    with Image.open(path) as im:
        return np.asarray(im)


def load_image(filename):
    """PIL view of :func:`read_array` (API of the reference's helper, data_loading.py:20-27)."""
    from PIL import Image

    return Image.fromarray(read_array(filename))


def _resized(arr: np.ndarray, scale: float, nearest: bool) -> np.ndarray:
    h, w = arr.shape[:2]
    size = (int(scale * w), int(scale * h))
    if size[0] <= 0 or size[1] <= 0:
        raise ValueError(f"scale {scale} leaves no pixel of a {w}x{h} image")
    if size == (w, h):
        return arr
    from PIL import Image

    mode = Image.NEAREST if nearest else Image.BICUBIC
    return np.asarray(Image.fromarray(arr).resize(size, resample=mode))


def _row_keys(arr: np.ndarray) -> np.ndarray:
    """One sortable integer key per pixel: the value itself for single-channel masks, the channel
    tuple packed into an unsigned integer (lexicographic order preserved) otherwise."""
    if arr.ndim <= 2:
        return arr.reshape(-1)
    flat = np.ascontiguousarray(arr.reshape(-1, arr.shape[-1]))
    if flat.dtype.kind in "ui" and flat.dtype.itemsize <= 2 and flat.shape[1] * 16 <= 64:
        bits = 8 * flat.dtype.itemsize
        u = flat.astype(np.int64) - (np.iinfo(flat.dtype).min if flat.dtype.kind == "i" else 0)
        key = np.zeros(len(flat), dtype=np.uint64)
        for c in range(flat.shape[1]):
            key = (key << np.uint64(bits)) | u[:, c].astype(np.uint64)
        return key
    # generic fallback: a structured view sorts lexicographically as well
    return flat.view([("", flat.dtype)] * flat.shape[1]).reshape(-1)


class SegmentationDataset(Dataset):
    """Image / mask pairs for the UNet trainer (semantics of the reference's ``BasicDataset``,
    /root/reference/pytorch/unet/data_loading.py:52-134; re-implemented, not transcribed):

    * the sample list is built ONCE by pairing ``images_dir/<id>.*`` with
      ``mask_dir/<id><mask_suffix>.*`` (duplicate or missing files are rejected up front, not on
      every ``__getitem__``);
    * the table of distinct mask values (pixel values, or channel tuples of colour masks) is found
      by a thread-parallel scan of the masks;
    * a mask is mapped to class indices by one vectorised ``searchsorted`` into that table (no loop
      over the values), then binarised (index > 0) to float32 -- the reference's training target;
    * images are resized by ``scale`` (bicubic; nearest for masks), laid out CHW, divided by 255
      when any value exceeds 1, float32;
    * ``cache=True`` decodes each sample once and keeps the tensors (the device-resident variant is
      ``data.DeviceCachedDataset``).

    Returns ``{'image': float32 [C, H, W], 'mask': float32 [H, W]}``."""

    def __init__(self, images_dir, mask_dir, scale=1.0, mask_suffix="", cache=False, workers=None):
        if not 0 < scale <= 1:
            raise ValueError(f"scale must be in (0, 1], got {scale}")
        self.images_dir, self.mask_dir = str(images_dir), str(mask_dir)
        self.scale, self.mask_suffix = float(scale), mask_suffix
        self._pairs = self._pair_files()
        self.ids = [k for k, _, _ in self._pairs]
        self._table = self._value_table(workers)
        self._cache = {} if cache else None

    # ------------------------------------------------------------------ indexing
    def _pair_files(self):
        def by_stem(d, suffix):
            out = {}
            for f in sorted(os.listdir(d)):
                full = join(d, f)
                if f.startswith(".") or not isfile(full):
                    continue
                stem = splitext(f)[0]
                if suffix:
                    if not stem.endswith(suffix):
                        continue
                    stem = stem[: -len(suffix)]
                out.setdefault(stem, []).append(full)
            return out

        imgs = by_stem(self.images_dir, "")
        if not imgs:
            raise RuntimeError(f"{self.images_dir} holds no image files")
        masks = by_stem(self.mask_dir, self.mask_suffix)
        pairs = []
        for stem in sorted(imgs):
            if len(imgs[stem]) != 1:
                raise RuntimeError(f"sample {stem!r}: expected one image file, got {imgs[stem]}")
            m = masks.get(stem, [])
            if len(m) != 1:
                raise RuntimeError(f"sample {stem!r}: expected one mask file '{stem}{self.mask_suffix}.*' in "
                                   f"{self.mask_dir}, got {m}")
            pairs.append((stem, imgs[stem][0], m[0]))
        return pairs

    def _value_table(self, workers):
        from concurrent.futures import ThreadPoolExecutor

        def distinct(path):
            a = read_array(path)
            if a.ndim not in (2, 3):
                raise ValueError(f"mask {path}: expected a 2-D or 3-D array, got {a.ndim}-D")
            return a.ndim, (np.unique(a) if a.ndim == 2 else np.unique(a.reshape(-1, a.shape[-1]), axis=0))

        n = workers or min(16, os.cpu_count() or 1, len(self._pairs))
        with ThreadPoolExecutor(max_workers=max(1, n)) as ex:
            found = list(ex.map(distinct, [m for _, _, m in self._pairs]))
        ndims = {d for d, _ in found}
        if len(ndims) != 1:
            raise ValueError("masks mix single-channel and multi-channel files")
        vals = np.unique(np.concatenate([u for _, u in found]), axis=0)   # sorted (lexicographic rows)
        self.mask_values = vals.tolist()
        return np.sort(_row_keys(vals if vals.ndim == 1 else vals[None]))

    # ------------------------------------------------------------------ samples
    def mask_indices(self, mask: np.ndarray) -> np.ndarray:
        """Class index of every pixel (its value's rank in the table); int64 [H, W]."""
        keys = _row_keys(mask)
        idx = np.searchsorted(self._table, keys)
        idx = np.minimum(idx, len(self._table) - 1)
        idx = np.where(self._table[idx] == keys, idx, 0)   # values outside the table -> class 0
        return idx.astype(np.int64).reshape(mask.shape[:2])

    def load(self, i):
        stem, ipath, mpath = self._pairs[i]
        img, mask = read_array(ipath), read_array(mpath)
        if img.shape[:2] != mask.shape[:2]:
            raise ValueError(f"sample {stem!r}: image {img.shape[:2]} and mask {mask.shape[:2]} differ in size")
        img = _resized(img, self.scale, nearest=False)
        mask = _resized(mask, self.scale, nearest=True)
        chw = np.ascontiguousarray(img[None] if img.ndim == 2 else np.moveaxis(img, -1, 0))
        if bool((chw > 1).any()):
            chw = chw / 255.0
        image = torch.tensor(chw).float()
        target = torch.from_numpy(self.mask_indices(mask) > 0).float()
        return {"image": image.contiguous(), "mask": target.contiguous()}

    def __len__(self):
        return len(self._pairs)

    def __getitem__(self, i):
        if self._cache is None:
            return self.load(i)
        if i not in self._cache:
            self._cache[i] = self.load(i)
        return self._cache[i]


class CarvanaDataset(SegmentationDataset):
    """Name kept for the reference's entry points (data_loading.py:132-134): no mask suffix."""

    def __init__(self, images_dir, mask_dir, scale=1.0, **kw):
        super().__init__(images_dir, mask_dir, scale, mask_suffix="", **kw)
