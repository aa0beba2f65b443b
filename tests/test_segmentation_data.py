"""Segmentation dataset outputs pinned against a fixture (tests/fixtures/segmentation_expected.pt,
written by the round-1 implementation, whose outputs matched the reference's BasicDataset
semantics, /root/reference/pytorch/unet/data_loading.py:52-134) on a generated file set: RGB PNG
images with 3-level grayscale PNG masks and a mask suffix (scale 1.0 and 0.5), and float32 .npy
images with RGB .npy colour masks (scale 0.75)."""
import os

import numpy as np
import pytest
import torch

from deeplearning_mpi_amd.data.datasets import CarvanaDataset, SegmentationDataset

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "segmentation_expected.pt")


def _make(root):
    from PIL import Image

    g = np.random.default_rng(7)
    os.makedirs(f"{root}/a/img")
    os.makedirs(f"{root}/a/mask")
    for i in range(4):
        Image.fromarray(g.integers(0, 256, (30, 40, 3), dtype=np.uint8)).save(f"{root}/a/img/s{i}.png")
        Image.fromarray((g.integers(0, 3, (30, 40)) * 127).astype(np.uint8)).save(f"{root}/a/mask/s{i}_mask.png")
    os.makedirs(f"{root}/b/img")
    os.makedirs(f"{root}/b/mask")
    for i in range(3):
        np.save(f"{root}/b/img/t{i}.npy", g.random((24, 32)).astype(np.float32))
        cols = np.array([[0, 0, 0], [255, 0, 0], [0, 255, 0]], dtype=np.uint8)
        np.save(f"{root}/b/mask/t{i}.npy", cols[g.integers(0, 3, (24, 32))])


@pytest.mark.parametrize("cache", [False, True])
def test_segmentation_outputs_match_fixture(tmp_path, cache):
    pytest.importorskip("PIL")
    _make(tmp_path)
    want = torch.load(FIX, weights_only=True)
    for name, d, sfx, sc in (("a10", "a", "_mask", 1.0), ("a05", "a", "_mask", 0.5), ("b075", "b", "", 0.75)):
        ds = SegmentationDataset(tmp_path / d / "img", tmp_path / d / "mask", sc, mask_suffix=sfx, cache=cache)
        assert torch.equal(torch.tensor(ds.mask_values), want[f"{name}/mask_values"])
        for i, k in enumerate(ds.ids):
            for _ in range(2 if cache else 1):
                s = ds[i]
                assert s["image"].dtype == torch.float32 and s["mask"].dtype == torch.float32
                assert torch.equal(s["image"], want[f"{name}/{k}/image"]), (name, k)
                assert torch.equal(s["mask"], want[f"{name}/{k}/mask"]), (name, k)


def test_segmentation_rejects_bad_sets(tmp_path):
    pytest.importorskip("PIL")
    _make(tmp_path)
    with pytest.raises(ValueError):
        SegmentationDataset(tmp_path / "a" / "img", tmp_path / "a" / "mask", 0.0)
    with pytest.raises(RuntimeError, match="mask"):
        CarvanaDataset(tmp_path / "a" / "img", tmp_path / "a" / "mask")   # masks carry a suffix
    os.remove(tmp_path / "b" / "mask" / "t1.npy")
    with pytest.raises(RuntimeError, match="t1"):
        SegmentationDataset(tmp_path / "b" / "img", tmp_path / "b" / "mask")
