"""Segmentation dataset (reference: pytorch/unet/data_loading.py) -- re-exported from the framework."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from deeplearning_mpi_amd.data.datasets import CarvanaDataset, SegmentationDataset as BasicDataset, load_image  # noqa: E402,F401

if __name__ == "__main__":
    ds = CarvanaDataset(images_dir=os.path.join("data", "images"), mask_dir=os.path.join("data", "masks"), scale=0.2)
    s = ds[0]
    print(len(ds), s["image"].shape, s["mask"].shape, ds.mask_values)
