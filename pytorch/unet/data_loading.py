"""Segmentation dataset (reference: pytorch/unet/data_loading.py) -- re-exported from the framework."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from deeplearning_mpi_amd.data.datasets import CarvanaDataset, SegmentationDataset as BasicDataset, load_image  # noqa: E402,F401

if __name__ == "__main__":
    # Manual data check (reference data_loading.py:137-180 plots the first pair with matplotlib,
    # which this image does not ship): print the dataset summary and write image | mask side by
    # side to data_check.png with PIL.
    import numpy as np
    from PIL import Image

    ds = CarvanaDataset(images_dir=os.path.join("data", "images"), mask_dir=os.path.join("data", "masks"), scale=0.2)
    s = ds[0]
    print(len(ds), s["image"].shape, s["mask"].shape, ds.mask_values)
    img = (s["image"].permute(1, 2, 0).numpy() * 255).clip(0, 255).astype(np.uint8)
    if img.shape[2] == 1:
        img = np.repeat(img, 3, axis=2)
    msk = np.repeat((s["mask"].numpy() * 255).astype(np.uint8)[..., None], 3, axis=2)
    Image.fromarray(np.concatenate([img, msk], axis=1)).save("data_check.png")
    print("wrote data_check.png")
