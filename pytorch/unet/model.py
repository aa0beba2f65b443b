"""UNet model (reference: pytorch/unet/model.py) -- re-exported from the framework; running this
file does the reference's shape smoke test (model.py:84-89)."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from deeplearning_mpi_amd.models.unet import DoubleConv, DownBlock, UNet, UpBlock  # noqa: E402,F401

if __name__ == "__main__":
    import torch

    model = UNet(out_classes=2, up_sample_mode="conv_transpose")
    print(model)
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    model = model.to(dev).eval()
    with torch.no_grad():
        y = model(torch.randn(1, 3, 512, 512, device=dev))
    print(y.shape)
