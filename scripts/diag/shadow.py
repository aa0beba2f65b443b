"""Op-level shadow check of one training step (deeplearning_mpi_amd/utils/shadow.py): every
backend call of the native engine repeated on the fp64 reference backend with the same inputs.

python scripts/diag/shadow.py --model unet|unet_bilinear|resnet18|resnet50 [--precision fp32|bf16] [--tol 1e-5]
"""
import argparse
import os
import sys

os.environ.setdefault("DLMPI_WGRAD_STREAM", "0")
os.environ.setdefault("DLMPI_BRANCH_STREAM", "0")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from deeplearning_mpi_amd.ops.backend import RefBackend  # noqa: E402
from deeplearning_mpi_amd.utils.shadow import ShadowBackend  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="unet")
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--tol", type=float, default=1e-5)
    a = ap.parse_args()
    from deeplearning_mpi_amd.models import UNet, resnet18, resnet50
    from deeplearning_mpi_amd.ops import bce_with_logits, cross_entropy

    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(5)
    torch.manual_seed(0)
    if a.model.startswith("unet"):
        m = UNet(out_classes=1, up_sample_mode="bilinear" if "bilinear" in a.model else "conv_transpose").to(dev)
        x = torch.randn(2, 3, 64, 64, device=dev, generator=g)
        y = (torch.rand(2, 64, 64, device=dev, generator=g) > 0.5).float()
        lossf = lambda o: bce_with_logits(o.squeeze(1), y)   # noqa: E731
    else:
        m = (resnet18 if a.model == "resnet18" else resnet50)(num_classes=10).to(dev)
        side = 32 if a.model == "resnet18" else 64
        x = torch.randn(16, 3, side, side, device=dev, generator=g)
        y = torch.randint(10, (16,), device=dev, generator=g)
        lossf = lambda o: cross_entropy(o, y)   # noqa: E731
    m.precision = a.precision
    m.train()
    m.engine_setup(dev)
    sh = ShadowBackend(m._be, RefBackend(dev, torch.float64), a.tol)
    m._be = sh
    lossf(m(x)).backward()
    torch.cuda.synchronize()
    print(f"{sh.calls} backend calls shadowed; {len(sh.records)} above tol {a.tol}")
    for op, e in sorted(sh.worst.items(), key=lambda t: -t[1]):
        print(f"  {op:20s} worst {e:.2e}")
    for r in sh.records:
        print(*r)


if __name__ == "__main__":
    main()
