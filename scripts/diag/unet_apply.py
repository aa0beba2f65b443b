"""BN-apply pass bandwidth on the UNet-512 shapes (bs 16: 512^2 x 64, 256^2 x 128, 128^2 x 256) vs the
ResNet-50 layer-1 shape, in isolation: contiguous output and the cat-slice output (ld 192 / 384 / 768).

usage: python scripts/diag/unet_apply.py
"""
import torch

from deeplearning_mpi_amd.ops.act import Act
from deeplearning_mpi_amd.ops.backend import NativeBackend

DEV = "cuda"


def timeit(f, it=20):
    f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1000.0   # us


def main():
    be = NativeBackend(torch.device(DEV))
    for M, C, ldy in [(16 * 512 * 512, 64, 64), (16 * 512 * 512, 64, 192), (16 * 256 * 256, 128, 128),
                      (16 * 256 * 256, 128, 384), (16 * 128 * 128, 256, 256), (256 * 56 * 56, 64, 64)]:
        z = torch.randn(M, C, device=DEV).to(torch.bfloat16)
        yb = torch.empty(M, ldy, device=DEV, dtype=torch.bfloat16)
        sc = torch.rand(C, device=DEV) + 0.5
        sh = torch.randn(C, device=DEV) * 0.1
        mb = torch.empty(M, C // 8, dtype=torch.uint8, device=DEV)
        za = Act(z, M, 1, 1, C)
        ya = Act(yb, M, 1, 1, ldy).slice(ldy - C, C)
        us = timeit(lambda: be.bn_apply(za, sc, sh, None, True, ya, mbits=mb))
        nbytes = 2 * M * C * 2 + M * C // 8
        print(f"M {M:>9} C {C:>4} ldy {ldy:>4}: {us:7.1f} us  {nbytes / us / 1e6:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
