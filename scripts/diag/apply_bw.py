"""Bandwidth of the BN-apply pass (the ResNet-50 layer-1 output apply: 802,816 rows x 256 channels,
bf16, residual, ReLU, mask bits) against the relative placement of its three streams (z, residual,
y), plus a plain device copy of the same bytes as the reference.  Each tensor is a slice of a
private buffer at a chosen byte offset past its 2 MB-aligned start.

usage: python scripts/diag/apply_bw.py
"""
import torch

from deeplearning_mpi_amd.ops.act import Act
from deeplearning_mpi_amd.ops.backend import NativeBackend

DEV = "cuda"
M, C = 802816, 256


def sliced(off_bytes):
    n = M * C
    extra = off_bytes // 2
    buf = torch.empty(n + extra + 4096, dtype=torch.bfloat16, device=DEV)
    return buf, buf[extra:extra + n].view(M, C)


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
    sc = torch.rand(C, device=DEV) + 0.5
    sh = torch.randn(C, device=DEV) * 0.1
    nbytes = 3 * M * C * 2 + M * C // 8
    for oz, orr, oy in [(0, 0, 0), (0, 4096, 8192), (0, 65536, 131072), (0, 1 << 20, 1 << 21 | 4096),
                        (0, 2048, 4096), (0, 256, 512), (0, 12288, 24576)]:
        _, z = sliced(oz)
        _, r = sliced(orr)
        _, y = sliced(oy)
        z.normal_()
        r.normal_()
        mb = torch.empty(M, C // 8, dtype=torch.uint8, device=DEV)
        za, ra, ya = Act(z, M, 1, 1, C), Act(r, M, 1, 1, C), Act(y, M, 1, 1, C)
        us = timeit(lambda: be.bn_apply(za, sc, sh, ra, True, ya, mbits=mb))
        print(f"offsets z {oz:>8} res {orr:>8} y {oy:>8}: {us:7.1f} us  {nbytes / us / 1e6:5.2f} TB/s", flush=True)
    _, a = sliced(0)
    _, b = sliced(4096)
    us = timeit(lambda: b.copy_(a))
    print(f"torch copy (read + write {2 * M * C * 2 / 1e6:.0f} MB): {us:7.1f} us  {2 * M * C * 2 / us / 1e6:5.2f} TB/s")


if __name__ == "__main__":
    main()
