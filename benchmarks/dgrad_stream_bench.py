"""Time the ResNet-50 (bs 256) 1x1 data gradients with the fused BN-backward epilogue through the
streaming kernel (conv1x1_dgrad_stream.hip) and through the general implicit-GEMM kernel.

python benchmarks/dgrad_stream_bench.py [--iters 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

CASES = [
    # name, N, H, W, K (A channels), C (dx channels), residual, mask mode, bias
    ("layer1 conv1 dual (2x64 -> 256)", 256, 56, 56, 128, 256, True, "bits", True),
    ("layer1.1 conv1 dual + z2 (2x64 -> 256)", 256, 56, 56, 128, 256, True, "bits_z2", True),
    ("layer2.0 conv1 dual (2x128 -> 256)", 256, 56, 56, 256, 256, True, "bits", True),
    ("layer2 conv1 dual (2x128 -> 512)", 256, 28, 28, 256, 512, True, "bits", True),
    ("layer3 conv1 (256 -> 1024)", 256, 14, 14, 256, 1024, True, "bits", False),
    ("layer3.0 conv1 dual (2x256 -> 512)", 256, 28, 28, 512, 512, True, "bits", True),
    ("layer4 conv1 (512 -> 2048)", 256, 7, 7, 512, 2048, True, "bits", False),
    ("layer1 conv1 no-res (2x64 -> 256), z-mask", 256, 56, 56, 128, 256, False, "z", True),
    ("layer1 conv3 dual (2x256 -> 64), z-mask", 256, 56, 56, 512, 64, False, "z", True),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from deeplearning_mpi_amd.models.engine import BwdFuse
    from deeplearning_mpi_amd.ops.act import Act
    from deeplearning_mpi_amd.ops.backend import NativeBackend

    nb = NativeBackend("cuda")
    dev = "cuda"
    for name, N, H, W, K, C, has_res, mm, has_bias in CASES:
        rows = N * H * W
        dy = Act(torch.randn(rows, K, device=dev).to(torch.bfloat16), N, H, W, K)
        wT = (torch.randn(C, 1, 1, K, device=dev) / K ** 0.5).to(torch.bfloat16)
        res = Act(torch.randn(rows, C, device=dev).to(torch.bfloat16), N, H, W, C) if has_res else None
        z = Act(torch.randn(rows, C, device=dev).to(torch.bfloat16), N, H, W, C)
        bias = torch.randn(C, device=dev) if has_bias else None
        if mm.startswith("bits"):
            mb = torch.randint(0, 256, (rows, C // 8), device=dev, dtype=torch.uint8)
            z2 = Act(torch.randn(rows, C, device=dev).to(torch.bfloat16), N, H, W, C) if mm == "bits_z2" else None
            fuse = BwdFuse(None, z, z2, mbits=mb)
            mbytes = mb.numel() + (rows * C * 2 if z2 is not None else 0)
        else:
            fuse = BwdFuse(None, z, None, torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev))
            mbytes = 0
        dx = Act.empty(N, H, W, C, torch.bfloat16, dev)
        byts = rows * 2 * (K + C * (2 + (1 if has_res else 0))) + mbytes
        out = []
        for on in (0, 1, 0, 1):
            nb.C.set_dgrad_stream(on)
            fn = lambda: nb.conv_dgrad(dy, wT, C, 1, 1, 1, 0, dx, res=res, fuse=fuse, bias=bias)  # noqa: E731
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(a.iters):
                fn()
            ev[1].record()
            torch.cuda.synchronize()
            t = ev[0].elapsed_time(ev[1]) / a.iters * 1e-3
            out.append((on, nb.C.dgrad_stream_last(), t))
        nb.C.set_dgrad_stream(-1)
        gen = min(t for on, _, t in out if on == 0)
        st = min(t for on, _, t in out if on == 1)
        ran = [r for on, r, _ in out if on == 1][0]
        print(f"{name:44s} general {gen * 1e6:7.1f} us ({byts / gen / 1e12:4.2f} TB/s)  "
              f"stream {st * 1e6:7.1f} us ({byts / st / 1e12:4.2f} TB/s) ran={ran}  x{gen / st:4.2f}", flush=True)


if __name__ == "__main__":
    main()
