"""ONE 1x1 data gradient with the fused BN-backward epilogue, repeated (for rocprofv3 counters):
ResNet-50 layer-1 conv1, dual operand [dy | z] (2 x 64) -> 256 channels at 56^2, bs 256, + residual
gradient + mask bits + BN partials.  --stream 1: the streaming kernel, 0: the general kernel.

python benchmarks/dgrad_one.py --stream 1 [--iters 5]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stream", type=int, default=1)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    from deeplearning_mpi_amd.models.engine import BwdFuse
    from deeplearning_mpi_amd.ops.act import Act
    from deeplearning_mpi_amd.ops.backend import NativeBackend

    nb = NativeBackend("cuda")
    dev = "cuda"
    N, H, W, K, C = 256, 56, 56, 128, 256
    rows = N * H * W
    dy = Act(torch.randn(rows, K, device=dev).to(torch.bfloat16), N, H, W, K)
    wT = (torch.randn(C, 1, 1, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    res = Act(torch.randn(rows, C, device=dev).to(torch.bfloat16), N, H, W, C)
    z = Act(torch.randn(rows, C, device=dev).to(torch.bfloat16), N, H, W, C)
    mb = torch.randint(0, 256, (rows, C // 8), device=dev, dtype=torch.uint8)
    bias = torch.randn(C, device=dev)
    dx = Act.empty(N, H, W, C, torch.bfloat16, dev)
    nb.C.set_dgrad_stream(a.stream)
    for _ in range(a.iters):
        nb.conv_dgrad(dy, wT, C, 1, 1, 1, 0, dx, res=res, fuse=BwdFuse(None, z, None, mbits=mb), bias=bias)
    torch.cuda.synchronize()
    print("ran stream" if nb.C.dgrad_stream_last() else "ran general", flush=True)


if __name__ == "__main__":
    main()
