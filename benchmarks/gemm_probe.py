"""Probe: hipBLASLt (via torch.mm / torch.matmul with bf16 inputs) on the plain GEMMs of 1x1
stride-1 weight gradients (dW[Ko][C] = dY^T X over N*H*W pixels), vs our split-K wgrad kernel."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def t(fn, iters=20):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(iters):
        fn()
    e[1].record()
    torch.cuda.synchronize()
    return e[0].elapsed_time(e[1]) / iters * 1e3


def main():
    from deeplearning_mpi_amd.ops.act import Act
    from deeplearning_mpi_amd.ops.backend import NativeBackend

    be = NativeBackend("cuda")
    shapes = [(256, 14, 256, 1024), (256, 14, 1024, 256), (256, 28, 512, 128), (256, 28, 128, 512),
              (256, 7, 512, 2048), (256, 7, 2048, 512), (256, 56, 64, 256), (256, 56, 256, 64),
              (256, 56, 256, 128), (256, 28, 512, 256), (256, 14, 1024, 512), (256, 56, 64, 64)]
    for N, H, C, K in shapes:
        M = N * H * H
        x = torch.randn(M, C, device="cuda").to(torch.bfloat16)
        dy = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        g = torch.zeros(K * C, device="cuda")
        xa, dya = Act(x, N, H, H, C), Act(dy, N, H, H, K)
        ours = t(lambda: be.conv_wgrad(dya, xa, 1, 1, 1, 0, g, C, K))
        mm = t(lambda: torch.mm(dy.t(), x))
        mmf = t(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32)) if hasattr(torch.mm, "__call__") else float("nan")
        fl = 2.0 * M * C * K
        print(f"M={M:7d} C={C:5d} K={K:5d}: ours {ours:7.1f} us ({fl / ours / 1e6:6.0f} TF)  "
              f"torch.mm bf16 {mm:7.1f} us ({fl / mm / 1e6:6.0f} TF)  out fp32 {mmf:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
