"""Run the production forward dispatch of a few ResNet-50 shapes (as benchmarks/conv_bench.py does)
10 times each, to be traced with rocprofv3 --kernel-trace: which kernel each one runs, and its time."""
import torch

from deeplearning_mpi_amd.ops.act import Act
from deeplearning_mpi_amd.ops.backend import NativeBackend

SHAPES = [(256, 14, 14, 256, 256, 3, 1, 1), (256, 7, 7, 2048, 512, 1, 1, 0), (256, 7, 7, 512, 512, 3, 1, 1)]


def main():
    be = NativeBackend(torch.device("cuda"))
    for N, H, W, C, K, R, s, p in SHAPES:
        P = (H + 2 * p - R) // s + 1
        x = Act(torch.randn(N * H * W, C, device="cuda").to(torch.bfloat16), N, H, W, C)
        w = (torch.randn(K, R, R, C, device="cuda") * 0.05).to(torch.bfloat16)
        y = Act.empty(N, P, P, K, torch.bfloat16, "cuda")
        st = torch.empty(be.conv_mtiles(N, H, W, C, K, R, R, s, p), 2, K, device="cuda")
        for _ in range(10):
            be.conv_fwd(x, w, K, R, R, s, p, y, stats=st)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
