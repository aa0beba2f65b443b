"""Per-shape A/B of the 256 x 128 halo conv tiles: conv_halo_pipe_kernel (double-buffered weight tile)
vs the single-stage conv_igemm_kernel halo mode, forward (+ BN statistics) and data gradient, on the
UNet 3x3 shapes with >= 256 output channels.  Interleaved rounds, CUDA events, min over rounds.

python benchmarks/halo_lab.py [--n 16] [--scale 1] [--iters 20] [--rounds 3]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

SHAPES = [  # H, Cin, Cout at 512^2 input (scale 2: 1024^2)
    (128, 128, 256), (128, 256, 256), (128, 768, 256),
    (64, 256, 512), (64, 512, 512), (64, 1536, 512),
    (32, 512, 1024), (32, 1024, 1024),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--scale", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    from deeplearning_mpi_amd.ops.act import Act
    from deeplearning_mpi_amd.ops.backend import NativeBackend

    be = NativeBackend("cuda")
    dev = "cuda"
    tot = {0: 0.0, 1: 0.0}
    for H0, Cin, K in SHAPES:
        H = H0 * a.scale
        N = a.n
        x = Act(torch.randn(N * H * H, Cin, device=dev).to(torch.bfloat16), N, H, H, Cin)
        w = (torch.randn(K, 3, 3, Cin, device=dev) * 0.02).to(torch.bfloat16)
        wT = w.permute(3, 1, 2, 0).contiguous()
        y = Act.empty(N, H, H, K, torch.bfloat16, dev)
        dy = Act(torch.randn(N * H * H, K, device=dev).to(torch.bfloat16), N, H, H, K)
        dx = Act.empty(N, H, H, Cin, torch.bfloat16, dev)
        st = torch.empty(be.conv_mtiles(N, H, H, Cin, K, 3, 3, 1, 1), 2, K, device=dev)
        fns = {"fwd": lambda: be.conv_fwd(x, w, K, 3, 3, 1, 1, y, stats=st),
               "dgrad": lambda: be.conv_dgrad(dy, wT, Cin, 3, 3, 1, 1, dx)}
        for ps, fn in fns.items():
            best = {0: 1e9, 1: 1e9}
            for r in range(a.rounds):
                for on in ((1, 0) if r % 2 == 0 else (0, 1)):
                    be.C.set_halo_pipe(on)
                    fn()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.iters):
                        fn()
                    e1.record()
                    e1.synchronize()
                    best[on] = min(best[on], e0.elapsed_time(e1) * 1000 / a.iters)
            flop = 2.0 * N * H * H * K * 9 * Cin
            halo = be.C.conv_halo_last()
            print(f"{N}x{H}^2 {Cin}->{K} {ps:5s} halo={halo} pipe {best[1]:8.1f} us ({flop / best[1] / 1e6:6.0f} TF/s)"
                  f"  single {best[0]:8.1f} us ({flop / best[0] / 1e6:6.0f} TF/s)  {best[1] / best[0]:.3f}", flush=True)
            tot[0] += best[0]
            tot[1] += best[1]
    be.C.set_halo_pipe(1)
    print(f"total pipe {tot[1]:.1f} us single {tot[0]:.1f} us ratio {tot[1] / tot[0]:.3f}")


if __name__ == "__main__":
    main()
