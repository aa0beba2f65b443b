"""Per-shape A/B of the 256 x 128 halo conv tiles: conv_halo_pipe_kernel (double-buffered weight tile)
vs the single-stage conv_igemm_kernel halo mode, forward (+ BN statistics) and data gradient, on the
UNet 3x3 shapes with >= 256 output channels.  Interleaved rounds, CUDA events, min over rounds.

python benchmarks/halo_lab.py [--n 16] [--scale 1] [--iters 20] [--rounds 3]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

SHAPES = [  # H, Cin, Cout at 512^2 input (scale 2: 1024^2); 256 x 128 halo tiles
    (128, 128, 256), (128, 256, 256), (128, 768, 256),
    (64, 256, 512), (64, 512, 512), (64, 1536, 512),
    (32, 512, 1024), (32, 1024, 1024),
]
SHAPES_SMALL = [  # 128 x 128 (128-channel outputs) and 256 x 64 (64-channel) halo tiles
    (256, 64, 128), (256, 128, 128), (256, 384, 128), (512, 192, 64),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--scale", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--modes", default="1,0", help="set_halo_pipe values to compare (first = the candidate)")
    ap.add_argument("--small", type=int, default=0, help="1: the 128 x 128 / 256 x 64 halo shapes instead")
    a = ap.parse_args()
    modes = [int(v) for v in a.modes.split(",")]
    from deeplearning_mpi_amd.ops.act import Act
    from deeplearning_mpi_amd.ops.backend import NativeBackend

    be = NativeBackend("cuda")
    dev = "cuda"
    tot = {m: 0.0 for m in modes}
    for H0, Cin, K in (SHAPES_SMALL if a.small else SHAPES):
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
            best = {m: 1e9 for m in modes}
            for r in range(a.rounds):
                for on in (modes if r % 2 == 0 else modes[::-1]):
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
            cols = "  ".join(f"mode {m}: {best[m]:8.1f} us ({flop / best[m] / 1e6:5.0f} TF/s)" for m in modes)
            print(f"{N}x{H}^2 {Cin}->{K} {ps:5s} halo={halo}  {cols}  {best[modes[0]] / best[modes[-1]]:.3f}", flush=True)
            for m in modes:
                tot[m] += best[m]
    be.C.set_halo_pipe(1)
    print("total " + "  ".join(f"mode {m}: {tot[m]:.1f} us" for m in modes) +
          f"  ratio {tot[modes[0]] / tot[modes[-1]]:.3f}")


if __name__ == "__main__":
    main()
