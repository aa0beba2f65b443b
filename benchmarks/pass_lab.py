"""Forward / data-gradient A/B lab through the production dispatch: each shape, pass and arm (a set of
extension setters) in interleaved rounds on the same operands; outputs of every arm are compared with
arm 0 (bitwise by default).  The forward runs with BN statistics, the data gradient with the fused
BN-backward epilogue (mask from z), as in the training step.

python benchmarks/pass_lab.py --shapes "16,512,512,64,64;256,56,56,64,64" --arms "halo:set_conv3_stream=0;stream:"
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

RESET = {"set_conv3_stream": -1, "set_conv_halo": -1}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="16,512,512,64,64;256,56,56,64,64")
    ap.add_argument("--arms", default="base:")
    ap.add_argument("--passes", default="fwd,dgrad")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    from deeplearning_mpi_amd.models.engine import BwdFuse
    from deeplearning_mpi_amd.ops.act import Act
    from deeplearning_mpi_amd.ops.backend import NativeBackend

    be = NativeBackend("cuda")
    C_ = be.C
    dev = "cuda"
    arms = []
    for part in args.arms.split(";"):
        name, _, sets = part.partition(":")
        arms.append((name, [(k, int(v)) for k, v in (kv.split("=") for kv in sets.split(",") if kv)]))

    def apply(kv):
        for k, v in RESET.items():
            getattr(C_, k)(v)
        for k, v in kv:
            getattr(C_, k)(v)

    for sh in args.shapes.split(";"):
        N, H, W, C, K = map(int, sh.split(","))
        x = Act(torch.randn(N * H * W, C, device=dev).to(torch.bfloat16), N, H, W, C)
        w = (torch.randn(K, 3, 3, C, device=dev) / (9 * C) ** 0.5).to(torch.bfloat16)
        wT = w.permute(3, 1, 2, 0).contiguous()
        bias = torch.randn(K, device=dev) * 0.1
        dy = Act(torch.randn(N * H * W, K, device=dev).to(torch.bfloat16), N, H, W, K)
        z = Act(torch.randn(N * H * W, C, device=dev).to(torch.bfloat16), N, H, W, C)
        sc, shf = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.5
        y = Act.empty(N, H, W, K, torch.bfloat16, dev)
        dx = Act.empty(N, H, W, C, torch.bfloat16, dev)
        flops = 2.0 * N * H * W * C * K * 9
        for ps in args.passes.split(","):
            def fn():
                if ps == "fwd":
                    st = torch.empty(be.conv_mtiles(N, H, W, C, K, 3, 3, 1, 1), 2, K, device=dev)
                    be.conv_fwd(x, w, K, 3, 3, 1, 1, y, bias=bias, stats=st)
                elif ps == "dgradp":   # plain data gradient (no BN fusion)
                    be.conv_dgrad(dy, wT, C, 3, 3, 1, 1, dx)
                else:
                    be.conv_dgrad(dy, wT, C, 3, 3, 1, 1, dx, fuse=BwdFuse(None, z, None, sc, shf))
            outs = []
            for name, kv in arms:
                apply(kv)
                fn()
                torch.cuda.synchronize()
                outs.append((y if ps == "fwd" else dx).buf.clone())
            same = ["=" if torch.equal(o, outs[0]) else "DIFF" for o in outs[1:]]
            times = {n: [] for n, _ in arms}
            for _ in range(args.rounds):
                for name, kv in arms:
                    apply(kv)
                    for _ in range(3):
                        fn()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(args.iters):
                        fn()
                    e1.record()
                    torch.cuda.synchronize()
                    times[name].append(e0.elapsed_time(e1) / args.iters * 1e3)
            apply([])
            cells = []
            for name, _ in arms:
                t = sorted(times[name])[len(times[name]) // 2]
                cells.append(f"{name} {t:7.1f} us {flops / t / 1e6:6.0f} TF/s")
            print(f"{sh:22s} {ps:5s} " + " | ".join(cells) + "  " + " ".join(same), flush=True)


if __name__ == "__main__":
    main()
