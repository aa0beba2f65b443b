"""Weight-gradient lab: every distinct weight-gradient shape of ResNet-50 (bs 256) and UNet-512 (bs 16)
through the production dispatch (`NativeBackend.conv_wgrad`: kernel + split reduction), under a list of
extension setter configurations, in interleaved rounds (box drift hits every arm alike).  Each arm is
checked against the first (bitwise or to --tol) and the first against the fp32 reference once.

python benchmarks/wgrad_lab.py [--net resnet50|unet512|all] [--only3x3] [--rounds 3] [--iters 20]
       [--arms "base:;gen:set_wgrad3=0;full:set_wgrad3_blocks=256"]
Arm syntax: name:setter=value,setter=value (setters of deeplearning_mpi_amd._C; restored to -1/0 after).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from conv_bench import resnet50_shapes, unet_shapes  # noqa: E402

RESET = {"set_wgrad3_blocks": 0, "set_wgrad3": -1, "set_wgrad_fast": 1}


def parse_arms(spec):
    arms = []
    for part in spec.split(";"):
        name, _, sets = part.partition(":")
        kv = []
        for s in filter(None, sets.split(",")):
            k, v = s.split("=")
            kv.append((k, int(v)))
        arms.append((name, kv))
    return arms


def apply(C, kv):
    for k, v in RESET.items():
        if hasattr(C, k):
            getattr(C, k)(v)
    for k, v in kv:
        getattr(C, k)(v)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--net", default="all")
    ap.add_argument("--only3x3", action="store_true")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--arms", default="base:")
    ap.add_argument("--tol", type=float, default=0.0, help="max rel. difference to arm 0 (0: bitwise)")
    ap.add_argument("--shapes", default="", help="N,H,W,Cin,Cout,R,s,p;... (overrides --net)")
    args = ap.parse_args()
    from deeplearning_mpi_amd.ops.act import Act, padc
    from deeplearning_mpi_amd.ops.backend import NativeBackend, RefBackend

    be, rb = NativeBackend("cuda"), RefBackend("cuda")
    C = be.C
    dev = "cuda"
    arms = parse_arms(args.arms)
    shapes = {}
    if args.shapes:
        for s in args.shapes.split(";"):
            shapes[tuple(map(int, s.split(",")))] = 1
    else:
        if args.net in ("resnet50", "all"):
            shapes.update(resnet50_shapes(256))
        if args.net in ("unet512", "all"):
            for k, v in unet_shapes(16).items():
                shapes[k] = shapes.get(k, 0) + v
    tot = {n: 0.0 for n, _ in arms}
    bad = 0
    for shape, cnt in sorted(shapes.items(), key=lambda kv: (kv[0][0], -kv[0][3] * kv[0][1])):
        N, H, W, Cin, K, R, s, p = shape
        if args.only3x3 and not (R == 3 and s == 1):
            continue
        if Cin < 8:
            continue
        Cp, Kp = padc(Cin), padc(K)
        P = (H + 2 * p - R) // s + 1
        flops = 2.0 * N * P * P * K * Cin * R * R
        x = Act(torch.randn(N * H * W, Cp, device=dev).to(torch.bfloat16), N, H, W, Cp)
        dy = Act(torch.randn(N * P * P, Kp, device=dev).to(torch.bfloat16), N, P, P, Kp)
        g = torch.zeros(K * R * R * Cin, device=dev)
        outs = []
        for name, kv in arms:
            apply(C, kv)
            g.zero_()
            be.conv_wgrad(dy, x, R, R, s, p, g, Cin, K)
            torch.cuda.synchronize()
            outs.append(g.clone())
        ref = torch.zeros_like(g)
        if N * H * W <= 1 << 22:
            rb.conv_wgrad(Act(dy.buf.float(), N, P, P, Kp), Act(x.buf.float(), N, H, W, Cp), R, R, s, p, ref, Cin, K)
            rel0 = ((outs[0] - ref).norm() / ref.norm()).item()
        else:
            rel0 = float("nan")
        diffs = []
        for o in outs[1:]:
            d = ((o - outs[0]).norm() / outs[0].norm()).item()
            diffs.append(d)
            if d > args.tol:
                bad += 1
        times = {n: [] for n, _ in arms}
        for _ in range(2 * args.iters):   # clocks up after the fp32 reference, before any arm is timed
            be.conv_wgrad(dy, x, R, R, s, p, g, Cin, K)
        for _ in range(args.rounds):
            for name, kv in arms:
                apply(C, kv)
                fn = lambda: be.conv_wgrad(dy, x, R, R, s, p, g, Cin, K)  # noqa: E731
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
        apply(C, [])
        cells = []
        for name, _ in arms:
            t = min(times[name])   # best of the interleaved rounds
            tot[name] += t * cnt
            cells.append(f"{name} {t:7.1f} us {flops / t / 1e6:6.0f} TF/s")
        print(f"{str(shape):38s} x{cnt}  ref {rel0:.1e}  " + " | ".join(cells)
              + ("  diff " + " ".join(f"{d:.1e}" for d in diffs) if diffs else ""), flush=True)
    print("total (count-weighted, us): " + " | ".join(f"{n} {v:.1f}" for n, v in tot.items()))
    print(f"arms differing from arm 0 beyond tol: {bad}")


if __name__ == "__main__":
    main()
