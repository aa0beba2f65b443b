"""Tile / kernel-variant A/B for the implicit-GEMM conv forward, interleaved in ONE process
(cdna_hip_programming.md §5.4 rule 24), with a bit-exactness check of every variant against the
default choice (every tile reduces K in the same order, so outputs and BN partial sums per 256 rows
must agree exactly).

python benchmarks/conv_ab.py [--net resnet50|unet512] [--rounds 3] [--iters 10]
Variants: name=(bm, bn); every variant must be bit-exact against the default.  The 1-block/CU ring-pipelined 256-row kernel measured with this script
(profiles/r1_conv_pipe_rejected) lost to the occupancy-hidden kernels and was not kept.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("DLMPI_AB_ROOT"):   # A/B against another build of the package (e.g. a saved copy)
    sys.path.insert(0, os.path.abspath(os.environ["DLMPI_AB_ROOT"]))

import torch  # noqa: E402

from benchmarks.conv_bench import resnet50_shapes, unet_shapes  # noqa: E402

VARIANTS = {   # name: (bm, bn, reserved); a 32x32x16-MFMA variant was measured: profiles/r1_mfma32_rejected
    "default": (0, 0, 0),
    "64x128": (64, 128, 0),
    "128x64": (128, 64, 0),
    "128x128": (128, 128, 0),
    "256x128": (256, 128, 0),
    "256x256": (256, 256, 0),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--net", default="resnet50", choices=["resnet50", "unet512"])
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--variants", default=",".join(VARIANTS))
    args = ap.parse_args()
    from deeplearning_mpi_amd.ops.act import padc
    from deeplearning_mpi_amd.ops.backend import NativeBackend

    be = NativeBackend("cuda")
    C = be.C
    dev = "cuda"
    batch = args.batch or (256 if args.net == "resnet50" else 16)
    shapes = resnet50_shapes(batch) if args.net == "resnet50" else unet_shapes(batch)
    names = args.variants.split(",")
    tot = {n: 0.0 for n in names}
    for shape, cnt in sorted(shapes.items(), key=lambda kv: -kv[1]):
        N, H, W, Cin, K, R, s, p = shape
        Cp, Kp = padc(Cin), padc(K)
        if Cp < 64 or Kp < 64:
            continue
        P = (H + 2 * p - R) // s + 1
        M = N * P * P
        flops = 2.0 * M * K * Cin * R * R
        torch.manual_seed(0)
        x = torch.randn(N * H * W, Cp, device=dev).to(torch.bfloat16)
        w = (torch.randn(Kp, R, R, Cp, device=dev) * 0.05).to(torch.bfloat16)
        ys = {n: torch.empty(M, Kp, device=dev, dtype=torch.bfloat16) for n in names}
        sts = {n: torch.zeros((M + 63) // 64, 2, Kp, device=dev) for n in names}

        def run(n):
            bm, bn, _ = VARIANTS[n]
            C.conv2d_fwd(x, N, H, W, Cp, Cp, 0, w, Kp, R, R, s, p, ys[n], Kp, 0, None, None, 0, 0, None, None,
                         False, sts[n], bm, 0, bn)

        times = {n: [] for n in names}
        for _ in range(args.rounds):
            for n in names:
                run(n)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    run(n)
                e1.record()
                torch.cuda.synchronize()
                times[n].append(e0.elapsed_time(e1) / args.iters * 1e3)
        ref = ys["default"] if "default" in ys else ys[names[0]]
        rec = {"shape": shape, "count": cnt}
        for n in names:
            t = sorted(times[n])[len(times[n]) // 2]
            tot[n] += t * cnt
            exact = bool(torch.equal(ys[n], ref))
            d = ((ys[n].float() - ref.float()).abs().max() / ref.float().abs().max()).item()
            rec[n] = {"us": round(t, 1), "tf": round(flops / t / 1e6, 1), "exact": exact, "maxrel": float(f"{d:.2e}")}
        print(json.dumps(rec), flush=True)
    print(json.dumps({"total_us_weighted": {n: round(v, 1) for n, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
