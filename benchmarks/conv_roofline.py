"""Memory-roofline probe of the memory-bound 1x1 convolutions (ResNet-50, batch 256): for every
distinct 1x1 shape, our forward with the fused BN-statistics epilogue, without it, other tiles,
and MIOpen (torch conv2d, bf16 channels_last), each as time and effective HBM bandwidth
((input + output bytes) / time), next to a device copy of the same output size.

python benchmarks/conv_roofline.py [--iters 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from benchmarks.conv_bench import resnet50_shapes  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(3):
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / iters * 1e3)
    return sorted(ts)[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    from deeplearning_mpi_amd.ops.act import padc
    from deeplearning_mpi_amd.ops.backend import NativeBackend

    be = NativeBackend("cuda")
    C = be.C
    dev = "cuda"
    for shape, cnt in sorted(resnet50_shapes(a.batch).items(), key=lambda kv: -kv[1]):
        N, H, W, Cin, K, R, s, p = shape
        if R != 1 or Cin < 64:
            continue
        Cp, Kp = padc(Cin), padc(K)
        P = (H - 1) // s + 1
        M = N * P * P
        x = torch.randn(N * H * W, Cp, device=dev).to(torch.bfloat16)
        w = (torch.randn(Kp, 1, 1, Cp, device=dev) * 0.05).to(torch.bfloat16)
        y = torch.empty(M, Kp, device=dev, dtype=torch.bfloat16)
        st = torch.zeros((M + 63) // 64, 2, Kp, device=dev)
        rec = {"shape": shape, "count": cnt}
        byts = (x.numel() * (1 if s == 1 else 0.25) + y.numel()) * 2
        flops = 2.0 * M * K * Cin

        def ours(bm, bn, stats):
            return lambda: C.conv2d_fwd(x, N, H, W, Cp, Cp, 0, w, Kp, 1, 1, s, 0, y, Kp, 0, None, None, 0, 0, None,
                                        None, False, st if stats else None, bm, 0, bn)
        for name, fn in (("stats", ours(0, 0, True)), ("nostats", ours(0, 0, False)),
                         ("128x64", ours(128, 64, True)), ("64x128", ours(64, 128, True)),
                         ("256x128", ours(256, 128, True))):
            try:
                t = timeit(fn, a.iters)
            except Exception as e:  # noqa: BLE001  (a variant the shape does not support)
                rec[name] = str(e)[:60]
                continue
            rec[name] = {"us": round(t, 1), "TBps": round(byts / t / 1e6, 2), "TF": round(flops / t / 1e6, 1)}
        xt = x[:, :Cin].reshape(N, H, W, Cin).permute(0, 3, 1, 2)
        wt = w[:K, :, :, :Cin].permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        t = timeit(lambda: F.conv2d(xt, wt, None, s), a.iters)
        rec["miopen"] = {"us": round(t, 1), "TBps": round(byts / t / 1e6, 2)}
        src = torch.empty_like(y)
        t = timeit(lambda: y.copy_(src), a.iters)
        rec["copy_out"] = {"us": round(t, 1), "TBps": round(2 * y.numel() * 2 / t / 1e6, 2)}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
