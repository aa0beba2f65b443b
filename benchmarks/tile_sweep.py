"""Forward-conv tile sweep: every (BM, BN[, split-K]) plan the conv kernels offer, timed on one shape
through the production entry point with forced tiles (conv2d_fwd bm_req / bn_req; 256-column tiles
are the pipelined 8-wave kernel), next to the static rule's choice and MIOpen.  Statistics epilogue
on (the training forward).

python benchmarks/tile_sweep.py [--shapes N,H,W,Cin,Cout,R,stride,pad;...] [--iters 30]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

DEFAULT = ("256,7,7,512,2048,1,1,0;256,28,28,512,128,1,1,0;256,56,56,64,256,1,1,0;256,28,28,512,256,1,1,0;"
           "256,56,56,128,128,3,2,1;256,14,14,256,1024,1,1,0;256,14,14,1024,256,1,1,0;256,7,7,2048,512,1,1,0")


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=DEFAULT)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--reps", type=int, default=3, help="round-robin repetitions per plan (min taken)")
    ap.add_argument("--plans", default="", help="only these plans, e.g. 128x128,256x256 (plus default)")
    a = ap.parse_args()
    from deeplearning_mpi_amd.ops.act import Act
    from deeplearning_mpi_amd.ops.backend import NativeBackend

    be = NativeBackend("cuda")
    C_ = be.C
    dev = "cuda"
    for sh in a.shapes.split(";"):
        N, H, W, Cin, K, R, s, p = map(int, sh.split(","))
        P = (H + 2 * p - R) // s + 1
        M = N * P * P
        flops = 2.0 * M * K * Cin * R * R
        x = torch.randn(N * H * W, Cin, device=dev).to(torch.bfloat16)
        w = (torch.randn(K, R, R, Cin, device=dev) * 0.05).to(torch.bfloat16)
        y = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        st = torch.empty(M // 16 + 64, 2, K, device=dev)

        def run(bm, bn, sk=0):
            C_.set_conv_splitk(sk)
            try:
                return timeit(lambda: C_.conv2d_fwd(x, N, H, W, Cin, Cin, 0, w, K, R, R, s, p, y, K, 0, None, None, 0, 0,
                                                    None, None, False, st, bm, 0, bn), a.iters)
            finally:
                C_.set_conv_splitk(0)

        plans = [("default", 0, 0, 0)]
        for bm, bn in ((64, 64), (64, 128), (128, 64), (128, 128), (256, 64), (256, 128), (128, 256), (256, 256)):
            if bn > K and not (bn == 64 and K < 64):
                continue
            for sk in (0, 2):
                name = f"{bm}x{bn}" + (f"/k{sk}" if sk else "")
                if a.plans and name not in a.plans.split(","):
                    continue
                plans.append((name, bm, bn, sk))
        res = {"shape": sh}
        for _ in range(a.reps):   # round robin: clock / thermal drift hits every plan alike
            for name, bm, bn, sk in plans:
                try:
                    t = round(run(bm, bn, sk), 1)
                    res[name] = min(res.get(name, 1e9), t)
                except RuntimeError as e:
                    res[name] = str(e)[:40]
        xt = x.view(N, H, W, Cin).permute(0, 3, 1, 2)
        wt = w.permute(0, 3, 1, 2)
        res["miopen"] = round(timeit(lambda: F.conv2d(xt, wt, None, s, p), a.iters), 1)
        best = min((v, k) for k, v in res.items() if isinstance(v, float) and k not in ("miopen",))
        res["best"] = best[1]
        res["best_tflops"] = round(flops / best[0] / 1e6, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
