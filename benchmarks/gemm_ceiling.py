"""Library ceiling for the convolution GEMMs: hipBLASLt (torch.mm, bf16 in / bf16 out) on the dense
GEMM of every ResNet-50 bs-256 convolution (M = N*P*Q pixels, N = Cout, K = R*S*Cin; no im2col
cost for the library) next to our implicit-GEMM forward kernel on the real convolution (with and
without the fused BN-statistics epilogue), plus a square 8192^3 GEMM as the chip's practical bf16
peak.  One JSON line per shape.

python benchmarks/gemm_ceiling.py [--iters 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(iters):
        fn()
    e[1].record()
    torch.cuda.synchronize()
    return e[0].elapsed_time(e[1]) / iters * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from conv_bench import resnet50_shapes

    from deeplearning_mpi_amd.ops.act import Act, padc
    from deeplearning_mpi_amd.ops.backend import NativeBackend

    be = NativeBackend("cuda")
    dev = "cuda"
    A = torch.randn(8192, 8192, device=dev).to(torch.bfloat16)
    us = timeit(lambda: torch.mm(A, A), a.iters)
    print(json.dumps({"gemm": "8192^3", "us": round(us, 1), "tflops": round(2 * 8192 ** 3 / us / 1e6, 1)}), flush=True)
    del A
    for shape, cnt in sorted(resnet50_shapes(256).items()):
        N, H, W, Cin, K, R, s, p = shape
        if R == 7:
            continue
        Cp, Kp = padc(Cin), padc(K)
        P = (H + 2 * p - R) // s + 1
        M, KK = N * P * P, R * R * Cp
        fl = 2.0 * M * Kp * KK
        x = Act(torch.randn(N * H * W, Cp, device=dev).to(torch.bfloat16), N, H, W, Cp)
        w = (torch.randn(Kp, R, R, Cp, device=dev) * 0.05).to(torch.bfloat16)
        y = Act.empty(N, P, P, Kp, torch.bfloat16, dev)
        st = torch.empty(be.conv_mtiles(N, H, W, Cp, Kp, R, R, s, p), 2, Kp, device=dev)
        ours = timeit(lambda: be.conv_fwd(x, w, Kp, R, R, s, p, y), a.iters)
        ours_st = timeit(lambda: be.conv_fwd(x, w, Kp, R, R, s, p, y, stats=st), a.iters)
        am = torch.randn(M, KK, device=dev).to(torch.bfloat16)
        bm = torch.randn(KK, Kp, device=dev).to(torch.bfloat16)
        lib = timeit(lambda: torch.mm(am, bm), a.iters)
        byt = 2.0 * (N * H * W * Cp + M * Kp)   # activation bytes in + out (weights ignored)
        print(json.dumps({"shape": shape, "count": cnt, "M": M, "N": Kp, "K": KK,
                          "ours_us": round(ours, 1), "ours_tf": round(fl / ours / 1e6, 1),
                          "ours_stats_us": round(ours_st, 1), "hipblaslt_us": round(lib, 1),
                          "hipblaslt_tf": round(fl / lib / 1e6, 1),
                          "ours_tbps": round(byt / ours / 1e6, 2)}), flush=True)
        del x, w, y, st, am, bm


if __name__ == "__main__":
    main()
