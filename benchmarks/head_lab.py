"""UNet head (1x1 conv, 64 -> 1, fp32 logits, bias) and input conv (3x3, 8-channel padded image -> 64,
bias, BN statistics) at bench scale: the streaming dot-product kernel (csrc/kernels/head.hip) vs the
GEMM path (set_head1x1 0), the 8-channel 3x3 kernel (csrc/kernels/conv_small.hip) vs the GEMM path
(set_conv_c8 0), and the 2x2/s2 up-sampling into its concat slice (streaming 1x1 kernel over 4 Cout
columns vs the 4-phase implicit GEMM, set_convT_stream 0), interleaved rounds.

python benchmarks/head_lab.py [--iters 20] [--rounds 3]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


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
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    from deeplearning_mpi_amd.ops.act import Act
    from deeplearning_mpi_amd.ops.backend import NativeBackend

    be = NativeBackend("cuda")
    for N, H, W in ((16, 512, 512), (16, 1024, 1024)):
        M, C, Kp = N * H * W, 64, 8
        x = Act(torch.randn(M, C, device="cuda").to(torch.bfloat16), N, H, W, C)
        w = (torch.randn(Kp, C, device="cuda") / 8).to(torch.bfloat16)
        b = torch.randn(Kp, device="cuda")
        y = Act(torch.empty(M, 1, device="cuda"), N, H, W, 1)
        res = {}
        for _ in range(a.rounds):
            for name, on in (("head", 1), ("gemm", 0)):
                be.C.set_head1x1(on)
                try:
                    t = timeit(lambda: be.conv_fwd(x, w, Kp, 1, 1, 1, 0, y, bias=b, kvalid=1), a.iters)
                finally:
                    be.C.set_head1x1(1)
                res[name] = round(min(res.get(name, 1e9), t), 1)
        res["head_TBps"] = round(M * C * 2 / res["head"] / 1e6, 2)
        print(json.dumps({"shape": [N, H, W, C], "us": res}), flush=True)
        xi = Act(torch.randn(M, 8, device="cuda").to(torch.bfloat16), N, H, W, 8)
        wi = (torch.randn(64, 3, 3, 8, device="cuda") / 8).to(torch.bfloat16)
        bi = torch.randn(64, device="cuda")
        z = Act(torch.empty(M, 64, device="cuda", dtype=torch.bfloat16), N, H, W, 64)
        res = {}
        for _ in range(a.rounds):
            for name, on in (("c8", 1), ("gemm", 0)):
                be.C.set_conv_c8(on)
                try:
                    st = torch.empty(be.C.conv2d_fwd_mtiles(N, H, W, 8, 64, 3, 3, 1, 1, 0), 2, 64, device="cuda")
                    t = timeit(lambda: be.conv_fwd(xi, wi, 64, 3, 3, 1, 1, z, bias=bi, stats=st), a.iters)
                finally:
                    be.C.set_conv_c8(1)
                res[name] = round(min(res.get(name, 1e9), t), 1)
        res["c8_TBps_out"] = round(M * 64 * 2 / res["c8"] / 1e6, 2)
        print(json.dumps({"input_conv": [N, H, W, 8, 64], "us": res}), flush=True)
        for C, skip in ((128, 64), (256, 128)):
            h, w_ = H * 128 // C // 2, W * 128 // C // 2   # the level below: 256^2 x 128, 128^2 x 256
            xt = Act(torch.randn(N * h * w_, C, device="cuda").to(torch.bfloat16), N, h, w_, C)
            wt = (torch.randn(C, 2, 2, C, device="cuda") / C ** 0.5).to(torch.bfloat16)
            bt = torch.randn(C, device="cuda")
            cat = Act(torch.empty(N * 4 * h * w_, C + skip, device="cuda", dtype=torch.bfloat16), N, 2 * h, 2 * w_,
                      C + skip)
            res, outs = {}, {}
            for _ in range(a.rounds):
                for name, on in (("stream", 1), ("igemm", 0)):
                    be.C.set_convT_stream(on)
                    try:
                        t = timeit(lambda: be.convT_fwd(xt, wt, C, cat.slice(0, C), bt), a.iters)
                        outs[name] = cat.buf[:, :C].clone() if name not in outs else outs[name]
                        assert on == be.C.convT_stream_last()
                    finally:
                        be.C.set_convT_stream(1)
                    res[name] = round(min(res.get(name, 1e9), t), 1)
            d = (outs["stream"].float() - outs["igemm"].float()).abs().max().item()
            res["max_abs_diff"] = d
            del outs
            res["stream_TBps"] = round((N * h * w_ * C * 2 + N * 4 * h * w_ * C * 2) / res["stream"] / 1e6, 2)
            print(json.dumps({"convT": [N, h, w_, C, C], "us": res}), flush=True)


if __name__ == "__main__":
    main()
