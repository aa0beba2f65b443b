"""Producer BN-apply fused into the 1x1 consumer conv (pro 3) vs the apply pass + plain conv, on the
ResNet-50 bs-256 shapes: per variant the time of the pair (apply + conv + finalize) and the check that
y / mask bits / conv output are bit-identical to the unfused schedule.

python benchmarks/apply_lab.py [--iters 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

SHAPES = [  # N, H, W, C (apply channels), K (conv out), BN-output residual
    (256, 56, 56, 256, 64, False),
    (256, 28, 28, 512, 128, False),
    (256, 14, 14, 1024, 256, False),
    (256, 14, 14, 1024, 256, True),
]


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
    a = ap.parse_args()
    from deeplearning_mpi_amd._ext import native

    C_ = native()
    dev = "cuda"
    for N, H, W, C, K, bnres in SHAPES:
        M = N * H * W
        g = torch.Generator(device=dev).manual_seed(C + K)
        z3 = torch.randn(M, C, device=dev, generator=g).to(torch.bfloat16)
        res = torch.randn(M, C, device=dev, generator=g).to(torch.bfloat16)
        sc, sh = torch.rand(C, device=dev, generator=g) + 0.5, torch.randn(C, device=dev, generator=g) * 0.2
        rs, rh = (torch.rand(C, device=dev, generator=g) + 0.5, torch.randn(C, device=dev, generator=g) * 0.2) \
            if bnres else (None, None)
        w = (torch.randn(K, C, device=dev, generator=g) / C ** 0.5).to(torch.bfloat16)
        gamma, beta = torch.rand(K, device=dev, generator=g) + 0.5, torch.randn(K, device=dev, generator=g)
        vec = torch.empty(4, K, device=dev)
        rm, rv = torch.zeros(K, device=dev), torch.ones(K, device=dev)
        st = torch.empty(M // 32 + 8, 2, K, device=dev)
        y = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
        mb = torch.empty(M, C // 8, device=dev, dtype=torch.uint8)
        zo = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        fin = (float(M), gamma, beta, rm, rv, 0.1, 1e-5, vec[0], vec[1], vec[2], vec[3])

        def fused():
            C_.conv2d_fwd_bn_apply(z3, N, H, W, C, C, 0, w, K, zo, K, 0, None, st, sc, sh, res, C, 0, rs, rh, y, C, 0,
                                   mb, *fin)

        def unfused():
            C_.bn_apply(z3, C, 0, M, C, sc, sh, res, C, 0, True, y, C, 0, mb, rs, rh)
            C_.conv2d_fwd_bn(y, N, H, W, C, C, 0, w, K, 1, 1, 1, 0, zo, K, 0, None, st, 0, None, None, None, 0, 0,
                             *fin)

        out, res_t = {}, {}
        for name, setv, fn in (("unfused", -1, unfused), ("fused_old", 0, fused), ("fused_new", -1, fused)):
            C_.set_conv_apply(setv)
            try:
                fn()
                torch.cuda.synchronize()
                out[name] = (y.clone(), mb.clone(), zo.clone())
                res_t[name] = round(timeit(fn, a.iters), 1)
            finally:
                C_.set_conv_apply(-1)
        ref = out["unfused"]
        same = {k: [bool(torch.equal(v[i].view(torch.int16) if v[i].dtype == torch.bfloat16 else v[i],
                                     ref[i].view(torch.int16) if ref[i].dtype == torch.bfloat16 else ref[i]))
                    for i in range(3)] for k, v in out.items()}
        gb = (3 * M * C * 2 + M * C // 8 + M * K * 2) / 1e9
        print(json.dumps({"shape": [N, H, W, C, K, bnres], "us": res_t, "bit_identical_y_mbits_out": same,
                          "new_TBps": round(gb / res_t["fused_new"] * 1e6 / 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
