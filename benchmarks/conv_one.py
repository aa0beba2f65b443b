"""Run ONE convolution pass repeatedly (for rocprofv3 counter collection on a single kernel).

python benchmarks/conv_one.py --shape N,H,W,Cin,Cout,R,stride,pad --pass fwd|dgrad|wgrad [--iters 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="16,64,64,512,512,3,1,1")
    ap.add_argument("--pass", dest="ps", default="fwd")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--set", default="", help="extension setters for A/B: name=value,name=value")
    a = ap.parse_args()
    from deeplearning_mpi_amd.ops.act import Act, padc
    from deeplearning_mpi_amd.ops.backend import NativeBackend

    N, H, W, Cin, K, R, s, p = map(int, a.shape.split(","))
    be = NativeBackend("cuda")
    for kv in filter(None, a.set.split(",")):
        k, v = kv.split("=")
        getattr(be.C, k)(int(v))
    dev = "cuda"
    Cp, Kp = padc(Cin), padc(K)
    P = (H + 2 * p - R) // s + 1
    x = Act(torch.randn(N * H * W, Cp, device=dev).to(torch.bfloat16), N, H, W, Cp)
    w = (torch.randn(Kp, R, R, Cp, device=dev) * 0.05).to(torch.bfloat16)
    y = Act.empty(N, P, P, Kp, torch.bfloat16, dev)
    dy = Act(torch.randn(N * P * P, Kp, device=dev).to(torch.bfloat16), N, P, P, Kp)
    dx = Act.empty(N, H, W, Cp, torch.bfloat16, dev)
    g = torch.zeros(K * R * R * Cin, device=dev)
    st = torch.empty(be.conv_mtiles(N, H, W, Cp, Kp, R, R, s, p), 2, Kp, device=dev)
    fn = {"fwd": lambda: be.conv_fwd(x, w, Kp, R, R, s, p, y, stats=st),
          "dgrad": lambda: be.conv_dgrad(dy, w.transpose(0, 3).contiguous(), Cp, R, R, s, p, dx),
          "wgrad": lambda: be.conv_wgrad(dy, x, R, R, s, p, g, Cin, K)}[a.ps]
    for _ in range(a.iters):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(a.iters):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    t = ev[0].elapsed_time(ev[1]) / a.iters * 1e-3
    print(f"{a.ps} {a.shape}: {t * 1e6:.1f} us, {2.0 * N * P * P * K * Cin * R * R / t / 1e12:.1f} TFLOP/s")


if __name__ == "__main__":
    main()
