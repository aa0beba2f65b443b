"""Per-shape convolution benchmark: our gfx950 implicit-GEMM kernels vs MIOpen (torch conv2d,
bf16, channels_last) on every distinct ResNet-50 conv shape at batch 256,
forward / data-gradient / weight-gradient.  Prints one JSON line per (shape, pass) and a summary
weighted by how often each shape occurs in the network.

python benchmarks/conv_bench.py [--batch 256] [--iters 20] [--only fwd|dgrad|wgrad]
"""
import argparse
import json
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def resnet50_shapes(N, img=224):
    """(N, H, W, Cin, Cout, R, stride, pad) of every conv of torchvision resnet50, with counts."""
    from deeplearning_mpi_amd.models import resnet50

    m = resnet50()
    shapes = []
    H = img

    def add(conv, h):
        k = conv.kernel_size[0]
        s, p = conv.stride[0], conv.padding[0]
        shapes.append((N, h, h, conv.in_channels, conv.out_channels, k, s, p))
        return (h + 2 * p - k) // s + 1

    h = add(m.conv1, H)
    h = (h + 2 - 3) // 2 + 1
    for layer in (m.layer1, m.layer2, m.layer3, m.layer4):
        for b in layer:
            h1 = add(b.conv1, h)
            h2 = add(b.conv2, h1)
            add(b.conv3, h2)
            if b.downsample is not None:
                add(b.downsample[0], h)
            h = h2
    return Counter(shapes)


def unet_shapes(N, img=512, cin=3):
    """3x3 convs of the reference UNet (/root/reference/pytorch/unet/model.py:51-81) + the 1x1 head."""
    sh = Counter()
    h, c = img, cin
    for co in (64, 128, 256, 512):
        sh[(N, h, h, c, co, 3, 1, 1)] += 1
        sh[(N, h, h, co, co, 3, 1, 1)] += 1
        c, h = co, h // 2
    sh[(N, h, h, 512, 1024, 3, 1, 1)] += 1
    sh[(N, h, h, 1024, 1024, 3, 1, 1)] += 1
    c = 1024
    for co in (512, 256, 128, 64):
        h *= 2
        # after concat: c up-sampled (ConvTranspose2d keeps the channel count) + co skip channels
        # (UpBlock(c + co, co), /root/reference/pytorch/unet/model.py:36-47, 66-69)
        sh[(N, h, h, c + co, co, 3, 1, 1)] += 1
        sh[(N, h, h, co, co, 3, 1, 1)] += 1
        c = co
    sh[(N, h, h, 64, 1, 1, 1, 0)] += 1
    return sh


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
    return s.elapsed_time(e) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default=None)
    ap.add_argument("--no_miopen", action="store_true")
    ap.add_argument("--net", default="resnet50", choices=["resnet50", "unet512"])
    args = ap.parse_args()
    if args.net == "unet512" and args.batch == 256:
        args.batch = 16
    from deeplearning_mpi_amd.ops.act import Act, padc
    from deeplearning_mpi_amd.ops.backend import NativeBackend

    be = NativeBackend("cuda")
    dev = "cuda"
    torch.backends.cudnn.benchmark = True
    tot = Counter()
    shapes = resnet50_shapes(args.batch) if args.net == "resnet50" else unet_shapes(args.batch)
    for shape, cnt in sorted(shapes.items(), key=lambda kv: -kv[1]):
        N, H, W, Cin, K, R, s, p = shape
        Cp, Kp = padc(Cin), padc(K)
        P = (H + 2 * p - R) // s + 1
        flops = 2.0 * N * P * P * K * Cin * R * R
        x = Act(torch.randn(N * H * W, Cp, device=dev).to(torch.bfloat16), N, H, W, Cp)
        w = (torch.randn(Kp, R, R, Cp, device=dev) * 0.05).to(torch.bfloat16)
        y = Act.empty(N, P, P, Kp, torch.bfloat16, dev)
        dy = Act(torch.randn(N * P * P, Kp, device=dev).to(torch.bfloat16), N, P, P, Kp)
        dx = Act.empty(N, H, W, Cp, torch.bfloat16, dev)
        wT = (torch.randn(Cp, R, R, Kp, device=dev) * 0.05).to(torch.bfloat16)
        g = torch.zeros(K * R * R * Cin, device=dev)
        mt = be.conv_mtiles(N, H, W, Cp, Kp, R, R, s, p)
        st = torch.empty(mt, 2, Kp, device=dev)
        ours = {
            "fwd": lambda: be.conv_fwd(x, w, Kp, R, R, s, p, y, stats=st),
            "dgrad": lambda: be.conv_dgrad(dy, wT, Cp, R, R, s, p, dx),
            "wgrad": lambda: be.conv_wgrad(dy, x, R, R, s, p, g, Cin, K),
        }
        xt = torch.randn(N, Cin, H, W, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        wt = (torch.randn(K, Cin, R, R, device=dev, dtype=torch.bfloat16) * 0.05).to(memory_format=torch.channels_last)
        gy = torch.randn(N, K, P, P, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        ref = {
            "fwd": lambda: F.conv2d(xt, wt, None, s, p),
            "dgrad": lambda: torch.ops.aten.convolution_backward(gy, xt, wt, None, [s, s], [p, p], [1, 1], False,
                                                                 [0, 0], 1, [True, False, False]),
            "wgrad": lambda: torch.ops.aten.convolution_backward(gy, xt, wt, None, [s, s], [p, p], [1, 1], False,
                                                                 [0, 0], 1, [False, True, False]),
        }
        for ps in ("fwd", "dgrad", "wgrad"):
            if args.only and ps != args.only:
                continue
            if ps == "dgrad" and shape[3] == 3:
                continue
            t_o = timeit(ours[ps], args.iters)
            t_r = timeit(ref[ps], args.iters) if not args.no_miopen else float("nan")
            tot[("ours", ps)] += t_o * cnt
            tot[("miopen", ps)] += t_r * cnt
            print(json.dumps({"shape": shape, "count": cnt, "pass": ps, "ours_us": round(t_o * 1e6, 1),
                              "ours_tflops": round(flops / t_o / 1e12, 1), "miopen_us": round(t_r * 1e6, 1),
                              "miopen_tflops": round(flops / t_r / 1e12, 1)}), flush=True)
    print(json.dumps({"summary_ms_per_network": {f"{k[0]}_{k[1]}": round(v * 1e3, 3) for k, v in tot.items()}}))


if __name__ == "__main__":
    main()
