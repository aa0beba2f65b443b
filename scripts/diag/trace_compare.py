"""Record every backend call of one UNet training step on two engines (native fp32 and the fp64
reference) and compare the calls pairwise in order: inputs and outputs, per tensor, per statistic
row.  Prints the first calls whose tensors disagree by more than --tol (Frobenius-relative).

python scripts/diag/trace_compare.py [--tol 1e-4]
"""
import argparse
import copy
import os
import sys

os.environ.setdefault("DLMPI_WGRAD_STREAM", "0")
os.environ.setdefault("DLMPI_BRANCH_STREAM", "0")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from deeplearning_mpi_amd.ops.act import Act  # noqa: E402

SKIP = {"cast_weights", "conv_mtiles", "set_aux_stream", "materialize"}


def snap(a):
    if isinstance(a, Act):
        return ("act", a.nhwc().detach().double().clone() if a.buf.is_floating_point() else None)
    if isinstance(a, torch.Tensor):
        return ("t", a.detach().double().clone() if a.is_floating_point() else None)
    if isinstance(a, (list, tuple)):
        return ("seq", [snap(x) for x in a])
    return ("o", None)


def leaves(s, path="a"):
    kind, v = s
    if kind == "seq":
        for i, x in enumerate(v):
            yield from leaves(x, f"{path}.{i}")
    elif v is not None:
        yield path, v


class Rec:
    def __init__(self, be, log):
        self.__dict__.update(be=be, log=log)

    def __setattr__(self, k, v):
        setattr(self.be, k, v)

    def __getattr__(self, name):
        f = getattr(self.be, name)
        if not callable(f) or name in SKIP or name.startswith("_"):
            return f

        def wrapped(*args, **kw):
            torch.cuda.synchronize()
            pre = snap((list(args), kw.get("pre"), kw.get("fuse"), kw.get("res")))
            out = f(*args, **kw)
            torch.cuda.synchronize()
            post = snap((list(args), [kw[k] for k in sorted(kw) if k != "pre"]))
            self.log.append((name, pre, post, snap(out)))
            return out

        return wrapped


def err(a, b):
    if a.shape != b.shape:
        if a.dim() == 3 and b.dim() == 3 and a.shape[1:] == b.shape[1:]:
            a, b = a.sum(0), b.sum(0)
            return max(((x - y).norm() / y.norm().clamp_min(1e-30)).item() for x, y in zip(a, b))
        return None
    if a.dim() == 3:   # partials: per statistic row of the sums
        a, b = a.sum(0), b.sum(0)
        return max(((x - y).norm() / y.norm().clamp_min(1e-30)).item() for x, y in zip(a, b))
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tol", type=float, default=1e-4)
    ap.add_argument("--show", type=int, default=12)
    a = ap.parse_args()
    from deeplearning_mpi_amd.models import UNet
    from deeplearning_mpi_amd.ops import bce_with_logits

    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(2, 3, 64, 64, device=dev, generator=g)
    y = (torch.rand(2, 64, 64, device=dev, generator=g) > 0.5).float()
    torch.manual_seed(0)
    m0 = UNet(out_classes=1).to(dev)
    logs = []
    for prec, dt in (("fp32", torch.float32), ("ref", torch.float64)):
        m = copy.deepcopy(m0).to(dt)
        m.precision = prec
        m.train()
        m.engine_setup(dev)
        log = []
        m._be = Rec(m._be, log)
        loss = bce_with_logits(m(x.to(dt)).squeeze(1), y.to(dt))
        loss.backward()
        torch.cuda.synchronize()
        logs.append(log)
    print(len(logs[0]), len(logs[1]), "calls")
    shown = 0
    for i, (c0, c1) in enumerate(zip(*logs)):
        if c0[0] != c1[0]:
            print(f"#{i}: schedule differs: {c0[0]} vs {c1[0]}")
            break
        rows = []
        for tag, s0, s1 in (("arg", c0[2], c1[2]), ("ret", c0[3], c1[3])):   # args after the call
            l1 = dict(leaves(s1))
            for p, v in leaves(s0):
                if p in l1:
                    e = err(v, l1[p])
                    if e is not None and e > a.tol:
                        rows.append(f"{tag}:{p}{tuple(v.shape)}={e:.1e}")
        if rows:
            print(f"#{i} {c0[0]}: " + " ".join(rows[:8]))
            shown += 1
            if shown >= a.show:
                break


if __name__ == "__main__":
    main()


def mask_flips(call=78):
    """For a fused conv_dgrad call: ReLU-mask decisions (z*scale + shift > 0) of the two runs."""
    import deeplearning_mpi_amd.models.engine as E  # noqa: F401
    from deeplearning_mpi_amd.models import UNet
    from deeplearning_mpi_amd.ops import bce_with_logits

    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(2, 3, 64, 64, device=dev, generator=g)
    y = (torch.rand(2, 64, 64, device=dev, generator=g) > 0.5).float()
    torch.manual_seed(0)
    m0 = UNet(out_classes=1).to(dev)
    fuses = []
    for prec, dt in (("fp32", torch.float32), ("ref", torch.float64)):
        m = copy.deepcopy(m0).to(dt)
        m.precision = prec
        m.train()
        m.engine_setup(dev)
        log = []
        m._be = Rec(m._be, log)
        loss = bce_with_logits(m(x.to(dt)).squeeze(1), y.to(dt))
        loss.backward()
        torch.cuda.synchronize()
        fuses.append(log[call][2])
    leaves0 = dict(leaves(fuses[0]))
    leaves1 = dict(leaves(fuses[1]))
    for k in sorted(leaves0):
        print(k, tuple(leaves0[k].shape))
    return leaves0, leaves1


if __name__ == "__main__" and os.environ.get("MASK_FLIPS"):
    l0, l1 = mask_flips(int(os.environ["MASK_FLIPS"]))
    # kw order (sorted): colsum, fuse, res -> a.1.1 is the fuse tuple (mask, z, z2, scale, shift, mbits)
    z0, z1 = l0["a.1.1.1"], l1["a.1.1.1"]
    s0, s1 = l0["a.1.1.3"], l1["a.1.1.3"]
    h0, h1 = l0["a.1.1.4"], l1["a.1.1.4"]
    v0 = z0 * s0 + h0
    v1 = z1 * s1 + h1
    flips = (v0 > 0) != (v1 > 0)
    print("elements", v0.numel(), "mask flips", int(flips.sum()))
    C = v0.shape[-1]
    fc = flips.reshape(-1, C).sum(0)
    print("flips per channel (nonzero):", {int(c): int(n) for c, n in enumerate(fc) if n})
    zz = z1.reshape(-1, C)
    print("channels with the smallest std of z:", zz.std(0).sort().values[:5].tolist())
    print("|v| at flips (max):", v1[flips].abs().max().item() if flips.any() else None)
    print("scale at flipped channels:", [float(s1.reshape(-1)[c]) for c in range(C) if fc[c]][:8])
