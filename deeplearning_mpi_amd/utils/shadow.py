"""Op-level numerics shadow of the execution engine.

:class:`ShadowBackend` wraps a compute backend (normally the native one): every backend call of a
forward/backward is repeated on a second backend (normally the float64 reference) with float64
copies of the inputs the first call saw, and every floating output -- tensors written in place,
returned BN-statistics partials -- is compared.  Because each op is checked on identical inputs,
the check isolates kernel error from the chaotic part of end-to-end comparisons (a forward value
within rounding of a ReLU's zero flips its mask, and one flipped element moves whole gradients by
1e-3; see tests/test_fp32_gpu.py).  Per-tile partials ([T][ns][C], tilings differ between backends)
are compared as sums, every statistic row on its own scale.

Used by tests/test_fp32_gpu.py and scripts/diag/shadow.py.
"""
from __future__ import annotations

import torch

from ..ops.act import Act, Deferred

# ops whose outputs the reference cannot reproduce bit-compatibly: max-pool window indices (native
# uint8 window slots vs torch flat indices) feed maxpool_bwd; cast_weights / conv_mtiles are layout
# bookkeeping
SKIP = frozenset({"maxpool_bwd", "cast_weights", "conv_mtiles", "materialize"})
# fused ops whose inputs are engine objects the shadow cannot copy (engine.PendingApply): hidden, so
# the engine takes the unfused path (the same values, op by op)
# (wgrad_defer: the weight gradients are compared call by call, so their reductions must not queue)
HIDDEN = frozenset({"conv_fwd_bn_apply", "wgrad_defer", "wgrad_flush", "wgrad_bypass"})
# positional index of the BN-partials buffer of ops that take it positionally
STATS_ARG = {"conv_fwd_bn": 9}


def to64(a):
    """float64 copy of every floating tensor inside ``a`` (Acts, tensors, (named)tuples, lists)."""
    if isinstance(a, Act):
        b = a.buf.detach()
        return Act(b.double().clone() if b.is_floating_point() else b.clone(), a.N, a.H, a.W, a.C, a.off)
    if isinstance(a, torch.Tensor):
        return a.detach().double().clone() if a.is_floating_point() else a.clone()
    if isinstance(a, Deferred):
        return Deferred(a.kind, to64(a.src), to64(a.z), to64(a.k0), to64(a.k1))
    if isinstance(a, tuple) and hasattr(a, "_fields"):
        return type(a)(*[to64(x) for x in a])
    if isinstance(a, (list, tuple)):
        return type(a)(to64(x) for x in a)
    return a


def tensors(a):
    if isinstance(a, Act):
        return [a.nhwc()]
    if isinstance(a, torch.Tensor):
        return [a]
    if isinstance(a, (list, tuple)):
        return [t for x in a for t in tensors(x)]
    return []


def max_rel(x: torch.Tensor, y: torch.Tensor):
    """max |x - y| / max |y|; partials [T][ns][C] as per-row sums; None if not comparable."""
    x, y = x.double(), y.double()
    if x.dim() == 3 and y.dim() == 3 and x.shape[1:] == y.shape[1:]:
        x, y = x.sum(0), y.sum(0)
        return max(((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item() for a, b in zip(x, y))
    if x.shape != y.shape:
        return None
    return ((x - y).abs().max() / y.abs().max().clamp_min(1e-30)).item()


class ShadowBackend:
    """Delegates to ``primary``; re-runs every call on ``shadow`` and records ops whose outputs
    differ by more than ``tol`` in ``self.records`` as (call index, op, error)."""

    def __init__(self, primary, shadow, tol=1e-5):
        self.__dict__.update(primary=primary, shadow=shadow, tol=tol, records=[], calls=0, worst={})

    def __setattr__(self, k, v):   # engine-side settings (aux_on, ...) go to the primary
        setattr(self.primary, k, v)

    def __getattr__(self, name):
        if name in HIDDEN:
            raise AttributeError(name)
        f = getattr(self.primary, name)
        if not callable(f) or name in SKIP or name.startswith("_") or not hasattr(self.shadow, name):
            return f

        def call(*args, **kw):
            sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)
            sync()
            a64, k64 = to64(args), {k: to64(v) for k, v in kw.items()}
            if k64.get("stats") is not None:   # the reference fills row 0 of the partials only
                k64["stats"].zero_()
            if name in STATS_ARG and len(a64) > STATS_ARG[name] and isinstance(a64[STATS_ARG[name]], torch.Tensor):
                a64[STATS_ARG[name]].zero_()
            out = f(*args, **kw)
            sync()
            ref = getattr(self.shadow, name)(*a64, **k64)
            self.__dict__["calls"] += 1
            pairs = list(zip(tensors(args) + tensors(list(kw.values())), tensors(a64) + tensors(list(k64.values()))))
            if out is not None and ref is not None:
                pairs += list(zip(tensors(out), tensors(ref)))
            worst = 0.0
            for x, y in pairs:
                if x.is_floating_point() and y.is_floating_point():
                    e = max_rel(x, y)
                    if e is not None:
                        worst = max(worst, e)
            self.worst[name] = max(self.worst.get(name, 0.0), worst)
            if worst > self.tol:
                self.records.append((self.calls, name, worst))
            return out

        return call
