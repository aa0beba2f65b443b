"""Fused optimizers over the ParamArena flat buffers (one kernel launch per step for the whole
model) with torch.optim semantics, plus a launch-free ``clip_grad_norm_``.

Replaces ``optim.SGD(momentum=0.9, weight_decay=1e-5)`` (/root/reference/pytorch/resnet/main.py:114),
``optim.Adam`` (/root/reference/pytorch/unet/train.py:160-161) and
``torch.nn.utils.clip_grad_norm_`` (train.py:194).  When the parameters are not backed by a
single arena the optimizers fall back to one kernel per parameter tensor.
"""
from __future__ import annotations

import torch

from ..ops.backend import make_backend
from ..utils.arena import arena_of
from ..utils.profiler import range as trace_range


def _single_arena(params):
    ars = {id(arena_of(p)) for p in params}
    if len(ars) != 1:
        return None
    a = arena_of(params[0])
    if a is None or len(params) != len(a.params):
        return None
    return a


class _FusedBase(torch.optim.Optimizer):
    def __init__(self, params, defaults):
        super().__init__(params, defaults)
        allp = [p for g in self.param_groups for p in g["params"]]
        self._arena = _single_arena(allp) if len(self.param_groups) == 1 else None
        dev = allp[0].device
        self._be = self._arena.backend if self._arena is not None else make_backend(dev)
        self._step_count = 0

    def zero_grad(self, set_to_none: bool = True):
        self._resolve_arena()
        if self._arena is not None:
            self._arena.zero_grad()   # grads are views of the flat buffer: one memset
        else:
            super().zero_grad(set_to_none=set_to_none)

    def _resolve_arena(self):
        # the engine builds its arena lazily (first forward / DDP construction), possibly after the
        # optimizer was created: pick it up as soon as it exists
        if (self._arena is None or not self._arena.valid()) and len(self.param_groups) == 1:
            a = _single_arena(self.param_groups[0]["params"])
            if a is not None:
                self._arena = a
                self._be = a.backend

    def _groups(self):
        """Yield (group, p, g, state-key-prefix) as flat (arena) or per-tensor views."""
        self._resolve_arena()
        if self._arena is not None:
            g = self.param_groups[0]
            yield g, self._arena.flat, self._arena.grad, "__flat__"
        else:
            for g in self.param_groups:
                for p in g["params"]:
                    if p.grad is None:
                        continue
                    if not (p.is_contiguous() and p.grad.is_contiguous()):
                        raise RuntimeError("fused optimizer fallback needs contiguous params/grads")
                    yield g, p.data.view(-1), p.grad.view(-1), p

    def _buf(self, key, name, like):
        st = self.state[key] if not isinstance(key, str) else self.state.setdefault(key, {})
        if name not in st:
            st[name] = torch.zeros_like(like)
        return st[name]


class SGD(_FusedBase):
    def __init__(self, params, lr=1e-3, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False):
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                                      nesterov=nesterov))
        self.skip_flag = None   # optional device scalar: non-zero -> skip the update on every rank

    @torch.no_grad()
    def step(self, closure=None):
        with trace_range("dlmpi.sgd_step"):
            return self._step(closure)

    def _step(self, closure):
        loss = closure() if closure is not None else None
        for g, p, gr, key in self._groups():
            first = "momentum_buffer" not in (self.state[key] if not isinstance(key, str) else
                                              self.state.get(key, {}))
            m = self._buf(key, "momentum_buffer", p) if g["momentum"] != 0 else p
            self._be.sgd(p, gr, m, g["lr"], g["momentum"], g["dampening"], g["weight_decay"], g["nesterov"],
                         first, self.skip_flag)
        if self._arena is not None:
            self._arena.mark_updated()
        self._step_count += 1
        return loss


class Adam(_FusedBase):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, decoupled=False):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.decoupled = decoupled
        self.clip = None   # device [coef, nonfinite] from clip_grad_norm_ (applied & used to skip)
        self._clip_handoff = False   # clip_grad_norm_ left the in-place scaling to this step (see there)

    @torch.no_grad()
    def step(self, closure=None):
        with trace_range("dlmpi.adam_step"):
            return self._step(closure)

    def _step(self, closure):
        loss = closure() if closure is not None else None
        self._step_count += 1
        t = self._step_count
        for g, p, gr, key in self._groups():
            b1, b2 = g["betas"]
            m = self._buf(key, "exp_avg", p)
            v = self._buf(key, "exp_avg_sq", p)
            # the step count lives on the device: the kernel uses step + 1 and advances it only when
            # the update is applied (a collective NaN/Inf skip leaves it unchanged), so a captured
            # step replayed from a hipGraph keeps correct bias corrections
            st = self.state[key] if not isinstance(key, str) else self.state.setdefault(key, {})
            if "step" not in st:
                st["step"] = torch.zeros(1, dtype=torch.float32, device=p.device)
            self._be.adam(p, gr, m, v, g["lr"], b1, b2, g["eps"], g["weight_decay"], self.decoupled,
                          1 - b1 ** t, 1 - b2 ** t, self.clip, st["step"], clip_writeback=self._clip_handoff)
        if self._clip_handoff:   # a handed-off coefficient is used once
            self.clip = None
            self._clip_handoff = False
        if self._arena is not None:
            self._arena.mark_updated()
        return loss


class AdamW(Adam):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        super().__init__(params, lr, betas, eps, weight_decay, decoupled=True)


def clip_grad_norm_(parameters, max_norm: float, norm_type: float = 2.0, optimizer=None):
    """L2 gradient clipping without a host synchronisation.  Returns the total norm as a device
    tensor.  With ``optimizer`` (our Adam) the clip coefficient is also handed to it so a
    non-finite norm skips the update (the same decision on every rank, because gradients are
    identical after the all-reduce).  With ``optimizer`` and arena-backed parameters (norm_type 2)
    the in-place scaling of the gradients is left to that optimizer's next ``step()``: its kernel
    stores g * coef back while it reads g (one pass over the gradients less, the same products:
    bit-identical update and gradients), so until ``step()`` the gradients are still unscaled.

    ``norm_type`` 2 runs the fused single-pass kernel; any other p (including ``inf``) is the
    torch.nn.utils.clip_grad_norm_ contract computed with device-side torch reductions (still no
    host synchronisation, still capturable)."""
    params = [p for p in parameters if p.grad is not None] if not isinstance(parameters, torch.Tensor) \
        else [parameters]
    a = _single_arena(params)
    dev = params[0].device
    be = a.backend if a is not None else make_backend(dev)
    norm = torch.empty(1, dtype=torch.float32, device=dev)
    # [scale, nonfinite, 1, nonfinite]: the last pair is the optimizer's (scale, skip) once the
    # gradients are scaled in place (written by the same kernel: no copy or fill per step)
    coef = torch.empty(4, dtype=torch.float32, device=dev)
    if float(norm_type) != 2.0:
        grads = [a.grad] if a is not None else [p.grad.reshape(-1) for p in params]
        p = float(norm_type)
        if p == float("inf"):
            n = torch.stack([g.float().abs().max() for g in grads]).max()
        else:
            n = torch.stack([g.double().abs().pow(p).sum() for g in grads]).sum().pow(1.0 / p).float()
        norm.copy_(n.reshape(1))
        coef[0] = torch.clamp(max_norm / (n + 1e-6), max=1.0)
        coef[1] = (~torch.isfinite(n)).float()
        coef[2] = 1.0
        coef[3] = coef[1]
        for g in grads:
            g.mul_(coef[0].to(g.dtype))
    elif a is not None:
        be.grad_norm(a.grad, float(max_norm), norm, coef)
        if optimizer is not None and hasattr(optimizer, "_clip_handoff") and \
                (optimizer._resolve_arena() or getattr(optimizer, "_arena", None) is a):
            optimizer.clip = coef[0:2]   # (scale, skip): applied and stored back by the optimizer's step
            optimizer._clip_handoff = True
            return norm[0]
        be.scale_(a.grad, coef)
    else:
        flat = torch.cat([p.grad.reshape(-1).float() for p in params])
        be.grad_norm(flat, float(max_norm), norm, coef)
        for p in params:
            be.scale_(p.grad.view(-1), coef)
    if optimizer is not None and hasattr(optimizer, "clip"):
        optimizer.clip = coef[2:4]   # grads already scaled in place: scale 1, keep the skip flag
    return norm[0]
