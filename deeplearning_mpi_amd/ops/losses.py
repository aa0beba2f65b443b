"""Fused losses and evaluation metrics (HIP kernels on GPU, torch reference on CPU).

``CrossEntropyLoss`` / ``BCEWithLogitsLoss`` are drop-in for the torch modules the reference uses
(/root/reference/pytorch/resnet/main.py:113, /root/reference/pytorch/unet/train.py:162) for the
``reduction='mean'`` case: one kernel for the loss, one for the gradient, deterministic reductions.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .backend import make_backend

_BE = {}
_ONES = {}


def backward(loss: torch.Tensor):
    """``loss.backward()`` with a cached unit seed gradient (autograd's own seed is an ATen fill
    launch every step; with this the training step launches our kernels only)."""
    key = (loss.device, loss.dtype)
    one = _ONES.get(key)
    if one is None:
        one = _ONES[key] = torch.ones((), dtype=loss.dtype, device=loss.device)
    loss.backward(one)


def _be(device, dtype=None):
    dt = torch.float64 if dtype == torch.float64 else torch.float32
    key = (str(device), dt)
    b = _BE.get(key)
    if b is None:
        b = _BE[key] = make_backend(device, dt)
    return b


class _CE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        logits = logits.contiguous()
        be = _be(logits.device, logits.dtype)
        loss, lse = be.ce_fwd(logits.to(be.dt), labels)
        ctx.save_for_backward(logits, labels, lse)
        return loss

    @staticmethod
    def backward(ctx, go):
        logits, labels, lse = ctx.saved_tensors
        be = _be(logits.device, logits.dtype)
        g = be.ce_bwd(logits.to(be.dt), labels, lse, go.reshape(1).to(be.dt).contiguous())
        return g.to(logits.dtype), None


class _BCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target):
        logits = logits.contiguous()
        target = target.contiguous().to(_be(logits.device, logits.dtype).dt)
        be = _be(logits.device, logits.dtype)
        loss = be.bce_fwd(logits.to(be.dt), target)
        ctx.save_for_backward(logits, target)
        return loss

    @staticmethod
    def backward(ctx, go):
        logits, target = ctx.saved_tensors
        be = _be(logits.device, logits.dtype)
        g = be.bce_bwd(logits.to(be.dt), target, go.reshape(1).to(be.dt).contiguous())
        return g.view(logits.shape).to(logits.dtype), None


def cross_entropy(logits, labels):
    return _CE.apply(logits, labels)


def bce_with_logits(logits, target):
    return _BCE.apply(logits, target)


class CrossEntropyLoss(nn.Module):
    def forward(self, logits, labels):
        return cross_entropy(logits, labels)


class BCEWithLogitsLoss(nn.Module):
    def forward(self, logits, target):
        return bce_with_logits(logits, target)


@torch.no_grad()
def top1_correct(logits, labels) -> torch.Tensor:
    """Device int32[1] count of argmax(logits) == labels (reference main.py:65-71)."""
    return _be(logits.device, logits.dtype).argmax_correct(logits.float().contiguous(), labels)


@torch.no_grad()
def dice_per_sample(logits, target) -> torch.Tensor:
    """Per-sample Dice of (sigmoid(logits) > 0.5) vs target, 1.0 when both are empty
    (reference train.py:121-137).  logits [N,1,H,W] or [N,H,W]; target [N,H,W]."""
    lg = logits.reshape(target.shape).float().contiguous()
    return _be(logits.device, logits.dtype).dice(lg, target.float().contiguous())
