"""Execution engine: explicit forward / backward schedules over fused layer units.

The models keep torch ``nn.Module`` parameter containers with the reference's exact names (so
``state_dict`` is key-compatible with torchvision / the reference UNet), but they never run
``nn.Conv2d.forward``.  Instead a model's ``forward`` runs a hand-written schedule of fused units
(conv + BatchNorm statistics in the GEMM epilogue + BN-apply/ReLU/residual, pooling, ...) on a
compute backend (gfx950 kernels on GPU, torch reference on CPU), and its backward is the
matching hand-written reverse schedule:

* parameter gradients are written (accumulated) straight into the arena's flat gradient buffer
  and announced to the DDP reducer the moment they are final, so bucket all-reduces start while
  the rest of the backward is still running;
* the block-input gradient of a residual block is formed in the data-gradient GEMM epilogue
  (dgrad(conv1) + identity-grad), never as a separate add;
* nothing is traced or compiled: the schedule is plain code, so a whole training step can be
  captured into a hipGraph and replayed.

One ``torch.autograd.Function`` bridges the engine to autograd (loss.backward() works as usual).
"""
from __future__ import annotations

import contextlib
import os
from typing import NamedTuple, Optional

import torch
import torch.nn as nn

from ..ops.act import Act, Deferred, padc
from ..ops.backend import make_backend
from ..utils.arena import ParamArena
from ..utils.profiler import range as trace_range


@contextlib.contextmanager
def grad_side(be, *tensors):
    """Run parameter-gradient work -- weight-gradient GEMMs, their split reductions, bias sums and
    the DDP ``ready`` announcements that launch bucket all-reduces -- on the backend's side stream,
    ordered after everything issued so far on the current stream.  Only the data-gradient chain
    (dgrad -> BN backward -> dgrad ...) stays on the main stream, so weight gradients fill the
    GPU beside it (tails of under-filled grids, the small BN finalize launches).  Every ``ready``
    is issued here, so a bucket's all-reduce always fences on the side stream, which has waited
    for the main stream's BN-parameter gradients.  ``tensors``: buffers read on the side stream
    (kept alive for it in the caching allocator).  The engine backward joins the side stream
    before the optimizer (``_EngineFn.backward``).

    Keeping them alive: the buffers are held in ``be.held``
    until that join and then dropped, so their blocks go back to the main stream's pool already
    ordered after the side-stream work.  ``record_stream`` instead defers each block's reuse to an
    event the host polls only at the next allocation; the host runs a whole backward ahead of the
    GPU, so during backward nearly every freed block was still pending, every allocation took fresh
    memory, and at UNet 1024^2 the cache grew to 170-272 GB reserved for 53 GB allocated with
    step times from 146 to 871 ms (profiles/r1_stream_hold)."""
    side = getattr(be, "side_stream", None)
    if side is None:
        yield
        return
    # set_stream instead of the torch.cuda.stream() context manager: this runs ~300 times per
    # ResNet-152 backward, and the context manager's device bookkeeping cost ~18 us of host time each
    # (bench.py --pyprof, profiles/r3_host)
    cur = torch.cuda.current_stream()
    side.wait_stream(cur)
    torch.cuda.set_stream(side)
    try:
        yield
    finally:
        torch.cuda.set_stream(cur)
    if _STREAM_HOLD:
        be.held.extend(t for t in tensors if t is not None)
        return
    for t in tensors:
        if t is not None:
            t.record_stream(side)


def record_on(stream, *objs):
    """Mark every tensor (or Act buffer) inside ``objs`` (nested tuples / lists allowed) as used on
    ``stream``, so the caching allocator does not recycle it before that stream's work is done.

    With ``_STREAM_HOLD`` (always) this is a no-op: its callers (the ResNet downsample
    branch, models/resnet.py:_BlockExec) keep the main-pool tensors they hand to the branch stream
    referenced until the main stream has waited for it, and the branch stream waits for the main
    stream every time it is entered, so a branch-pool block freed after a main-stream read is only
    reused by branch work ordered after that read."""
    if _STREAM_HOLD:
        return
    for o in objs:
        if o is None:
            continue
        if isinstance(o, torch.Tensor):
            if o.is_cuda:
                o.record_stream(stream)
        elif isinstance(o, Deferred):
            record_on(stream, *o.bufs())
        elif hasattr(o, "buf") and isinstance(getattr(o, "buf"), torch.Tensor):
            record_on(stream, o.buf)
        elif isinstance(o, (tuple, list)):
            record_on(stream, *o)


# Cross-stream buffer lifetimes are held by the issuing step (grad_side) rather than record_stream.
_STREAM_HOLD = True

# One-output-channel 1x1 data gradients as a streaming outer product (bn.hip outer_dgrad_bn_kernel).
_OUTER_DGRAD = True

# BN-backward apply of a unit whose input needs no gradient (the ResNet stem, UNet's first conv) is
# rebuilt in its weight-gradient GEMM's operand prologue instead of stored (ops.act.Deferred).
# (Deferring the other BatchNorm elementwise passes -- forward BN-apply rebuilt by every consumer
# conv, every BN-backward apply rebuilt by its data gradient -- was bit-identical but measured
# slower, ResNet-50 9,924 vs 11,655 img/s, profiles/r2_defer_bn_rejected, and was removed.)
DEFER_BN_WGRAD = True

# Dual data gradient of 1x1 stride-1 convolutions behind a training BN (ConvUnit.dual): the forward
# stores the BN input z in the right half of a [rows][2K] buffer whose left half later receives the
# BN's output gradient dy, so the data gradient reduces over [dy | z] with weights {W*k1, W*k2} and
# bias W.k3 -- dx = dz.W without dz -- and the BN-backward apply pass (dz = k1 dy + k2 z + k3, needed
# only by the weight gradient now) moves to the side stream, off the data-gradient critical path.
# Only for layers with at least DUAL_MIN_ROWS output pixels (N*P*Q): since the streaming 1x1 data
# gradient (conv1x1_dgrad_stream.hip) the layer-2 shapes (200,704 rows at bs 256) gain nothing from
# the doubled reduction: 401,408 keeps it for ResNet-50 layer 1 and the ResNet-152 (bs 128) layer 1
# (ResNet-50 12,948-12,968 vs 12,882-12,901 img/s with layer 2 included, profiles/r3_cifar_ab2).
DUAL_DGRAD = True
DUAL_MIN_ROWS = 2 * 256 * 28 * 28
# The dual path's weight gradient rebuilds dz in its operand prologue (PA 2) from the same [dy | z]
# buffer (an apply pass materialising dz on the side stream first measured slower: it competes with
# the main stream for HBM, profiles/r2_dual_dgrad).
DUAL_WGRAD_PRO = True

# A residual block's BN-apply (+ residual + ReLU) whose first consumer is a 1x1 / stride-1
# convolution of up to FUSE_APPLY_MAX_K output channels (the next bottleneck's conv1 in ResNet-50
# layer1 / layer2) is left pending (PendingApply) and computed by that convolution's operand
# prologue, which also stores it and its ReLU mask bits (backend conv_fwd_bn_apply): no element is
# transformed twice, and the apply's output is written once and never re-read by the consumer.
# With several output tile columns the blocks of every column rebuild y in their prologue: correct
# but measured slower at 256 (ResNet-50 12,730-12,746 vs 12,889-12,916 img/s, profiles/
# r3_fuse_apply_2col_rejected).  (Running the apply in two image chunks beside the consumer's GEMM on
# two streams measured slower too -- a cross-stream join before every BN finalize,
# profiles/r2_chunk_fwd_rejected -- and was removed, as was rebuilding bn2 in the streaming conv3's
# prologue: bit-identical but neutral, profiles/r3_stream_pro.)
FUSE_APPLY = True
# Consumers of one 64 / 128 / 256-channel output column (ResNet-50 conv1 of layers 1-3) run the
# register-staged kernel (conv_igemm.hip conv1x1_apply_kernel): isolated, 56^2 256->64 277 us vs 292
# (the single-stage pro-3 kernel) / 335 (apply pass + conv), 28^2 512->128 162 vs 214 / 194, 14^2
# 1024->256 103 vs 194 / 106 (107 vs 202 / 119 with a BN-output residual), profiles/r5_apply.  (With the
# single-stage kernel only 64 channels paid: 128 lost in the step, profiles/r5_policy.)
FUSE_APPLY_MAX_K = 256
# A BN-apply + ReLU without residual feeding a 64 -> 64 3x3 / s1 / p1 conv (UNet level-1 DoubleConv,
# ResNet layer-1 conv2) is computed by the streaming 3x3 kernel on its staged input tiles, which also
# stores it once (backend conv3_fwd_bn_apply, conv3x3_stream.hip PRO): the apply pass's read of z and
# its launch go; the stored output is what the weight gradient reads (profiles/r6_c3pro).  Per unit
# (ConvUnit.fuse3): the UNet level-1 DoubleConvs take it; ResNet layer 1 does not (its first block's
# conv2 runs beside the downsample branch, where the fused kernel lost what the others gained).
FUSE_APPLY_3X3 = True

# The step's last weight gradient (a unit with ``wgrad_main``: the ResNet stem, whose input needs no
# gradient) runs on the main stream -- idle by then -- instead of queueing behind the side stream's
# last weight gradients (profiles/r3_tail).
WGRAD_TAIL_MAIN = True


def img_rows(a, n0: int, n1: int):
    """Images [n0, n1) of an Act (a row range of its 2-D buffer, same ld / channel offset) or of a
    Deferred.bn operand."""
    if a is None:
        return None
    if isinstance(a, Deferred):
        return Deferred(a.kind, img_rows(a.src, n0, n1), img_rows(a.z, n0, n1), a.k0, a.k1)
    hw = a.H * a.W
    return Act(a.buf[n0 * hw:n1 * hw], n1 - n0, a.H, a.W, a.C, a.off)


class PendingApply:
    """A training BN-apply (+ residual) (+ ReLU) (+ mask bits) whose output ``y`` is allocated but
    not yet computed: a 1x1 consumer convolution computes (and stores) it in its operand prologue
    (FUSE_APPLY, ``ConvUnit.fwd``); any other consumer calls ``resolve`` (one whole apply)."""

    __slots__ = ("y", "z", "scale", "shift", "res", "relu", "mbits", "done")

    def __init__(self, y, z, scale, shift, res, relu, mbits):
        self.y, self.z, self.scale, self.shift, self.res, self.relu, self.mbits = y, z, scale, shift, res, relu, mbits
        self.done = False

    N = property(lambda self: self.y.N)
    H = property(lambda self: self.y.H)
    W = property(lambda self: self.y.W)
    C = property(lambda self: self.y.C)
    device = property(lambda self: self.y.device)

    def resolve(self, be) -> Act:
        if not self.done:
            be.bn_apply(self.z, self.scale, self.shift, self.res, self.relu, self.y, mbits=self.mbits)
            self.done = True
        return self.y


def resolve(be, a):
    return a.resolve(be) if isinstance(a, PendingApply) else a


def bufs(*objs):
    """The storage tensors behind Acts / Deferred operands (None skipped)."""
    out = []
    for o in objs:
        if o is None:
            continue
        if isinstance(o, Deferred):
            out.extend(o.bufs())
        elif isinstance(o, Act):
            out.append(o.buf)
        else:
            out.append(o)
    return out


class BwdFuse(NamedTuple):
    """What a data-gradient GEMM needs to produce the gradient of a BN+ReLU output fused: the ReLU
    mask (``mask`` = the saved output y, or -- for BN+ReLU without a residual -- recomputed from the
    BN input as z*scale + shift > 0, saving the read of y), the BN input(s) z (z2: a second BN
    consuming the same gradient, the ResNet downsample branch) for the backward statistics."""
    mask: Optional[Act]
    z: Act
    z2: Optional[Act] = None
    scale: Optional[torch.Tensor] = None
    shift: Optional[torch.Tensor] = None
    mbits: Optional[torch.Tensor] = None   # [pixels][C/8] ReLU mask bits from the forward BN-apply


class ConvUnit:
    """conv2d / linear (+ training or folded-eval BatchNorm) (+ residual) (+ ReLU)."""

    wgrad_main = False   # see WGRAD_TAIL_MAIN
    fuse3 = False        # FUSE_APPLY_3X3 for this unit (set by the model where it measured faster)

    def __init__(self, arena: ParamArena, conv, bn=None, relu=True, cin_pad=None, need_dgrad=True):
        self.arena, self.conv, self.bn, self.relu = arena, conv, bn, relu
        w = conv.weight
        self.linear = isinstance(conv, nn.Linear)
        if self.linear:
            self.K, self.Cin = w.shape
            self.R = self.S = 1
            self.stride, self.pad = 1, 0
        else:
            self.K, self.Cin, self.R, self.S = w.shape
            assert conv.stride[0] == conv.stride[1] and conv.padding[0] == conv.padding[1]
            assert conv.dilation == (1, 1) and conv.groups == 1
            self.stride, self.pad = conv.stride[0], conv.padding[0]
        self.Cp = cin_pad or padc(self.Cin)
        self.Kp = padc(self.K)
        R, S, K, C = self.R, self.S, self.K, self.Cin
        if self.linear:   # weight [K, C]
            self.h_fwd = arena.add_compute(w, (self.Kp, 1, 1, self.Cp), (K, 1, 1, C), (0, None, None, 1))
            self.h_dg = arena.add_compute(w, (self.Cp, 1, 1, self.Kp), (C, 1, 1, K), (1, None, None, 0)) \
                if need_dgrad else None
        else:             # weight [K, C, R, S]
            self.h_fwd = arena.add_compute(w, (self.Kp, R, S, self.Cp), (K, R, S, C), (0, 2, 3, 1))
            self.h_dg = arena.add_compute(w, (self.Cp, R, S, self.Kp), (C, R, S, K), (1, 2, 3, 0)) \
                if need_dgrad else None
        self.bias = conv.bias
        self._bias_pad = None

    dual = False   # set by the model for 1x1 stride-1 convs behind a training BN (DUAL_DGRAD)

    def dy_slot(self, ctx) -> Optional[Act]:
        """Where the producer of this unit's output gradient should write it: the left half of the
        forward's [rows][2K] z buffer when the dual data gradient is on for this step, else None."""
        if not self.dual or ctx is None:
            return None
        z = ctx[1]
        if z is None or z.off != z.C or z.ld != 2 * z.C:
            return None
        return Act(z.buf, z.N, z.H, z.W, z.C, 0)

    def out_hw(self, H, W):
        return ((H + 2 * self.pad - self.R) // self.stride + 1, (W + 2 * self.pad - self.S) // self.stride + 1)

    def _weight_fwd(self):
        return self.arena.get_compute(self.h_fwd)

    def prep_input(self, be, x: torch.Tensor) -> Act:
        """The network input (fp32 NCHW) in this unit's input layout."""
        return be.nchw_to_nhwc(x, self.Cp)

    def _wgrad(self, be, dz: Act, x: Act):
        be.conv_wgrad(dz, x, self.R, self.S, self.stride, self.pad, self.arena.grad_flat(self.conv.weight),
                      self.Cin, self.K)

    def _bias_vec(self):
        if self.bias is None:
            return None
        if self.Kp == self.K:
            return self.bias.data
        if self._bias_pad is None or self._bias_pad.device != self.bias.device:
            self._bias_pad = torch.zeros(self.Kp, dtype=self.bias.dtype, device=self.bias.device)
            idx = torch.arange(self.Kp)
            idx[self.K:] = -1   # zero padding
            self._bias_idx = idx.to(self.bias.device)
        self.arena.backend.gather_(self._bias_pad, self.bias.data, self._bias_idx)   # one launch of ours
        return self._bias_pad

    def can_fuse_apply(self, be, x, train: bool, save=True) -> bool:
        """True if ``fwd`` computes the pending BN-apply ``x`` inside its GEMM's operand prologue
        (FUSE_APPLY): a 1x1 / stride-1 conv of <= FUSE_APPLY_MAX_K outputs behind a residual BN + ReLU,
        or (FUSE_APPLY_3X3) a 64 -> 64 3x3 conv behind a BN + ReLU without residual."""
        if self._fuse3(be, x, train, save):
            return True
        return (FUSE_APPLY and train and save and isinstance(x, PendingApply) and not x.done
                and self.bn is not None and self.R == 1 and self.S == 1 and self.stride == 1 and self.pad == 0
                and self.Kp <= FUSE_APPLY_MAX_K and x.relu and x.res is not None and x.mbits is not None
                and x.C == self.Cp and hasattr(be, "conv_fwd_bn_apply") and not getattr(be, "f32", False))

    def _fuse3(self, be, x, train, save) -> bool:
        if not (FUSE_APPLY_3X3 and self.fuse3 and train and save and isinstance(x, PendingApply) and not x.done
                and self.bn is not None and self.R == 3 and self.S == 3 and self.stride == 1 and self.pad == 1
                and self.Cp == 64 and self.Kp == 64 and x.C == 64 and x.relu and x.res is None and x.mbits is None
                and hasattr(be, "conv3_fwd_bn_apply") and not getattr(be, "f32", False)):
            return False
        ok = getattr(be, "conv3_pro_ok", None)
        return ok is None or ok(x.z, x.y)

    def fwd(self, be, x, train: bool, res: Act = None, out: Act = None, save=True, defer_apply=False,
            before_res=None, lazy=False):
        """Returns (output, saved context).  x: an Act or a Deferred operand (rebuilt by the GEMM's
        operand prologue).  before_res: called right before the first kernel that reads ``res`` (a
        residual produced on another stream is joined there, after this unit's GEMM).  defer_apply (training BN + ReLU, no residual): skip the BN-apply + ReLU;
        True returns the BN input z -- the consumer applies scale/shift (ctx[5:7]) itself (the ResNet
        stem's max-pool) --, "act" returns Deferred.affine(z, scale, shift) for the next
        convolution, "bn" (BN without ReLU) Deferred.bn(z, scale, shift) for a residual consumer
        (the ResNet downsample branch, applied inside the block's last BN-apply).  Either way the BN
        output is never materialised.  lazy (training BN, not deferred): return a PendingApply instead
        of running the BN-apply -- for a consumer that computes it in its operand prologue."""
        fuse_apply = self.can_fuse_apply(be, x, train, save)
        if isinstance(x, PendingApply) and not fuse_apply:
            x = x.resolve(be)
        assert x.C == self.Cp, (x, self.Cp)
        P, Q = self.out_hw(x.H, x.W)
        N, dev = x.N, x.device
        wf = self._weight_fwd()
        if defer_apply == "act" and not (train and save and res is None and self.relu and self.bn is not None):
            defer_apply = False
        if defer_apply == "bn" and not (train and save and res is None and not self.relu and self.bn is not None):
            defer_apply = False
        y = None if defer_apply and out is None else (
            out if out is not None else Act.empty(N, P, Q, self.Kp, be.act_dtype, dev))
        bn = self.bn
        if bn is None:
            if before_res is not None and res is not None:
                before_res()
            be.conv_fwd(x, wf, self.Kp, self.R, self.S, self.stride, self.pad, y, bias=self._bias_vec(), res=res,
                        relu=self.relu, kvalid=y.C if y.C < self.Kp else 0)
            return y, ((x, y) if save else None)
        if train:
            if (self.dual and DUAL_DGRAD and save and not defer_apply and self.stride == 1 and self.R == 1
                    and self.S == 1 and N * P * Q >= DUAL_MIN_ROWS and hasattr(be, "dual_weights")):
                # [dy | z]: z on the right, the BN's output gradient later on the left (dy_slot)
                z = Act(torch.empty(N * P * Q, 2 * self.Kp, dtype=be.act_dtype, device=dev), N, P, Q, self.Kp,
                        self.Kp)
            else:
                z = Act.empty(N, P, Q, self.Kp, be.act_dtype, dev)
            vec = torch.empty(4, self.Kp, dtype=be.dt, device=dev)
            scale, shift, mean, invstd = vec[0], vec[1], vec[2], vec[3]
            mom = bn.momentum
            if mom is None:   # cumulative moving average
                mom = 1.0 / float(bn.num_batches_tracked.item())
            fin = (N * P * Q, bn.weight.data if bn.affine else None, bn.bias.data if bn.affine else None,
                   bn.running_mean if bn.track_running_stats else None,
                   bn.running_var if bn.track_running_stats else None, mom, bn.eps, scale, shift, mean, invstd)
            if fuse_apply and self.R == 3:   # the producer's BN-apply inside the streaming 3x3 kernel
                mt = be.conv_mtiles(N, x.H, x.W, x.C, self.Kp, 3, 3, 1, 1)
                stats = torch.empty(mt, 2, self.Kp, dtype=be.dt, device=dev)
                self.arena.wait_buffers()
                be.conv3_fwd_bn_apply(x, wf, self.Kp, z, self._bias_vec(), stats, *fin)
                x.done = True
                x = x.y
            elif fuse_apply:   # the producer's BN-apply runs (and is stored) inside this GEMM
                mt = be.conv_mtiles(N, x.H, x.W, x.C, self.Kp, 1, 1, 1, 0, pro=3)
                stats = torch.empty(mt, 2, self.Kp, dtype=be.dt, device=dev)
                self.arena.wait_buffers()
                be.conv_fwd_bn_apply(x, wf, self.Kp, z, self._bias_vec(), stats, *fin)
                x.done = True
                x = x.y
            else:
                mt = be.conv_mtiles(N, x.H, x.W, x.C, self.Kp, self.R, self.S, self.stride, self.pad,
                                    pro=(1 if x.kind == "affine" else 2) if isinstance(x, Deferred) else 0)
                stats = torch.empty(mt, 2, self.Kp, dtype=be.dt, device=dev)
                # the finalize (in the conv launch itself when possible) reads / updates the running
                # statistics: DDP's asynchronous buffer broadcast must land before the conv
                self.arena.wait_buffers()
                be.conv_fwd_bn(x, wf, self.Kp, self.R, self.S, self.stride, self.pad, z, self._bias_vec(), stats,
                               *fin)
            if defer_apply and save and res is None:
                ctx = (x, z, None, mean, invstd, scale, shift, False, None)
                if defer_apply == "act":
                    return Deferred.affine(z, scale, shift), ctx
                if defer_apply == "bn":
                    return Deferred.bn(z, scale, shift), ctx
                return z, ctx
            # residual units: the backward mask (y > 0) cannot be recomputed from z alone, so keep it
            # as bits (1/16 of y's bytes) for the fused data-gradient epilogue
            mbits = None
            if save and res is not None and self.relu and self.Kp % 8 == 0:
                mbits = torch.empty(y.rows, self.Kp // 8, dtype=torch.uint8, device=dev)
            if before_res is not None and res is not None:
                before_res()
            ctx = (x, z, y, mean, invstd, scale, shift, res is not None, mbits) if save else None
            if lazy and FUSE_APPLY and out is None:
                return PendingApply(y, z, scale, shift, res, self.relu, mbits), ctx
            be.bn_apply(z, scale, shift, res, self.relu, y, mbits=mbits)
            return y, ctx
        # eval: fold BN (and conv bias) into the GEMM epilogue
        if before_res is not None and res is not None:
            before_res()
        invstd = torch.rsqrt(bn.running_var + bn.eps)
        scale = bn.weight.data * invstd if bn.affine else invstd
        shift = (bn.bias.data if bn.affine else 0.0) - bn.running_mean * scale
        if self.bias is not None:
            shift = shift + self.bias.data * scale
        be.conv_fwd(x, wf, self.Kp, self.R, self.S, self.stride, self.pad, y, res=res, scale=scale.contiguous(),
                    shift=shift.contiguous(), relu=self.relu)
        return y, None

    @staticmethod
    def fuse_spec(ctx, z2=None) -> BwdFuse:
        """What a producer of this (trained BN+ReLU) unit's output gradient needs to fuse the
        unit's BN-backward reduction into its data-gradient epilogue."""
        x, z, y, mean, invstd, scale, shift, has_res, mbits = ctx
        if has_res or z2 is not None:
            return BwdFuse(None if mbits is not None else y, z, z2, mbits=mbits)
        return BwdFuse(None, z, None, scale, shift)

    def bwd(self, be, ctx, dy: Act, need_dx=True, dx_res: Act = None, dyr_out: Act = None, ymask: Act = None,
            use_own_mask=True, pre=None, k2=1, fuse_next=None, colsum=False, before_res=None, dx_out: Act = None):
        """Backward of the unit.

        pre:       BN-backward partials already produced by the dgrad epilogue that wrote ``dy``
                   (then ``dy`` is already ReLU-masked; row ``k2`` holds sum dy*z for this BN).
        fuse_next: (mask, z, z2) of the consumer of this unit's dx -- the dgrad epilogue masks dx and
                   emits that consumer's partials; returns (dx, partials) instead of dx.
        colsum:    (without fuse_next) the dgrad epilogue also emits per-tile column sums of dx;
                   returns (dx, partials [tiles][2][C]).
        before_res: called right before the data-gradient GEMM that adds ``dx_res`` (a residual
                   gradient produced on another stream is joined there, after this unit's BN backward).
        dx_out:    where to write dx (the consumer's dy_slot), else a fresh buffer.
        """
        ar = self.arena
        bn = self.bn
        dg_in, dg_w, dg_b = None, None, None   # data-gradient GEMM operand / weights / bias (dual path)
        if bn is not None and need_dx and pre is not None and dyr_out is None and self.dual:
            x, z = ctx[0], ctx[1]
            if (z.off == z.C and z.ld == 2 * z.C and dy.off == 0 and dy.ld == z.ld
                    and dy.buf.data_ptr() == z.buf.data_ptr()):
                # dual: finalize only on this stream; dz for the weight gradient on the side stream
                mean, invstd = ctx[3], ctx[4]
                gam = bn.weight.data if bn.affine else None
                dzd = be.bn_bwd_deferred(dy, z, mean, invstd, gam, ar.grad_flat(bn.weight) if bn.affine else None,
                                         ar.grad_flat(bn.bias) if bn.affine else None, pre=pre, k2=k2)
                with grad_side(be, *bufs(dzd, x)):
                    if bn.affine:
                        ar.ready(bn.weight, bn.bias)
                    if self.bias is not None:
                        ar.ready(self.bias)
                    self._wgrad(be, dzd if (DUAL_WGRAD_PRO and getattr(be, "prologue", False)) else be.materialize(dzd), x)
                    ar.ready(self.conv.weight)
                dg_w, dg_b = be.dual_weights(ar.get_compute(self.h_dg), self.Cp, self.Kp, dzd.k0)
                dg_in = Act(z.buf, z.N, z.H, z.W, 2 * z.C)
                bn = None   # handled
        if dg_in is not None:
            x = ctx[0]
        elif bn is not None:
            x, z, y, mean, invstd = ctx[:5]
            if pre is not None:
                mask = None
            else:
                mask = ymask if ymask is not None else (y if (self.relu and use_own_mask) else None)
            gam = bn.weight.data if bn.affine else None
            dgam = ar.grad_flat(bn.weight) if bn.affine else None
            dbet = ar.grad_flat(bn.bias) if bn.affine else None
            # deferred when the weight gradient is dz's only consumer (need_dx False: the ResNet stem, the UNet input conv) -- then the
            # BN-backward apply pass (read dy, z; write dz) is replaced by the wgrad reading dy and z
            defer = not need_dx and DEFER_BN_WGRAD and getattr(be, "prologue", False)
            if pre is not None and mask is None and dyr_out is None and defer:
                # finalize only: dz = k1 dy + k2 z + k3 is rebuilt inside the wgrad / dgrad GEMMs
                dz = be.bn_bwd_deferred(dy, z, mean, invstd, gam, dgam, dbet, pre=pre, k2=k2)
            else:
                dz = Act.empty(z.N, z.H, z.W, z.C, be.act_dtype, z.device)
                be.bn_bwd(dy, mask, z, mean, invstd, gam, dgam, dbet, dz, dyr_out, pre=pre, k2=k2)
            if self.wgrad_main and WGRAD_TAIL_MAIN and not need_dx:
                # the last weight gradient of the step (the stem): on the main stream, which has
                # nothing left to do, beside the side stream's last weight gradients; the DDP
                # announcements still go through the side stream (ordered after both)
                self._wgrad(be, dz, x)
                with grad_side(be, *bufs(dz, x)):
                    if bn.affine:
                        ar.ready(bn.weight, bn.bias)
                    if self.bias is not None:
                        ar.ready(self.bias)
                    ar.ready(self.conv.weight)
            else:
                with grad_side(be, *bufs(dz, x)):
                    if bn.affine:
                        ar.ready(bn.weight, bn.bias)
                    if self.bias is not None:
                        # d(bias) of a conv followed by training-mode BN is exactly zero (BN removes the mean)
                        ar.ready(self.bias)
                    self._wgrad(be, dz, x)
                    ar.ready(self.conv.weight)
        else:
            x, y = ctx
            assert not self.relu, "ReLU without BN is not used by the engine models"
            dz = dy
            with grad_side(be, *bufs(dz, x)):
                if self.bias is not None:
                    if self.Kp == self.K:
                        be.channel_sum(dz, ar.grad_flat(self.bias))
                    else:
                        tmp = torch.empty(self.Kp, dtype=be.dt, device=dz.device)
                        be.fill_(tmp, 0.0)
                        be.channel_sum(dz, tmp)
                        if getattr(self, "_kidx", None) is None or self._kidx.device != dz.device:
                            self._kidx = torch.arange(self.K, device=dz.device)
                        be.gather_(ar.grad_flat(self.bias), tmp, self._kidx, accumulate=True)
                    ar.ready(self.bias)
                self._wgrad(be, dz, x)
                ar.ready(self.conv.weight)
        if not need_dx:
            return None
        if before_res is not None:
            before_res()
        if dx_out is not None:
            assert (dx_out.N, dx_out.H, dx_out.W, dx_out.C) == (x.N, x.H, x.W, self.Cp), (dx_out, x, self.Cp)
            dx = dx_out
        else:
            dx = Act.empty(x.N, x.H, x.W, self.Cp, be.act_dtype, x.device)
        if dg_in is not None:
            part = be.conv_dgrad(dg_in, dg_w, self.Cp, 1, 1, 1, 0, dx, res=dx_res, fuse=fuse_next, colsum=colsum,
                                 bias=dg_b)
            return (dx, part) if (fuse_next is not None or colsum) else dx
        if (self.K == 1 and self.R == 1 and self.S == 1 and self.stride == 1 and dx_res is None and not colsum
                and fuse_next is not None and fuse_next.scale is not None and fuse_next.z2 is None
                and hasattr(be, "outer_dgrad_bn") and _OUTER_DGRAD):
            # one output channel (the UNet head): the data gradient is an outer product
            part = be.outer_dgrad_bn(be.materialize(dz), ar.get_compute(self.h_dg), self.Kp, dx, fuse_next)
            return dx, part
        part = be.conv_dgrad(dz, ar.get_compute(self.h_dg), self.Cp, self.R, self.S, self.stride, self.pad, dx,
                             res=dx_res, fuse=fuse_next, colsum=colsum)
        return (dx, part) if (fuse_next is not None or colsum) else dx


class S2DConvUnit(ConvUnit):
    """A stride-2 convolution with few input channels (the ResNet 7x7/s2/p3 stem) computed as a
    dense stride-1 convolution over a 2x2 space-to-depth image of the zero-padded input.

    With u = p + a, slot (vh, vw) = (r % 2, s % 2) and a = r // 2, b = s // 2:
        y[p, q] = sum_{r,s,c} x[2p + r - pad, 2q + s - pad, c] w[r, s, c]
                = sum_{a,b,slot,c} X2[p + a, q + b, slot, c] w[2a + vh, 2b + vw, c]
    where X2[u, v, slot, c] = x[2u + vh - pad, 2v + vw - pad, c].  For the 7x7 stem over 3 channels
    the GEMM reduction becomes 4x4 taps x 16 channels = 256 (4 K-steps) instead of 7x7 taps x 8
    padded channels = 392 (7 K-steps), the im2col gather has no out-of-image taps (the padding is
    in the image), and the bf16 input image is half the bytes.  The weight is re-laid out as
    W2[k][a][b][slot * CS + c] (zero for 2a + vh >= R); the weight gradient is computed in that
    layout and scattered back into the [K][R][S][C] gradient slot.  Only the forward and the
    weight gradient exist (the stem's input needs no gradient)."""

    CS = 4   # channels per sub-pixel slot (input channels <= 4)

    def __init__(self, arena: ParamArena, conv, bn=None, relu=True):
        w = conv.weight
        K, Cin, R, S = w.shape
        assert conv.stride == (2, 2) and conv.padding[0] == conv.padding[1] and conv.groups == 1
        assert Cin <= self.CS and conv.dilation == (1, 1)
        self.arena, self.conv, self.bn, self.relu = arena, conv, bn, relu
        self.linear = False
        self.K, self.Cin, self.R0, self.S0, self.pad0 = K, Cin, R, S, conv.padding[0]
        self.R, self.S = (R + 1) // 2, (S + 1) // 2   # taps of the stride-1 conv
        self.stride, self.pad = 1, 0
        self.Cp = 4 * self.CS
        self.Kp = padc(K)
        self.bias = conv.bias
        self._bias_pad = None
        self.h_dg = None
        # one forward compute copy per sub-pixel slot: w[:, :, vh::2, vw::2] -> [Kp][R][S][CS]
        self.h_slots = []
        for vh in (0, 1):
            for vw in (0, 1):
                v = w.data[:, :, vh::2, vw::2]
                self.h_slots.append(arena.add_compute(v, (self.Kp, self.R, self.S, self.CS),
                                                      (K, v.shape[2], v.shape[3], Cin), (0, 2, 3, 1)))
        self.w2 = None
        self._w2idx = None
        arena.post_refresh.append(self._build_w2)
        self._gidx = None

    def _build_w2(self):
        """w2[k][a][b][slot * CS + c] = slot copy [k][a][b][c]: one gather launch from the compute
        copies (index map built once)."""
        ar = self.arena
        comp = ar.compute
        if self._w2idx is None or self._w2idx.device != comp.device:
            k, a, b, sl, c = torch.meshgrid(torch.arange(self.Kp), torch.arange(self.R), torch.arange(self.S),
                                            torch.arange(4), torch.arange(self.CS), indexing="ij")
            offs = torch.tensor([h[0] for h in self.h_slots])
            idx = offs[sl] + (((k * self.R + a) * self.S + b) * self.CS + c)
            self._w2idx = idx.reshape(-1).to(comp.device)
        if self.w2 is None or self.w2.device != comp.device or self.w2.dtype != comp.dtype:
            self.w2 = torch.empty(self.Kp, self.R, self.S, 4 * self.CS, dtype=comp.dtype, device=comp.device)
        ar.backend.gather_(self.w2, comp, self._w2idx)

    def prep_input(self, be, x: torch.Tensor) -> Act:
        N, _, H, W = x.shape
        P = (H + 2 * self.pad0 - self.R0) // 2 + 1
        Q = (W + 2 * self.pad0 - self.S0) // 2 + 1
        return be.s2d(x, self.pad0, P + self.R - 1, Q + self.S - 1, self.CS)

    def fwd(self, be, x: Act, train: bool, res: Act = None, out: Act = None, save=True, defer_apply=False):
        if self.w2 is None:
            self._build_w2()
        return super().fwd(be, x, train, res=res, out=out, save=save, defer_apply=defer_apply)

    def _weight_fwd(self):
        return self.w2.view(-1)

    def _wgrad(self, be, dz: Act, x: Act):
        K, R, S, CT = self.K, self.R, self.S, 4 * self.CS
        g2 = torch.empty(K * R * S * CT, dtype=be.dt, device=dz.device)
        be.fill_(g2, 0.0)
        # g2 is read right below: its reduction runs now, on this stream (the queued ones stay queued)
        bypass = getattr(be, "wgrad_bypass", None)
        if bypass is not None:
            bypass(True)
        try:
            be.conv_wgrad(dz, x, R, S, 1, 0, g2, CT, K)
        finally:
            if bypass is not None:
                bypass(False)
        if self._gidx is None or self._gidx.device != dz.device:
            # grad[k][r][s][c] <- g2[k][r // 2][s // 2][((r % 2) * 2 + s % 2) * CS + c]
            k, r, s_, c = torch.meshgrid(torch.arange(K), torch.arange(self.R0), torch.arange(self.S0),
                                         torch.arange(self.Cin), indexing="ij")
            idx = (((k * R + r // 2) * S + s_ // 2) * CT + ((r % 2) * 2 + s_ % 2) * self.CS + c)
            self._gidx = idx.reshape(-1).to(dz.device)
        be.gather_(self.arena.grad_flat(self.conv.weight), g2, self._gidx, accumulate=True)


class ConvTUnit:
    """ConvTranspose2d(k=2, s=2) with bias (UNet up-sampling, reference model.py:36-38)."""

    def __init__(self, arena: ParamArena, convT: nn.ConvTranspose2d):
        self.arena, self.m = arena, convT
        Ci, Co, kh, kw = convT.weight.shape
        assert (kh, kw) == (2, 2) and convT.stride == (2, 2) and convT.padding == (0, 0)
        self.Cin, self.Cout = Ci, Co
        self.Cip, self.Cop = padc(Ci), padc(Co)
        w = convT.weight
        # forward layout [Cout][i][j][Cin]; data-grad layout [Cin][i][j][Cout] (a stride-2 2x2 conv)
        self.h_fwd = arena.add_compute(w, (self.Cop, 2, 2, self.Cip), (Co, 2, 2, Ci), (1, 2, 3, 0))
        self.h_dg = arena.add_compute(w, (self.Cip, 2, 2, self.Cop), (Ci, 2, 2, Co), (0, 2, 3, 1))

    def fwd(self, be, x: Act, out: Act):
        be.convT_fwd(x, self.arena.get_compute(self.h_fwd), self.Cop, out,
                     self.m.bias.data if self.m.bias is not None else None)
        return x

    def bwd(self, be, x: Act, dout: Act, fuse_next=None, bias_part=None):
        """fuse_next (BwdFuse of the BN+ReLU unit that produced x): the data gradient is written
        ReLU-masked with that BN's backward partials -> returns (dx, partials).  bias_part: per-tile
        column sums of ``dout`` already produced by the GEMM that wrote it ([tiles][ns][C] partials,
        row 0 = sum dout, channels [0, Cout) = this up-sampling's slice); the bias gradient is then
        their column sum (one reduction launch over tiles rows) instead of another pass over ``dout``."""
        ar = self.arena
        with grad_side(be, dout.buf, x.buf, bias_part):
            if self.m.bias is not None:
                src = dout
                if bias_part is not None:
                    T = bias_part.shape[0]
                    src = Act(bias_part.reshape(T, -1), T, 1, 1, self.Cop)   # ld = ns * C: row 0 per tile
                if self.Cop == self.Cout:
                    be.channel_sum(src, ar.grad_flat(self.m.bias))
                else:
                    tmp = torch.empty(self.Cop, dtype=be.dt, device=dout.device)
                    be.fill_(tmp, 0.0)
                    be.channel_sum(src, tmp)
                    if getattr(self, "_kidx", None) is None or self._kidx.device != dout.device:
                        self._kidx = torch.arange(self.Cout, device=dout.device)
                    be.gather_(ar.grad_flat(self.m.bias), tmp, self._kidx, accumulate=True)
                ar.ready(self.m.bias)
            # dW[ci][i][j][co] = sum_pix x[pix][ci] * dout[2p+i, 2q+j][co]: the wgrad of a 2x2/s2 conv
            be.conv_wgrad(x, dout, 2, 2, 2, 0, ar.grad_flat(self.m.weight), self.Cout, self.Cin)
            ar.ready(self.m.weight)
        dx = Act.empty(x.N, x.H, x.W, self.Cip, be.act_dtype, x.device)
        if fuse_next is not None:
            return dx, be.conv_fwd_bnbwd(dout, ar.get_compute(self.h_dg), self.Cip, 2, 2, 2, 0, dx, fuse_next)
        be.conv_fwd(dout, ar.get_compute(self.h_dg), self.Cip, 2, 2, 2, 0, dx)
        return dx


class _EngineFn(torch.autograd.Function):
    """roctx ranges "dlmpi.forward" / "dlmpi.backward" (rocprofv3 --marker-trace) bracket the
    schedules; DDP bucket launches and optimizers add their own ranges."""

    @staticmethod
    def forward(ctx, mod, x, anchor):
        with trace_range(f"dlmpi.forward[{type(mod).__name__}]"):
            out, state = mod._engine_forward(x, train=True, save=True)
            mod._arena.end_cast()   # the side-stream weight recast joined (normally long since, lazily)
        ctx.mod = mod
        ctx.state = state
        ctx.aux_on = getattr(mod._be, "aux_on", None)   # the backward uses the forward's stream plan
        return out

    @staticmethod
    def backward(ctx, gout):
        mod = ctx.mod
        state = ctx.state
        ctx.state = None
        if ctx.aux_on is not None:
            mod._be.aux_on = ctx.aux_on
        with trace_range(f"dlmpi.backward[{type(mod).__name__}]"):
            prof = BWD_PROFILER   # bench.py --pyprof: the backward runs on autograd's worker thread
            if prof is not None:
                prof.enable()
            be = mod._be
            # weight-gradient split reductions are queued and launched in batches (at DDP bucket
            # launches, every kWgradBatch gradients, and below): a handful of launches per step
            defer = getattr(be, "wgrad_defer", None)   # (the shadow backend checks every call: never)
            if defer is not None:
                defer(True)
            try:
                mod._engine_backward(state, gout)
            except BaseException:
                # a failed backward (e.g. a capture torn down inside it): its queued reductions point at
                # slabs that were never computed and at abandoned streams -- drop them, never launch them
                if defer is not None:
                    be.wgrad_discard()
                raise
            try:
                side = getattr(be, "side_stream", None)
                if side is not None:
                    if defer is not None:   # the queue's tail on the side stream, beside the main
                        with torch.cuda.stream(side):   # stream's last work (the stem's weight gradient)
                            be.wgrad_flush()
                    torch.cuda.current_stream().wait_stream(side)   # every gradient final before the optimizer
            finally:
                if defer is not None:
                    defer(False)   # (flushes what is still queued -- nothing with a side stream)
            if prof is not None:
                prof.disable()
            held = getattr(mod._be, "held", None)
            if held:   # buffers read on the side stream: freed now, ordered after it (grad_side)
                held.clear()
        with trace_range("dlmpi.ddp_finalize"):
            mod._arena.end_backward()
        return None, None, None


# a cProfile.Profile enabled around every engine backward (bench.py --pyprof), else None
BWD_PROFILER = None


class EngineModule(nn.Module):
    """Base class: lazily builds the backend + arena on the device of the parameters."""

    def __init__(self):
        super().__init__()
        self._arena = None
        self._be = None
        self._anchor = torch.zeros(0, requires_grad=True)
        # BN-backward reductions fused into the producing dgrad epilogue (False: separate passes)
        self.fuse_bn_bwd = True
        self.precision = "bf16"    # "fp32": fp32 activations / weights in the same kernels (set before first use)

    def engine_setup(self, device=None):
        if device is None:
            device = next(self.parameters()).device
        device = torch.device(device)
        if device.type == "cuda" and device.index is None:   # "cuda" and "cuda:0" are one arena
            device = torch.device("cuda", torch.cuda.current_device())
        if self._arena is not None and self._arena.device == device and self._arena.valid():
            return self._arena
        self._be = make_backend(device, next(self.parameters()).dtype, self.precision)
        self._arena = ParamArena(self, device, self._be, order_names=self._grad_ready_names())
        self._build_units(self._arena)
        self._arena.refresh(force=True)
        return self._arena

    @property
    def arena(self) -> ParamArena:
        return self.engine_setup()

    def _build_units(self, arena):
        raise NotImplementedError

    def _grad_ready_names(self):
        """Parameter names in the order the engine backward announces them ready (the flat
        gradient layout, hence the DDP bucket order).  None: reverse registration order."""
        return None

    @staticmethod
    def unit_ready_names(conv: str, bn: str = None, conv_bias=False):
        """The ``ready`` order of one ConvUnit (ConvUnit.bwd): BN weight, BN bias, conv bias, conv
        weight; a ConvTUnit / bias-only unit: bias, weight."""
        out = [f"{bn}.weight", f"{bn}.bias"] if bn else []
        if conv_bias:
            out.append(f"{conv}.bias")
        return out + [f"{conv}.weight"]

    def forward(self, x):
        self.engine_setup(x.device)
        be = self._be
        if hasattr(be, "aux_min_pixels"):   # auxiliary streams only for steps big enough to use them
            be.aux_on = x.shape[0] * x.shape[-2] * x.shape[-1] >= be.aux_min_pixels
        self._arena.refresh(split=True)   # (the rest of a split recast goes out at the model's launch_cast)
        if self.training and torch.is_grad_enabled():
            self._arena.attach_grads()
            if self._arena.ibuf_total:   # every BatchNorm's num_batches_tracked, one launch
                be.add_i64_(self._arena.ibuf, 1)
            return _EngineFn.apply(self, x, self._anchor)
        with torch.no_grad():
            if self.training and self._arena.ibuf_total:
                be.add_i64_(self._arena.ibuf, 1)
            out, _ = self._engine_forward(x, train=self.training, save=False)
            self._arena.end_cast()
        return out

    # implemented by the model
    def _engine_forward(self, x, train, save):
        raise NotImplementedError

    def _engine_backward(self, state, gout):
        raise NotImplementedError
