"""Compute backends of the execution engine.

* :class:`NativeBackend` -- the product path: bf16 NHWC activations, every op is one of our
  gfx950 HIP kernels (``_C``), launched on the current HIP stream (graph-capturable).  With
  ``act_dtype=torch.float32`` the same kernels run instantiated for fp32 storage (fp32 MFMA
  v_mfma_f32_16x16x4_f32 in the GEMMs): the ``--precision fp32`` path.
* :class:`RefBackend` -- fp32 torch reference of exactly the same op set and semantics.  It runs
  on CPU (CPU test-suite, gloo multi-process tests) and is the numerics oracle for the kernels.

Both expose the same methods; the engine (models/*) is written once against this interface.
"""
from __future__ import annotations

import os
import weakref
import struct

import torch
import torch.nn.functional as F

from .act import Act, Deferred


# --------------------------------------------------------------------------------------------
_AUX_STREAMS = {}
_BACKENDS = weakref.WeakSet()   # NativeBackend instances (their aux stream references)


def _new_aux_stream(idx, C, role):
    with torch.cuda.device(idx):
        # a raw HIP stream, not a torch pool stream: if a failed hipGraph capture leaves it stuck in
        # capture mode it is abandoned (replace_poisoned_aux_streams), never handed out again
        st = torch.cuda.ExternalStream(C.create_stream(), device=torch.device("cuda", idx))
        C.set_aux_stream(st.cuda_stream, role)
    return st


def _aux_stream(device, C, role):
    """Auxiliary streams, one per (device, role), shared by every backend instance: role 1 = the
    weight-gradient side stream, role 2 = the residual-branch stream.  The kernels keep a separate
    last-arriver ticket array per role (bn.hip:fin_tickets)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    st = _AUX_STREAMS.get((idx, role))
    if st is None:
        st = _AUX_STREAMS[(idx, role)] = _new_aux_stream(idx, C, role)
    return st


def replace_poisoned_aux_streams() -> int:
    """After a failed hipGraph capture (utils/graphs.py): every auxiliary stream that the capture
    had forked and that HIP left in capture mode is replaced by a fresh one, in the registry, in the
    kernels' role table and in every live backend.  Returns the number replaced."""
    if not _AUX_STREAMS:
        return 0
    from .._ext import native

    C = native()
    n = 0
    for (idx, role), st in list(_AUX_STREAMS.items()):
        if not C.stream_capturing(st.cuda_stream):
            continue
        fresh = _AUX_STREAMS[(idx, role)] = _new_aux_stream(idx, C, role)
        for be in list(_BACKENDS):
            if be._side is st:
                be._side = fresh
            if be._branch is st:
                be._branch = fresh
        n += 1
    return n


class NativeBackend:
    name = "native"
    use_side_stream = True     # False: weight gradients on the current stream (A/B)
    use_branch_stream = True   # False: the ResNet downsample branch on the current stream (A/B)
    dt = torch.float32

    def __init__(self, device, act_dtype=torch.bfloat16):
        from .._ext import native

        if act_dtype not in (torch.bfloat16, torch.float32):
            raise ValueError(f"native activations are bf16 or fp32, got {act_dtype}")
        self.C = native()
        self.device = torch.device(device)
        self.act_dtype = act_dtype
        self.f32 = act_dtype == torch.float32
        # the GEMM operand prologues (deferred BN passes) are instantiated for bf16 only
        self.prologue = not self.f32
        self._cast_cache = {}
        self.held = []   # buffers read on the side stream, dropped at the backward's join (engine.grad_side)
        # parameter-gradient work (weight-gradient GEMMs + split reductions, DDP bucket launches)
        # runs on this side stream, off the data-gradient critical path (models/engine.py:grad_side);
        self._side = _aux_stream(self.device, self.C, 1) if self.use_side_stream \
            else None
        # independent residual branches (the ResNet downsample conv + BN) run on this stream beside
        # the main branch, forward and backward (models/resnet.py:_BlockExec)
        self._branch = _aux_stream(self.device, self.C, 2) \
            if self.use_branch_stream else None
        # The auxiliary streams pay off when kernels are long enough to leave idle CUs beside each
        # other; a launch-bound step (ResNet-18 on 32x32 CIFAR: ~300 kernels of a few us) only pays
        # their per-launch event traffic (measured 31-36k vs 58-60k img/s eager).  The engine turns
        # them on per step when the input has >= aux_min_pixels (N*H*W) pixels
        # (EngineModule.forward; DLMPI_AUX_MIN_PIXELS, default 1M: on for ResNet-50 bs 256 at 224^2 and
        # UNet bs 16 at 512^2, off for CIFAR).
        self.aux_min_pixels = int(os.environ.get("DLMPI_AUX_MIN_PIXELS", str(1 << 20)))
        self.aux_on = True
        _BACKENDS.add(self)

    @property
    def side_stream(self):
        return self._side if self.aux_on else None

    @side_stream.setter
    def side_stream(self, s):
        self._side = s

    @property
    def branch_stream(self):
        return self._branch if self.aux_on else None

    @branch_stream.setter
    def branch_stream(self, s):
        self._branch = s

    # ---------------- conv family ----------------
    # the weight-gradient GEMM consumes ops.act.Deferred operands directly in its operand prologues
    # (bf16); the forward / data-gradient GEMMs take them materialized (one elementwise pass)
    prologue = True

    @staticmethod
    def _pro(op):
        """(source Act, prologue mode, k0, k1, Z buffer, Z ld, Z offset) of a GEMM operand."""
        if not isinstance(op, Deferred):
            return op, 0, None, None, None, 0, 0
        if op.kind == "affine":
            return op.src, 1, op.k0, op.k1, None, 0, 0
        return op.src, 2, op.k0, None, op.z.buf, op.z.ld, op.z.off

    def materialize(self, d) -> Act:
        """The stored form of a Deferred operand (one elementwise pass)."""
        if not isinstance(d, Deferred):
            return d
        src = d.src
        out = Act.empty(src.N, src.H, src.W, src.C, self.act_dtype, src.device)
        if d.kind in ("affine", "bn"):
            self.bn_apply(src, d.k0, d.k1, None, d.kind == "affine", out)
        else:
            self.C.bn_bwd_apply(src.buf, src.ld, src.off, None, 0, 0, d.z.buf, d.z.ld, d.z.off, src.rows, src.C,
                                d.k0, out.buf, None)
        return out

    def conv_mtiles(self, N, H, W, C, K, R, S, stride, pad, pro=0):
        """BN-statistics rows the forward conv will write; pro: 3 = the consumer GEMM of a pending
        residual BN-apply (conv_fwd_bn_apply), else 0."""
        return self.C.conv2d_fwd_mtiles_pro(N, H, W, C, K, R, S, stride, pad, 0, 3 if pro == 3 else 0,
                                            int(self.f32))

    def conv_fwd(self, x, w, K, R, S, stride, pad, y: Act, bias=None, res: Act = None, scale=None,
                 shift=None, relu=False, stats=None, kvalid=0):
        """Returns the number of BN-statistics rows written (stats given).  A Deferred.affine input is
        materialized, except for the <= 4-output 1x1 head, which applies it on the fly."""
        if (isinstance(x, Deferred) and x.kind == "affine" and R == 1 and S == 1 and stride == 1 and pad == 0
                and 0 < kvalid <= 4 and res is None and scale is None and not relu and stats is None
                and not self.f32 and x.C in (16, 32, 64, 128, 256, 512) and self.C.head1x1_on()):
            z = x.src
            self.C.conv1x1_head_affine(z.buf, z.N, z.H, z.W, z.C, z.ld, z.off, w, w.shape[-1], int(kvalid), x.k0,
                                       x.k1, y.buf, y.ld, y.off, bias)
            return 0
        x = self.materialize(x)
        return self.C.conv2d_fwd(x.buf, x.N, x.H, x.W, x.C, x.ld, x.off, w, K, R, S, stride, pad, y.buf, y.ld,
                                 y.off, bias, res.buf if res is not None else None,
                                 res.ld if res is not None else 0, res.off if res is not None else 0, scale, shift,
                                 bool(relu), stats, 0, int(kvalid), 0)

    def conv_fwd_bn(self, x, w, K, R, S, stride, pad, z: Act, bias, stats, count, gamma, beta, rm, rv, momentum,
                    eps, scale, shift, save_mean, save_invstd):
        """conv_fwd into z with the BN-statistics epilogue AND the training-BN finalize of those
        statistics (scale / shift / mean / invstd / running stats): the conv, then the column-reduce +
        finalize launch."""
        x = self.materialize(x)
        self.C.conv2d_fwd_bn(x.buf, x.N, x.H, x.W, x.C, x.ld, x.off, w, K, R, S, stride, pad, z.buf, z.ld, z.off,
                             bias, stats, 0, None, None, None, 0, 0, float(count), gamma, beta, rm, rv,
                             float(momentum), float(eps), scale, shift, save_mean, save_invstd)

    def conv_fwd_bn_apply(self, xp, w, K, z: Act, bias, stats, count, gamma, beta, rm, rv, momentum, eps, scale,
                          shift, save_mean, save_invstd):
        """conv_fwd_bn (1x1, stride 1) whose input is a pending BN-apply (engine.PendingApply: y =
        relu(z * scale + shift + res), res an Act or a Deferred.bn): the conv's operand prologue computes y,
        uses it and stores it with its ReLU mask bits (pro 3) -- no separate apply pass."""
        x, res = xp.z, xp.res
        rs = rh = None
        if isinstance(res, Deferred):
            assert res.kind == "bn", res
            res, rs, rh = res.src, res.k0, res.k1
        y = xp.y
        self.C.conv2d_fwd_bn_apply(x.buf, x.N, x.H, x.W, x.C, x.ld, x.off, w, K, z.buf, z.ld, z.off, bias, stats,
                                   xp.scale, xp.shift, res.buf, res.ld, res.off, rs, rh, y.buf, y.ld, y.off, xp.mbits,
                                   float(count), gamma, beta, rm, rv, float(momentum), float(eps), scale, shift,
                                   save_mean, save_invstd)

    def conv3_pro_ok(self, z: Act, y: Act) -> bool:
        """The fused BN-apply + streaming 3x3 launch applies to this input z / applied output y."""
        return bool(self.C.conv3_pro_ok(z.N, z.H, z.W, z.C, 64, z.ld, z.off, y.ld, y.off, y.ld, y.off))

    def conv3_fwd_bn_apply(self, xp, w, K, z: Act, bias, stats, count, gamma, beta, rm, rv, momentum, eps, scale,
                           shift, save_mean, save_invstd):
        """conv_fwd_bn of a 3x3 / s1 / p1 64 -> 64 conv whose input is a pending BN-apply + ReLU without
        residual (engine.PendingApply): the streaming 3x3 kernel applies it to its staged input tiles and
        stores it to xp.y (each pixel once) -- no separate apply pass.  Falls back to the apply pass +
        conv_fwd_bn where the fused launch does not apply."""
        x, y = xp.z, xp.y
        r = self.C.conv3x3_fwd_bn_apply(x.buf, x.N, x.H, x.W, x.ld, x.off, w, z.buf, z.ld, z.off, bias, stats,
                                        xp.scale, xp.shift, y.buf, y.ld, y.off, float(count), gamma, beta, rm, rv,
                                        float(momentum), float(eps), scale, shift, save_mean, save_invstd)
        if r < 0:
            self.bn_apply(xp.z, xp.scale, xp.shift, None, True, y)
            self.conv_fwd_bn(y, w, K, 3, 3, 1, 1, z, bias, stats, count, gamma, beta, rm, rv, momentum, eps, scale,
                             shift, save_mean, save_invstd)

    def conv_fwd_bnbwd(self, x: Act, w, K, R, S, stride, pad, y: Act, fuse):
        """Forward conv producing the gradient of relu(BN(z)) (fuse = BwdFuse(None, z, None, scale,
        shift)): masked in the epilogue, BN-backward partials [tiles][2][K] returned."""
        z = fuse.z
        return self.C.conv2d_fwd_bnbwd(x.buf, x.N, x.H, x.W, x.C, x.ld, x.off, w, K, R, S, stride, pad, y.buf, y.ld,
                                       y.off, z.buf, z.ld, z.off, fuse.scale, fuse.shift)

    def conv_dgrad(self, dy: Act, wT, C, R, S, stride, pad, dx: Act, res: Act = None, fuse=None, colsum=False,
                   bias=None):
        """fuse = BwdFuse(mask, z, z2, scale, shift): dx is the gradient of relu(BN(z) [+ BN2(z2)]);
        the epilogue applies the ReLU mask (y > 0, or z*scale + shift > 0 without a residual) and
        returns BN-backward partials [tiles][2|3][C].  colsum (no fuse): returns per-tile
        {sum dx, sum dx^2} [tiles][2][C] of the stored dx instead.  bias: fp32 [C] added to the
        GEMM result first (the dual 1x1 data gradient's W . k3 term)."""
        m, z, z2, sc, sh, mb = fuse if fuse is not None else (None, None, None, None, None, None)

        def t(a):
            return (a.buf, a.ld, a.off) if a is not None else (None, 0, 0)

        dy = self.materialize(dy)
        return self.C.conv2d_dgrad_pro(dy.buf, dy.N, dy.H, dy.W, dy.C, dy.ld, dy.off, wT, C, R, S, stride, pad, dx.H,
                                       dx.W, dx.buf, dx.ld, dx.off, *t(res), *t(m), *t(z), *t(z2), sc, sh, mb,
                                       bool(colsum and fuse is None), 0, None, None, None, 0, 0, bias)

    def dual_weights(self, wT, C, K, coef):
        """[dy | z] weights of the dual 1x1 data gradient (engine.ConvUnit, dual path): w2 [C][2K] =
        {wT * coef[0], wT * coef[1]} in the storage type, b [C] = wT . coef[2] in fp32."""
        w2 = torch.empty(C, 2 * K, dtype=self.act_dtype, device=self.device)
        b = torch.empty(C, dtype=torch.float32, device=self.device)
        self.C.dual_dgrad_weights(wT, C, K, coef, w2, b)
        return w2, b

    def convT_fwd(self, x: Act, wf, Cout, y: Act, bias=None):
        self.C.convT2x2_fwd(x.buf, x.N, x.H, x.W, x.C, x.ld, x.off, wf, Cout, y.buf, y.ld, y.off, bias)

    def wgrad_defer(self, on: bool):
        """Queue weight-gradient split reductions (on) / flush the queue and launch them at once
        again (off); ops.cpp wgrad_reduce_or_defer."""
        self.C.set_wgrad_defer(bool(on))

    def wgrad_flush(self):
        self.C.wgrad_flush()

    def wgrad_discard(self):
        """Drop the queued reductions of a failed backward and turn deferral off."""
        self.C.wgrad_discard()

    def wgrad_bypass(self, on: bool):
        """Reduce the next weight gradients right away (their consumer reads them next), queue kept."""
        self.C.set_wgrad_bypass(bool(on))

    def conv_wgrad(self, dy, x, R, S, stride, pad, grad, Creal, Ko_real):
        direct = R == 1 and S == 1 and stride == 1 and pad == 0
        if isinstance(dy, Deferred) and isinstance(x, Deferred) or (isinstance(x, Deferred) and not direct):
            x = self.materialize(x)   # (prologue combinations the kernel is not built for: dlmpi_wgrad_pro_ok)
        dy, pa, ca, _, zb, zld, zoff = self._pro(dy)
        x, pb, sb, hb, _, _, _ = self._pro(x)
        assert pa in (0, 2) and pb in (0, 1)
        self.C.conv2d_wgrad_pro(dy.buf, dy.ld, dy.off, dy.C, x.buf, x.N, x.H, x.W, x.C, x.ld, x.off, R, S, stride,
                                pad, dy.H, dy.W, grad, Creal, Ko_real, pa, ca, zb, zld, zoff, pb, sb, hb)

    # ---------------- batch norm ----------------
    def bn_finalize(self, stats, ntiles, C, count, gamma, beta, rm, rv, momentum, eps, scale, shift, save_mean,
                    save_invstd):
        self.C.bn_finalize(stats, ntiles, C, float(count), gamma, beta, rm, rv, float(momentum), float(eps), scale,
                           shift, save_mean, save_invstd)

    def bn_stats(self, x: Act):
        nblk = self.C.reduce_blocks(x.rows, x.C)
        part = torch.empty(nblk, 2, x.C, dtype=torch.float32, device=x.device)
        self.C.bn_stats(x.buf, x.rows, x.C, x.ld, x.off, part, nblk)
        return part, nblk

    def bn_apply(self, x: Act, scale, shift, res, relu, y: Act, mbits=None):
        """res: an Act, or a Deferred.bn residual (applied on the fly, never materialised)."""
        rs = rh = None
        if isinstance(res, Deferred):
            assert res.kind == "bn", res
            res, rs, rh = res.src, res.k0, res.k1
        self.C.bn_apply(x.buf, x.ld, x.off, x.rows, x.C, scale, shift, res.buf if res is not None else None,
                        res.ld if res is not None else 0, res.off if res is not None else 0, bool(relu), y.buf, y.ld,
                        y.off, mbits, rs, rh)

    def bn_bwd_deferred(self, dy: Act, x: Act, mean, invstd, gamma, dgamma, dbeta, pre, k2=1) -> Deferred:
        """BN backward from the producer's fused partials (``pre``): finalize only (dgamma, dbeta and
        the apply coefficients); dz stays a Deferred operand of the unit's wgrad / dgrad GEMMs."""
        coef = torch.empty(3, x.C, dtype=torch.float32, device=x.device)
        self.C.bn_bwd_finalize_fused(pre, k2, x.C, float(x.rows), gamma, mean, invstd, dgamma, dbeta, coef)
        return Deferred.bnbwd(dy, x, coef)

    def bn_bwd(self, dy: Act, ymask: Act, x: Act, mean, invstd, gamma, dgamma, dbeta, dx: Act, dyr_out: Act = None,
               pre=None, k2=1):
        M, Cc = x.rows, x.C
        coef = torch.empty(3, Cc, dtype=torch.float32, device=x.device)
        if pre is not None:   # partials {sum dyr, sum dyr*z} came from the producer's dgrad epilogue
            assert ymask is None
            self.C.bn_bwd_finalize_fused(pre, k2, Cc, float(M), gamma, mean, invstd, dgamma, dbeta, coef)
        else:
            nblk = self.C.reduce_blocks(M, Cc)
            part = torch.empty(nblk, 2, Cc, dtype=torch.float32, device=x.device)
            self.C.bn_bwd_reduce(dy.buf, dy.ld, dy.off, ymask.buf if ymask is not None else None,
                                 ymask.ld if ymask is not None else 0, ymask.off if ymask is not None else 0, x.buf,
                                 x.ld, x.off, M, Cc, mean, invstd, part, nblk)
            self.C.bn_bwd_finalize(part, nblk, Cc, float(M), gamma, mean, invstd, dgamma, dbeta, coef)
        assert dx.ld == Cc and dx.off == 0
        if dyr_out is not None:
            assert dyr_out.ld == Cc and dyr_out.off == 0
        self.C.bn_bwd_apply(dy.buf, dy.ld, dy.off, ymask.buf if ymask is not None else None,
                            ymask.ld if ymask is not None else 0, ymask.off if ymask is not None else 0, x.buf, x.ld,
                            x.off, M, Cc, coef, dx.buf, dyr_out.buf if dyr_out is not None else None)

    def channel_sum(self, x: Act, out_acc):
        self.C.channel_sum(x.buf, x.rows, x.C, x.ld, x.off, out_acc)

    # ---------------- pooling / layout ----------------
    def maxpool_fwd(self, x: Act, k, s, p, y: Act, bn=None, store: Act = None):
        """bn = (scale, shift): pool relu(x * scale + shift) -- a BN-apply + ReLU fused into the pool;
        store (2x2 / s2 only): also write that applied input there (the BN-apply's own output)."""
        idx = torch.empty(y.rows * y.C, dtype=torch.uint8, device=x.device)
        assert y.ld == y.C and y.off == 0
        sc, sh = bn if bn is not None else (None, None)
        self.C.maxpool_fwd(x.buf, x.N, x.H, x.W, x.C, x.ld, x.off, k, s, p, y.buf, idx, y.H, y.W, sc, sh,
                           store.buf if store is not None else None, store.ld if store is not None else 0,
                           store.off if store is not None else 0)
        return idx

    def maxpool_bwd(self, dy: Act, idx, x: Act, k, s, p, dx: Act, add: Act = None, fuse=None):
        """fuse = BwdFuse(None, z, scale=, shift=): dx is the gradient of relu(BN(z)); it is written
        masked and the BN-backward partials are returned (for bn_bwd(pre=...)).  add: a second
        gradient of the pool input, summed in before the mask."""
        if fuse is not None:
            assert fuse.scale is not None and dx.ld == dx.C and fuse.z.ld == fuse.z.C
            assert dy.ld == dy.C and dy.off == 0 and dx.off == 0 and fuse.z.off == 0
            return self.C.maxpool_bwd_bn(dy.buf, idx, x.N, x.H, x.W, x.C, k, s, p, dy.H, dy.W, fuse.z.buf,
                                         fuse.scale, fuse.shift, add.buf if add is not None else None,
                                         add.ld if add is not None else 0, add.off if add is not None else 0,
                                         dx.buf)
        self.C.maxpool_bwd(dy.buf, idx, x.N, x.H, x.W, x.C, k, s, p, dy.H, dy.W, add.buf if add is not None else None,
                           add.ld if add is not None else 0, add.off if add is not None else 0, dx.buf, dx.ld, dx.off)

    def outer_dgrad_bn(self, dy: Act, wT, ldw, dx: Act, fuse):
        """Data gradient of a 1x1 conv with one output channel: dx[m, c] = dy[m, 0] * wT[c * ldw],
        as the masked gradient of relu(BN(z)) (fuse = BwdFuse(None, z, None, scale, shift)); returns
        the BN-backward partials [blocks][2][C]."""
        assert fuse.scale is not None and fuse.z2 is None and fuse.mask is None and fuse.mbits is None
        assert dx.ld == dx.C and dx.off == 0 and fuse.z.ld == fuse.z.C and fuse.z.off == 0
        return self.C.outer_dgrad_bn(dy.buf[:, dy.off:], dy.ld, dx.rows, dx.C, wT, ldw, fuse.z.buf, fuse.scale,
                                     fuse.shift, dx.buf)

    def avgpool_fwd(self, x: Act, y: Act):
        self.C.avgpool_fwd(x.buf, x.N, x.H * x.W, x.C, y.buf)

    def avgpool_bwd(self, dy: Act, dx: Act):
        self.C.avgpool_bwd(dy.buf, dx.N, dx.H * dx.W, dx.C, dx.buf)

    def nchw_to_nhwc(self, x: torch.Tensor, Cpad) -> Act:
        N, Cc, H, W = x.shape
        x = x.contiguous().to(self.dt)
        y = Act.empty(N, H, W, Cpad, self.act_dtype, x.device)
        self.C.nchw_to_nhwc(x, N, Cc, H, W, Cpad, y.buf)
        return y

    def s2d(self, x: torch.Tensor, pad, U, V, CS) -> Act:
        """2x2 space-to-depth of the zero-padded NCHW image -> [N, U, V, 4*CS] NHWC."""
        N, Cc, H, W = x.shape
        x = x.contiguous().to(self.dt)
        y = Act.empty(N, U, V, 4 * CS, self.act_dtype, x.device)
        self.C.s2d_nchw(x, N, Cc, H, W, pad, U, V, CS, y.buf)
        return y

    def upsample_fwd(self, x: Act, y: Act):
        self.C.upsample2x_fwd(x.buf, x.N, x.H, x.W, x.C, x.ld, x.off, y.buf, y.ld, y.off)

    def upsample_bwd(self, dy: Act, dx: Act):
        assert dx.ld == dx.C and dx.off == 0
        self.C.upsample2x_bwd(dy.buf, dx.N, dx.H, dx.W, dx.C, dy.ld, dy.off, dx.buf)

    # ---------------- weights ----------------
    def cast_weights(self, entries, total, dst_flat):
        """entries: list of (src fp32 tensor view, dst offset, dims[4], valid[4], src strides[4])."""
        key = (id(entries), len(entries), dst_flat.data_ptr())
        ent = self._cast_cache.get(key)
        if ent is None or ent[0] is not entries:
            blob = bytearray()
            base, esz = dst_flat.data_ptr(), dst_flat.element_size()
            assert dst_flat.dtype == self.act_dtype
            bmap = []
            for k, (src, doff, d, v, st) in enumerate(entries):
                blob += struct.pack("<QQ4i4i4qq", src.data_ptr(), base + esz * doff, *d, *v, *st, doff)
                # ~one block per 4096 destination elements (one 64x64 tile of the transpose path)
                nb = max(1, min(1024, -(-d[0] * d[1] * d[2] * d[3] // 4096)))
                bmap += [(k, j, nb, 0) for j in range(nb)]
            dev = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(self.device)
            bm = torch.tensor(bmap, dtype=torch.int32).to(self.device)
            self._cast_cache[key] = ent = (entries, dev, bm)
        self.C.cast_weights(ent[1], ent[2], self.f32)

    # ---------------- losses / eval ----------------
    def ce_fwd(self, logits, labels):
        N, K = logits.shape
        loss_rows = torch.empty(N, dtype=torch.float32, device=logits.device)
        lse = torch.empty(N, dtype=torch.float32, device=logits.device)
        loss = torch.empty((), dtype=torch.float32, device=logits.device)
        self.C.softmax_ce_fwd(logits, logits.stride(0), labels, N, K, loss_rows, lse, loss)
        return loss, lse

    def ce_bwd(self, logits, labels, lse, go):
        N, K = logits.shape
        d = torch.empty(N, K, dtype=torch.float32, device=logits.device)
        self.C.softmax_ce_bwd(logits, logits.stride(0), labels, lse, N, K, K, go, 1.0 / N, d)
        return d

    def bce_fwd(self, logits, target):
        loss = torch.empty((), dtype=torch.float32, device=logits.device)
        self.C.bce_fwd(logits, 1, target, logits.numel(), loss)
        return loss

    def bce_bwd(self, logits, target, go):
        d = torch.empty_like(logits, memory_format=torch.contiguous_format)
        self.C.bce_bwd(logits, 1, target, logits.numel(), go, 1.0 / logits.numel(), d)
        return d

    def argmax_correct(self, logits, labels):
        c = torch.zeros(1, dtype=torch.int32, device=logits.device)
        self.C.argmax_correct(logits, logits.stride(0), labels, logits.shape[0], logits.shape[1], c)
        return c

    def dice(self, logits, target):
        N = target.shape[0]
        out = torch.empty(N, dtype=torch.float32, device=logits.device)
        self.C.dice(logits, 1, target, N, target[0].numel(), out)
        return out

    # ---------------- optimizers ----------------
    def sgd(self, p, g, m, lr, momentum, dampening, wd, nesterov, first, skip_flag=None):
        self.C.sgd_step(p, g, m, lr, momentum, dampening, wd, nesterov, first, skip_flag)

    def adam(self, p, g, m, v, lr, b1, b2, eps, wd, adamw, bc1, bc2, clip=None, tstep=None, clip_writeback=False):
        self.C.adam_step(p, g, m, v, lr, b1, b2, eps, wd, adamw, bc1, bc2, clip, tstep, bool(clip_writeback))

    def grad_norm(self, g, max_norm, norm_out, coef_out):
        self.C.grad_norm(g, max_norm, norm_out, coef_out)

    def scale_(self, x, coef):
        self.C.scale_(x, coef)

    # ---------------- utilities (per-step glue on our own kernels) ----------------
    def fill_(self, t, v):
        self.C.fill_(t, float(v))

    def add_i64_(self, t, v):
        self.C.add_i64_(t, int(v))

    def gather_(self, dst, src, idx, accumulate=False):
        """dst.view(-1)[i] (+)= src.view(-1)[idx[i]] (idx < 0: zero)."""
        self.C.gather_(dst, src, idx, bool(accumulate))


# --------------------------------------------------------------------------------------------
class RefBackend:
    """fp32 torch reference with identical semantics (CPU tests / numerics oracle)."""

    name = "ref"

    def __init__(self, device="cpu", dtype=torch.float32):
        self.device = torch.device(device)
        self.dt = dtype            # float64 turns the whole engine into an fp64 oracle run
        self.act_dtype = dtype

    @staticmethod
    def _store(y: Act, v_nchw):
        y.nhwc().copy_(v_nchw[:, :y.C].permute(0, 2, 3, 1))

    prologue = False   # Deferred operands are materialized (same values) before each consumer

    def materialize(self, d) -> Act:
        if not isinstance(d, Deferred):
            return d
        src = d.src
        out = Act.empty(src.N, src.H, src.W, src.C, self.act_dtype, src.device)
        if d.kind in ("affine", "bn"):
            self.bn_apply(src, d.k0, d.k1, None, d.kind == "affine", out)
        else:
            c = d.k0.to(self.dt)
            out.nhwc().copy_(c[0] * src.nhwc().to(self.dt) + c[1] * d.z.nhwc().to(self.dt) + c[2])
        return out

    def bn_bwd_deferred(self, dy: Act, x: Act, mean, invstd, gamma, dgamma, dbeta, pre, k2=1) -> Deferred:
        """bn_bwd's result as coefficients: dz = k1*(dy - s1/M - xhat*s2/M) = c0*dy + c1*x + c2."""
        ps = pre.sum(0)
        s1 = ps[0]
        s2 = invstd * (ps[k2] - mean * s1)
        if dbeta is not None:
            dbeta.add_(s1)
        if dgamma is not None:
            dgamma.add_(s2)
        M = x.rows
        k1 = (gamma if gamma is not None else torch.ones_like(mean)) * invstd
        c0 = k1
        c1 = -k1 * invstd * s2 / M
        c2 = -k1 * s1 / M + k1 * mean * invstd * s2 / M
        return Deferred.bnbwd(dy, x, torch.stack([c0, c1, c2]).to(self.dt))

    def conv_mtiles(self, N, H, W, C, K, R, S, stride, pad, pro=False):
        return 1

    def conv_fwd(self, x, w, K, R, S, stride, pad, y: Act, bias=None, res=None, scale=None, shift=None,
                 relu=False, stats=None, kvalid=0):
        x = self.materialize(x)
        wk = w.view(K, R, S, x.C).permute(0, 3, 1, 2).to(self.dt)
        out = F.conv2d(x.nchw().to(self.dt), wk, None, stride, pad)
        if bias is not None:
            out = out + bias.view(1, -1, 1, 1)
        if stats is not None:
            stats.view(-1, 2, K)[0, 0].copy_(out.sum((0, 2, 3)))
            stats.view(-1, 2, K)[0, 1].copy_((out * out).sum((0, 2, 3)))
        if scale is not None:
            out = out * scale.view(1, -1, 1, 1) + shift.view(1, -1, 1, 1)
        if res is not None:
            out = out + res.nchw().to(self.dt)
        if relu:
            out = F.relu(out)
        self._store(y, out)

    def conv_fwd_bn(self, x, w, K, R, S, stride, pad, z: Act, bias, stats, count, gamma, beta, rm, rv, momentum,
                    eps, scale, shift, save_mean, save_invstd):
        self.conv_fwd(x, w, K, R, S, stride, pad, z, bias=bias, stats=stats)
        self.bn_finalize(stats, stats.shape[0], K, count, gamma, beta, rm, rv, momentum, eps, scale, shift,
                         save_mean, save_invstd)

    def dual_weights(self, wT, C, K, coef):
        w = wT.reshape(C, K).to(self.dt)
        c = coef.to(self.dt)
        w2 = torch.cat([w * c[0], w * c[1]], 1).to(self.act_dtype)
        return w2, (w * c[2]).sum(1)

    def conv_dgrad(self, dy, wT, C, R, S, stride, pad, dx: Act, res=None, fuse=None, colsum=False, bias=None):
        dy = self.materialize(dy)
        K = dy.C
        wk = wT.view(C, R, S, K).permute(3, 0, 1, 2).to(self.dt)
        g = torch.nn.grad.conv2d_input((dx.N, C, dx.H, dx.W), wk, dy.nchw().to(self.dt), stride, pad)
        if bias is not None:
            g = g + bias.to(self.dt).view(1, -1, 1, 1)
        if res is not None:
            g = g + res.nchw().to(self.dt)
        if fuse is None:
            self._store(dx, g)
            if colsum:
                v = dx.nhwc().to(self.dt)
                return torch.stack([v.sum((0, 1, 2)), (v * v).sum((0, 1, 2))]).unsqueeze(0)
            return None
        m, z, z2, sc, sh, mb = fuse
        if mb is not None:
            g = g * self._unpack_bits(mb, z).permute(0, 3, 1, 2)
        elif m is not None:
            g = g * (m.nchw() > 0)
        else:   # mask recomputed from the BN input, as the forward BN-apply computed y
            keep = (z.nhwc().to(self.dt) * sc + sh) > 0
            g = g * keep.permute(0, 3, 1, 2)
        self._store(dx, g)
        v = dx.nhwc().to(self.dt)
        rows = [v.sum((0, 1, 2)), (v * z.nhwc().to(self.dt)).sum((0, 1, 2))]
        if z2 is not None:
            rows.append((v * z2.nhwc().to(self.dt)).sum((0, 1, 2)))
        return torch.stack(rows).unsqueeze(0)

    def conv_fwd_bn_apply(self, xp, w, K, z: Act, bias, stats, *fin):
        """Reference form of the fused consumer: the pending BN-apply as its own pass, then conv_fwd_bn."""
        self.bn_apply(xp.z, xp.scale, xp.shift, xp.res, xp.relu, xp.y, mbits=xp.mbits)
        self.conv_fwd_bn(xp.y, w, K, 1, 1, 1, 0, z, bias, stats, *fin)

    def conv3_fwd_bn_apply(self, xp, w, K, z: Act, bias, stats, *fin):
        """Reference form of the fused 3x3 consumer (the engine schedule is the same on every backend)."""
        self.bn_apply(xp.z, xp.scale, xp.shift, None, True, xp.y)
        self.conv_fwd_bn(xp.y, w, K, 3, 3, 1, 1, z, bias, stats, *fin)

    def conv_fwd_bnbwd(self, x: Act, w, K, R, S, stride, pad, y: Act, fuse):
        wk = w.view(K, R, S, x.C).permute(0, 3, 1, 2).to(self.dt)
        out = F.conv2d(x.nchw().to(self.dt), wk, None, stride, pad)
        zz = fuse.z.nhwc().to(self.dt)
        keep = (zz * fuse.scale + fuse.shift) > 0
        self._store(y, out * keep.permute(0, 3, 1, 2))
        v = y.nhwc().to(self.dt)
        return torch.stack([v.sum((0, 1, 2)), (v * zz).sum((0, 1, 2))]).unsqueeze(0)

    def convT_fwd(self, x: Act, wf, Cout, y: Act, bias=None):
        Cin = x.C
        wk = wf.view(Cout, 2, 2, Cin).permute(3, 0, 1, 2).to(self.dt)
        out = F.conv_transpose2d(x.nchw().to(self.dt), wk, bias, stride=2)
        self._store(y, out)

    def wgrad_defer(self, on: bool):
        pass

    def wgrad_flush(self):
        pass

    def wgrad_discard(self):
        pass

    def wgrad_bypass(self, on: bool):
        pass

    def conv_wgrad(self, dy, x, R, S, stride, pad, grad, Creal, Ko_real):
        dy, x = self.materialize(dy), self.materialize(x)
        Ko, Cc = dy.C, x.C
        gw = torch.nn.grad.conv2d_weight(x.nchw().to(self.dt), (Ko, Cc, R, S), dy.nchw().to(self.dt), stride, pad)
        gw = gw.permute(0, 2, 3, 1)[:Ko_real, :, :, :Creal]
        grad.view(Ko_real, R, S, Creal).add_(gw)

    def bn_finalize(self, stats, ntiles, C, count, gamma, beta, rm, rv, momentum, eps, scale, shift, save_mean,
                    save_invstd):
        s = stats.view(-1, 2, C)[:ntiles].double().sum(0)
        mean = s[0] / count
        var = (s[1] / count - mean * mean).clamp_min(0)
        invstd = 1.0 / torch.sqrt(var + eps)
        g = gamma.double() if gamma is not None else torch.ones_like(mean)
        b = beta.double() if beta is not None else torch.zeros_like(mean)
        sc = (g * invstd).to(self.dt)
        scale.copy_(sc)
        shift.copy_((b - mean * g * invstd).to(self.dt))
        if save_mean is not None:
            save_mean.copy_(mean.to(self.dt))
        if save_invstd is not None:
            save_invstd.copy_(invstd.to(self.dt))
        if rm is not None:
            unb = var * count / (count - 1) if count > 1 else var
            rm.mul_(1 - momentum).add_(momentum * mean.to(self.dt))
            rv.mul_(1 - momentum).add_(momentum * unb.to(self.dt))

    def bn_stats(self, x: Act):
        v = x.nhwc().to(self.dt)
        part = torch.stack([v.sum((0, 1, 2)), (v * v).sum((0, 1, 2))]).unsqueeze(0)
        return part, 1

    def bn_apply(self, x: Act, scale, shift, res, relu, y: Act, mbits=None):
        v = x.nhwc().to(self.dt) * scale + shift
        if isinstance(res, Deferred):   # a BN output applied on the fly (no storage rounding)
            assert res.kind == "bn", res
            v = v + (res.src.nhwc().to(self.dt) * res.k0.to(self.dt) + res.k1.to(self.dt))
        elif res is not None:
            v = v + res.nhwc().to(self.dt)
        if relu:
            v = F.relu(v)
        y.nhwc().copy_(v)
        if mbits is not None:   # bit e of byte (row, g): y[row][8g + e] > 0
            pos = (y.nhwc().reshape(-1, y.C // 8, 8) > 0).to(torch.uint8)
            w = (2 ** torch.arange(8, device=pos.device, dtype=torch.uint8))
            mbits.copy_((pos * w).sum(-1).to(torch.uint8).view(mbits.shape))

    @staticmethod
    def _unpack_bits(mbits, like: Act):
        b = mbits.view(-1, like.C // 8, 1).to(torch.int32)
        bits = (b >> torch.arange(8, device=b.device, dtype=torch.int32)) & 1
        return bits.view(like.N, like.H, like.W, like.C).bool()

    def bn_bwd(self, dy: Act, ymask, x: Act, mean, invstd, gamma, dgamma, dbeta, dx: Act, dyr_out=None, pre=None,
               k2=1):
        g = dy.nhwc().to(self.dt)
        if ymask is not None:
            g = g * (ymask.nhwc() > 0)
        M = x.rows
        xhat = (x.nhwc().to(self.dt) - mean) * invstd
        if pre is not None:
            assert ymask is None
            ps = pre.sum(0)
            s1 = ps[0]
            s2 = invstd * (ps[k2] - mean * s1)
        else:
            s1 = g.sum((0, 1, 2))
            s2 = (g * xhat).sum((0, 1, 2))
        if dbeta is not None:
            dbeta.add_(s1)
        if dgamma is not None:
            dgamma.add_(s2)
        k1 = (gamma if gamma is not None else torch.ones_like(mean)) * invstd
        dx.nhwc().copy_(k1 * (g - s1 / M - xhat * s2 / M))
        if dyr_out is not None:
            dyr_out.nhwc().copy_(g)

    def channel_sum(self, x: Act, out_acc):
        out_acc.add_(x.nhwc().to(self.dt).sum((0, 1, 2)))

    def maxpool_fwd(self, x: Act, k, s, p, y: Act, bn=None, store: Act = None):
        v = x.nchw().to(self.dt)
        if bn is not None:
            v = F.relu(v * bn[0].view(1, -1, 1, 1) + bn[1].view(1, -1, 1, 1)).to(x.dtype).to(self.dt)
        if store is not None:
            self._store(store, v)
        out, idx = F.max_pool2d(v, k, s, p, return_indices=True)
        self._store(y, out)
        return idx

    def maxpool_bwd(self, dy: Act, idx, x: Act, k, s, p, dx: Act, add=None, fuse=None):
        g = torch.ops.aten.max_pool2d_with_indices_backward(dy.nchw().to(self.dt).contiguous(), x.nchw().to(self.dt), [k, k],
                                                            [s, s], [p, p], [1, 1], False, idx)
        if add is not None:
            g = g + add.nchw().to(self.dt)
        if fuse is None:
            self._store(dx, g)
            return None
        zz = fuse.z.nhwc().to(self.dt)
        keep = (zz * fuse.scale + fuse.shift) > 0
        self._store(dx, g * keep.permute(0, 3, 1, 2))
        v = dx.nhwc().to(self.dt)
        return torch.stack([v.sum((0, 1, 2)), (v * zz).sum((0, 1, 2))]).unsqueeze(0)

    def outer_dgrad_bn(self, dy: Act, wT, ldw, dx: Act, fuse):
        """dx[m, c] = dy[m, 0] * wT[c * ldw], ReLU-masked by relu(BN(z)); BN-backward partials."""
        d = dy.nhwc()[..., :1].to(self.dt)
        w = wT.reshape(-1)[::ldw][:dx.C].to(self.dt)
        zz = fuse.z.nhwc().to(self.dt)
        keep = (zz * fuse.scale + fuse.shift) > 0
        dx.nhwc().copy_(d * w * keep)
        v = dx.nhwc().to(self.dt)
        return torch.stack([v.sum((0, 1, 2)), (v * zz).sum((0, 1, 2))]).unsqueeze(0)

    def avgpool_fwd(self, x: Act, y: Act):
        y.nhwc().copy_(x.nhwc().to(self.dt).mean((1, 2), keepdim=True))

    def avgpool_bwd(self, dy: Act, dx: Act):
        dx.nhwc().copy_(dy.nhwc().to(self.dt).expand(dx.N, dx.H, dx.W, dx.C) / (dx.H * dx.W))

    def nchw_to_nhwc(self, x: torch.Tensor, Cpad) -> Act:
        N, Cc, H, W = x.shape
        y = Act.zeros(N, H, W, Cpad, self.dt, x.device)
        y.nhwc()[..., :Cc].copy_(x.permute(0, 2, 3, 1))
        return y

    def s2d(self, x: torch.Tensor, pad, U, V, CS) -> Act:
        N, Cc, H, W = x.shape
        xp = torch.zeros(N, CS, 2 * U, 2 * V, dtype=self.dt, device=x.device)
        hh, ww = min(H, 2 * U - pad), min(W, 2 * V - pad)
        xp[:, :Cc, pad:pad + hh, pad:pad + ww] = x[:, :, :hh, :ww].to(self.dt)
        # [N, CS, U, vh, V, vw] -> [N, U, V, vh, vw, CS]
        y = xp.view(N, CS, U, 2, V, 2).permute(0, 2, 4, 3, 5, 1).reshape(N * U * V, 4 * CS)
        return Act(y.contiguous(), N, U, V, 4 * CS)

    def upsample_fwd(self, x: Act, y: Act):
        out = F.interpolate(x.nchw().to(self.dt), scale_factor=2, mode="bilinear", align_corners=True)
        self._store(y, out)

    def upsample_bwd(self, dy: Act, dx: Act):
        xin = torch.zeros(dx.N, dx.C, dx.H, dx.W, dtype=self.dt, device=dy.device, requires_grad=True)
        with torch.enable_grad():
            out = F.interpolate(xin, scale_factor=2, mode="bilinear", align_corners=True)
            (g,) = torch.autograd.grad(out, xin, dy.nchw().to(self.dt))
        self._store(dx, g)

    def cast_weights(self, entries, total, dst_flat):
        for (src, doff, d, v, st) in entries:
            n = d[0] * d[1] * d[2] * d[3]
            dst = dst_flat[doff:doff + n].view(*d)
            dst.zero_()
            dst[:v[0], :v[1], :v[2], :v[3]].copy_(src.as_strided(tuple(v), tuple(st)))

    def ce_fwd(self, logits, labels):
        lse = torch.logsumexp(logits.to(self.dt), 1)
        loss = F.cross_entropy(logits.to(self.dt), labels)
        return loss, lse

    def ce_bwd(self, logits, labels, lse, go):
        p = torch.exp(logits.to(self.dt) - lse[:, None])
        p[torch.arange(len(labels)), labels] -= 1.0
        return p * (go if go is not None else 1.0) / logits.shape[0]

    def bce_fwd(self, logits, target):
        return F.binary_cross_entropy_with_logits(logits.to(self.dt), target.to(self.dt))

    def bce_bwd(self, logits, target, go):
        return (torch.sigmoid(logits.to(self.dt)) - target) * (go if go is not None else 1.0) / logits.numel()

    def argmax_correct(self, logits, labels):
        return (logits.argmax(1) == labels).sum().to(torch.int32).view(1)

    def dice(self, logits, target):
        pred = (logits.reshape(target.shape) > 0).to(self.dt)
        inter = (pred * target).flatten(1).sum(1)
        uni = pred.flatten(1).sum(1) + target.flatten(1).sum(1)
        return torch.where(uni > 0, (2 * inter + 1e-8) / (uni + 1e-8), torch.ones_like(uni))

    def sgd(self, p, g, m, lr, momentum, dampening, wd, nesterov, first, skip_flag=None):
        if skip_flag is not None and float(skip_flag.reshape(-1)[0]) != 0:
            return
        d = g + wd * p if wd != 0 else g.clone()
        if momentum != 0:
            if first:
                m.copy_(d)
            else:
                m.mul_(momentum).add_(d, alpha=1 - dampening)
            d = d + momentum * m if nesterov else m
        p.add_(d, alpha=-lr)

    def adam(self, p, g, m, v, lr, b1, b2, eps, wd, adamw, bc1, bc2, clip=None, tstep=None, clip_writeback=False):
        coef = 1.0
        if clip is not None:
            if float(clip[1]) != 0:
                return
            coef = clip[0]
        if tstep is not None:   # tstep = updates applied so far; advanced only when this one is applied
            t = float(tstep.reshape(-1)[0]) + 1
            bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
            tstep.add_(1)
        gin = g
        g = g * coef
        if clip_writeback and float(coef) != 1.0:   # the clipped gradients stay visible (torch's in-place clip)
            gin.copy_(g)
        if wd != 0:
            if adamw:
                p.mul_(1 - lr * wd)
            else:
                g = g + wd * p
        m.lerp_(g, 1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        denom = v.sqrt() / (bc2 ** 0.5) + eps
        p.addcdiv_(m, denom, value=-lr / bc1)

    def grad_norm(self, g, max_norm, norm_out, coef_out):
        n = g.double().pow(2).sum().sqrt().to(self.dt)
        norm_out.reshape(-1)[0] = n
        coef_out[0] = torch.clamp(max_norm / (n + 1e-6), max=1.0)
        coef_out[1] = 0.0 if torch.isfinite(n) else 1.0
        if coef_out.numel() >= 4:
            coef_out[2] = 1.0
            coef_out[3] = coef_out[1]

    def scale_(self, x, coef):
        x.mul_(coef[0])

    def fill_(self, t, v):
        t.fill_(v)

    def add_i64_(self, t, v):
        t.add_(v)

    def gather_(self, dst, src, idx, accumulate=False):
        d, sv = dst.view(-1)[:idx.numel()], src.reshape(-1)
        v = torch.where(idx >= 0, sv[idx.clamp_min(0)], torch.zeros((), dtype=sv.dtype, device=sv.device))
        if accumulate:
            d.add_(v)
        else:
            d.copy_(v)


def make_backend(device, dtype=torch.float32, precision: str = "bf16") -> "NativeBackend | RefBackend":
    """GPU: the native gfx950 kernels with bf16 activations (default) or, ``precision='fp32'`` (the
    apps' ``--precision fp32``), the same kernels instantiated for fp32 activations and weights.
    ``precision='ref'`` on GPU: the torch reference backend in the parameters' dtype (numerics
    oracle, e.g. fp64 against the fp32 kernels).  CPU: the
    reference backend in the parameters' dtype."""
    device = torch.device(device)
    if device.type == "cuda":
        if precision == "ref":
            return RefBackend(device, dtype)
        if precision not in ("bf16", "fp32"):
            raise ValueError(f"precision must be bf16 or fp32, got {precision!r}")
        return NativeBackend(device, torch.float32 if precision == "fp32" else torch.bfloat16)
    return RefBackend(device, dtype)
