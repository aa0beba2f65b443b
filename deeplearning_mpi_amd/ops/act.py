"""NHWC activation descriptor used by the execution engine.

An :class:`Act` is a (possibly channel-sliced) NHWC tensor stored as a 2-D buffer
``[N*H*W, ld]``.  Channel slices (``off``, ``C`` < ``ld``) are how the UNet skip concatenation
is made free: the encoder writes its skip output straight into the decoder's concat buffer
(replaces ``torch.cat`` at /root/reference/pytorch/unet/model.py:47).
"""
from __future__ import annotations

import torch


class Act:
    __slots__ = ("buf", "N", "H", "W", "C", "off")

    def __init__(self, buf: torch.Tensor, N: int, H: int, W: int, C: int, off: int = 0):
        assert buf.dim() == 2 and buf.shape[0] == N * H * W, (tuple(buf.shape), N, H, W)
        assert off + C <= buf.shape[1]
        self.buf, self.N, self.H, self.W, self.C, self.off = buf, N, H, W, C, off

    @property
    def ld(self) -> int:
        return self.buf.shape[1]

    @property
    def rows(self) -> int:
        return self.N * self.H * self.W

    @property
    def dtype(self):
        return self.buf.dtype

    @property
    def device(self):
        return self.buf.device

    def nhwc(self) -> torch.Tensor:
        return self.buf.view(self.N, self.H, self.W, self.ld)[..., self.off:self.off + self.C]

    def nchw(self) -> torch.Tensor:
        return self.nhwc().permute(0, 3, 1, 2)

    def slice(self, off: int, C: int) -> "Act":
        return Act(self.buf, self.N, self.H, self.W, C, self.off + off)

    @staticmethod
    def empty(N, H, W, C, dtype, device, ld=None) -> "Act":
        ld = C if ld is None else ld
        return Act(torch.empty(N * H * W, ld, dtype=dtype, device=device), N, H, W, C)

    @staticmethod
    def zeros(N, H, W, C, dtype, device, ld=None) -> "Act":
        ld = C if ld is None else ld
        return Act(torch.zeros(N * H * W, ld, dtype=dtype, device=device), N, H, W, C)

    def __repr__(self):
        return f"Act(N={self.N},H={self.H},W={self.W},C={self.C},ld={self.ld},off={self.off},{self.dtype})"


class Deferred:
    """A GEMM operand that is never stored: the convolution kernels rebuild it from ``src`` in their
    operand prologue (in LDS, right after the tile lands), which removes a full elementwise pass
    (read + write) over the tensor and its re-read by the consumer.

    * ``Deferred.affine(z, scale, shift)`` = relu(z * scale + shift): a training BatchNorm-apply +
      ReLU without residual (the ResNet bottleneck's bn1 / bn2, the first BN of a UNet DoubleConv),
      consumed by the next convolution's forward and weight gradient;
    * ``Deferred.bn(z, scale, shift)`` = z * scale + shift: a training BatchNorm output without ReLU
      used only as a residual (the ResNet downsample branch), applied inside the consumer's BN-apply;
    * ``Deferred.bnbwd(dy, z, coef)`` = coef[0] * dy + coef[1] * z + coef[2]: the BatchNorm-backward
      apply, consumed by the unit's own weight-gradient and data-gradient GEMMs.

    Backends without operand prologues call ``materialize`` (same values)."""

    __slots__ = ("kind", "src", "z", "k0", "k1")

    def __init__(self, kind, src: Act, z: Act = None, k0=None, k1=None):
        self.kind, self.src, self.z, self.k0, self.k1 = kind, src, z, k0, k1

    @staticmethod
    def affine(z: Act, scale, shift) -> "Deferred":
        return Deferred("affine", z, None, scale, shift)

    @staticmethod
    def bn(z: Act, scale, shift) -> "Deferred":
        """z * scale + shift (a training BatchNorm output without ReLU): the ResNet downsample
        branch, read only as the residual of the block's last BN-apply, which applies it on the fly."""
        return Deferred("bn", z, None, scale, shift)

    @staticmethod
    def bnbwd(dy: Act, z: Act, coef) -> "Deferred":
        return Deferred("bnbwd", dy, z, coef)

    N = property(lambda self: self.src.N)
    H = property(lambda self: self.src.H)
    W = property(lambda self: self.src.W)
    C = property(lambda self: self.src.C)
    rows = property(lambda self: self.src.rows)
    dtype = property(lambda self: self.src.dtype)
    device = property(lambda self: self.src.device)

    def bufs(self):
        """Storage the deferred value is computed from (kept alive across streams by the engine)."""
        return (self.src.buf,) + ((self.z.buf,) if self.z is not None else ()) + \
            tuple(k for k in (self.k0, self.k1) if isinstance(k, torch.Tensor))   # the per-channel coefficients too

    def __repr__(self):
        return f"Deferred({self.kind}, {self.src!r})"


def pad8(c: int) -> int:
    return (c + 7) // 8 * 8


def padc(c: int) -> int:
    """Compute-layout channel count: the GEMM kernels reduce 64 channels per step, so channel
    counts are 8, 16, 32 or a multiple of 64 (zero padded)."""
    for v in (8, 16, 32):
        if c <= v:
            return v
    return (c + 63) // 64 * 64
