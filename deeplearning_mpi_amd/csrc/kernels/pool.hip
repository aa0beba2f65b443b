// Pooling / layout / resampling kernels (NHWC, 8 channels per thread; every kernel is templated on
// the activation storage type T: uint16_t = bf16, float = the fp32 precision path).
// Replace ATen MaxPool2d (ResNet stem 3x3/s2/p1, UNet 2x2/s2: /root/reference/pytorch/unet/model.py:25),
// AdaptiveAvgPool2d(1) (ResNet head), the host-side NCHW fp32 -> NHWC bf16 input conversion, and
// nn.Upsample(scale_factor=2, mode='bilinear', align_corners=True) (model.py:39-40).
#include "common.h"

namespace dlmpi {

static inline unsigned ew_blocks(int64_t total) {
  int64_t b = (total + 255) / 256;
  if (b > 16384) b = 16384;
  if (b < 1) b = 1;
  return (unsigned)b;
}

// Max pool forward; idx stores the winning window position (kh*k + kw) per channel, first max
// in scan order wins (torch semantics).  Padding never wins.
// scale/shift (optional): the pooled input is relu(x * scale + shift) rounded to bf16, i.e. the
// training-mode BN-apply + ReLU of the ResNet stem fused into the pool -- the stem's BN output is
// never written or re-read (identical values and argmax to pooling the materialised bf16 tensor).
template <typename T>
__global__ void maxpool_fwd_kernel(const T* __restrict__ x, int N, int H, int W, int C, int ldx, int xoff,
                                   int k, int stride, int pad, T* __restrict__ y, uint8_t* __restrict__ idx,
                                   int OH, int OW, const float* __restrict__ scale, const float* __restrict__ shift,
                                   FastDiv fdCC, FastDiv fdOW, FastDiv fdOH) {
  const int CC = C >> 3;
  const int64_t total = (int64_t)N * OH * OW * CC;   // < 2^31 (launcher): 32-bit magic divisions
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t ui = (uint32_t)i;
    const uint32_t upix = fdiv(ui, fdCC);
    const int cc = (int)(ui - upix * CC);
    const int64_t pix = upix;
    const uint32_t t2 = fdiv(upix, fdOW);
    const int ow = (int)(upix - t2 * OW);
    const uint32_t n_ = fdiv(t2, fdOH);
    const int oh = (int)(t2 - n_ * OH);
    const int n = (int)n_;
    float best[8], sc[8], sh[8];
    uint8_t bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; bi[e] = 0; }
    if (scale) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { sc[e] = scale[cc * 8 + e]; sh[e] = shift[cc * 8 + e]; }
    }
    for (int kh = 0; kh < k; ++kh) {
      const int ih = oh * stride - pad + kh;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int kw = 0; kw < k; ++kw) {
        const int iw = ow * stride - pad + kw;
        if ((unsigned)iw >= (unsigned)W) continue;
        float v[8];
        load8(x + (((int64_t)n * H + ih) * W + iw) * ldx + xoff + cc * 8, v);
        if (scale) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = stored<T>(fmaxf(v[e] * sc[e] + sh[e], 0.f));
        }
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (v[e] > best[e] || (v[e] != v[e] && best[e] == best[e])) { best[e] = v[e]; bi[e] = (uint8_t)(kh * k + kw); }
      }
    }
    store8(y + pix * C + cc * 8, best);
    uint64_t packed = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) packed |= (uint64_t)bi[e] << (8 * e);
    *reinterpret_cast<uint64_t*>(idx + pix * C + cc * 8) = packed;
  }
}

// Max pool forward with a compile-time K x K window and stride S (the ResNet stem's 3x3/s2, the UNet's
// 2x2/s2): every tap's load is issued before the first compare (out-of-image taps read a clamped
// in-image address and are masked to -inf, which never wins), instead of one dependent round trip per
// tap of the runtime-k loop (182 -> ~100 us for the ResNet-50 bs-256 stem pool).  Same scan order and
// compares as maxpool_fwd_kernel: identical values and indices.
//
// ys (with scale / shift, K == S: every input pixel in exactly one window): the applied values
// relu(fma(x, scale, shift)) -- bn_apply_kernel's arithmetic, bit-identical -- are also stored to ys, so
// a BN-apply whose output is both kept and pooled (the UNet encoder skip) needs one pass, not two.
template <int K, int S, typename T>
__global__ __launch_bounds__(256) void maxpool_fwd_fixed_kernel(const T* __restrict__ x, int N, int H, int W, int C,
                                                                int ldx, int xoff, int pad, T* __restrict__ y,
                                                                uint8_t* __restrict__ idx, int OH, int OW,
                                                                const float* __restrict__ scale,
                                                                const float* __restrict__ shift, FastDiv fdCC,
                                                                FastDiv fdOW, FastDiv fdOH, T* __restrict__ ys,
                                                                int ldys, int ysoff) {
  const int CC = C >> 3;
  const int64_t total = (int64_t)N * OH * OW * CC;   // < 2^31 (launcher)
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t ui = (uint32_t)i;
    const uint32_t upix = fdiv(ui, fdCC);
    const int cc = (int)(ui - upix * CC);
    const uint32_t t2 = fdiv(upix, fdOW);
    const int ow = (int)(upix - t2 * OW);
    const uint32_t n_ = fdiv(t2, fdOH);
    const int oh = (int)(t2 - n_ * OH);
    typename Vec8<T>::type raw[K][K];
    bool ok[K][K];
#pragma unroll
    for (int kh = 0; kh < K; ++kh)
#pragma unroll
      for (int kw = 0; kw < K; ++kw) {
        const int ih = oh * S - pad + kh, iw = ow * S - pad + kw;
        ok[kh][kw] = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
        const int ihc = min(max(ih, 0), H - 1), iwc = min(max(iw, 0), W - 1);
        raw[kh][kw] = raw8(x + (((int64_t)n_ * H + ihc) * W + iwc) * ldx + xoff + cc * 8);
      }
    float best[8], sc[8], sh[8];
    uint8_t bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; bi[e] = 0; }
    if (scale) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { sc[e] = scale[cc * 8 + e]; sh[e] = shift[cc * 8 + e]; }
    }
#pragma unroll
    for (int kh = 0; kh < K; ++kh)
#pragma unroll
      for (int kw = 0; kw < K; ++kw) {
        if (!ok[kh][kw]) continue;
        float v[8];
        unpack8(raw[kh][kw], v);
        if (scale) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = stored<T>(fmaxf(__builtin_fmaf(v[e], sc[e], sh[e]), 0.f));
          if (ys) {
            const int ih = oh * S - pad + kh, iw = ow * S - pad + kw;
            store8(ys + (((int64_t)n_ * H + ih) * W + iw) * ldys + ysoff + cc * 8, v);
          }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (v[e] > best[e] || (v[e] != v[e] && best[e] == best[e])) { best[e] = v[e]; bi[e] = (uint8_t)(kh * K + kw); }
      }
    store8(y + (int64_t)upix * C + cc * 8, best);
    uint64_t packed = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) packed |= (uint64_t)bi[e] << (8 * e);
    *reinterpret_cast<uint64_t*>(idx + (int64_t)upix * C + cc * 8) = packed;
  }
}

// Max pool backward as a gather (no atomics): each input pixel sums the gradients of the windows
// that selected it; optionally adds a second gradient source (UNet skip-concat slice).
template <typename T>
__global__ void maxpool_bwd_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ idx, int N, int H,
                                   int W, int C, int k, int stride, int pad, int OH, int OW,
                                   const T* __restrict__ add, int ldadd, int addoff, T* __restrict__ dx,
                                   int lddx, int dxoff, FastDiv fdCC, FastDiv fdW, FastDiv fdH) {
  const int CC = C >> 3;
  const int64_t total = (int64_t)N * H * W * CC;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int cc, iw, ih, n;
    int64_t pix;
    if (total < (1ll << 31)) {   // 32-bit fast division (the 64-bit divisions dominated this kernel)
      const uint32_t q = fdiv((uint32_t)i, fdCC);
      cc = (int)((uint32_t)i - q * CC);
      pix = q;
      const uint32_t t2 = fdiv(q, fdW);
      iw = (int)(q - t2 * W);
      const uint32_t nn = fdiv(t2, fdH);
      ih = (int)(t2 - nn * H);
      n = (int)nn;
    } else {
      cc = (int)(i % CC);
      pix = i / CC;
      iw = (int)(pix % W);
      const int64_t t2 = pix / W;
      ih = (int)(t2 % H);
      n = (int)(t2 / H);
    }
    float g[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (add) load8(add + pix * ldadd + addoff + cc * 8, g);
    // windows oh with oh*stride - pad <= ih <= oh*stride - pad + k - 1
    int oh_lo = ih + pad - k + 1;
    oh_lo = oh_lo <= 0 ? 0 : (oh_lo + stride - 1) / stride;
    const int oh_hi = min((ih + pad) / stride, OH - 1);
    int ow_lo = iw + pad - k + 1;
    ow_lo = ow_lo <= 0 ? 0 : (ow_lo + stride - 1) / stride;
    const int ow_hi = min((iw + pad) / stride, OW - 1);
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const uint8_t want = (uint8_t)((ih - (oh * stride - pad)) * k + (iw - (ow * stride - pad)));
        const int64_t op = ((int64_t)n * OH + oh) * OW + ow;
        const uint64_t id = *reinterpret_cast<const uint64_t*>(idx + op * C + cc * 8);
        float d[8];
        load8(dy + op * C + cc * 8, d);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (((id >> (8 * e)) & 0xff) == want) g[e] += d[e];
      }
    }
    store8(dx + pix * lddx + dxoff + cc * 8, g);
  }
}

// Global average pool [N][HW][C] -> [N][C]
template <typename T>
__global__ void avgpool_fwd_kernel(const T* __restrict__ x, int N, int HW, int C, T* __restrict__ y) {
  const int CC = C >> 3;
  const int64_t total = (int64_t)N * CC;
  const float inv = 1.f / (float)HW;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int cc = (int)(i % CC);
    const int n = (int)(i / CC);
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int p = 0; p < HW; ++p) {
      float v[8];
      load8(x + ((int64_t)n * HW + p) * C + cc * 8, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += v[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] *= inv;
    store8(y + (int64_t)n * C + cc * 8, s);
  }
}

template <typename T>
__global__ void avgpool_bwd_kernel(const T* __restrict__ dy, int N, int HW, int C, T* __restrict__ dx) {
  const int CC = C >> 3;
  const int64_t total = (int64_t)N * HW * CC;
  const float inv = 1.f / (float)HW;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int cc = (int)(i % CC);
    const int64_t pix = i / CC;
    const int n = (int)(pix / HW);
    float v[8];
    load8(dy + (int64_t)n * C + cc * 8, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= inv;
    store8(dx + pix * C + cc * 8, v);
  }
}

// NCHW fp32 -> NHWC T with channel zero-padding to Cpad (multiple of 8).
template <typename T>
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, int N, int C, int H, int W, int Cpad,
                                    T* __restrict__ y) {
  const int CC = Cpad >> 3;
  const int64_t HW = (int64_t)H * W;
  const int64_t total = (int64_t)N * HW * CC;
  if (total < (1ll << 31) && N * HW * C < (1ll << 31)) {   // 32-bit index math (no 64-bit divisions)
    const uint32_t ut = (uint32_t)total, uCC = CC, uHW = (uint32_t)HW;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < ut; i += gridDim.x * blockDim.x) {
      const uint32_t pix = i / uCC;
      const int cc = (int)(i - pix * uCC);
      const uint32_t n = pix / uHW, hw = pix - n * uHW;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = cc * 8 + e;
        v[e] = c < C ? x[(n * (uint32_t)C + c) * uHW + hw] : 0.f;
      }
      store8(y + (int64_t)pix * Cpad + cc * 8, v);
    }
    return;
  }
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t pix = i / CC;   // cc-major inner loop keeps reads of one channel plane coalesced
    const int cc = (int)(i - pix * CC);
    const int64_t n = pix / HW, hw = pix - n * HW;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = cc * 8 + e;
      v[e] = c < C ? x[(n * C + c) * HW + hw] : 0.f;
    }
    store8(y + pix * Cpad + cc * 8, v);
  }
}

// 2x2 space-to-depth of a zero-padded fp32 NCHW image into bf16 NHWC (the strided-stem layout,
// models/engine.py:S2DConvUnit): y[n][u][v][(vh*2 + vw)*CS + c] = x[n][c][2u+vh-pad][2v+vw-pad]
// (zero outside the image and for c >= C).  One thread = 8 output channels of one pixel.
template <typename T>
__global__ void s2d_nchw_kernel(const float* __restrict__ x, int N, int C, int H, int W, int pad, int U, int V, int CS,
                                T* __restrict__ y) {
  const int CT = 4 * CS, CC = CT >> 3;
  const int64_t total = (int64_t)N * U * V * CC;
  if (total < (1ll << 31)) {
    // 32-bit index math (the 64-bit divisions of the general loop dominated it: 90 us at ResNet-50
    // bs 256, 2.9 TB/s); one thread per (pixel, 8-channel group), the same loads and values
    const uint32_t ut = (uint32_t)total, uCC = CC, uV = V, uU = U;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < ut; i += gridDim.x * blockDim.x) {
      const uint32_t pix = i / uCC;
      const int g = (int)(i - pix * uCC);
      const uint32_t t = pix / uV;
      const int v = (int)(pix - t * uV);
      const uint32_t n = t / uU;
      const int u = (int)(t - n * uU);
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int j = g * 8 + e, slot = j / CS, c = j - slot * CS;
        const int h = 2 * u + (slot >> 1) - pad, w = 2 * v + (slot & 1) - pad;
        o[e] = (c < C && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W)
                   ? x[(int64_t)(((int)n * C + c) * H + h) * W + w]
                   : 0.f;
      }
      store8(y + (int64_t)pix * CT + g * 8, o);
    }
    return;
  }
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t pix = i / CC;
    const int g = (int)(i - pix * CC);
    const int v = (int)(pix % V);
    const int64_t t = pix / V;
    const int u = (int)(t % U);
    const int64_t n = t / U;
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int j = g * 8 + e, slot = j / CS, c = j - slot * CS;
      const int h = 2 * u + (slot >> 1) - pad, w = 2 * v + (slot & 1) - pad;
      o[e] = (c < C && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) ? x[((n * C + c) * H + h) * W + w]
                                                                               : 0.f;
    }
    store8(y + pix * CT + g * 8, o);
  }
}

// Bilinear x2 upsample, align_corners=True: src = o * (in-1)/(out-1).
template <typename T>
__global__ void upsample2x_fwd_kernel(const T* __restrict__ x, int N, int H, int W, int C, int ldx, int xoff,
                                      T* __restrict__ y, int ldy, int yoff) {
  const int OH = 2 * H, OW = 2 * W, CC = C >> 3;
  const float sh = OH > 1 ? (float)(H - 1) / (float)(OH - 1) : 0.f;
  const float sw = OW > 1 ? (float)(W - 1) / (float)(OW - 1) : 0.f;
  const int64_t total = (int64_t)N * OH * OW * CC;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int cc = (int)(i % CC);
    const int64_t pix = i / CC;
    const int ow = (int)(pix % OW);
    const int64_t t2 = pix / OW;
    const int oh = (int)(t2 % OH);
    const int n = (int)(t2 / OH);
    const float fh = oh * sh, fw = ow * sw;
    const int h0 = (int)fh, w0 = (int)fw;
    const int h1 = min(h0 + 1, H - 1), w1 = min(w0 + 1, W - 1);
    const float lh = fh - h0, lw = fw - w0;
    float a[8], b[8], c[8], d[8], o[8];
    const int64_t base = (int64_t)n * H;
    load8(x + ((base + h0) * W + w0) * ldx + xoff + cc * 8, a);
    load8(x + ((base + h0) * W + w1) * ldx + xoff + cc * 8, b);
    load8(x + ((base + h1) * W + w0) * ldx + xoff + cc * 8, c);
    load8(x + ((base + h1) * W + w1) * ldx + xoff + cc * 8, d);
#pragma unroll
    for (int e = 0; e < 8; ++e)
      o[e] = (1.f - lh) * ((1.f - lw) * a[e] + lw * b[e]) + lh * ((1.f - lw) * c[e] + lw * d[e]);
    store8(y + pix * ldy + yoff + cc * 8, o);
  }
}

// Bilinear x2 backward as a GATHER (deterministic, no atomics): input pixel (h, w) sums, in
// ascending (oh, ow) order, the output gradients whose interpolation footprint contains it, with the
// forward's own weights (same fh = oh * sh, h0 = (int) fh, lh = fh - h0 arithmetic).  An output row
// oh touches input rows h0(oh) and h1(oh) = min(h0 + 1, H - 1) with h0 = floor(oh * sh) monotone in
// oh, so h receives from h0 in {h - 1, h}: oh in [(h - 1) / sh, (h + 1) / sh), widened by one row
// each side against rounding (sh = (H-1)/(2H-1) < 1/2: at most ~2/sh + 3 candidate rows).
__device__ __forceinline__ void bilin_rows(int o, float s, int n_in, int& i0, int& i1, float& l) {
  const float f = o * s;
  i0 = (int)f;
  i1 = min(i0 + 1, n_in - 1);
  l = f - i0;
}

template <typename T>
__global__ void upsample2x_bwd_kernel(const T* __restrict__ dy, int N, int H, int W, int C, int lddy, int dyoff,
                                      T* __restrict__ dx) {
  const int OH = 2 * H, OW = 2 * W, CC = C >> 3;
  const float sh = OH > 1 ? (float)(H - 1) / (float)(OH - 1) : 0.f;
  const float sw = OW > 1 ? (float)(W - 1) / (float)(OW - 1) : 0.f;
  const int64_t total = (int64_t)N * H * W * CC;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int cc = (int)(i % CC);
    const int64_t pix = i / CC;
    const int w = (int)(pix % W);
    const int64_t t2 = pix / W;
    const int h = (int)(t2 % H);
    const int n = (int)(t2 / H);
    int oh_lo = 0, oh_hi = OH - 1, ow_lo = 0, ow_hi = OW - 1;
    if (sh > 0.f) {
      oh_lo = max(0, (int)floorf((h - 1) / sh) - 1);
      oh_hi = min(OH - 1, (int)((h + 1) / sh) + 1);
    }
    if (sw > 0.f) {
      ow_lo = max(0, (int)floorf((w - 1) / sw) - 1);
      ow_hi = min(OW - 1, (int)((w + 1) / sw) + 1);
    }
    float g[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      int h0, h1;
      float lh;
      bilin_rows(oh, sh, H, h0, h1, lh);
      const float wh = (h0 == h ? 1.f - lh : 0.f) + (h1 == h ? lh : 0.f);
      if (h0 != h && h1 != h) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        int w0, w1;
        float lw;
        bilin_rows(ow, sw, W, w0, w1, lw);
        if (w0 != w && w1 != w) continue;
        const float ww = (w0 == w ? 1.f - lw : 0.f) + (w1 == w ? lw : 0.f);
        float d[8];
        load8(dy + (((int64_t)n * OH + oh) * OW + ow) * lddy + dyoff + cc * 8, d);
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] += wh * ww * d[e];
      }
    }
    store8(dx + pix * C + cc * 8, g);
  }
}

}  // namespace dlmpi

using namespace dlmpi;

// f32: 1 = fp32 activations (the fp32 precision path), 0 = bf16 (uint16_t storage)
extern "C" hipError_t dlmpi_maxpool_fwd(const void* x, int N, int H, int W, int C, int ldx, int xoff, int k,
                                        int stride, int pad, void* y, uint8_t* idx, int OH, int OW,
                                        const float* scale, const float* shift, void* ys, int ldys, int ysoff,
                                        int f32, hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;
  // ys: K == S, no padding, the windows tile the input exactly, an applied input (scale / shift)
  if (ys && (!scale || !shift || k != 2 || stride != 2 || pad != 0 || H != 2 * OH || W != 2 * OW || ldys % 8 ||
             ysoff % 8))
    return hipErrorInvalidValue;
  const int64_t total = (int64_t)N * OH * OW * (C / 8);
  if (total >= (1ll << 31)) return hipErrorInvalidValue;
  const FastDiv a = make_fastdiv(C / 8), b = make_fastdiv(OW), c = make_fastdiv(OH);
#define LAUNCH_MPF(K_, S_)                                                                                          \
  do {                                                                                                            \
    if (f32)                                                                                                      \
      hipLaunchKernelGGL((maxpool_fwd_fixed_kernel<K_, S_, float>), dim3(ew_blocks(total)), dim3(256), 0, s,      \
                         (const float*)x, N, H, W, C, ldx, xoff, pad, (float*)y, idx, OH, OW, scale, shift, a, b, c, \
                         (float*)ys, ldys, ysoff);                                                                \
    else                                                                                                          \
      hipLaunchKernelGGL((maxpool_fwd_fixed_kernel<K_, S_, uint16_t>), dim3(ew_blocks(total)), dim3(256), 0, s,   \
                         (const uint16_t*)x, N, H, W, C, ldx, xoff, pad, (uint16_t*)y, idx, OH, OW, scale, shift, a, \
                         b, c, (uint16_t*)ys, ldys, ysoff);                                                       \
    return hipGetLastError();                                                                                     \
  } while (0)
  if (k == 3 && stride == 2 && H > 0 && W > 0) LAUNCH_MPF(3, 2);
  if (k == 2 && stride == 2 && H > 0 && W > 0) LAUNCH_MPF(2, 2);
#undef LAUNCH_MPF
  if (f32)
    hipLaunchKernelGGL(maxpool_fwd_kernel<float>, dim3(ew_blocks(total)), dim3(256), 0, s, (const float*)x, N, H, W, C,
                       ldx, xoff, k, stride, pad, (float*)y, idx, OH, OW, scale, shift, a, b, c);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<uint16_t>, dim3(ew_blocks(total)), dim3(256), 0, s, (const uint16_t*)x, N, H,
                       W, C, ldx, xoff, k, stride, pad, (uint16_t*)y, idx, OH, OW, scale, shift, a, b, c);
  return hipGetLastError();
}

extern "C" hipError_t dlmpi_maxpool_bwd(const void* dy, const uint8_t* idx, int N, int H, int W, int C, int k,
                                        int stride, int pad, int OH, int OW, const void* add, int ldadd,
                                        int addoff, void* dx, int lddx, int dxoff, int f32, hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;
  const int64_t total = (int64_t)N * H * W * (C / 8);
  const dim3 g(ew_blocks(total));
  if (f32)
    hipLaunchKernelGGL(maxpool_bwd_kernel<float>, g, dim3(256), 0, s, (const float*)dy, idx, N, H, W, C, k, stride,
                       pad, OH, OW, (const float*)add, ldadd, addoff, (float*)dx, lddx, dxoff, make_fastdiv(C / 8),
                       make_fastdiv(W), make_fastdiv(H));
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel<uint16_t>, g, dim3(256), 0, s, (const uint16_t*)dy, idx, N, H, W, C, k,
                       stride, pad, OH, OW, (const uint16_t*)add, ldadd, addoff, (uint16_t*)dx, lddx, dxoff,
                       make_fastdiv(C / 8), make_fastdiv(W), make_fastdiv(H));
  return hipGetLastError();
}

extern "C" hipError_t dlmpi_avgpool_fwd(const void* x, int N, int HW, int C, void* y, int f32, hipStream_t s) {
  const dim3 g(ew_blocks((int64_t)N * (C / 8)));
  if (f32) hipLaunchKernelGGL(avgpool_fwd_kernel<float>, g, dim3(256), 0, s, (const float*)x, N, HW, C, (float*)y);
  else hipLaunchKernelGGL(avgpool_fwd_kernel<uint16_t>, g, dim3(256), 0, s, (const uint16_t*)x, N, HW, C, (uint16_t*)y);
  return hipGetLastError();
}

extern "C" hipError_t dlmpi_avgpool_bwd(const void* dy, int N, int HW, int C, void* dx, int f32, hipStream_t s) {
  const dim3 g(ew_blocks((int64_t)N * HW * (C / 8)));
  if (f32) hipLaunchKernelGGL(avgpool_bwd_kernel<float>, g, dim3(256), 0, s, (const float*)dy, N, HW, C, (float*)dx);
  else hipLaunchKernelGGL(avgpool_bwd_kernel<uint16_t>, g, dim3(256), 0, s, (const uint16_t*)dy, N, HW, C,
                          (uint16_t*)dx);
  return hipGetLastError();
}

extern "C" hipError_t dlmpi_nchw_to_nhwc(const float* x, int N, int C, int H, int W, int Cpad, void* y, int f32,
                                         hipStream_t s) {
  if (Cpad % 8 || Cpad < C) return hipErrorInvalidValue;
  const dim3 g(ew_blocks((int64_t)N * H * W * (Cpad / 8)));
  if (f32) hipLaunchKernelGGL(nchw_to_nhwc_kernel<float>, g, dim3(256), 0, s, x, N, C, H, W, Cpad, (float*)y);
  else hipLaunchKernelGGL(nchw_to_nhwc_kernel<uint16_t>, g, dim3(256), 0, s, x, N, C, H, W, Cpad, (uint16_t*)y);
  return hipGetLastError();
}

extern "C" hipError_t dlmpi_s2d_nchw(const float* x, int N, int C, int H, int W, int pad, int U, int V, int CS,
                                     void* y, int f32, hipStream_t s) {
  if ((4 * CS) % 8 || C > CS) return hipErrorInvalidValue;
  const dim3 g(ew_blocks((int64_t)N * U * V * (CS / 2)));
  if (f32) hipLaunchKernelGGL(s2d_nchw_kernel<float>, g, dim3(256), 0, s, x, N, C, H, W, pad, U, V, CS, (float*)y);
  else hipLaunchKernelGGL(s2d_nchw_kernel<uint16_t>, g, dim3(256), 0, s, x, N, C, H, W, pad, U, V, CS, (uint16_t*)y);
  return hipGetLastError();
}

extern "C" hipError_t dlmpi_upsample2x_fwd(const void* x, int N, int H, int W, int C, int ldx, int xoff, void* y,
                                           int ldy, int yoff, int f32, hipStream_t s) {
  const dim3 g(ew_blocks((int64_t)N * 4 * H * W * (C / 8)));
  if (f32)
    hipLaunchKernelGGL(upsample2x_fwd_kernel<float>, g, dim3(256), 0, s, (const float*)x, N, H, W, C, ldx, xoff,
                       (float*)y, ldy, yoff);
  else
    hipLaunchKernelGGL(upsample2x_fwd_kernel<uint16_t>, g, dim3(256), 0, s, (const uint16_t*)x, N, H, W, C, ldx, xoff,
                       (uint16_t*)y, ldy, yoff);
  return hipGetLastError();
}

extern "C" hipError_t dlmpi_upsample2x_bwd(const void* dy, int N, int H, int W, int C, int lddy, int dyoff, void* dx,
                                           int f32, hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;
  const dim3 g(ew_blocks((int64_t)N * H * W * (C / 8)));
  if (f32)
    hipLaunchKernelGGL(upsample2x_bwd_kernel<float>, g, dim3(256), 0, s, (const float*)dy, N, H, W, C, lddy, dyoff,
                       (float*)dx);
  else
    hipLaunchKernelGGL(upsample2x_bwd_kernel<uint16_t>, g, dim3(256), 0, s, (const uint16_t*)dy, N, H, W, C, lddy,
                       dyoff, (uint16_t*)dx);
  return hipGetLastError();
}
