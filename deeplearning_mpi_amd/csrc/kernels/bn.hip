// Training-mode BatchNorm2d on NHWC bf16 activations (fp32 statistics), fused with ReLU and the
// bottleneck residual add.  Replaces the cuDNN BN fwd/bwd + ATen ReLU/add kernels the reference
// runs implicitly (/root/reference/pytorch/unet/model.py:9-14, torchvision
// BasicBlock/Bottleneck used by /root/reference/pytorch/resnet/main.py:40).
//
// Forward statistics normally come for free from the conv epilogue (per-tile partial sums);
// bn_finalize reduces them in double precision in a fixed order (deterministic, no atomics),
// updates the running statistics with torch semantics (unbiased running_var) and emits the
// per-channel scale/shift consumed by bn_apply (y = relu(x*scale + shift [+ residual])).
// Backward: bn_bwd_reduce -> bn_bwd_finalize -> bn_bwd_apply, i.e.
//   dyr = dy * [y > 0];  dbeta = sum dyr;  dgamma = sum dyr * xhat;
//   dx  = k1*dyr + k2*x + k3   (k* folded per channel by the finalize kernel).
// All tensors may be channel slices of a wider buffer (ld*, *off) so UNet's skip concat is free.
#include <cstdlib>

#include "common.h"
#include "bnfin.h"

namespace dlmpi {

// ---------------- generic chunked row reduction layout --------------------------------------
// A block of 256 threads walks rows; thread -> (chunk of 8 channels cc, row lane rr).
struct RowMap {
  int CC, RPB, cc, rr;
  bool active;
};
__device__ __forceinline__ RowMap rowmap(int C) {
  RowMap m;
  m.CC = C >> 3;
  m.RPB = 256 / m.CC;
  m.cc = threadIdx.x % m.CC;
  m.rr = threadIdx.x / m.CC;
  m.active = m.rr < m.RPB;
  return m;
}

// Block-level combine of per-thread [8] sums over threads that share a channel chunk; writes
// partial[blk][k][C] for k < NS.
// Fixed summation order over the row lanes -> bit-reproducible partials.
template <int NS>
__device__ void block_combine(float (*acc)[8], const RowMap& rm, int C, float* partial) {
  __shared__ float buf[256 * NS * 8];
#pragma unroll
  for (int k = 0; k < NS; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) buf[(threadIdx.x * NS + k) * 8 + e] = acc[k][e];
  __syncthreads();
  for (int i = threadIdx.x; i < NS * C; i += 256) {
    const int k = i / C, c = i - k * C, cc = c >> 3, e = c & 7;
    float s = 0.f;
    for (int r = 0; r < rm.RPB; ++r) s += buf[((r * rm.CC + cc) * NS + k) * 8 + e];
    partial[(int64_t)blockIdx.x * NS * C + i] = s;
  }
}

// Max-pool backward (gather, no atomics) fused with the BN-backward statistics of the BN+ReLU
// that produced the pool input (the ResNet stem): dx = [z*scale + shift > 0] * sum of the window
// gradients that selected the element, written as the masked gradient dyr, and per-block partials
// {sum dyr, sum dyr*z} for the fused finalize (raw_z).  Replaces maxpool_bwd + bn_bwd_reduce and
// the mask read of bn_bwd_apply.  `add` (optional): a second gradient of the pool input summed in
// before the mask (the UNet encoder output also feeds the decoder's skip concat).
// NWIN > 0: at most NWIN x NWIN windows hold an input pixel (ceil(k / stride): 2 for the ResNet
// stem's 3x3/s2, 1 for the UNet's 2x2/s2); the candidate loop is unrolled with predication so all
// window loads (index + gradient) are in flight at once instead of one dependent round trip per
// window.  Same summation order as the generic loop (oh, then ow, ascending) -> identical results.
template <int NWIN, typename T>
__global__ __launch_bounds__(256) void maxpool_bwd_bn_kernel(const T* __restrict__ dy,
                                                             const uint8_t* __restrict__ idx, int N, int H, int W,
                                                             int C, int k, int stride, int pad, int OH, int OW,
                                                             FastDiv fdW, FastDiv fdH, const T* __restrict__ z,
                                                             const float* __restrict__ msc,
                                                             const float* __restrict__ msh,
                                                             const T* __restrict__ add, int ldadd, int addoff,
                                                             T* __restrict__ dx, float* __restrict__ partial) {
  const RowMap rm = rowmap(C);
  float acc[2][8] = {};
  const int64_t M = (int64_t)N * H * W;
  if (rm.active) {
    const int c0 = rm.cc * 8;
    float sc[8], sh[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { sc[e] = msc[c0 + e]; sh[e] = msh[c0 + e]; }
    for (int64_t row = (int64_t)blockIdx.x * rm.RPB + rm.rr; row < M; row += (int64_t)gridDim.x * rm.RPB) {
      const uint32_t pix = (uint32_t)row;
      const uint32_t t2 = fdiv(pix, fdW);
      const int iw = (int)(pix - t2 * W);
      const uint32_t n = fdiv(t2, fdH);
      const int ih = (int)(t2 - n * H);
      float g[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      int oh_lo = ih + pad - k + 1;
      oh_lo = oh_lo <= 0 ? 0 : (oh_lo + stride - 1) / stride;
      const int oh_hi = min((ih + pad) / stride, OH - 1);
      int ow_lo = iw + pad - k + 1;
      ow_lo = ow_lo <= 0 ? 0 : (ow_lo + stride - 1) / stride;
      const int ow_hi = min((iw + pad) / stride, OW - 1);
      if constexpr (NWIN > 0) {
        uint64_t id[NWIN * NWIN];
        typename Vec8<T>::type dv[NWIN * NWIN];
#pragma unroll
        for (int a = 0; a < NWIN; ++a)
#pragma unroll
          for (int b = 0; b < NWIN; ++b) {
            const bool ok = oh_lo + a <= oh_hi && ow_lo + b <= ow_hi;
            const int64_t op = ok ? ((int64_t)n * OH + oh_lo + a) * OW + ow_lo + b : 0;   // 0: a valid address
            id[a * NWIN + b] = *reinterpret_cast<const uint64_t*>(idx + op * C + c0);
            dv[a * NWIN + b] = raw8(dy + op * C + c0);
          }
#pragma unroll
        for (int a = 0; a < NWIN; ++a)
#pragma unroll
          for (int b = 0; b < NWIN; ++b) {
            const bool ok = oh_lo + a <= oh_hi && ow_lo + b <= ow_hi;
            const int want = ok ? (ih - ((oh_lo + a) * stride - pad)) * k + (iw - ((ow_lo + b) * stride - pad)) : 256;
            float d[8];
            unpack8(dv[a * NWIN + b], d);
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if ((int)((id[a * NWIN + b] >> (8 * e)) & 0xff) == want) g[e] += d[e];
          }
      } else {
        for (int oh = oh_lo; oh <= oh_hi; ++oh) {
          for (int ow = ow_lo; ow <= ow_hi; ++ow) {
            const uint8_t want = (uint8_t)((ih - (oh * stride - pad)) * k + (iw - (ow * stride - pad)));
            const int64_t op = ((int64_t)n * OH + oh) * OW + ow;
            const uint64_t id = *reinterpret_cast<const uint64_t*>(idx + op * C + c0);
            float d[8];
            load8(dy + op * C + c0, d);
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (((id >> (8 * e)) & 0xff) == want) g[e] += d[e];
          }
        }
      }
      if (add) {   // second gradient source of the pool input (UNet: its skip-concat slice)
        float a2[8];
        load8(add + row * ldadd + addoff + c0, a2);
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] += a2[e];
      }
      float zz[8];
      load8(z + row * C + c0, zz);
#pragma unroll
      for (int e = 0; e < 8; ++e) g[e] = zz[e] * sc[e] + sh[e] > 0.f ? g[e] : 0.f;
      store8(dx + row * C + c0, g);
#pragma unroll
      for (int e = 0; e < 8; ++e) {   // statistics of the stored gradient
        const float r = stored<T>(g[e]);
        acc[0][e] += r;
        acc[1][e] += r * zz[e];
      }
    }
  }
  block_combine<2>(acc, rm, C, partial);
}

// Data gradient of a 1x1 convolution with ONE output channel (the UNet head, reference
// model.py:68) into the gradient of the BN+ReLU output below it: dx[m, c] = dy[m] * w[c] -- an
// outer product, so a streaming kernel instead of a GEMM tile with 63 of 64 reduction lanes zero
// -- masked by [z*scale + shift > 0], stored, and the BN-backward partials {sum dx, sum dx*z} per
// block.  The bf16 x bf16 product is exact in fp32, as in the GEMM path: identical dx.
template <typename T>
__global__ __launch_bounds__(256) void outer_dgrad_bn_kernel(const T* __restrict__ dy, int lddy, int64_t M,
                                                             int C, const T* __restrict__ w, int ldw,
                                                             const T* __restrict__ z,
                                                             const float* __restrict__ msc,
                                                             const float* __restrict__ msh,
                                                             T* __restrict__ dx, float* __restrict__ partial) {
  const RowMap rm = rowmap(C);
  float acc[2][8] = {};
  if (rm.active) {
    const int c0 = rm.cc * 8;
    float wv[8], sc[8], sh[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      wv[e] = load1(w + (int64_t)(c0 + e) * ldw);
      sc[e] = msc[c0 + e];
      sh[e] = msh[c0 + e];
    }
    for (int64_t row = (int64_t)blockIdx.x * rm.RPB + rm.rr; row < M; row += (int64_t)gridDim.x * rm.RPB) {
      const float d = load1(dy + row * lddy);
      float zz[8], g[8];
      load8(z + row * C + c0, zz);
#pragma unroll
      for (int e = 0; e < 8; ++e) g[e] = zz[e] * sc[e] + sh[e] > 0.f ? d * wv[e] : 0.f;
      store8(dx + row * C + c0, g);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float r = stored<T>(g[e]);
        acc[0][e] += r;
        acc[1][e] += r * zz[e];
      }
    }
  }
  block_combine<2>(acc, rm, C, partial);
}

template <typename T>
__global__ __launch_bounds__(256) void bn_stats_kernel(const T* __restrict__ x, int64_t M, int C, int ldx,
                                                       int xoff, float* __restrict__ partial) {
  const RowMap rm = rowmap(C);
  float acc[2][8] = {};
  if (rm.active) {
    for (int64_t row = (int64_t)blockIdx.x * rm.RPB + rm.rr; row < M; row += (int64_t)gridDim.x * rm.RPB) {
      float v[8];
      load8(x + row * ldx + xoff + rm.cc * 8, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) { acc[0][e] += v[e]; acc[1][e] += v[e] * v[e]; }
    }
  }
  block_combine<2>(acc, rm, C, partial);
}

// Stage 1 of every per-channel column reduction over [T][2][C] fp32 partials:
// dpart[s][k][c] = sum of partial[t][k][c] over row slice s (double).  Grid (ceil(C/64), S) so the
// whole chip works on it (the partial tensors are up to 6272 x 2 x 2048); fixed summation order.
// Sums rows 0 and k2 of per-tile partials laid out [T][ns][C] (fwd stats: ns = 2, k2 = 1; fused
// backward stats from a GEMM epilogue: ns = 2 or 3 with the second BN consumer at k2 = 2).
__global__ __launch_bounds__(256) void colsum2_kernel(const float* __restrict__ partial, int T, int C, int ns,
                                                      int k2, double* __restrict__ dpart) {
  __shared__ double r[2][4][64];
  const int lc = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lc;
  const int S = gridDim.y, s = blockIdx.y;
  const int per = (T + S - 1) / S;
  const int t0 = s * per, t1 = min(T, t0 + per);
  double a = 0.0, b = 0.0;
  if (c < C) {
#pragma unroll 8
    for (int t = t0 + rl; t < t1; t += 4) {
      a += (double)partial[(int64_t)t * ns * C + c];
      b += (double)partial[(int64_t)t * ns * C + k2 * C + c];
    }
  }
  r[0][rl][lc] = a;
  r[1][rl][lc] = b;
  __syncthreads();
  if (rl == 0 && c < C) {
    for (int g = 1; g < 4; ++g) { a += r[0][g][lc]; b += r[1][g][lc]; }
    dpart[(int64_t)s * 2 * C + c] = a;
    dpart[(int64_t)s * 2 * C + C + c] = b;
  }
}

__device__ __forceinline__ void colsum2_final(const double* __restrict__ dpart, int S, int C, int c, double& s1,
                                              double& s2) {
  s1 = 0.0;
  s2 = 0.0;
#pragma unroll 8
  for (int s = 0; s < S; ++s) {
    s1 += dpart[(int64_t)s * 2 * C + c];
    s2 += dpart[(int64_t)s * 2 * C + C + c];
  }
}

static inline int colsum_slices(int T) {
  // tiles per slice / slice cap (measured, profiles/r2_*)
  constexpr int tps = 32, smax = 64;
  int S = (T + tps - 1) / tps;
  return S < 1 ? 1 : (S > smax ? smax : S);
}

__global__ __launch_bounds__(256) void finalize_kernel(const double* __restrict__ dpart, int S, int C, FinArgs f) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c < C) {
    double s1, s2;
    colsum2_final(dpart, S, C, c, s1, s2);
    if (f.mode == 0) fin_fwd(f, c, s1, s2);
    else fin_bwd(f, c, s1, s2, C);
  }
}

// Fused column reduction + finalize: colsum2 for slice s of channel group g, then the LAST block
// of group g to finish (ticket, cdna_hip_programming.md "In-launch split-K reduction") sums the S
// slice partials in a fixed order and finalizes the group's 64 channels.  Saves the second launch
// of every BN finalize.  Tickets self-reset.
// SC1 (default): the slice partials are stored write-through (8-B agent-scope relaxed atomic
// stores = sc1) and drained before the ticket, and the last arriver reads them with sc1 loads, so
// neither side fences (Guideline 16 R1).  A release fence here would write back every dirty line
// of the XCD's L2 -- right after a conv kernel, megabytes of its output (the fenced form measured
// ResNet-50 -1.5 %, profiles/r1_fin_sc1).
typedef __attribute__((address_space(1))) unsigned long long gu64_t;
typedef __attribute__((address_space(1))) int gi32_t;

// Direct form for short partial columns (T <= 512 rows: the 14^2 / 7^2 ResNet layers): one
// 1024-thread block per 16-channel group, 64 row lanes x 16 channels; every lane issues all of its
// <= 8 row loads at once (predicated, no dependent chain), sums them in double, then a fixed-order
// pairwise tree over the row lanes (rl += rl + s, s = 32 .. 1): s = 32 .. 4 cross waves through one
// 8 KB LDS buffer, s = 2 and 1 are shuffles inside wave 0; one lane per channel finalizes -- no slice
// stores, ticket or second pass.  (The first form, 16 row lanes per 64 channels, walked up to 32
// dependent loads per lane: 14 us per call vs ~11 us for the sliced kernel.  The 17 KB all-LDS tree of
// the same order often could not start beside a streaming conv on another stream holding 146 of the
// CU's 160 KB of LDS: 19-103 us instead of ~5 in the ResNet-50 step.  256-thread forms with 4 row lanes
// per thread ran ~9 us per call: 4x the load instructions per wave, profiles/r5_fin256.)
constexpr int kDirectMaxT = 512;
__global__ __launch_bounds__(1024) void colsum_fin_direct_kernel(const float* __restrict__ partial, int T, int C,
                                                                 int ns, int k2, FinArgs f) {
  __shared__ double r[2][32][16];
  const int lc = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + lc;
  constexpr int NR = kDirectMaxT / 64;
  float va[NR], vb[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int t = rl + 64 * i;
    const bool ok = c < C && t < T;
    const int64_t o = ok ? (int64_t)t * ns * C + c : 0;
    va[i] = ok ? partial[o] : 0.f;
    vb[i] = ok ? partial[o + (int64_t)k2 * C] : 0.f;
  }
  double a = 0.0, b = 0.0;
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    a += (double)va[i];
    b += (double)vb[i];
  }
#pragma unroll
  for (int s = 32; s >= 4; s >>= 1) {
    if (rl >= s && rl < 2 * s) {
      r[0][rl - s][lc] = a;
      r[1][rl - s][lc] = b;
    }
    __syncthreads();
    if (rl < s) {
      a += r[0][rl][lc];
      b += r[1][rl][lc];
    }
    __syncthreads();
  }
  // s = 2, 1: row lanes 0..3 are wave 0 (row lane rl + s is lane + 16 s)
  const double a2 = __shfl_down(a, 32, 64), b2 = __shfl_down(b, 32, 64);
  if (rl < 2) { a += a2; b += b2; }
  const double a1 = __shfl_down(a, 16, 64), b1 = __shfl_down(b, 16, 64);
  if (rl == 0 && c < C) {
    a += a1;
    b += b1;
    if (f.mode == 0) fin_fwd(f, c, a, b);
    else fin_bwd(f, c, a, b, C);
  }
}

__global__ __launch_bounds__(256) void colsum_fin_kernel(const float* __restrict__ partial, int T, int C, int ns,
                                                         int k2, double* __restrict__ dpart, int* __restrict__ tickets,
                                                         FinArgs f) {
  __shared__ double r[2][4][64];
  __shared__ int last;
  const int lc = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lc;
  const int S = gridDim.y, s = blockIdx.y;
  const int per = (T + S - 1) / S;
  const int t0 = s * per, t1 = min(T, t0 + per);
  double a = 0.0, b = 0.0;
  if (c < C) {
#pragma unroll 8
    for (int t = t0 + rl; t < t1; t += 4) {
      a += (double)partial[(int64_t)t * ns * C + c];
      b += (double)partial[(int64_t)t * ns * C + k2 * C + c];
    }
  }
  r[0][rl][lc] = a;
  r[1][rl][lc] = b;
  __syncthreads();
  if (rl == 0 && c < C) {
    for (int g = 1; g < 4; ++g) { a += r[0][g][lc]; b += r[1][g][lc]; }
    __hip_atomic_store((gu64_t*)(dpart + (int64_t)s * 2 * C + c), (unsigned long long)__double_as_longlong(a),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((gu64_t*)(dpart + (int64_t)s * 2 * C + C + c), (unsigned long long)__double_as_longlong(b),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains
  __syncthreads();
  if (threadIdx.x == 0) {
    last = __hip_atomic_fetch_add((gi32_t*)&tickets[blockIdx.x], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == S - 1;
  }
  __syncthreads();
  if (!last) return;
  if (threadIdx.x == 0)
    __hip_atomic_store((gi32_t*)&tickets[blockIdx.x], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler barrier only: loads stay below
  a = 0.0;
  b = 0.0;
  if (c < C) {
#pragma unroll 4
    for (int q = rl; q < S; q += 4) {
      // every load of the handed-off slices is an sc1 load (no L1 copy)
      a += __longlong_as_double((long long)__hip_atomic_load((gu64_t*)(dpart + (int64_t)q * 2 * C + c),
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      b += __longlong_as_double((long long)__hip_atomic_load((gu64_t*)(dpart + (int64_t)q * 2 * C + C + c),
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
  }
  __syncthreads();   // r is reused
  r[0][rl][lc] = a;
  r[1][rl][lc] = b;
  __syncthreads();
  if (rl == 0 && c < C) {
    for (int g = 1; g < 4; ++g) { a += r[0][g][lc]; b += r[1][g][lc]; }
    if (f.mode == 0) fin_fwd(f, c, a, b);
    else fin_bwd(f, c, a, b, C);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void bn_apply_kernel(const T* __restrict__ x, int ldx, int xoff, int64_t M,
                                                       int C, FastDiv fdCC, const float* __restrict__ scale,
                                                       const float* __restrict__ shift,
                                                       const T* __restrict__ res, int ldres, int resoff,
                                                       int relu, T* __restrict__ y, int ldy, int yoff,
                                                       uint8_t* __restrict__ mbits, const float* __restrict__ rscale,
                                                       const float* __restrict__ rshift) {
  const int CC = C >> 3;
  const int64_t total = M * CC;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t row;
    int cc;
    if (total < (1ll << 31)) {
      row = fdiv((uint32_t)i, fdCC);
      cc = (int)(i - row * CC);
    } else {
      row = i / CC;
      cc = (int)(i - row * CC);
    }
    const int c0 = cc * 8;
    float v[8];
    load8(x + row * ldx + xoff + c0, v);
    const f32x4 s0 = *reinterpret_cast<const f32x4*>(scale + c0), s1 = *reinterpret_cast<const f32x4*>(scale + c0 + 4);
    const f32x4 h0 = *reinterpret_cast<const f32x4*>(shift + c0), h1 = *reinterpret_cast<const f32x4*>(shift + c0 + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      // explicit fma: the conv prologue (conv_igemm.hip, pro 1) recomputes exactly this value
      v[e] = __builtin_fmaf(v[e], s0[e], h0[e]);
      v[e + 4] = __builtin_fmaf(v[e + 4], s1[e], h1[e]);
    }
    if (res) {
      float r[8];
      load8(res + row * ldres + resoff + c0, r);
      if (rscale) {   // the residual is itself a BN output (ResNet downsample): r * rscale + rshift,
                      // applied here instead of in a pass of its own (never rounded to bf16)
        const f32x4 a0 = *reinterpret_cast<const f32x4*>(rscale + c0), a1 = *reinterpret_cast<const f32x4*>(rscale + c0 + 4);
        const f32x4 b0 = *reinterpret_cast<const f32x4*>(rshift + c0), b1 = *reinterpret_cast<const f32x4*>(rshift + c0 + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          r[e] = __builtin_fmaf(r[e], a0[e], b0[e]);
          r[e + 4] = __builtin_fmaf(r[e + 4], a1[e], b1[e]);
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += r[e];
    }
    if (relu) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    if constexpr (sizeof(T) == 2) {
      const u32x4 pk = pack8(v);
      *reinterpret_cast<u32x4*>(y + row * ldy + yoff + c0) = pk;
      if (mbits) {   // ReLU mask bits of the stored bf16 values (bit e: y[c0 + e] > 0), 1/16 of y's bytes
        uint32_t b = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          b |= (uint32_t)((pk[k] & 0xffffu) != 0u && !(pk[k] & 0x8000u)) << (2 * k);
          b |= (uint32_t)((pk[k] >> 16) != 0u && !(pk[k] & 0x80000000u)) << (2 * k + 1);
        }
        mbits[row * CC + cc] = (uint8_t)b;
      }
    } else {
      store8(y + row * ldy + yoff + c0, v);
      if (mbits) {
        uint32_t b = 0;
#pragma unroll
        for (int e = 0; e < 8; ++e) b |= (uint32_t)(v[e] > 0.f) << e;
        mbits[row * CC + cc] = (uint8_t)b;
      }
    }
  }
}

// partial[blk][0][C] = sum dyr, partial[blk][1][C] = sum dyr * xhat  (x == null: only the first)
template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const T* __restrict__ dy, int lddy, int dyoff,
                                                            const T* __restrict__ ym, int ldym, int ymoff,
                                                            const T* __restrict__ x, int ldx, int xoff,
                                                            int64_t M, int C, const float* __restrict__ mean,
                                                            const float* __restrict__ invstd,
                                                            float* __restrict__ partial) {
  const RowMap rm = rowmap(C);
  float acc[2][8] = {};
  if (rm.active) {
    const int c0 = rm.cc * 8;
    float mu[8], is[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      mu[e] = x ? mean[c0 + e] : 0.f;
      is[e] = x ? invstd[c0 + e] : 0.f;
    }
    for (int64_t row = (int64_t)blockIdx.x * rm.RPB + rm.rr; row < M; row += (int64_t)gridDim.x * rm.RPB) {
      float g[8];
      load8(dy + row * lddy + dyoff + c0, g);
      if (ym) {
        float m[8];
        load8(ym + row * ldym + ymoff + c0, m);
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = m[e] > 0.f ? g[e] : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[0][e] += g[e];
      if (x) {
        float xv[8];
        load8(x + row * ldx + xoff + c0, xv);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[1][e] += g[e] * (xv[e] - mu[e]) * is[e];
      }
    }
  }
  block_combine<2>(acc, rm, C, partial);
}

template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const T* __restrict__ dy, int lddy, int dyoff,
                                                           const T* __restrict__ ym, int ldym, int ymoff,
                                                           const T* __restrict__ x, int ldx, int xoff,
                                                           int64_t M, int C, FastDiv fdCC,
                                                           const float* __restrict__ coef, T* __restrict__ dx,
                                                           T* __restrict__ dyr_out) {
  const int CC = C >> 3;
  const int64_t total = M * CC;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t row;
    int cc;
    if (total < (1ll << 31)) {
      row = fdiv((uint32_t)i, fdCC);
      cc = (int)(i - row * CC);
    } else {
      row = i / CC;
      cc = (int)(i - row * CC);
    }
    const int c0 = cc * 8;
    float g[8], xv[8];
    load8(dy + row * lddy + dyoff + c0, g);
    if (ym) {
      float m[8];
      load8(ym + row * ldym + ymoff + c0, m);
#pragma unroll
      for (int e = 0; e < 8; ++e) g[e] = m[e] > 0.f ? g[e] : 0.f;
    }
    if (dyr_out) store8(dyr_out + row * C + c0, g);
    load8(x + row * ldx + xoff + c0, xv);
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e)   // this fma order is shared with the conv prologues (pro 2 / PA 2)
      o[e] = __builtin_fmaf(coef[c0 + e], g[e], __builtin_fmaf(coef[C + c0 + e], xv[e], coef[2 * C + c0 + e]));
    store8(dx + row * C + c0, o);
  }
}


// Weights of the "dual" data gradient of a 1x1 stride-1 convolution whose input gradient passes
// through a training BatchNorm (models/engine.py:ConvUnit, dual path): instead of materialising
// dz = k1*dy + k2*z + k3 (coef [3][K]) and running dx = dz . W, the GEMM reduces over [dy | z]
// (2K channels, stored side by side) with
//   w2[c][k] = W[c][k] * k1[k],   w2[c][K + k] = W[c][k] * k2[k]   (rounded to the storage type),
//   b[c] = sum_k W[c][k] * k3[k]   (fp32 epilogue bias; fixed-order tree, deterministic).
// W is the data-gradient compute copy [C][K] (CRSK of a 1x1 conv); one block per row c.
template <typename T>
__global__ __launch_bounds__(256) void dual_dgrad_weights_kernel(const T* __restrict__ w, int K,
                                                                 const float* __restrict__ coef,
                                                                 T* __restrict__ w2, float* __restrict__ b) {
  __shared__ float red[4];
  const int c = blockIdx.x;
  const T* wr = w + (int64_t)c * K;
  T* o = w2 + (int64_t)c * 2 * K;
  float acc = 0.f;
  for (int k = threadIdx.x; k < K; k += 256) {
    const float wv = load1(wr + k);
    store1(o + k, wv * coef[k]);
    store1(o + K + k, wv * coef[K + k]);
    acc = __builtin_fmaf(wv, coef[2 * K + k], acc);
  }
  acc = warp_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) b[c] = (red[0] + red[1]) + (red[2] + red[3]);
}

static inline unsigned ew_blocks(int64_t total) {
  int64_t b = (total + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (unsigned)b;
}

}  // namespace dlmpi

using namespace dlmpi;

extern "C" int dlmpi_reduce_blocks(int64_t M, int C) {
  const int CC = C / 8;
  const int rpb = 256 / CC;
  int64_t b = (M + (int64_t)rpb * 16 - 1) / ((int64_t)rpb * 16);
  if (b > 1024) b = 1024;
  if (b < 1) b = 1;
  return (int)b;
}

// Storage-type dispatch of the templated kernels: f32 = 1 -> float activations (fp32 precision
// path), 0 -> bf16.  TA(p) casts a `const void*` / `void*` launcher argument to the chosen type.
#define LAUNCH_TLAUNCH(KER, GRID, ...)                                               \
  do {                                                                             \
    if (f32) {                                                                     \
      typedef float T;                                                             \
      hipLaunchKernelGGL(KER<T>, GRID, dim3(256), 0, s, __VA_ARGS__);              \
    } else {                                                                       \
      typedef uint16_t T;                                                          \
      hipLaunchKernelGGL(KER<T>, GRID, dim3(256), 0, s, __VA_ARGS__);              \
    }                                                                              \
  } while (0)
#define CT(p) static_cast<const T*>(p)
#define MT(p) static_cast<T*>(p)

extern "C" hipError_t dlmpi_bn_stats(const void* x, int64_t M, int C, int ldx, int xoff, float* partial, int nblk,
                                     int f32, hipStream_t s) {
  if (C % 8 || C > 2048) return hipErrorInvalidValue;
  LAUNCH_TLAUNCH(bn_stats_kernel, dim3(nblk), CT(x), M, C, ldx, xoff, partial);
  return hipGetLastError();
}

extern "C" int dlmpi_colsum_ws_doubles(int T, int C) { return colsum_slices(T) * 2 * C; }

// Self-resetting per-channel-group tickets of colsum_fin_kernel, one array per device, zeroed once
// (the first use happens before any hipGraph capture: the warm-up steps run eagerly).
// Last-arriver tickets of the fused finalize: one self-resetting array per device and stream
// ROLE.  Launches on one stream are serialised, so they can share an array; the engine's auxiliary
// streams (models/engine.py: the weight-gradient side stream and the residual-branch stream) run
// colsum_fin launches concurrently with the main stream's, so each role gets its own array.
// (Per role rather than per stream: a graph capture runs the main role on a fresh capture stream,
// where no allocation may happen.)
constexpr int kTicketRoles = 4;   // 0 = main (any unregistered stream), 1..3 = registered aux streams
static int* g_tickets[64] = {};
static hipStream_t g_aux_stream[64][kTicketRoles] = {};

static int* tickets_for_device(int dev) {
  if (!g_tickets[dev]) {
    int* p = nullptr;
    if (hipMalloc(&p, kTicketRoles * 4096 * sizeof(int)) != hipSuccess) return nullptr;
    if (hipMemset(p, 0, kTicketRoles * 4096 * sizeof(int)) != hipSuccess) return nullptr;
    g_tickets[dev] = p;
  }
  return g_tickets[dev];
}

static int* fin_tickets(hipStream_t s) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  int* t = tickets_for_device(dev);
  if (!t) return nullptr;
  for (int r = 1; r < kTicketRoles; ++r)
    if (s != nullptr && s == g_aux_stream[dev][r]) return t + r * 4096;
  return t;
}

static int role_of(hipStream_t s, int dev) {
  for (int r = 1; r < kTicketRoles; ++r)
    if (s != nullptr && s == g_aux_stream[dev][r]) return r;
  return 0;
}

// Split-K workspaces of the conv kernel (conv_igemm.hip), per device and stream role like the
// finalize tickets.  The slab grows on demand outside graph captures (the eager warm-up steps
// size it); inside a capture a too-small slab makes the launcher fall back to no split.
static float* g_sk_slab[64][kTicketRoles] = {};
static size_t g_sk_slab_floats[64][kTicketRoles] = {};
static int* g_sk_tk[64][kTicketRoles] = {};
constexpr int kSplitTickets = 4096;

extern "C" float* dlmpi_splitk_slab(hipStream_t s, size_t floats) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  const int r = role_of(s, dev);
  if (g_sk_slab_floats[dev][r] >= floats) return g_sk_slab[dev][r];
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return nullptr;
  // the old slab is never freed: a captured hipGraph may still reference it (a few MB, kept)
  const size_t n = floats + floats / 2;   // head room
  float* p = nullptr;
  if (hipMalloc(&p, n * sizeof(float)) != hipSuccess) return nullptr;
  g_sk_slab[dev][r] = p;
  g_sk_slab_floats[dev][r] = n;
  return p;
}

extern "C" int* dlmpi_splitk_tickets(hipStream_t s, int n) {
  int dev = 0;
  if (n > kSplitTickets || hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  const int r = role_of(s, dev);
  if (!g_sk_tk[dev][r]) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return nullptr;
    int* p = nullptr;
    if (hipMalloc(&p, kSplitTickets * sizeof(int)) != hipSuccess) return nullptr;
    if (hipMemsetAsync(p, 0, kSplitTickets * sizeof(int), s) != hipSuccess) return nullptr;   // ordered before the kernel
    g_sk_tk[dev][r] = p;
  }
  return g_sk_tk[dev][r];
}

static int colsum_direct_max() { return kDirectMaxT; }   // the kernel holds <= kDirectMaxT rows

static hipError_t colsum_finalize(const float* partial, int T, int C, int ns, int k2, double* ws, const FinArgs& f,
                                  hipStream_t s) {
  const int S = colsum_slices(T);
  const int G = (C + 63) / 64;
  if (T <= colsum_direct_max()) {
    hipLaunchKernelGGL(colsum_fin_direct_kernel, dim3((C + 15) / 16), dim3(1024), 0, s, partial, T, C, ns, k2, f);
    return hipGetLastError();
  }
  int* tk = G <= 4096 ? fin_tickets(s) : nullptr;
  if (tk) {
    hipLaunchKernelGGL(colsum_fin_kernel, dim3(G, S), dim3(256), 0, s, partial, T, C, ns, k2, ws, tk, f);
  } else {
    hipLaunchKernelGGL(colsum2_kernel, dim3(G, S), dim3(256), 0, s, partial, T, C, ns, k2, ws);
    hipLaunchKernelGGL(finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, s, ws, S, C, f);
  }
  return hipGetLastError();
}

extern "C" hipError_t dlmpi_outer_dgrad_bn(const void* dy, int lddy, int64_t M, int C, const void* w, int ldw,
                                         const void* z, const float* mscale, const float* mshift, void* dx,
                                         float* partial, int nblk, int f32, hipStream_t s) {
  if (C % 8 || C > 2048 || M <= 0) return hipErrorInvalidValue;
  LAUNCH_TLAUNCH(outer_dgrad_bn_kernel, dim3(nblk), CT(dy), lddy, M, C, CT(w), ldw, CT(z), mscale, mshift, MT(dx),
                partial);
  return hipGetLastError();
}

extern "C" hipError_t dlmpi_set_aux_stream(hipStream_t s, int role) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= 64 || role < 1 || role >= kTicketRoles || !tickets_for_device(dev))
    return hipErrorInvalidValue;   // (allocates outside any capture)
  g_aux_stream[dev][role] = s;
  return hipSuccess;
}

extern "C" hipError_t dlmpi_bn_finalize(const float* partial, int ntiles, int C, double count, const float* gamma,
                                        const float* beta, float* running_mean, float* running_var, float momentum,
                                        float eps, float* scale, float* shift, float* save_mean, float* save_invstd,
                                        double* ws, hipStream_t s) {
  FinArgs f{};
  f.mode = 0;
  f.count = count;
  f.gamma = gamma;
  f.beta = beta;
  f.running_mean = running_mean;
  f.running_var = running_var;
  f.momentum = momentum;
  f.eps = eps;
  f.scale = scale;
  f.shift = shift;
  f.save_mean = save_mean;
  f.save_invstd = save_invstd;
  return colsum_finalize(partial, ntiles, C, 2, 1, ws, f, s);
}

extern "C" hipError_t dlmpi_bn_apply2(const void* x, int ldx, int xoff, int64_t M, int C, const float* scale,
                                      const float* shift, const void* res, int ldres, int resoff, const float* rscale,
                                      const float* rshift, int relu, void* y, int ldy, int yoff, uint8_t* mbits,
                                      int f32, hipStream_t s) {
  if (C % 8 || ((rscale != nullptr) != (rshift != nullptr)) || (rscale && !res)) return hipErrorInvalidValue;
  const int64_t total = M * (C / 8);
  LAUNCH_TLAUNCH(bn_apply_kernel, dim3(ew_blocks(total)), CT(x), ldx, xoff, M, C, make_fastdiv(C / 8), scale, shift,
                CT(res), ldres, resoff, relu, MT(y), ldy, yoff, mbits, rscale, rshift);
  return hipGetLastError();
}

extern "C" hipError_t dlmpi_bn_apply(const void* x, int ldx, int xoff, int64_t M, int C, const float* scale,
                                     const float* shift, const void* res, int ldres, int resoff, int relu,
                                     void* y, int ldy, int yoff, uint8_t* mbits, int f32, hipStream_t s) {
  return dlmpi_bn_apply2(x, ldx, xoff, M, C, scale, shift, res, ldres, resoff, nullptr, nullptr, relu, y, ldy, yoff,
                         mbits, f32, s);
}

extern "C" hipError_t dlmpi_bn_bwd_reduce(const void* dy, int lddy, int dyoff, const void* ymask, int ldym,
                                          int ymoff, const void* x, int ldx, int xoff, int64_t M, int C,
                                          const float* mean, const float* invstd, float* partial, int nblk,
                                          int f32, hipStream_t s) {
  if (C % 8 || C > 2048) return hipErrorInvalidValue;
  LAUNCH_TLAUNCH(bn_bwd_reduce_kernel, dim3(nblk), CT(dy), lddy, dyoff, CT(ymask), ldym, ymoff, CT(x), ldx, xoff, M, C,
                mean, invstd, partial);
  return hipGetLastError();
}

extern "C" hipError_t dlmpi_bn_bwd_finalize_ex(const float* partial, int nblk, int ns, int k2, int raw_z, int C,
                                               double count, const float* gamma, const float* mean,
                                               const float* invstd, float* dgamma, float* dbeta, float* coef,
                                               double* ws, hipStream_t s) {
  if (ns < 2 || ns > 3 || k2 < 1 || k2 >= ns) return hipErrorInvalidValue;
  FinArgs f{};
  f.mode = 1;
  f.count = count;
  f.gamma = gamma;
  f.mean = mean;
  f.invstd = invstd;
  f.dgamma = dgamma;
  f.dbeta = dbeta;
  f.coef = coef;
  f.raw_z = raw_z;
  return colsum_finalize(partial, nblk, C, ns, k2, ws, f, s);
}

extern "C" hipError_t dlmpi_bn_bwd_finalize(const float* partial, int nblk, int C, double count, const float* gamma,
                                            const float* mean, const float* invstd, float* dgamma, float* dbeta,
                                            float* coef, double* ws, hipStream_t s) {
  return dlmpi_bn_bwd_finalize_ex(partial, nblk, 2, 1, 0, C, count, gamma, mean, invstd, dgamma, dbeta, coef, ws, s);
}

extern "C" hipError_t dlmpi_bn_bwd_apply(const void* dy, int lddy, int dyoff, const void* ymask, int ldym,
                                         int ymoff, const void* x, int ldx, int xoff, int64_t M, int C,
                                         const float* coef, void* dx, void* dyr_out, int f32, hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;
  const int64_t total = M * (C / 8);
  LAUNCH_TLAUNCH(bn_bwd_apply_kernel, dim3(ew_blocks(total)), CT(dy), lddy, dyoff, CT(ymask), ldym, ymoff, CT(x), ldx,
                xoff, M, C, make_fastdiv(C / 8), coef, MT(dx), MT(dyr_out));
  return hipGetLastError();
}


extern "C" hipError_t dlmpi_dual_dgrad_weights(const void* w, int C, int K, const float* coef, void* w2, float* b,
                                               int f32, hipStream_t s) {
  if (C <= 0 || K <= 0) return hipErrorInvalidValue;
  LAUNCH_TLAUNCH(dual_dgrad_weights_kernel, dim3(C), CT(w), K, coef, MT(w2), b);
  return hipGetLastError();
}

extern "C" hipError_t dlmpi_channel_sum(const void* x, int64_t M, int C, int ldx, int xoff, float* out_acc,
                                        float* partial, int nblk, double* ws, int f32, hipStream_t s) {
  hipError_t e = dlmpi_bn_bwd_reduce(x, ldx, xoff, nullptr, 0, 0, nullptr, 0, 0, M, C, nullptr, nullptr, partial,
                                     nblk, f32, s);
  if (e != hipSuccess) return e;
  return dlmpi_bn_bwd_finalize(partial, nblk, C, (double)M, nullptr, nullptr, nullptr, nullptr, out_acc, nullptr, ws,
                               s);
}

extern "C" hipError_t dlmpi_maxpool_bwd_bn(const void* dy, const uint8_t* idx, int N, int H, int W, int C, int k,
                                           int stride, int pad, int OH, int OW, const void* z, const float* mscale,
                                           const float* mshift, const void* add, int ldadd, int addoff,
                                           void* dx, float* partial, int nblk, int f32, hipStream_t s) {
  if (C % 8 || C > 2048 || (int64_t)N * H * W >= (1ll << 31)) return hipErrorInvalidValue;
  const int nw = (k + stride - 1) / stride;
#define LAUNCH_MPB1(NW, T)                                                                                          \
  hipLaunchKernelGGL((maxpool_bwd_bn_kernel<NW, T>), dim3(nblk), dim3(256), 0, s, CT(dy), idx, N, H, W, C, k, stride, \
                     pad, OH, OW, make_fastdiv(W), make_fastdiv(H), CT(z), mscale, mshift, CT(add), ldadd, addoff,   \
                     MT(dx), partial)
#define LAUNCH_MPB(NW)          \
  do {                         \
    if (f32) {                 \
      typedef float T;         \
      LAUNCH_MPB1(NW, T);       \
    } else {                   \
      typedef uint16_t T;      \
      LAUNCH_MPB1(NW, T);       \
    }                          \
  } while (0)
  // fixed window extents for the 2x2/s2 and 3x3/s2 pools; NW 0: the general window loop
  if (nw == 1) LAUNCH_MPB(1);
  else if (nw == 2) LAUNCH_MPB(2);
  else LAUNCH_MPB(0);
#undef LAUNCH_MPB
#undef LAUNCH_MPB1
  return hipGetLastError();
}
