// 3x3 / stride 1 / pad 1 convolution of an 8-channel input (the padded RGB / grey image) into 64
// channels -- the UNet input conv (/root/reference/pytorch/unet/model.py:10, DoubleConv of
// in_channels -> 64) -- with bias and the BN-statistics epilogue.
//
// Through the generic implicit GEMM this shape ran at 1.9 TB/s of output (289 us at 16 x 512^2,
// 8-wide K slices of a 64-wide K step).  The reduction is only 9 taps x 8 channels = 72, so here it is
// three K = 32 steps of v_mfma_f32_16x16x32_bf16 with (tap, channel) as the K index: the 8 K values a
// lane supplies are ONE tap's 8 channels -- one 16-byte global load of the shifted pixel (zero outside
// the image, taps 9-11 zero) -- and the weights (64 x 96, zero padded) live in registers for the
// whole persistent loop.  The product is computed transposed, D[channel][pixel] (weights as the A
// operand), so a lane holds 4 consecutive channels of one pixel; the wave assembles its 64 output
// rows in LDS (XOR-swizzled 16-B chunks) and stores them as whole 128-B rows, 16 B per lane (the
// 8-byte scattered stores straight from the accumulators ran at 2.3 TB/s).  Each wave takes 2 groups
// of 16 consecutive pixels of a row per iteration.
// BN statistics: per-lane fp32 sums of the stored (bf16) values, a fixed shuffle tree over the 16
// pixels of a lane group, the 4 waves combined in LDS in wave order -> stats[block][2][64].
#include "common.h"

namespace dlmpi {

// The same scheme, generalized (conv_small_kernel<CIN, TR, TS, PAD, GP>): a TR x TS / stride-1 / pad-PAD
// convolution of a CIN-channel input (CIN 8 or 16) into 64 channels.  K index = tap * CIN + channel;
// a lane group supplies 8 channels of one tap (CIN / 8 lane groups per tap, 32 / CIN taps per K
// step).  Instances:
//   <8, 3, 3, 1, 2>  the UNet input conv (3 K steps, taps 9-11 zero);
//   <16, 4, 4, 0, 1> the ResNet stem as the 4x4 stride-1 conv over its 2x2 space-to-depth image
//                    (models/engine.py S2DConvUnit: 16 taps x 16 channels = 8 K steps, the padding is
//                    in the image, so no bounds checks).  Through the generic GEMM (256 x 64 tiles of
//                    16-B-piece taps) it ran at 1.5 TB/s of output: 268 us at bs 256 for a 411 MB store.
template <int CIN, int TR, int TS, int PAD, int GP>
__global__ __launch_bounds__(256) void conv_small_kernel(const uint16_t* __restrict__ x, int ldx, int xoff, int N,
                                                        int H, int W, int P, int Q, const uint16_t* __restrict__ w,
                                                        const float* __restrict__ bias, uint16_t* __restrict__ y,
                                                        int ldy, int yoff, float* __restrict__ stats) {
  constexpr int LPT = CIN / 8;                    // lane groups per tap
  constexpr int TPK = 4 / LPT;                    // taps per K step
  constexpr int NTAP = TR * TS, KTOT = NTAP * CIN;
  constexpr int KS = (NTAP + TPK - 1) / TPK;      // K steps of 32
  static_assert(CIN == 8 || CIN == 16, "8 or 16 input channels");
  // per wave: the 16 GP output pixels of an iteration, 128 B each, 16-B chunks XOR-swizzled by (pixel & 7)
  __shared__ __attribute__((aligned(16))) char tile[4][GP * 16 * 128];
  __shared__ float red[4][2][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g = lane >> 4, i = lane & 15;
  char* const wt = tile[wid];
  // weights: A operand of channel tile ct, K step k: row 16 ct + i, K 32 k + 8 g .. + 7 = tap TPK k + g / LPT,
  // channels 8 (g % LPT) ..
  bf16x8 wf[4][KS];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const int tap = TPK * k + g / LPT;
      u32x4 v = u32x4{0u, 0u, 0u, 0u};
      if (tap < NTAP) v = *reinterpret_cast<const u32x4*>(w + (16 * ct + i) * KTOT + tap * CIN + 8 * (g % LPT));
      wf[ct][k] = __builtin_bit_cast(bf16x8, v);
    }
  float bv[4][4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[ct][r] = bias ? bias[16 * ct + 4 * g + r] : 0.f;
  float ssum[4][4] = {}, ssq[4][4] = {};
  // this lane's tap of each K step: row / column offsets and channel chunk
  int dr[KS], ds[KS];
  bool tv[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) {
    const int tap = TPK * k + g / LPT;
    tv[k] = tap < NTAP;
    dr[k] = tap / TS - PAD;
    ds[k] = tap % TS - PAD;
  }
  const int cofs = xoff + 8 * (g % LPT);
  const uint32_t uQ = Q, uP = P;
  const uint32_t ngroups = (uint32_t)((int64_t)N * P * Q / 16);   // host: N P Q < 2^31, Q % 16 == 0
  const uint32_t nwaves = gridDim.x * 4;
  for (uint32_t g0 = (blockIdx.x * 4 + wid) * GP; g0 < ngroups; g0 += nwaves * GP) {
    bf16x8 xf[GP][KS];
#pragma unroll
    for (int q = 0; q < GP; ++q) {
      const uint32_t grp = g0 + q;
      const uint32_t row = grp * 16 / uQ;                 // output row n * P + p of the 16-pixel group
      const int wc = (int)(grp * 16 - row * uQ) + i;
      const uint32_t n = row / uP;
      const int h = (int)(row - n * uP);
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        const int hh = h + dr[k], ww = wc + ds[k];
        u32x4 v = u32x4{0u, 0u, 0u, 0u};
        const bool in = PAD == 0 || ((unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W);
        if (grp < ngroups && tv[k] && in)
          v = *reinterpret_cast<const u32x4*>(x + ((int64_t)((int)n * H + hh) * W + ww) * ldx + cofs);
        xf[q][k] = __builtin_bit_cast(bf16x8, v);
      }
    }
#pragma unroll
    for (int q = 0; q < GP; ++q) {
      f32x4 acc[4];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        acc[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < KS; ++k) acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ct][k], xf[q][k], acc[ct], 0, 0, 0);
      }
      const bool live = g0 + q < ngroups;
      const int px = q * 16 + i;
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[ct][r] + bv[ct][r];
        const u32x2 pk = u32x2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
        // channels 16 ct + 4 g .. +3 = bytes 32 ct + 8 g: 16-B chunk 2 ct + (g >> 1), half g & 1
        const int ch = (2 * ct + (g >> 1)) ^ (px & 7);
        *reinterpret_cast<u32x2*>(wt + px * 128 + ch * 16 + (g & 1) * 8) = pk;
        if (stats && live) {
          const float s0 = bf2f((uint16_t)(pk[0] & 0xffffu)), s1 = bf2f((uint16_t)(pk[0] >> 16));
          const float s2 = bf2f((uint16_t)(pk[1] & 0xffffu)), s3 = bf2f((uint16_t)(pk[1] >> 16));
          ssum[ct][0] += s0; ssq[ct][0] += s0 * s0;
          ssum[ct][1] += s1; ssq[ct][1] += s1 * s1;
          ssum[ct][2] += s2; ssq[ct][2] += s2 * s2;
          ssum[ct][3] += s3; ssq[ct][3] += s3 * s3;
        }
      }
    }
    // this wave's LDS writes have landed before its reads (same wave, in order)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // rows: 8 pixels x 8 chunks per wave instruction, 16 B per lane, 1 KB contiguous when ldy == 64
#pragma unroll
    for (int t = 0; t < GP * 2; ++t) {
      const int px = t * 8 + (lane >> 3), c = lane & 7;
      const u32x4 v = *reinterpret_cast<const u32x4*>(wt + px * 128 + ((c ^ (px & 7)) << 4));
      const uint32_t grp = g0 + (px >> 4);
      if (grp < ngroups)
        *reinterpret_cast<u32x4*>(y + ((int64_t)grp * 16 + (px & 15)) * ldy + yoff + c * 8) = v;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (!stats) return;
  // over the 16 pixels (lanes i) of each lane group, then the 4 waves in order
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) {
        ssum[ct][r] += __shfl_xor(ssum[ct][r], o, 64);
        ssq[ct][r] += __shfl_xor(ssq[ct][r], o, 64);
      }
  if (i == 0) {
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        red[wid][0][16 * ct + 4 * g + r] = ssum[ct][r];
        red[wid][1][16 * ct + 4 * g + r] = ssq[ct][r];
      }
  }
  __syncthreads();
  if (threadIdx.x < 128) {
    const int s = threadIdx.x >> 6, c = threadIdx.x & 63;
    stats[((int64_t)blockIdx.x * 2 + s) * 64 + c] = ((red[0][s][c] + red[1][s][c]) + red[2][s][c]) + red[3][s][c];
  }
}

}  // namespace dlmpi

using namespace dlmpi;

extern "C" int dlmpi_conv3x3_c8_blocks(int64_t pixels) {
  const int64_t groups = (pixels + 15) / 16;
  return (int)std::max<int64_t>(1, std::min<int64_t>(1024, (groups + 15) / 16));
}

extern "C" hipError_t dlmpi_conv3x3_c8(const void* x, int ldx, int xoff, int N, int H, int W, const void* w,
                                       const float* bias, void* y, int ldy, int yoff, float* stats, int G,
                                       hipStream_t s) {
  if (W % 16 || ldx % 8 || xoff % 8 || ldy % 8 || yoff % 8 || G <= 0 || (int64_t)N * H * W >= (1ll << 31))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL((conv_small_kernel<8, 3, 3, 1, 2>), dim3((unsigned)G), dim3(256), 0, s,
                     static_cast<const uint16_t*>(x), ldx, xoff, N, H, W, H, W, static_cast<const uint16_t*>(w), bias,
                     static_cast<uint16_t*>(y), ldy, yoff, stats);
  return hipGetLastError();
}

// The ResNet stem on its space-to-depth image: 4 x 4 taps, 16 channels, no padding (input U x V, output
// (U - 3) x (V - 3)).  Blocks: the same rule as the 8-channel kernel (~16 pixel groups per block).
extern "C" int dlmpi_conv4x4_c16_blocks(int64_t pixels) { return dlmpi_conv3x3_c8_blocks(pixels); }

extern "C" hipError_t dlmpi_conv4x4_c16(const void* x, int ldx, int xoff, int N, int U, int V, const void* w,
                                        const float* bias, void* y, int ldy, int yoff, float* stats, int G,
                                        hipStream_t s) {
  const int P = U - 3, Q = V - 3;
  if (P <= 0 || Q % 16 || ldx % 8 || xoff % 8 || ldy % 8 || yoff % 8 || G <= 0 ||
      (int64_t)N * U * V * ldx >= (1ll << 31) || (int64_t)N * P * Q * ldy >= (1ll << 31))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL((conv_small_kernel<16, 4, 4, 0, 1>), dim3((unsigned)G), dim3(256), 0, s,
                     static_cast<const uint16_t*>(x), ldx, xoff, N, U, V, P, Q, static_cast<const uint16_t*>(w), bias,
                     static_cast<uint16_t*>(y), ldy, yoff, stats);
  return hipGetLastError();
}
