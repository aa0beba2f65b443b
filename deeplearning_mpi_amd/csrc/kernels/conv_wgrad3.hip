// Weight gradient of a 3x3 / stride-1 / pad-1 convolution by SPATIAL tiles (bf16 MFMA, fp32 slabs):
//
//   dW[ko][r][s][c] = sum_{n,h,w} dY[n,h,w][ko] * X[n, h+r-1, w+s-1][c]
//
// The general weight-gradient kernel (conv_wgrad.hip) reduces over 64 consecutive output pixels per
// K-step and gathers X once per (pixel, tap): every X element is fetched 9 times per Ko tile and
// every K-step pays a per-lane im2col decode.  Here a K-step is an 8 x 8 block of output pixels of
// one image: its dY rows [64][KT] and the 10 x 10 X halo around it [100][CT] are staged once
// (LDS-DMA through a 3-stage ring, issued through glds16_raw, so the compiler adds no drain before
// the transposed reads -- with the builtin it did, and no DMA latency was hidden: profiles/r5_wgrad),
// and all 9 taps are 9 GEMMs over the SAME staged tiles --
// tap (r, s) reads the halo window shifted by (r, s).  Out-of-image halo pixels are staged as
// zeros, which IS the zero padding for every tap, so no per-tap masking exists anywhere.  The
// block owns dW for all 9 taps of a KT x CT (ko, c) tile: 9 x (KT x CT) fp32 accumulators over 8
// waves, A fragments (dY) shared by the 9 taps.
//
// Operands are pixel-major in LDS (the reduction index is the row), fed to
// v_mfma_f32_16x16x32_bf16 through the transposing read ds_read_b64_tr_b16 (T10), as in
// conv_wgrad.hip.  Halo rows are numbered line * 10 + col (line/col = halo row/column); the
// 16-byte chunk XOR of a halo row is a function of (line, col) chosen so that the 8 rows one
// half-wave's transposed read touches -- columns c0..c0+3 of lines L and L+1 -- land on disjoint
// bank groups for every tap shift.
//
// Split over pixel tiles: split z writes its 9 x KT x CT partial into the [splits][Ko][9C] fp32
// workspace of the general path, whose two reduction kernels (conv_wgrad.hip) sum the splits in a
// fixed order into the fp32 gradient (bit-reproducible, no atomics).
//
// Reference semantics: nn.Conv2d(3x3, padding=1) weight gradient of every UNet DoubleConv and the
// ResNet bottleneck conv2 (/root/reference/pytorch/unet/model.py:9-14, resnet main.py:40-41).
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace dlmpi {

typedef __attribute__((address_space(3))) i16x4 w3_lds_i16x4;

// 16-byte chunk XOR of a row holding 8 consecutive output pixels (dY tile: row = pixel k of the
// 8 x 8 block, a half-wave reads rows k0 + q, k0 + 8 + q, q < 4)
template <int ROW>
__device__ __forceinline__ int w3_dy_swz(int row) {
  if constexpr (ROW == 256) return ((row & 3) << 2) | ((row >> 2) & 3);
  else return (((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2);
}

// 16-byte chunk XOR of halo row (line, col): a half-wave reads cols c..c+3 of lines L, L+1.
//   128-B rows: rows of equal parity share a 32-bank half -> pair index ^ {col bit 1, line bit 0}
//   256-B rows: a row spans all banks -> pair index ^ {col & 3, line bit 0} (8 distinct pairs)
template <int ROW>
__device__ __forceinline__ int w3_halo_swz(int line, int col) {
  if constexpr (ROW == 256) return ((((col & 3) << 1) | (line & 1)) << 1);
  else return ((((col >> 1) & 1) | ((line & 1) << 1)) << 1);
}

// KT x CT block tile over WR x WC waves; every wave owns 64 (ko) x 16 (c) x 9 taps (144 fp32
// accumulators): 4 dY fragments shared by the 9 taps, 1 X fragment per tap -- (64 + 9 x 16) rows of
// transposed reads per 9 x 64 x 16 MACs.  128 x 64 = 2 x 4 waves, 64 x 128 = 1 x 8, 64 x 64 = 1 x 4
// (a 4-wave block, 2 per CU: the 2 x 2 grid of 32 x 16 wave tiles it replaced read 1.7x the LDS
// bytes per MFMA).
//
// Pipeline (round 6, profiles/r6_wgrad3: -9 to -10 % on every UNet / ResNet 3x3 shape against the
// round-5 double buffer, bit-identical):
//  * a 3-stage LDS ring: the DMA of step t + 2 is issued during step t (two steps of latency cover;
//    a 4th stage measured no better, and costs the 64 x 64 tile its second block per CU);
//  * a wave's AL + BL DMA pieces go out one per tap slot of the first 32 pixels, between its MFMAs,
//    instead of all at once after the barrier (where every wave of the CU issued at once);
//  * the step loop is unrolled by the 3 stages, so each stage index is a constant: LDS holds the
//    three A stages, then the three B stages, and every fragment read is a loop-invariant lane offset
//    plus an immediate (no address arithmetic per read);
//  * every step issues a DMA (past the split's last tile: that tile again, into the stage nobody
//    reads), so the vmcnt of a step is a constant.
template <int KT, int CT, int WR, int WC>
__global__ __launch_bounds__(64 * WR * WC) __attribute__((amdgpu_waves_per_eu(2, 8)))
void wgrad3x3_kernel(const Wgrad3Args a) {
  constexpr int STAGES = 3;
  constexpr int NT = 64 * WR * WC;
  constexpr int WM = KT / WR, WN = CT / WC;   // per-wave ko x c
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int A_ROW = KT * 2, B_ROW = CT * 2;
  constexpr int A_BYTES = 64 * A_ROW;         // 64 output pixels
  constexpr int B_BYTES = 128 * B_ROW;        // 100 halo rows, slots of rows 100..127 unused
  constexpr int AL = A_BYTES / (16 * NT), BL = B_BYTES / (16 * NT);
  constexpr int PER = AL + BL;                // DMA pieces per wave per step
  static_assert(AL >= 1 && BL >= 1 && TM >= 1 && TN >= 1 && PER <= 9, "tile shape");
  __shared__ __attribute__((aligned(16))) char smem[STAGES * (A_BYTES + B_BYTES)];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WC, wn = wid % WC;
  const uint32_t nkc = (uint32_t)a.mtiles * a.ntiles;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int z = bid / nkc;
  const int kc = bid - z * nkc;
  // consecutive blocks (one XCD's range, xcd_remap) walk the ko tiles fastest: an XCD's blocks share
  // a few X tiles AND a few dY tiles in its L2 (ko-slowest: every X tile of the row once per XCD; L2
  // hit rate 66 % -> 81 % at 64^2 1536 -> 512, profiles/r6_wgrad3)
  const int mt = kc % a.mtiles, nt = kc / a.mtiles;
  const int ko0 = mt * KT, c0 = nt * CT;
  const int t_beg = z * a.tiles_per_split;
  const int t_end = min(a.ntiles_pix, t_beg + a.tiles_per_split);
  if (t_beg >= t_end) return;   // (never: the host sizes the splits to the tiles)
  const char* zp = reinterpret_cast<const char*>(g_zero_page);
  const int H = a.H, W = a.W;

  // ---- per-thread staging pieces (fixed slot -> (row, chunk) map) --------------------------
  // A piece: pixel (pi, pj) of the 8 x 8 block; B piece: halo (line, col) (line 10+: unused slot).
  // The byte offset of a piece from its tile origin (pixel (h0, w0) of image n) is fixed per thread;
  // per K-step only the origin (a scalar) and the bounds test change.
  int a_pi[AL], a_pj[AL], a_off[AL];
#pragma unroll
  for (int i = 0; i < AL; ++i) {
    const int o = NT * i + tid;
    const int row = (o * 16) / A_ROW, pos = (o * 16 % A_ROW) / 16;
    a_pi[i] = row >> 3;
    a_pj[i] = row & 7;
    a_off[i] = 2 * ((a_pi[i] * W + a_pj[i]) * a.ldy + a.dyoff + ko0 + 8 * (pos ^ w3_dy_swz<A_ROW>(row)));
  }
  int b_li[BL], b_co[BL], b_off[BL];
#pragma unroll
  for (int i = 0; i < BL; ++i) {
    const int o = NT * i + tid;
    const int row = (o * 16) / B_ROW, pos = (o * 16 % B_ROW) / 16;
    const int line = row / 10, col = row - line * 10;
    b_li[i] = row < 100 ? line - 1 : -1000;   // halo line / col relative to the tile origin
    b_co[i] = col - 1;
    b_off[i] = row < 100 ? 2 * ((b_li[i] * W + b_co[i]) * a.ldx + a.xoff + c0 + 8 * (pos ^ w3_halo_swz<B_ROW>(line, col))) : 0;
  }
  const char* dyb = static_cast<const char*>(a.dy);
  const char* xb = static_cast<const char*>(a.x);
  char* const sA = smem;                        // A stages
  char* const sB = smem + STAGES * A_BYTES;     // B stages

  // the tile whose DMA goes out next (walked incrementally, wave-uniform; clamped to the last tile)
  int n = 0, ti = 0, tj = 0, t_iss = t_beg;
  {
    const int per_img = a.tiles_h * a.tiles_w;
    n = t_beg / per_img;
    const int rem = t_beg - n * per_img;
    ti = rem / a.tiles_w;
    tj = rem - ti * a.tiles_w;
  }
  const char* da = nullptr;   // origin of the tile being issued
  const char* db = nullptr;
  int ih0 = 0, iw0 = 0;
  auto set_origin = [&]() {
    ih0 = ti * 8;
    iw0 = tj * 8;
    const int64_t pix = ((int64_t)n * H + ih0) * W + iw0;
    da = dyb + 2 * pix * a.ldy;
    db = xb + 2 * pix * a.ldx;
    if (++t_iss < t_end && ++tj == a.tiles_w) {
      tj = 0;
      if (++ti == a.tiles_h) { ti = 0; ++n; }
    }
  };
  auto piece = [&](int buf, int i) {
    if (i < AL) {
      const bool ok = a_pi[i] < H - ih0 && a_pj[i] < W - iw0;
      glds16_raw(ok ? da + a_off[i] : zp, sA + buf * A_BYTES + 16 * (NT * i + 64 * wid));
    } else {
      const int j = i - AL;
      const bool ok = (unsigned)(ih0 + b_li[j]) < (unsigned)H && (unsigned)(iw0 + b_co[j]) < (unsigned)W;
      glds16_raw(ok ? db + b_off[j] : zp, sB + buf * B_BYTES + 16 * (NT * j + 64 * wid));
    }
  };

  // ---- fragment reads: loop-invariant lane byte offsets (kk = 0; kk = 1 adds an immediate) ------
  // dY fragment mi: ko columns 16 cb .. +15, pixels kk*32 + 8g + {q, q+4}; X fragment of tap t = (r, s):
  // c columns 16 cb .. +15, the same pixels -> halo (line, col) = (4 kk + g + r, {q, q+4} + s)
  const int g = lane >> 4, fi = lane & 15, q = fi >> 2, p = fi & 3;
  int a_ln[TM][2], b_ln[9][TN][2];
#pragma unroll
  for (int mi = 0; mi < TM; ++mi)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r0 = 8 * g + q + 4 * h;
      const int ch = 2 * ((wm * WM) / 16 + mi) + (p >> 1);
      a_ln[mi][h] = r0 * A_ROW + ((ch ^ w3_dy_swz<A_ROW>(r0)) << 4) + (p & 1) * 8;
    }
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int ni = 0; ni < TN; ++ni)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int line = g + t / 3, col = q + t % 3 + 4 * h;
        const int ch = 2 * ((wn * WN) / 16 + ni) + (p >> 1);
        b_ln[t][ni][h] = (line * 10 + col) * B_ROW + ((ch ^ w3_halo_swz<B_ROW>(line, col)) << 4) + (p & 1) * 8;
      }
  auto rd = [](const char* ptr) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((w3_lds_i16x4*)(ptr)); };
  auto frag = [](i16x4 v0, i16x4 v1) -> bf16x8 {
    typedef short i16x8 __attribute__((ext_vector_type(8)));
    return __builtin_bit_cast(bf16x8, (i16x8)__builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
  };

  f32x4 acc[9][TM][TN];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) acc[t][mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int st = 0; st < STAGES - 1; ++st) {
    set_origin();
#pragma unroll
    for (int i = 0; i < PER; ++i) piece(st, i);
  }
  // one K-step on stage S (a constant)
  auto step = [&](auto Sc) {
    constexpr int S = decltype(Sc)::value;
    constexpr int NB = (S + STAGES - 1) % STAGES;   // the stage refilled during this step
    // stage S landed (this wave's DMA: only the newer stage may still be in flight; every wave's: the
    // barrier); every wave's reads of stage NB (the previous step) have returned (lgkmcnt(0)).  The DMA
    // goes through glds16_raw, so no compiler wait drains it before the fragment reads.
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)" ::"n"((STAGES - 2) * PER) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    set_origin();
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const char* As = sA + S * A_BYTES + kk * 32 * A_ROW;
      const char* Bs = sB + S * B_BYTES + kk * 4 * 10 * B_ROW;
      bf16x8 af[TM];
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) af[mi] = frag(rd(As + a_ln[mi][0]), rd(As + a_ln[mi][1]));
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        bf16x8 bfr[TN];
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) bfr[ni] = frag(rd(Bs + b_ln[t][ni][0]), rd(Bs + b_ln[t][ni][1]));
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int ni = 0; ni < TN; ++ni)
            acc[t][mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfr[ni], acc[t][mi][ni], 0, 0, 0);
        if (kk == 0) {   // DMA piece i after tap slot (9 i) / PER
#pragma unroll
          for (int i = 0; i < PER; ++i)
            if ((9 * i) / PER == t) piece(NB, i);
        }
      }
    }
  };
  for (int t = t_beg; t < t_end; t += STAGES) {
    step(std::integral_constant<int, 0>{});
    if (t + 1 < t_end) step(std::integral_constant<int, 1>{});
    if (t + 2 < t_end) step(std::integral_constant<int, 2>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the trailing (unread) DMA lands before exit

  // ---- partial of this split: ws[z][ko][tap * C + c] (D: lane holds c = lane & 15, ko rows 4g + j)
  float* wsz = a.ws + (int64_t)z * a.Ko * (9 * a.C);
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int c = c0 + wn * WN + ni * 16 + fi;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int ko = ko0 + wm * WM + mi * 16 + 4 * g + j;
          wsz[(int64_t)ko * (9 * a.C) + t * a.C + c] = acc[t][mi][ni][j];
        }
      }
}

}  // namespace dlmpi

using namespace dlmpi;

// 128-row Ko tiles where they fit (64-row tiles everywhere -- 156 instead of 252 VGPRs, room on every
// SIMD for a wave of the concurrent data-gradient chain -- measured no better, profiles/r3_w3blocks)
extern "C" int dlmpi_wgrad3_plan(int Ko, int C, int* kt, int* ct) {
  if (Ko % 64 || C % 64) return 0;
  *kt = Ko % 128 == 0 ? 128 : 64;
  *ct = (*kt == 64 && C % 128 == 0) ? 128 : 64;
  return 1;
}

extern "C" hipError_t dlmpi_wgrad3x3(const Wgrad3Args* a, int kt, int ct, hipStream_t s) {
  const unsigned nwg = (unsigned)(a->mtiles * a->ntiles * a->splits);
  if (nwg == 0) return hipSuccess;
  const dim3 g(nwg);
  if (kt == 128 && ct == 64) hipLaunchKernelGGL((wgrad3x3_kernel<128, 64, 2, 4>), g, dim3(512), 0, s, *a);
  else if (kt == 64 && ct == 128) hipLaunchKernelGGL((wgrad3x3_kernel<64, 128, 1, 8>), g, dim3(512), 0, s, *a);
  else if (kt == 64 && ct == 64) hipLaunchKernelGGL((wgrad3x3_kernel<64, 64, 1, 4>), g, dim3(256), 0, s, *a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}
