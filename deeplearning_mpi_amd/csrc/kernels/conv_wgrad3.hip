// Weight gradient of a 3x3 / stride-1 / pad-1 convolution by SPATIAL tiles (bf16 MFMA, fp32 slabs):
//
//   dW[ko][r][s][c] = sum_{n,h,w} dY[n,h,w][ko] * X[n, h+r-1, w+s-1][c]
//
// The general weight-gradient kernel (conv_wgrad.hip) reduces over 64 consecutive output pixels per
// K-step and gathers X once per (pixel, tap): every X element is fetched 9 times per Ko tile and
// every K-step pays a per-lane im2col decode.  Here a K-step is an 8 x 8 block of output pixels of
// one image: its dY rows [64][KT] and the 10 x 10 X halo around it [100][CT] are staged once
// (LDS-DMA, double-buffered: the next block's DMA is issued right after the K-step's barrier through
// glds16_raw, so the compiler adds no drain before the transposed reads -- with the builtin it did,
// and no DMA latency was hidden: profiles/r5_wgrad), and all 9 taps are 9 GEMMs over the SAME staged tiles --
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
template <int KT, int CT, int WR, int WC>
__global__ __launch_bounds__(64 * WR * WC) __attribute__((amdgpu_waves_per_eu(2, 8)))
void wgrad3x3_kernel(const Wgrad3Args a) {
  constexpr int NT = 64 * WR * WC;
  constexpr int WM = KT / WR, WN = CT / WC;   // per-wave ko x c
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int A_ROW = KT * 2, B_ROW = CT * 2;
  constexpr int A_BYTES = 64 * A_ROW;         // 64 output pixels
  constexpr int B_BYTES = 128 * B_ROW;        // 100 halo rows, slots of rows 100..127 unused
  constexpr int SB = A_BYTES + B_BYTES;
  constexpr int AL = A_BYTES / (16 * NT), BL = B_BYTES / (16 * NT);
  static_assert(AL >= 1 && BL >= 1 && TM >= 1 && TN >= 1, "tile shape");
  __shared__ __attribute__((aligned(16))) char smem[2 * SB];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WC, wn = wid % WC;
  const uint32_t nkc = (uint32_t)a.mtiles * a.ntiles;
  const uint32_t bid = xcd_remap(blockIdx.x, gridDim.x);
  const int z = bid / nkc;
  const int kc = bid - z * nkc;
  const int mt = kc / a.ntiles, nt = kc - mt * a.ntiles;
  const int ko0 = mt * KT, c0 = nt * CT;
  const int t_beg = z * a.tiles_per_split;
  const int t_end = min(a.ntiles_pix, t_beg + a.tiles_per_split);
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

  auto issue = [&](int buf, int n, int h0, int w0) {
    char* As = smem + buf * SB;
    char* Bs = As + A_BYTES;
    const int64_t pix = ((int64_t)n * H + h0) * W + w0;   // wave-uniform tile origin
    const char* da = dyb + 2 * pix * a.ldy;
    const char* db = xb + 2 * pix * a.ldx;
    const int hl = H - h0, wl = W - w0;
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      const bool ok = a_pi[i] < hl && a_pj[i] < wl;
      const char* src = ok ? da + a_off[i] : zp;
      glds16_raw(src, As + 16 * (NT * i + 64 * wid));
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const bool ok = (unsigned)(h0 + b_li[i]) < (unsigned)H && (unsigned)(w0 + b_co[i]) < (unsigned)W;
      const char* src = ok ? db + b_off[i] : zp;
      glds16_raw(src, Bs + 16 * (NT * i + 64 * wid));
    }
  };

  // ---- fragment reads ------------------------------------------------------------------------
  const int g = lane >> 4, fi = lane & 15, q = fi >> 2, p = fi & 3;
  auto tr2 = [](const char* p0, const char* p1) -> bf16x8 {
    const i16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((w3_lds_i16x4*)(p0));
    const i16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((w3_lds_i16x4*)(p1));
    typedef short i16x8 __attribute__((ext_vector_type(8)));
    return __builtin_bit_cast(bf16x8, (i16x8)__builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  // dY fragment: ko columns 16 cb .. +15, pixels kk*32 + 8g + {q, q+4}
  auto a_frag = [&](const char* As, int kk, int cb) -> bf16x8 {
    const int r0 = kk * 32 + 8 * g + q;
    const int ch = 2 * cb + (p >> 1);
    const char* p0 = As + r0 * A_ROW + ((ch ^ w3_dy_swz<A_ROW>(r0)) << 4) + (p & 1) * 8;
    const char* p1 = As + (r0 + 4) * A_ROW + ((ch ^ w3_dy_swz<A_ROW>(r0 + 4)) << 4) + (p & 1) * 8;
    return tr2(p0, p1);
  };
  // X fragment of tap (r, s): c columns 16 cb .. +15, pixels kk*32 + 8g + {q, q+4} -> halo
  // (line, col) = (4 kk + g + r, {q, q+4} + s)
  auto b_frag = [&](const char* Bs, int kk, int r, int s, int cb) -> bf16x8 {
    const int line = 4 * kk + g + r, col = q + s;
    const int ch = 2 * cb + (p >> 1);
    const char* p0 = Bs + (line * 10 + col) * B_ROW + ((ch ^ w3_halo_swz<B_ROW>(line, col)) << 4) + (p & 1) * 8;
    const char* p1 = Bs + (line * 10 + col + 4) * B_ROW + ((ch ^ w3_halo_swz<B_ROW>(line, col + 4)) << 4) + (p & 1) * 8;
    return tr2(p0, p1);
  };

  f32x4 acc[9][TM][TN];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) acc[t][mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};

  // pixel-tile walk: tile t -> (n, ti, tj), advanced incrementally (wave-uniform)
  int n = 0, ti = 0, tj = 0;
  if (t_beg < t_end) {
    const int per_img = a.tiles_h * a.tiles_w;
    n = t_beg / per_img;
    const int rem = t_beg - n * per_img;
    ti = rem / a.tiles_w;
    tj = rem - ti * a.tiles_w;
    issue(0, n, ti * 8, tj * 8);
  }
  for (int t = t_beg; t < t_end; ++t) {
    const int cur = (t - t_beg) & 1;
    if (++tj == a.tiles_w) {
      tj = 0;
      if (++ti == a.tiles_h) { ti = 0; ++n; }
    }
    // stage cur landed (this wave's DMA: vmcnt(0); every wave's: the barrier); every wave's reads of
    // stage cur^1 (step t - 1) have returned (lgkmcnt(0)) -> it may be refilled.  The DMA is issued
    // through glds16_raw, so no compiler wait drains it before the fragment reads below: it has the
    // whole K-step to land.
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 1 < t_end) issue(cur ^ 1, n, ti * 8, tj * 8);
    const char* As = smem + cur * SB;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[TM];
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) af[mi] = a_frag(As, kk, (wm * WM) / 16 + mi);
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          bf16x8 bfr[TN];
#pragma unroll
          for (int ni = 0; ni < TN; ++ni) bfr[ni] = b_frag(Bs, kk, r, s, (wn * WN) / 16 + ni);
#pragma unroll
          for (int mi = 0; mi < TM; ++mi)
#pragma unroll
            for (int ni = 0; ni < TN; ++ni)
              acc[r * 3 + s][mi][ni] =
                  __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfr[ni], acc[r * 3 + s][mi][ni], 0, 0, 0);
        }
    }
  }

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
