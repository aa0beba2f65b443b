// Streaming 3x3 / stride-1 / pad-1 convolution of 64 input into 64 output channels (bf16, MFMA), forward
// and data gradient: the full-resolution layers of the UNet (level 1: 16 x 512^2 / 16 x 1024^2 pixels,
// /root/reference/pytorch/unet/model.py:5-18 DoubleConv(64, 64) of `inc` and `up4`) and ResNet layer 1's
// conv2 (56^2, /root/reference/pytorch/resnet/main.py:40-41).
//
// Why a kernel of its own: these layers run 576-long reductions into 64 channels over millions of
// pixels.  The 256 x 64 halo tile of the general kernel (conv_igemm.hip HALO) stages a tile's halo once
// and its 9 taps' weights tap by tap, with two barriers and a drained weight DMA per tap; every block
// then stores its tile in one burst and retires (PMC at 16 x 512^2: MFMA busy 0.29, 1.56 TB/s of HBM,
// profiles/r4_lab, profiles/r5_bytes).  Here, as in conv1x1_dgrad_stream.hip:
//   * persistent blocks (one per CU, 152 KB of LDS), each walking a strided sequence of 2-D output
//     tiles of th x tw <= 128 pixels;
//   * all 9 taps' weights (9 x 64 x 64 bf16 = 72 KB) are staged ONCE and stay resident: the tap loop
//     is 9 x 2 K-halves of MFMAs with no barrier inside;
//   * the next tile's halo ((th + 2) x (tw + 2) <= 192 rows, double-buffered) and its epilogue operand
//     (the consumer's BN input z, double-buffered) are DMA'd right after the current tile's barrier
//     and stream in under its MFMAs and epilogue.  Every DMA is issued through glds16_raw (common.h),
//     so the compiler adds no drain of its own; the only wait is `vmcnt(NSTORE)` at the top of a
//     tile (the previous tile's row stores, issued last, stay in flight);
//   * the epilogue runs on the D^T accumulator fragments (operands swapped: each lane holds 4
//     consecutive channels of one pixel), writes bf16 quads into an LDS staging tile and the tile
//     leaves as 16-byte row stores; BN partial sums accumulate per lane over all of the block's
//     tiles: one statistics row per block.
// MODE 0: forward (+ bias), statistics {sum y, sum y^2} of the stored values.  MODE 1: plain output.
// MODE 2: data gradient into a BN + ReLU output: mask z * mscale + mshift > 0, statistics
// {sum dx, sum dx * z}.  FLIP (data gradient): the weight of tap (r, s) applies to input offset
// (1 - r, 1 - s), i.e. wT[c][r][s][k] of a stride-1 dgrad.  Taps are visited in the general kernel's
// order with its per-element epilogue arithmetic; with the MFMA operands swapped (D^T) a few fp32 sums
// round the other way: outputs match the halo kernel's to one bf16 ulp in a small fraction of the
// elements (tests/test_kernels_gpu.py::test_conv3x3_stream_64).
#include "common.h"

namespace dlmpi {

constexpr int c3_vmcnt(int n) { return (n & 15) | 0x70 | 0xF00 | ((n >> 4) << 14); }
__device__ __forceinline__ void c3_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// 128-B epilogue rows (64 channels): 16-byte chunk j of row r at chunk j ^ ((r >> 1) & 7), so the 16
// rows of one D^T fragment column (8-byte reads) hit distinct bank slots (conv1x1_dgrad_stream.hip)
__device__ __forceinline__ int c3_eoff(int r, int col) {
  return r * 128 + ((((col >> 3) ^ ((r >> 1) & 7))) << 4) + ((col & 4) << 1);
}

// 8 waves of 32 x 32 (two per SIMD).  Measured alternatives (profiles/r5_conv3): 4 waves of 64 x 32
// (one per SIMD, a third fewer LDS reads per MFMA but nothing to hide their latency: 415 vs 370 us at
// 16 x 512^2, also with a register double buffer of the next tap's fragments); the weights held in
// registers (144 VGPRs per wave) instead of LDS: spills with the statistics epilogue, and only +6 %
// on the plain data gradient at 512^2 (-5 % at 56^2).
// PRO (forward only): the input is the producer BN's input z.  Once a tile's halo has landed, every
// lane rewrites its own in-image halo pieces in LDS as bf16(relu(fma(z, psc, psh))) -- bn_apply_kernel's
// arithmetic, bit-identical -- and stores the pieces of the tile's own pixels to py (every pixel is in
// exactly one tile: the applied activation is written once and the standalone apply pass, a read of z
// and a write of y, is gone); out-of-image pieces stay the zero padding.  One extra barrier per tile.
template <int MODE, bool FLIP, bool PRO = false>
__global__ __launch_bounds__(512) void conv3x3_stream_kernel(const Conv3StreamArgs a) {
  static_assert(!PRO || (MODE == 0 && !FLIP), "prologue: forward only");
  constexpr int NW = 8, NT = 64 * NW, BM = 128, BN = 64;
  constexpr int WGM = 4, WGN = 2, WM = BM / WGM, WN = BN / WGN;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int RP = NT / 8;                    // 128-B rows staged per pass
  constexpr int HROWS = 192;                    // halo rows (host: (th + 2) (tw + 2) <= 192)
  constexpr int HL = HROWS / RP, WL = 9 * BN / RP, EL = BM / RP;
  constexpr int NSTORE = BM / RP;               // 16-byte row stores per thread per tile
  constexpr bool Z = MODE == 2;
  constexpr int W_BYTES = 9 * BN * 128, A_BYTES = HROWS * 128, E_BYTES = BM * 128;
  constexpr int OFF_A0 = W_BYTES, OFF_A1 = OFF_A0 + A_BYTES, OFF_E0 = OFF_A1 + A_BYTES;
  constexpr int OFF_E1 = OFF_E0 + E_BYTES;
  constexpr int SMEM = OFF_E1 + (Z ? E_BYTES : 0);
  static_assert(SMEM <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WGN, wn = wid % WGN;
  const int fr = lane & 15, fg = lane >> 4;
  const int lrow = tid >> 3;                                 // staging row (+ RP i)
  const int jc = (tid & 7) ^ ((tid >> 3) & 7);               // swizzled 16-B chunk of a halo / weight row
  const int ej = tid & 7;                                    // epilogue tile: LDS chunk of row lrow (+ RP i)
  const char* zp = reinterpret_cast<const char*>(g_zero_page);
  const int H = a.H, W = a.W, tw = a.tw, th = a.th, hw = a.tw + 2;

  // ---- weights: all 9 taps, staged once (row t * 64 + n: out channel n of tap t) ----------------
#pragma unroll
  for (int i = 0; i < WL; ++i) {
    const int row = lrow + RP * i;                           // < 576
    const int t = row >> 6, n = row & 63;
    const char* src = reinterpret_cast<const char*>(a.w + (int64_t)n * a.ldw + t * 64 + 8 * jc);
    glds16_raw(src, smem + (RP * i + 8 * wid) * 128);
  }

  // halo piece i of this lane: halo row lrow + RP i = (line, col) relative to the tile origin - (1, 1)
  int hdh[HL], hdw[HL];
  uint32_t hok = 0;
#pragma unroll
  for (int i = 0; i < HL; ++i) {
    const int hr = lrow + RP * i;
    const int line = hr / hw;
    hdh[i] = line - 1;
    hdw[i] = hr - line * hw - 1;
    if (hr < (th + 2) * hw) hok |= 1u << i;
  }
  // epilogue-tile row piece i: tile pixel lrow + RP i = (pr, pc)
  int epr[EL], epc[EL];
#pragma unroll
  for (int i = 0; i < EL; ++i) {
    const int r = lrow + RP * i;
    epr[i] = r < th * tw ? r / tw : 1 << 20;
    epc[i] = r - (r / tw) * tw;
  }
  const int per_img = a.tiles_h * a.tiles_w;
  auto origin = [&](int t, int& n, int& h0, int& w0) {
    n = t / per_img;
    const int rem = t - n * per_img;
    const int ti = rem / a.tiles_w;
    h0 = ti * th;
    w0 = (rem - ti * a.tiles_w) * tw;
  };
  const char* xb = reinterpret_cast<const char*>(a.x + a.xoff) + 16 * jc;
  auto issue_a = [&](int t, int off) {   // the halo of tile t (past the last tile: the zero page)
    int n, h0, w0;
    origin(t, n, h0, w0);
    const bool tv = t < a.ntiles;
    const char* base = xb + 2 * ((int64_t)n * H * W) * a.ldx;
#pragma unroll
    for (int i = 0; i < HL; ++i) {
      const int ih = h0 + hdh[i], iw = w0 + hdw[i];
      const bool ok = tv && ((hok >> i) & 1) && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      const char* src = ok ? base + 2 * (int64_t)(ih * W + iw) * a.ldx : zp;
      glds16_raw(src, smem + off + (RP * i + 8 * wid) * 128);
    }
  };
  auto issue_e = [&](int t, int off) {   // the consumer's BN input z of tile t's output pixels
    if constexpr (Z) {
      int n, h0, w0;
      origin(t, n, h0, w0);
      const bool tv = t < a.ntiles;
      const char* base = reinterpret_cast<const char*>(a.z + a.zoff) + 2 * ((int64_t)n * H * W) * a.ldz;
#pragma unroll
      for (int i = 0; i < EL; ++i) {
        const int r = lrow + RP * i;
        const int oh = h0 + epr[i], ow = w0 + epc[i];
        const bool ok = tv && oh < H && ow < W;
        const int gj = ej ^ ((r >> 1) & 7);                  // global chunk stored at LDS chunk ej
        const char* src = ok ? base + 2 * ((int64_t)(oh * W + ow) * a.ldz + 8 * gj) : zp;
        glds16_raw(src, smem + off + (RP * i + 8 * wid) * 128);
      }
    }
  };

  // per-lane constants: bias / mask coefficients of this lane's output quads
  f32x4 bq[TN], ms[TN], mh[TN];
#pragma unroll
  for (int ni = 0; ni < TN; ++ni) {
    const int c = wn * WN + ni * 16 + 4 * fg;
    bq[ni] = a.bias ? *reinterpret_cast<const f32x4*>(a.bias + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (Z) {
      ms[ni] = *reinterpret_cast<const f32x4*>(a.mscale + c);
      mh[ni] = *reinterpret_cast<const f32x4*>(a.mshift + c);
    }
  }
  // fragment pixels of this lane: tile pixel wm * WM + 16 mi + fr -> halo row at tap (0, 0)
  int hb[TM];
#pragma unroll
  for (int mi = 0; mi < TM; ++mi) {
    const int r = wm * WM + mi * 16 + fr;
    hb[mi] = r < th * tw ? (r / tw) * hw + (r - (r / tw) * tw) : 0;
  }
  float s1[TN][4], s2[TN][4];
#pragma unroll
  for (int ni = 0; ni < TN; ++ni)
#pragma unroll
    for (int j = 0; j < 4; ++j) { s1[ni][j] = 0.f; s2[ni][j] = 0.f; }
  const int cg = tid & 7;   // store phase: chunk cg of rows lrow + RP i
  static_assert(HROWS % RP == 0 && (9 * BN) % RP == 0 && BM % RP == 0, "staging passes");
  const int img_bytes = H * W * a.ldy * 2;   // one image's output rows (host: < 2^31)

  // PRO: this lane's halo pieces -- channels 8 jc .. + 7 at LDS slot (tid & 7) of row lrow + RP i
  f32x4 psa = {}, psb = {}, pha = {}, phb = {};
  if constexpr (PRO) {
    psa = *reinterpret_cast<const f32x4*>(a.psc + 8 * jc);
    psb = *reinterpret_cast<const f32x4*>(a.psc + 8 * jc + 4);
    pha = *reinterpret_cast<const f32x4*>(a.psh + 8 * jc);
    phb = *reinterpret_cast<const f32x4*>(a.psh + 8 * jc + 4);
  }
  const int py_img = PRO ? H * W * a.ldpy * 2 : 0;   // one image of the applied output (host: < 2^31)

  int t = blockIdx.x;   // tiles t, t + G, ...: the grid holds one block per CU
  issue_a(t, OFF_A0);
  issue_e(t, OFF_E0);
  // weights + the first tile + the coefficient loads above (the builtin: the compiler folds it into its
  // scoreboard and then waits for nothing inside the loop, where a wait would drain the prefetch)
  __builtin_amdgcn_s_waitcnt(c3_vmcnt(0));
  for (int it = 0; t < a.ntiles; ++it, t += a.G) {
    const int offA = (it & 1) ? OFF_A1 : OFF_A0, offAn = (it & 1) ? OFF_A0 : OFF_A1;
    const int offE = Z ? ((it & 1) ? OFF_E1 : OFF_E0) : OFF_E0, offEn = Z ? ((it & 1) ? OFF_E0 : OFF_E1) : OFF_E0;
    // this tile's halo / z landed (the younger vector-memory operations of this wave are the previous
    // tile's NSTORE row stores, and with PRO its HL applied-input stores before them); every wave is
    // done with the previous tile's buffers
    __builtin_amdgcn_s_waitcnt(c3_vmcnt(NSTORE + (PRO ? HL : 0)));
    c3_barrier();
    issue_a(t + a.G, offAn);   // the next tile streams in under this tile's MFMAs and epilogue
    issue_e(t + a.G, offEn);
    if constexpr (PRO) {
      int n, h0, w0;
      origin(t, n, h0, w0);
      const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc(
          reinterpret_cast<char*>(a.py) + (int64_t)n * py_img, (short)0, py_img, 0x00020000);
#pragma unroll
      for (int i = 0; i < HL; ++i) {
        const int ih = h0 + hdh[i], iw = w0 + hdw[i];
        const bool in = ((hok >> i) & 1) && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
        u32x4* pc = reinterpret_cast<u32x4*>(smem + offA + (RP * i + lrow) * 128 + (tid & 7) * 16);
        u32x4 q = u32x4{0u, 0u, 0u, 0u};
        if (in) {
          float v[8];
          unpack8(*pc, v);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = fmaxf(__builtin_fmaf(v[e], psa[e], pha[e]), 0.f);
            v[e + 4] = fmaxf(__builtin_fmaf(v[e + 4], psb[e], phb[e]), 0.f);
          }
          q = pack8(v);
          *pc = q;
        }
        // the tile's own pixels (halo line / column 1 .. th / tw): stored once; others dropped by the
        // buffer range check (offset 2^31), so every lane issues exactly HL stores (the vmcnt above)
        const bool own = in && hdh[i] >= 0 && hdh[i] < th && hdw[i] >= 0 && hdw[i] < tw;
        const uint32_t off = (uint32_t)(((ih * W + iw) * a.ldpy + a.pyoff + 8 * jc) * 2);
        __builtin_amdgcn_raw_buffer_store_b128(q, pr, own ? off : 0x80000000u, 0, 0);
      }
      c3_barrier();   // every wave's pieces are applied before any fragment read
    }

    f32x4 acc[TM][TN];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* As = smem + offA;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int tr = tap / 3, ts = tap % 3;
      const int toff = FLIP ? (2 - tr) * hw + (2 - ts) : tr * hw + ts;
      const char* Bs = smem + tap * BN * 128;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int ch = kk * 4 + fg;
        bf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int mi = 0; mi < TM; ++mi) {
          const int r = hb[mi] + toff;
          af[mi] = *reinterpret_cast<const bf16x8*>(As + r * 128 + ((ch ^ (r & 7)) << 4));
        }
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) {
          const int r = wn * WN + ni * 16 + fr;
          bfr[ni] = *reinterpret_cast<const bf16x8*>(Bs + r * 128 + ((ch ^ (r & 7)) << 4));
        }
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int ni = 0; ni < TN; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[ni], af[mi], acc[mi][ni], 0, 0, 0);
      }
    }

    // epilogue on the D^T fragments: lane (fr, fg) holds tile pixel wm * WM + 16 mi + fr, channels
    // wn * WN + 16 ni + 4 fg + [0, 4); the output quads go to the staging tile (in place of z)
    int n, h0, w0;
    origin(t, n, h0, w0);
    char* Ot = smem + offE;
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const int row = wm * WM + mi * 16 + fr;
      const int pr = row / tw, pc = row - pr * tw;
      const float keep = row < th * tw && h0 + pr < H && w0 + pc < W ? 1.f : 0.f;
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int col = wn * WN + ni * 16 + 4 * fg;
        const int eo = c3_eoff(row, col);
        f32x4 v = acc[mi][ni] + bq[ni];
        if constexpr (MODE == 0) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float rv = bf2f(f2bf(v[j])) * keep;   // statistics of the stored value
            s1[ni][j] += rv;
            s2[ni][j] += rv * rv;
          }
        } else if constexpr (Z) {
          const u32x2 q = *reinterpret_cast<const u32x2*>(Ot + eo);
          const f32x4 zz{__uint_as_float(q[0] << 16), __uint_as_float(q[0] & 0xffff0000u), __uint_as_float(q[1] << 16),
                         __uint_as_float(q[1] & 0xffff0000u)};
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = __builtin_fmaf(zz[j], ms[ni][j], mh[ni][j]) > 0.f ? v[j] : 0.f;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float rv = bf2f(f2bf(v[j])) * keep;   // statistics of the stored gradient
            s1[ni][j] += rv;
            s2[ni][j] += rv * zz[j];
          }
        }
        *reinterpret_cast<u32x2*>(Ot + eo) = u32x2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
      }
    }
    c3_barrier();
    // rows out: 16 bytes per thread per row through a buffer resource on the tile's image (32-bit
    // offsets); rows outside the tile / image are dropped by the range check (offset 2^31)
    const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<char*>(a.y) + (int64_t)n * img_bytes, (short)0, img_bytes, 0x00020000);
#pragma unroll
    for (int i = 0; i < NSTORE; ++i) {
      const int row = lrow + RP * i;
      const u32x4 q = *reinterpret_cast<const u32x4*>(Ot + row * 128 + ((cg ^ ((row >> 1) & 7)) << 4));
      const int oh = h0 + epr[i], ow = w0 + epc[i];
      const uint32_t off0 = (uint32_t)(((oh * W + ow) * a.ldy + a.yoff + cg * 8) * 2);
      __builtin_amdgcn_raw_buffer_store_b128(q, yr, oh < H && ow < W ? off0 : 0x80000000u, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA in flight when the block retires

  if constexpr (MODE != 1) {
    // per-lane sums -> [WGM * 16][BN] (one statistic at a time, in the now free weight tile) -> one
    // row per block, summed in a fixed order
    constexpr int RR = WGM * 16;
    float* red = reinterpret_cast<float*>(smem);
    float* st = a.stats + (int64_t)blockIdx.x * 2 * BN + tid;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      __syncthreads();
#pragma unroll
      for (int ni = 0; ni < TN; ++ni)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          red[(wm * 16 + fr) * BN + wn * WN + ni * 16 + 4 * fg + j] = k == 0 ? s1[ni][j] : s2[ni][j];
      __syncthreads();
      if (tid < BN) {
        float s = 0.f;
        for (int q = 0; q < RR; ++q) s += red[q * BN + tid];
        st[k * BN] = s;
      }
    }
  }
}

}  // namespace dlmpi

using namespace dlmpi;

static int g_c3_override = -1;   // dlmpi_ext set_conv3_stream (tests / A/B): 0 off, 1 on
extern "C" void dlmpi_set_conv3_stream(int mode) { g_c3_override = mode; }

// Plan: tile th x tw (th * tw <= 128, (th + 2)(tw + 2) <= 192) with the fewest tiles, G blocks (one per
// CU, at most `blocks`); 0 if the kernel does not apply.
extern "C" int dlmpi_conv3_stream_plan(int N, int H, int W, int C, int K, int blocks, int* th, int* tw, int* G) {
  const int on = g_c3_override >= 0 ? g_c3_override : 1;
  if (!on || C != 64 || K != 64 || N <= 0 || H <= 0 || W <= 0) return 0;
  int best = 0x7fffffff;
  for (int w = 16; w >= 4; --w) {
    int h = 128 / w;
    while (h > 0 && (h + 2) * (w + 2) > 192) --h;
    if (h < 1) continue;
    const int t = ((H + h - 1) / h) * ((W + w - 1) / w);
    if (t < best) {
      best = t;
      *th = h;
      *tw = w;
    }
  }
  const int64_t tiles = (int64_t)N * best;
  if (tiles > 0x7fffffff) return 0;
  const int b = blocks > 0 ? blocks : 256;
  *G = (int)(tiles < b ? tiles : b);
  return 1;
}

extern "C" hipError_t dlmpi_conv3x3_stream(const Conv3StreamArgs* a, int mode, hipStream_t s) {
  if (a->G <= 0) return hipSuccess;
  if (a->th * a->tw > 128 || (a->th + 2) * (a->tw + 2) > 192) return hipErrorInvalidValue;
  const dim3 g((unsigned)a->G), b(512);
  if (mode == 0 && !a->flip && a->stats && a->psc) {
    if (!a->psh || !a->py || a->ldpy % 8 || a->pyoff % 8 || (int64_t)a->H * a->W * a->ldpy * 2 >= (1ll << 31))
      return hipErrorInvalidValue;
    hipLaunchKernelGGL((conv3x3_stream_kernel<0, false, true>), g, b, 0, s, *a);
  } else if (mode == 0 && !a->flip && a->stats) hipLaunchKernelGGL((conv3x3_stream_kernel<0, false>), g, b, 0, s, *a);
  else if (mode == 1 && !a->flip) hipLaunchKernelGGL((conv3x3_stream_kernel<1, false>), g, b, 0, s, *a);
  else if (mode == 1 && a->flip) hipLaunchKernelGGL((conv3x3_stream_kernel<1, true>), g, b, 0, s, *a);
  else if (mode == 2 && a->flip && a->stats && a->z && a->mscale && a->mshift)
    hipLaunchKernelGGL((conv3x3_stream_kernel<2, true>), g, b, 0, s, *a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}
