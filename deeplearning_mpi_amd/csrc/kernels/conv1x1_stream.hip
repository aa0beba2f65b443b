// Streaming 1x1 convolution forward for short reductions (C = 64 / 128 / 256 input channels): the
// memory-bound "expand" convolutions of the ResNet bottleneck (conv3 and the layer-1 downsample,
// 56^2 64->256, 28^2 128->512, 14^2 256->1024), whose output write dominates, the layer-1 block-1
// conv1 (56^2 64->64), and the stride-2 layer-2 projection (56^2 256->512, S2: gathered rows).
//
// Why a kernel of its own (profiles/r3_stream1x1): the general implicit-GEMM kernel runs one tile
// per block -- stage A and B, one or two K-steps of MFMA, then the epilogue's stores -- so while a
// block loads nothing is stored and while it stores nothing is loaded, and its 32 KB of output
// leave in a burst at the end of its life.  At 4 blocks per CU the output stream then reaches
// ~2.8 TB/s although the very same tile store pattern alone runs at 5.5 TB/s
// (benchmarks/micro/store_bw.hip).  Here each block is persistent over a column of M-tiles:
//   * the weight tile [BN out channels][C] is staged into LDS ONCE and stays resident;
//   * the next M-tile's activations are fetched global->LDS (global_load_lds) right after the
//     current tile's MFMAs, so the fetch runs under the current tile's epilogue and stores;
//   * the epilogue never waits for its stores: the only wait is `s_waitcnt vmcnt(NSTORE)` at the top
//     of the next tile -- the prefetch was issued BEFORE the NSTORE stores of the epilogue and
//     vmcnt retires in issue order, so that wait covers the prefetch and leaves the stores in
//     flight.  Every thread issues exactly NSTORE stores per tile (raw buffer stores; rows past M
//     get an out-of-range offset and are dropped by the buffer descriptor's range check).
// MFMA v_mfma_f32_16x16x32_bf16 with the operands swapped (D^T: each lane holds 4 consecutive
// output channels of one pixel) -> bf16 quads into an LDS row-major staging tile -> 16-byte rows out.
// BatchNorm statistics of the stored (bf16) values accumulate per thread over ALL of the block's
// tiles and are written as ONE partial row per block: the finalize reduces G rows per N-tile
// (G = blocks per N-tile, a few hundred) instead of one row per 64/128-pixel tile.
// UP2: ConvTranspose2d(kernel 2, stride 2) (the UNet up-sampling, reference model.py:60-63) as ONE
// 1x1 GEMM with 4 Cup output columns ordered (i, j, co): an N-tile lies inside one (i, j) block, so its
// rows are stored to output pixel (2h + i, 2w + j) -- the input tile is read once for all four
// sub-pixel positions instead of once per phase.
//
// Reference semantics: nn.Conv2d(k=1, bias=False) + BatchNorm2d statistics (torchvision Bottleneck
// conv3 / downsample, /root/reference/pytorch/resnet/main.py:40-41).
#include "common.h"

namespace dlmpi {

typedef __attribute__((address_space(3))) void s1x1_lds_void;

// Workgroup barrier for LDS hand-offs only.  __syncthreads() (and any LDS release fence) makes
// the compiler drain vmcnt to 0, because the global_load_lds prefetch counts as a pending LDS write
// -- i.e. it would wait for the prefetch and the epilogue's stores, the very overlap this kernel
// exists for.  Here: this wave's own LDS accesses complete (lgkmcnt 0), then s_barrier; the
// "memory" clobber keeps the compiler from moving memory operations across it.  The prefetched
// tile is made visible separately by the explicit vmcnt wait at the top of each tile.
// s_waitcnt immediate (gfx9 encoding) waiting for vmcnt <= n only: vmcnt[3:0] | expcnt[6:4]=7 |
// lgkmcnt[11:8]=15 | vmcnt[5:4] at [15:14]
constexpr int vmcnt_imm(int n) { return (n & 15) | 0x70 | 0xF00 | ((n >> 4) << 14); }

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int BM, int BN, int KS, bool STATS, bool S2, bool UP2 = false>
__global__ __launch_bounds__(256) void conv1x1_stream_kernel(const Stream1x1Args a) {
  constexpr int NT = 256;
  constexpr int WM = BM / 2, WN = BN / 2;       // 2 x 2 waves
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int RP = NT / 8;                    // LDS rows of 128 B staged per pass
  constexpr int AL = BM / RP, BL = BN / RP;     // 16-byte pieces per thread per K-step
  constexpr int W_BYTES = KS * BN * 128, A_BYTES = KS * BM * 128;
  constexpr int OP = BN * 2 + 16;               // staging row pitch (bytes), padded
  constexpr int CG = BN / 8, RG = NT / CG;      // epilogue: channel groups of 8, row groups
  constexpr int NSTORE = BM / RG;               // 16-byte stores per thread per tile
  constexpr int O_BYTES0 = BM * OP, RED_BYTES = RG * 2 * BN * 4;
  constexpr int O_BYTES = O_BYTES0 > RED_BYTES ? O_BYTES0 : RED_BYTES;
  static_assert(BM % RP == 0 && BN % RP == 0 && BM % RG == 0, "tile shape");
  // three distinct LDS objects: the compiler's LDS-DMA alias tracking can then see that the
  // staging-tile reads of the epilogue do not depend on the in-flight activation prefetch (one
  // array would make it wait for the prefetch before every staging read)
  __shared__ __attribute__((aligned(16))) char Ws[W_BYTES];
  __shared__ __attribute__((aligned(16))) char As[A_BYTES];
  __shared__ __attribute__((aligned(16))) char Os[O_BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int fr = lane & 15, fg = lane >> 4;
  const int lrow = tid >> 3;                                // staging row (+ RP i)
  const int jc = (tid & 7) ^ ((tid >> 3) & 7);              // swizzled 16-byte chunk this lane fetches
  const char* zp = reinterpret_cast<const char*>(g_zero_page);   // weight rows past Kout

  // block -> (N-tile, position in the N-tile's block group); the ntiles blocks that walk the same
  // M-tiles are contiguous after the XCD remap, i.e. share an XCD's L2 for the activation tile
  const uint32_t lb = xcd_remap(blockIdx.x, gridDim.x);
  const int nt = lb % a.ntiles, g = lb / a.ntiles;
  const int n0 = nt * BN;
  // UP2: sub-pixel block (i, j) = ub of this N-tile and its first output channel
  const int ub = UP2 ? n0 / a.Cup : 0, c0 = UP2 ? n0 - ub * a.Cup : n0;

  // ---- weights: staged once ----------------------------------------------------------------
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const int n = n0 + lrow + RP * i;
      const int wrow = UP2 ? (c0 + lrow + RP * i) * 4 + ub : n;   // w [Cup][2][2][C]
      const char* src = n < a.Kout ? reinterpret_cast<const char*>(a.w + (int64_t)wrow * a.C + ks * 64 + 8 * jc) : zp;
      __builtin_amdgcn_global_load_lds(src, (s1x1_lds_void*)(Ws + ks * BN * 128 + (RP * i + 8 * wid) * 128), 16, 0, 0);
    }
  auto issue_a = [&](int mt) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int i = 0; i < AL; ++i) {
        // rows past M re-read the last row (their outputs are dropped, their statistics masked):
        // no select / exec-masked region around the load, which keeps the compiler's vmcnt
        // scoreboard exact so that it adds no vmcnt(0) of its own (32-bit offsets: host-checked)
        const int m = min(mt * BM + lrow + RP * i, a.M - 1);
        int row = m;
        if constexpr (S2) {   // output pixel (n, p, q) reads input pixel (n, 2p, 2q)
          const uint32_t n = fdiv((uint32_t)m, a.fdPQ), rem = (uint32_t)m - n * a.fdPQ.d;
          const uint32_t p = fdiv(rem, a.fdQ), q = rem - p * a.fdQ.d;
          row = (int)((n * a.H + 2 * p) * a.W + 2 * q);
        }
        const char* src = reinterpret_cast<const char*>(a.x + (uint32_t)(row * a.ldx + a.xoff + ks * 64 + 8 * jc));
        __builtin_amdgcn_global_load_lds(src, (s1x1_lds_void*)(As + ks * BM * 128 + (RP * i + 8 * wid) * 128), 16, 0,
                                         0);
      }
  };

  // output: raw buffer stores, range-checked by the descriptor (rows past M dropped)
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(a.y, (short)0, a.y_bytes, 0x00020000);
  const int cg = tid % CG, rg = tid / CG;
  // bias of this lane's output quads, loaded up front (no global load inside the tile loop: the
  // compiler would wait for it -- and so for the prefetch issued before it)
  f32x4 bq[TN];
#pragma unroll
  for (int ni = 0; ni < TN; ++ni)
    bq[ni] = a.bias ? *reinterpret_cast<const f32x4*>(a.bias + c0 + wn * WN + ni * 16 + 4 * fg) : f32x4{0.f, 0.f, 0.f, 0.f};
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }

  int mt = g;
  if (mt < a.mtiles) issue_a(mt);
  __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));   // weights + the first tile (one wait in the loop below)
  for (int it = 0; mt < a.mtiles; ++it, mt += a.G) {
    // the tile's activations have landed: the only younger vector-memory operations of this wave
    // are the previous tile's NSTORE stores, which stay in flight
    // (the builtin, not inline asm: the compiler's waitcnt pass folds it into its scoreboard and then
    // adds no conservative vmcnt(0) of its own before the activation reads)
    __builtin_amdgcn_s_waitcnt(vmcnt_imm(NSTORE));
    lds_barrier();   // every wave's pieces are in LDS; the previous tile's staging reads are done

    f32x4 acc[TM][TN];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const char* A = As + ks * BM * 128;
      const char* B = Ws + ks * BN * 128;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int ch = kk * 4 + fg;
        bf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int mi = 0; mi < TM; ++mi) {
          const int r = wm * WM + mi * 16 + fr;
          af[mi] = *reinterpret_cast<const bf16x8*>(A + r * 128 + ((ch ^ (r & 7)) << 4));
        }
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) {
          const int r = wn * WN + ni * 16 + fr;
          bfr[ni] = *reinterpret_cast<const bf16x8*>(B + r * 128 + ((ch ^ (r & 7)) << 4));
        }
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int ni = 0; ni < TN; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[ni], af[mi], acc[mi][ni], 0, 0, 0);
      }
    }
    lds_barrier();   // every wave is done reading this tile's activations
    // the next tile streams in under this epilogue (unconditionally -- past the last tile every
    // row reads the zero page -- so that the instruction stream and the compiler's vmcnt
    // scoreboard are the same for every tile)
    issue_a(mt + a.G);

    // D^T fragments -> bf16 quads into the row-major staging tile
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int row = wm * WM + mi * 16 + fr, col = wn * WN + ni * 16 + 4 * fg;
        const f32x4 v = acc[mi][ni] + bq[ni];
        *reinterpret_cast<u32x2*>(Os + row * OP + col * 2) = u32x2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
      }
    lds_barrier();
    // UP2: the tile's output rows are addressed relative to its first one (a 64-bit base in a per-tile
    // buffer descriptor), so the concat buffer may exceed 2 GB
    uint32_t orow0 = 0;
    __amdgpu_buffer_rsrc_t yo = yr;
    if constexpr (UP2) {
      const uint32_t m0 = (uint32_t)(mt * BM);
      const uint32_t n = fdiv(m0, a.fdPQ), rem = m0 - n * a.fdPQ.d;
      const uint32_t h = fdiv(rem, a.fdQ), w = rem - h * a.fdQ.d;
      orow0 = (n * 2u * a.H + 2u * h + (uint32_t)(ub >> 1)) * 2u * a.W + 2u * w + (uint32_t)(ub & 1);
      yo = __builtin_amdgcn_make_buffer_rsrc(a.y + (int64_t)orow0 * a.ldy + a.yoff + c0, (short)0, 0x7fffffff,
                                             0x00020000);
    }
    // rows out: 16 bytes per thread per row, statistics of the stored values
#pragma unroll
    for (int i = 0; i < NSTORE; ++i) {
      const int row = rg + RG * i;
      const u32x4 q = *reinterpret_cast<const u32x4*>(Os + row * OP + cg * 16);
      const int m = mt * BM + row;
      if constexpr (STATS) {
        float v[8];
        unpack8(q, v);
        const float keep = m < a.M ? 1.f : 0.f;   // branch-free: rows past M add 0
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float u = v[e] * keep;
          s1[e] += u;
          s2[e] += u * u;
        }
      }
      if constexpr (UP2) {   // input pixel (n, h, w) -> output pixel (n, 2h + i, 2w + j), relative to the tile's
        const uint32_t mm = m < a.M ? (uint32_t)m : 0u;
        const uint32_t n = fdiv(mm, a.fdPQ), rem = mm - n * a.fdPQ.d;
        const uint32_t h = fdiv(rem, a.fdQ), w = rem - h * a.fdQ.d;
        const uint32_t orow = (n * 2u * a.H + 2u * h + (uint32_t)(ub >> 1)) * 2u * a.W + 2u * w + (uint32_t)(ub & 1);
        const uint32_t off = m < a.M ? ((orow - orow0) * a.ldy + cg * 8) * 2u : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(q, yo, off, 0, 0);
      } else {
        const uint32_t off0 = (uint32_t)(m * a.ldy + a.yoff + n0 + cg * 8) * 2u;   // 32-bit: host-checked
        const uint32_t off = m < a.M ? off0 : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(q, yr, off, 0, 0);
      }
    }
  }

  if constexpr (STATS) {
    __syncthreads();   // staging reads done: the region holds the statistics combine
    float* red = reinterpret_cast<float*>(Os);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(rg * 2 + 0) * BN + cg * 8 + e] = s1[e];
      red[(rg * 2 + 1) * BN + cg * 8 + e] = s2[e];
    }
    __syncthreads();
    if (tid < BN && n0 + tid < a.Kout) {
      float t1 = 0.f, t2 = 0.f;
      for (int q = 0; q < RG; ++q) {
        t1 += red[(q * 2 + 0) * BN + tid];
        t2 += red[(q * 2 + 1) * BN + tid];
      }
      float* st = a.stats + (int64_t)g * 2 * a.Kout + n0 + tid;
      st[0] = t1;
      st[a.Kout] = t2;
    }
  }
}

}  // namespace dlmpi

using namespace dlmpi;

// Tile plan of the streaming kernel: (BM, BN, blocks per N-tile G) or false if it does not apply.
// (C = 512, the layer-4 expand, measured slower than the general kernel: 144 KB of LDS leave one block
// per CU, 58.3 vs 50.7 us, profiles/r3_stream1x1; C = 256 on 64 x 128 tiles was neutral,
// profiles/r3_c256.)
static int g_stream_override = -1;   // dlmpi_ext set_conv_stream (tests)
extern "C" void dlmpi_set_conv_stream(int mode) { g_stream_override = mode; }

extern "C" int dlmpi_stream1x1_plan(int64_t M, int C, int Kout, int stride, int* bm, int* bn, int* G) {
  const int on = g_stream_override >= 0 ? g_stream_override : 1;
  if (!on || M <= 0) return 0;
  if (stride == 2 && !(C == 256 && Kout % 64 == 0)) return 0;
  if (C == 64 && Kout % 128 == 0) { *bm = 128; *bn = 128; }
  else if (C == 64 && Kout == 64) { *bm = 128; *bn = 64; }   // layer-1 block-1 conv1 (56^2 64 -> 64)
  else if (C == 128 && Kout % 128 == 0) { *bm = 64; *bn = 128; }
  else if (C == 256 && Kout % 64 == 0) { *bm = 64; *bn = 64; }
  else return 0;
  const int ntiles = Kout / *bn;
  const int64_t mtiles = (M + *bm - 1) / *bm;
  // ~2 resident blocks per CU over the whole chip (LDS 65-80 KB per block)
  int target = 512 / ntiles;
  if (target < 8) target = 8;
  *G = (int)(mtiles < target ? mtiles : target);
  return 1;
}

extern "C" hipError_t dlmpi_conv1x1_stream(const Stream1x1Args* a, int bm, int bn, hipStream_t s) {
  const dim3 grid((unsigned)(a->ntiles * a->G)), block(256);
#define LAUNCH_S1(BM_, BN_, KS_, S2_)                                                                              \
  do {                                                                                                           \
    if (a->stats) hipLaunchKernelGGL((conv1x1_stream_kernel<BM_, BN_, KS_, true, S2_>), grid, block, 0, s, *a);     \
    else hipLaunchKernelGGL((conv1x1_stream_kernel<BM_, BN_, KS_, false, S2_>), grid, block, 0, s, *a);          \
  } while (0)
  if (a->up2) {   // ConvTranspose2d(2, 2): no statistics
    if (a->stats || a->Kout != 4 * a->Cup || a->Cup % bn) return hipErrorInvalidValue;
    if (bm == 64 && bn == 128 && a->C == 128) hipLaunchKernelGGL((conv1x1_stream_kernel<64, 128, 2, false, false, true>), grid, block, 0, s, *a);
    else if (bm == 64 && bn == 64 && a->C == 256) hipLaunchKernelGGL((conv1x1_stream_kernel<64, 64, 4, false, false, true>), grid, block, 0, s, *a);
    else if (bm == 128 && bn == 128 && a->C == 64) hipLaunchKernelGGL((conv1x1_stream_kernel<128, 128, 1, false, false, true>), grid, block, 0, s, *a);
    else return hipErrorInvalidValue;
  } else if (a->s2) {   // the stride-2 projection (layer-2 downsample, 56^2 256 -> 512)
    if (bm == 64 && bn == 64 && a->C == 256) LAUNCH_S1(64, 64, 4, true);
    else return hipErrorInvalidValue;
  } else if (bm == 128 && bn == 128 && a->C == 64) LAUNCH_S1(128, 128, 1, false);
  else if (bm == 128 && bn == 64 && a->C == 64) LAUNCH_S1(128, 64, 1, false);
  else if (bm == 64 && bn == 128 && a->C == 128) LAUNCH_S1(64, 128, 2, false);
  else if (bm == 64 && bn == 64 && a->C == 256) LAUNCH_S1(64, 64, 4, false);
  else return hipErrorInvalidValue;
#undef LAUNCH_S1
  return hipGetLastError();
}
