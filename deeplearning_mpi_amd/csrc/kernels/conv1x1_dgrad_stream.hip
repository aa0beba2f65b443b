// Streaming 1x1 / stride-1 DATA GRADIENT with the fused BN-backward epilogue: the memory-bound
// GEMMs of the ResNet bottleneck backward whose epilogue, not the MFMA work, sets the time.
//
//   dx[m, c] = sum_k A[m, k] W[c, k] (+ bias[c]) (+ res[m, c]),  then the consumer's ReLU mask
//   (mask bits of the forward BN-apply, or z * mscale + mshift > 0) and its BN-backward partials
//   {sum dx, sum dx * z} of the stored (bf16) gradient.
//
// A is dy, or [dy | z] of the dual data gradient (engine.ConvUnit.dual, K = 2 x 64 / 2 x 128).
// Example (profiles/r3_s3_base/resnet50_step.txt): layer-1 conv1 of a bottleneck, 802,816 rows, K 128,
// 256 output channels, plus a residual gradient, the previous block's z and mask bits: 1.46 GB of
// traffic that the general implicit-GEMM kernel moved in 645 us (2.3 TB/s) -- every block stages
// A, runs 2 K-steps of MFMA and then waits on the dependent residual / z / mask loads of its
// epilogue rows, so loads and stores never overlap inside a block.
//
// Here (same idea as conv1x1_stream.hip, extended to the epilogue operands):
//   * persistent blocks (one per CU), each walking a column of 128-channel output tiles;
//     the weight tile [128][K] is staged into LDS once and stays resident;
//   * the NEXT tile's epilogue operands (residual, z, mask bits) and A are fetched global -> LDS
//     (global_load_lds; the operands into the other half of a double buffer) right after the
//     current tile's MFMAs, so they stream in under the current tile's epilogue math and stores
//     (issued before the MFMAs instead, the compiler cannot separate the in-flight operand DMA from
//     the A / W fragment reads and waits for it there);
//   * the epilogue runs on the D^T accumulator fragments (operands swapped: each lane holds 4
//     consecutive channels of one pixel) reading its residual / z / mask pieces from LDS
//     (XOR-swizzled rows: conflict-free 8-byte reads), writes bf16 quads into a staging tile and
//     the tile leaves as 16-byte row stores that are never waited for (the only wait is
//     vmcnt(NSTORE) at the top of the next tile: vmcnt retires in issue order and the stores were
//     issued last);
//   * BN partial sums accumulate per lane over ALL of the block's tiles: one partial row per block.
// The per-element arithmetic is the conv_igemm epilogue's (fp32: (acc + bias) + res, mask, round
// once to bf16), so dx is bit-identical to the general kernel; the partial sums differ only in
// fp32 summation order.
//
// Reference semantics: the autograd of nn.Conv2d(k=1) + BatchNorm2d + ReLU (+ residual add) in
// torchvision's Bottleneck (/root/reference/pytorch/resnet/main.py:40-41, loss.backward() at :128).
#include "common.h"

namespace dlmpi {

typedef __attribute__((address_space(3))) void dgs_lds_void;

// s_waitcnt immediate waiting for vmcnt <= n only (gfx9 encoding, as in conv1x1_stream.hip)
constexpr int dgs_vmcnt(int n) { return (n & 15) | 0x70 | 0xF00 | ((n >> 4) << 14); }
__device__ __forceinline__ void dgs_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void dgs_glds(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds(g, (dgs_lds_void*)lds, 16, 0, 0);
}

// Epilogue-operand tile of BM rows x 128 channels (256-byte rows): 16-byte chunk j of row r sits at
// chunk position j ^ (r & 15), so that the 16 rows read by one D^T fragment column hit 16 different
// chunk positions (all 64 banks once per lane pair)
__device__ __forceinline__ int dgs_eoff(int r, int col) {   // byte offset of channel col (multiple of 4)
  return r * 256 + ((((col >> 3) ^ (r & 15))) << 4) + ((col & 4) << 1);
}

// MASK: 1 = forward mask bits, 2 = z * mscale + mshift > 0, 0 = no mask and no statistics
template <int BM, int KS, int NW, int MASK>
__global__ __launch_bounds__(64 * NW) void conv1x1_dgrad_stream_kernel(const DgradStreamArgs a) {
  constexpr int BN = 128;
  constexpr bool Z = MASK != 0;
  constexpr int NT = 64 * NW;
  constexpr int WGM = 2, WGN = NW / 2;          // wave grid
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int RP = NT / 8;                    // 128-B rows staged per pass (A / W tiles)
  constexpr int AL = BM / RP, BL = BN / RP;
  constexpr int EP = NT / 16;                   // 256-B rows staged per pass (epilogue operand tiles)
  constexpr int EL = BM / EP;
  constexpr int NSTORE = BM / EP;               // 16-byte output row stores per thread per tile
  constexpr int MB_ROWS = BM > 64 ? BM : 64;    // mask-bit tile: one wave instruction (16 B / row)
  constexpr int E_BYTES = BM * 256;
  static_assert(AL >= 1 && BM % RP == 0 && BN % RP == 0 && BM % EP == 0 && TM >= 1 && TN >= 1, "tile shape");
  constexpr int W_BYTES = KS * BN * 128, A_BYTES = KS * BM * 128;
  // distinct LDS objects per buffer (the compiler's LDS-DMA alias tracking then sees that the
  // epilogue's reads of one buffer do not depend on the prefetch in flight into the other; the
  // double-buffer index is static: the tile loop is unrolled by two)
  __shared__ __attribute__((aligned(16))) char Ws[W_BYTES];
  __shared__ __attribute__((aligned(16))) char As[A_BYTES];
  // epilogue-operand double buffer: [residual | z | mask bits] per buffer (one LDS object each: the
  // compiler tracks a handful of LDS-DMA targets, more objects make it wait for all of them)
  constexpr int EZ_OFF = E_BYTES, EM_OFF = E_BYTES + (Z ? E_BYTES : 0);
  constexpr int EB_BYTES = EM_OFF + (MASK == 1 ? MB_ROWS * 16 : 0);
  __shared__ __attribute__((aligned(16))) char E0[EB_BYTES];
  __shared__ __attribute__((aligned(16))) char E1[EB_BYTES];
  __shared__ __attribute__((aligned(16))) char Os[E_BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WGN, wn = wid % WGN;
  const int fr = lane & 15, fg = lane >> 4;
  const int lrow = tid >> 3;                                 // A / W staging row (+ RP i)
  const int jc = (tid & 7) ^ ((tid >> 4) & 7);               // swizzled 16-B chunk this lane fetches
  const int erow = tid >> 4;                                 // epilogue-tile staging row (+ EP i)
  const char* zp = reinterpret_cast<const char*>(g_zero_page);

  const uint32_t lb = xcd_remap(blockIdx.x, gridDim.x);
  const int nt = lb % a.ntiles, g = lb / a.ntiles;
  const int n0 = nt * BN;
  const bool has_res = a.res != nullptr;

  // ---- weights: staged once --------------------------------------------------------------------
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const int n = n0 + lrow + RP * i;
      const char* src = n < a.Kout ? reinterpret_cast<const char*>(a.w + (int64_t)n * a.K + ks * 64 + 8 * jc) : zp;
      dgs_glds(src, Ws + ks * BN * 128 + (RP * i + 8 * wid) * 128);
    }
  // rows past M re-read row M - 1 (outputs dropped, statistics masked): unconditional loads keep the
  // compiler's vmcnt scoreboard exact (32-bit offsets: host-checked)
  auto issue_a = [&](int mt) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int i = 0; i < AL; ++i) {
        const int m = min(mt * BM + lrow + RP * i, a.M - 1);
        dgs_glds(a.x + (uint32_t)(m * a.ldx + a.xoff + ks * 64 + 8 * jc), As + ks * BM * 128 + (RP * i + 8 * wid) * 128);
      }
  };
  auto issue_e = [&](int mt, char* Rb, char* Zb, char* Mb) {
    const int ej = (tid & 15);
#pragma unroll
    for (int i = 0; i < EL; ++i) {
      const int r = erow + EP * i;
      const int m = min(mt * BM + r, a.M - 1);
      const int gj = ej ^ (r & 15);                           // global chunk stored at LDS chunk ej
      // LDS destination: lane-linear 1 KB per wave instruction = rows erow (+ EP i), chunk ej
      if (has_res)
        dgs_glds(a.res + (uint32_t)(m * a.ldres + a.resoff + n0 + gj * 8), Rb + i * EP * 256 + wid * 1024);
      if constexpr (Z)
        dgs_glds(a.z + (uint32_t)(m * a.ldz + a.zoff + n0 + gj * 8), Zb + i * EP * 256 + wid * 1024);
    }
    if constexpr (MASK == 1) {
      if (wid == 0) {   // one 16-B piece (128 mask bits) per row
        const int m = min(mt * BM + lane, a.M - 1);
        dgs_glds(a.mbits + (uint32_t)(m * (a.Kout >> 3) + (n0 >> 3)), Mb);
      }
    }
  };

  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(a.y, (short)0, a.y_bytes, 0x00020000);
  f32x4 bq[TN], ms[TN], mh[TN];
#pragma unroll
  for (int ni = 0; ni < TN; ++ni) {
    const int c = n0 + wn * WN + ni * 16 + 4 * fg;
    bq[ni] = a.bias ? *reinterpret_cast<const f32x4*>(a.bias + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (MASK == 2) {
      ms[ni] = *reinterpret_cast<const f32x4*>(a.mscale + c);
      mh[ni] = *reinterpret_cast<const f32x4*>(a.mshift + c);
    }
  }
  float s1[TN][4], s2[TN][4];
#pragma unroll
  for (int ni = 0; ni < TN; ++ni)
#pragma unroll
    for (int j = 0; j < 4; ++j) { s1[ni][j] = 0.f; s2[ni][j] = 0.f; }

  const int cg = tid & 15, rg = tid >> 4;   // row-store phase: 16 threads per 256-B row

  // one tile; Rc/Zc/Mc: this tile's epilogue operands, Rn/Zn/Mn: the next tile's (prefetched here)
  auto tile = [&](int mt, int it, const char* Rc, const char* Zc, const char* Mc, char* Rn, char* Zn, char* Mn) {
    (void)it;
    // this tile's A / epilogue operands: the only younger vector-memory operations of this wave are
    // the previous tile's NSTORE stores, which stay in flight (before the first tile: none)
    __builtin_amdgcn_s_waitcnt(dgs_vmcnt(NSTORE));
    dgs_barrier();   // this tile's A / epilogue operands landed in every wave; last tile's reads done

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
          af[mi] = *reinterpret_cast<const bf16x8*>(A + r * 128 + ((ch ^ ((r >> 1) & 7)) << 4));
        }
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) {
          const int r = wn * WN + ni * 16 + fr;
          bfr[ni] = *reinterpret_cast<const bf16x8*>(B + r * 128 + ((ch ^ ((r >> 1) & 7)) << 4));
        }
#pragma unroll
        for (int mi = 0; mi < TM; ++mi)
#pragma unroll
          for (int ni = 0; ni < TN; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[ni], af[mi], acc[mi][ni], 0, 0, 0);
      }
    }
    dgs_barrier();       // every wave is done reading this tile's A
    issue_e(mt + a.G, Rn, Zn, Mn);
    issue_a(mt + a.G);   // the next tile's A streams in under this epilogue

    // epilogue on the D^T fragments: lane (fr, fg) holds row wm*WM + 16 mi + fr, channels
    // wn*WN + 16 ni + 4 fg + [0, 4)
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const int row = wm * WM + mi * 16 + fr;
      const float keep = mt * BM + row < a.M ? 1.f : 0.f;
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int col = wn * WN + ni * 16 + 4 * fg;
        const int eo = dgs_eoff(row, col);
        f32x4 v = acc[mi][ni] + bq[ni];
        if (has_res) {
          const u32x2 q = *reinterpret_cast<const u32x2*>(Rc + eo);
          v += f32x4{__uint_as_float(q[0] << 16), __uint_as_float(q[0] & 0xffff0000u), __uint_as_float(q[1] << 16),
                      __uint_as_float(q[1] & 0xffff0000u)};
        }
        if constexpr (Z) {
          const u32x2 q = *reinterpret_cast<const u32x2*>(Zc + eo);
          const f32x4 zz{__uint_as_float(q[0] << 16), __uint_as_float(q[0] & 0xffff0000u), __uint_as_float(q[1] << 16),
                         __uint_as_float(q[1] & 0xffff0000u)};
          if constexpr (MASK == 1) {
            const uint32_t b = (uint32_t)(uint8_t)Mc[row * 16 + (col >> 3)] >> (col & 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = (b >> j) & 1u ? v[j] : 0.f;
          } else {   // same fma as the forward BN-apply -> same sign as its output
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = __builtin_fmaf(zz[j], ms[ni][j], mh[ni][j]) > 0.f ? v[j] : 0.f;
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float rv = bf2f(f2bf(v[j])) * keep;   // statistics of the stored gradient
            s1[ni][j] += rv;
            s2[ni][j] += rv * zz[j];
          }
        }
        *reinterpret_cast<u32x2*>(Os + eo) = u32x2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
      }
    }
    dgs_barrier();
#pragma unroll
    for (int i = 0; i < NSTORE; ++i) {
      const int row = rg + EP * i;
      const u32x4 q = *reinterpret_cast<const u32x4*>(Os + row * 256 + ((cg ^ (row & 15)) << 4));
      const int m = mt * BM + row;
      const uint32_t off0 = (uint32_t)(m * a.ldy + a.yoff + n0 + cg * 8) * 2u;   // 32-bit: host-checked
      __builtin_amdgcn_raw_buffer_store_b128(q, yr, m < a.M ? off0 : 0x80000000u, 0, 0);
    }
  };

  int mt = g;
  if (mt < a.mtiles) {
    issue_a(mt);
    issue_e(mt, E0, E0 + EZ_OFF, E0 + EM_OFF);
  }
  __builtin_amdgcn_s_waitcnt(dgs_vmcnt(0));
  for (int it = 0; mt < a.mtiles;) {
    tile(mt, it, E0, E0 + EZ_OFF, E0 + EM_OFF, E1, E1 + EZ_OFF, E1 + EM_OFF);
    mt += a.G;
    ++it;
    if (mt >= a.mtiles) break;
    tile(mt, it, E1, E1 + EZ_OFF, E1 + EM_OFF, E0, E0 + EZ_OFF, E0 + EM_OFF);
    mt += a.G;
    ++it;
  }
  __builtin_amdgcn_s_waitcnt(dgs_vmcnt(0));   // no LDS-DMA in flight when the block retires

  if constexpr (Z) {
    __syncthreads();
    // per-lane sums -> [2][WGM * 16][BN] (the weight tile is free now) -> one row per block
    float* red = reinterpret_cast<float*>(Ws);
    static_assert(2 * WGM * 16 * BN * 4 <= W_BYTES, "statistics combine fits the weight tile");
#pragma unroll
    for (int ni = 0; ni < TN; ++ni)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = wn * WN + ni * 16 + 4 * fg + j;
        red[(wm * 16 + fr) * BN + col] = s1[ni][j];
        red[(WGM * 16 + wm * 16 + fr) * BN + col] = s2[ni][j];
      }
    __syncthreads();
    if (tid < BN && n0 + tid < a.Kout) {
      float t1 = 0.f, t2 = 0.f;
      for (int q = 0; q < WGM * 16; ++q) {
        t1 += red[q * BN + tid];
        t2 += red[(WGM * 16 + q) * BN + tid];
      }
      float* st = a.stats + (int64_t)g * 2 * a.Kout + n0 + tid;
      st[0] = t1;
      st[a.Kout] = t2;
    }
  }
}

}  // namespace dlmpi

using namespace dlmpi;

// DLMPI_DGRAD_STREAM=0 disables the kernel (A/B); set_dgrad_stream(0|1) overrides (tests)
static int g_dgs_override = -1;
extern "C" void dlmpi_set_dgrad_stream(int mode) { g_dgs_override = mode; }

// Tile plan: BM rows per tile and G blocks per 128-channel column (one block per CU over the chip),
// or 0 if the kernel does not apply to this shape.
extern "C" int dlmpi_dgrad_stream_plan(int64_t M, int K, int Kout, int mask_mode, int* bm, int* G) {
  static const int env = [] {
    const char* e = getenv("DLMPI_DGRAD_STREAM");
    return e ? atoi(e) : 1;
  }();
  const int on = g_dgs_override >= 0 ? g_dgs_override : env;
  if (!on || M <= 0 || Kout % 128 != 0 || mask_mode < 0 || mask_mode > 2) return 0;
  if (K == 128) *bm = 64;
  else if (K == 256) *bm = 32;
  else return 0;
  const int ntiles = Kout / 128;
  const int64_t mtiles = (M + *bm - 1) / *bm;
  int target = 256 / ntiles;
  if (target < 8) target = 8;
  *G = (int)(mtiles < target ? mtiles : target);
  return 1;
}

extern "C" hipError_t dlmpi_conv1x1_dgrad_stream(const DgradStreamArgs* a, int bm, int mask_mode, hipStream_t s) {
  const dim3 grid((unsigned)(a->ntiles * a->G));
#define DLMPI_DGS(BM_, KS_, NW_)                                                                                    \
  do {                                                                                                             \
    if (mask_mode == 1) hipLaunchKernelGGL((conv1x1_dgrad_stream_kernel<BM_, KS_, NW_, 1>), grid, dim3(64 * NW_), 0, s, *a); \
    else if (mask_mode == 2) hipLaunchKernelGGL((conv1x1_dgrad_stream_kernel<BM_, KS_, NW_, 2>), grid, dim3(64 * NW_), 0, s, *a); \
    else hipLaunchKernelGGL((conv1x1_dgrad_stream_kernel<BM_, KS_, NW_, 0>), grid, dim3(64 * NW_), 0, s, *a);       \
  } while (0)
  if (bm == 64 && a->K == 128) DLMPI_DGS(64, 2, 8);
  else if (bm == 32 && a->K == 256) DLMPI_DGS(32, 4, 4);
  else return hipErrorInvalidValue;
#undef DLMPI_DGS
  return hipGetLastError();
}
