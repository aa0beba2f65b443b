// Streaming 1x1 / stride-1 DATA GRADIENT with the fused BN-backward epilogue: the memory-bound
// GEMMs of the ResNet bottleneck backward whose epilogue, not the MFMA work, sets the time.
//
//   dx[m, c] = sum_k A[m, k] W[c, k] (+ bias[c]) (+ res[m, c]),  then the consumer's ReLU mask
//   (mask bits of the forward BN-apply, or z * mscale + mshift > 0) and its BN-backward partials
//   {sum dx, sum dx * z [, sum dx * z2]} of the stored (bf16) gradient (z2: a second BN input
//   consuming the same gradient, the ResNet downsample branch).
//
// A is dy, or [dy | z] of the dual data gradient (engine.ConvUnit.dual, K = 2 x 64 / 2 x 256).
// Tiles by reduction length (dlmpi_dgrad_stream_plan): K 128 -> 64 x 128 (8 waves), K 256 -> 48 x 128
// (6 waves; 32 x 128 with z2), K 512 -> 64 x 64 (8 waves, z-mask only; 32 x 64 with a residual / mask
// bits / z2 is opt-in, measured slower).  One block per CU; 98-160 KB of LDS.
// Example (profiles/r3_s3_base/resnet50_step.txt): layer-1 conv1 of a bottleneck, 802,816 rows, K 128,
// 256 output channels, plus a residual gradient, the previous block's z and mask bits: 1.46 GB of
// traffic that the general implicit-GEMM kernel moved in 645 us (2.3 TB/s) -- every block stages
// A, runs 2 K-steps of MFMA and then waits on the dependent residual / z / mask loads of its
// epilogue rows, so loads and stores never overlap inside a block.
//
// Here (same idea as conv1x1_stream.hip, extended to the epilogue operands):
//   * persistent blocks (one per CU), each walking a column of 128- (or 64-) channel output tiles;
//     the weight tile [BN][K] is staged into LDS once and stays resident;
//   * the NEXT tile's epilogue operands (residual, z, mask bits) and A are fetched global -> LDS
//     (global_load_lds; the operands into the other half of a double buffer) right after the
//     current tile's MFMAs, so they stream in under the current tile's epilogue math and stores
//     (issued before the MFMAs instead, the compiler cannot separate the in-flight operand DMA from
//     the A / W fragment reads and waits for it there);
//   * the epilogue runs on the D^T accumulator fragments (operands swapped: each lane holds 4
//     consecutive channels of one pixel) reading its residual / z / mask pieces from LDS
//     (XOR-swizzled rows: conflict-free 8-byte reads), writes bf16 quads in place of the consumed
//     z tile (a staging tile of its own without statistics) and
//     the tile leaves as 16-byte row stores that are never waited for (the only wait is
//     vmcnt(NSTORE) at the top of the next tile: vmcnt retires in issue order and the stores were
//     issued last);
//   * BN partial sums accumulate per lane over ALL of the block's tiles: one partial row per block.
// The per-element arithmetic is the conv_igemm epilogue's (fp32: (acc + bias) + res, mask, round
// once to bf16), so dx is bit-identical to the general kernel (K <= 256; at K = 512 the general
// kernel may split K); the partial sums differ only in fp32 summation order.
// With an RCCL communicator the grid is 256 - (RCCL channels) blocks (parallel/comm.py): a block
// that cannot start because a collective's workgroup holds LDS on its CU would hold the kernel.
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

// Epilogue-operand tiles of BM rows x BN channels (2 BN-byte rows): 16-byte chunk j of row r sits at
// chunk position j ^ sw(r) -- for 256-B rows sw = r & 15, for 128-B rows (two rows per 256-B bank
// line) sw = (r >> 1) & 7 -- so the 16 rows read by one D^T fragment column hit 16 different
// 16-byte bank slots.
template <int BN>
__device__ __forceinline__ int dgs_sw(int r) { return BN == 128 ? (r & 15) : ((r >> 1) & 7); }
template <int BN>
__device__ __forceinline__ int dgs_eoff(int r, int col) {   // byte offset of channel col (multiple of 4)
  return r * (2 * BN) + ((((col >> 3) ^ dgs_sw<BN>(r))) << 4) + ((col & 4) << 1);
}

// MASK: 1 = forward mask bits, 2 = z * mscale + mshift > 0, 0 = no mask and no statistics;
// Z2: a second BN input (third partial row sum dx * z2);
// ADB: A double-buffered, the next tile's A issued at the top of the current tile (long reductions:
// the A tile is most of a tile's bytes), else single-buffered and issued after the MFMAs.
// WGM: wave-grid rows (WGM x NW / WGM waves; 48-row tiles: 3 x 2).
template <int BM, int BN, int KS, int NW, int WGM, int MASK, bool Z2, bool ADB>
__global__ __launch_bounds__(64 * NW) void conv1x1_dgrad_stream_kernel(const DgradStreamArgs a) {
  constexpr bool Z = MASK != 0;
  static_assert(!Z2 || Z, "z2 needs the fused statistics");
  static_assert(BN == 64 || BN == 128, "tile width");
  constexpr bool RES = !(BN == 64 && BM == 64);  // residual-gradient operand (64 x 64 tiles: none, LDS)
  constexpr int NS = Z2 ? 3 : 2;
  constexpr int NT = 64 * NW;
  constexpr int WGN = NW / WGM;                 // wave grid
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int RP = NT / 8;                    // 128-B rows staged per pass (A / W tiles)
  constexpr int AL = BM / RP;
  constexpr int BL = (BN + RP - 1) / RP, WROWS = BL * RP;   // weight rows staged (>= BN: padding rows)
  constexpr int ERB = 2 * BN, ECH = BN / 8;     // epilogue tiles: bytes / 16-B chunks per row
  constexpr int EP = NT / ECH;                  // epilogue-tile rows staged per pass
  constexpr int EL = BM / EP;
  constexpr int NSTORE = BM / EP;               // 16-byte output row stores per thread per tile
  // mask-bit tile: BN / 8 bytes per row, staged with 16-byte (BN 128) or 4-byte (BN 64) pieces, in
  // whole wave instructions (64 rows / 32 rows each)
  constexpr int MBR = BN / 8, MB_PIECE = BN == 128 ? 16 : 4, MB_WROWS = 64 * MB_PIECE / MBR;
  constexpr int MB_INSTR = (BM + MB_WROWS - 1) / MB_WROWS, MB_ROWS = MB_INSTR * MB_WROWS;
  static_assert(MB_INSTR <= NW, "mask-bit staging: one instruction per wave");
  constexpr int E_BYTES = BM * ERB;
  static_assert(AL >= 1 && BM % RP == 0 && BM % EP == 0 && EL >= 1 && TM >= 1 && TN >= 1 && WM % 16 == 0 &&
                WN % 16 == 0, "tile shape");
  constexpr int W_BYTES = KS * WROWS * 128, A_BYTES = KS * BM * 128;
  // distinct LDS objects per buffer (the compiler's LDS-DMA alias tracking then sees that the
  // epilogue's reads of one buffer do not depend on the prefetch in flight into the other; the
  // double-buffer index is static: the tile loop is unrolled by two)
  __shared__ __attribute__((aligned(16))) char Ws[W_BYTES];
  __shared__ __attribute__((aligned(16))) char A0[A_BYTES];
  __shared__ __attribute__((aligned(16))) char A1[ADB ? A_BYTES : 16];
  // epilogue-operand double buffer: [residual | z | z2 | mask bits] per buffer (one LDS object each:
  // the compiler tracks a handful of LDS-DMA targets, more objects make it wait for all of them).
  // With statistics the output tile is staged in place of the consumed z tile (each lane writes
  // exactly the positions it has read); without, in a tile of its own.
  constexpr int EZ_OFF = RES ? E_BYTES : 0, EZ2_OFF = EZ_OFF + (Z ? E_BYTES : 0), EM_OFF = EZ2_OFF + (Z2 ? E_BYTES : 0);
  constexpr int EB_BYTES0 = EM_OFF + (MASK == 1 ? MB_ROWS * MBR : 0);
  constexpr int EB_BYTES = EB_BYTES0 > 16 ? EB_BYTES0 : 16;
  __shared__ __attribute__((aligned(16))) char E0[EB_BYTES];
  __shared__ __attribute__((aligned(16))) char E1[EB_BYTES];
  __shared__ __attribute__((aligned(16))) char Os[Z ? 16 : E_BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WGN, wn = wid % WGN;
  const int fr = lane & 15, fg = lane >> 4;
  const int lrow = tid >> 3;                                 // A / W staging row (+ RP i)
  const int jc = (tid & 7) ^ ((tid >> 3) & 7);               // swizzled 16-B chunk this lane fetches
  const int erow = tid / ECH, ej = tid % ECH;                // epilogue-tile staging row (+ EP i), chunk
  const char* zp = reinterpret_cast<const char*>(g_zero_page);

  const uint32_t lb = xcd_remap(blockIdx.x, gridDim.x);
  const int nt = lb % a.ntiles, g = lb / a.ntiles;
  const int n0 = nt * BN;
  const bool has_res = RES && a.res != nullptr;

  // ---- weights: staged once --------------------------------------------------------------------
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const int n = n0 + lrow + RP * i;
      const char* src = (lrow + RP * i < BN && n < a.Kout)
                            ? reinterpret_cast<const char*>(a.w + (int64_t)n * a.K + ks * 64 + 8 * jc) : zp;
      dgs_glds(src, Ws + ks * WROWS * 128 + (RP * i + 8 * wid) * 128);
    }
  // rows past M re-read row M - 1 (outputs dropped, statistics masked): unconditional loads keep the
  // compiler's vmcnt scoreboard exact (32-bit offsets: host-checked)
  auto issue_a = [&](int mt, char* Ab) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int i = 0; i < AL; ++i) {
        const int m = min(mt * BM + lrow + RP * i, a.M - 1);
        dgs_glds(a.x + (uint32_t)(m * a.ldx + a.xoff + ks * 64 + 8 * jc), Ab + ks * BM * 128 + (RP * i + 8 * wid) * 128);
      }
  };
  auto issue_e = [&](int mt, char* Rb, char* Zb, char* Mb) {
#pragma unroll
    for (int i = 0; i < EL; ++i) {
      const int r = erow + EP * i;
      const int m = min(mt * BM + r, a.M - 1);
      const int gj = ej ^ dgs_sw<BN>(r);                      // global chunk stored at LDS chunk ej
      // LDS destination: lane-linear 1 KB per wave instruction = rows erow (+ EP i), chunk ej
      if (has_res)
        dgs_glds(a.res + (uint32_t)(m * a.ldres + a.resoff + n0 + gj * 8), Rb + i * EP * ERB + wid * 1024);
      if constexpr (Z)
        dgs_glds(a.z + (uint32_t)(m * a.ldz + a.zoff + n0 + gj * 8), Zb + i * EP * ERB + wid * 1024);
      if constexpr (Z2)
        dgs_glds(a.z2 + (uint32_t)(m * a.ldz2 + a.z2off + n0 + gj * 8), Zb + (EZ2_OFF - EZ_OFF) + i * EP * ERB + wid * 1024);
    }
    if constexpr (MASK == 1) {
      if (wid < MB_INSTR) {   // wave w: rows [w MB_WROWS, (w + 1) MB_WROWS) of the mask-bit tile
        const int piece = wid * 64 + lane;                     // MB_PIECE-byte piece of the tile
        const int r = piece * MB_PIECE / MBR;
        const int m = min(mt * BM + r, a.M - 1);
        const uint8_t* src = a.mbits + (uint32_t)(m * (a.Kout >> 3) + (n0 >> 3) + (piece * MB_PIECE) % MBR);
        if constexpr (MB_PIECE == 16) __builtin_amdgcn_global_load_lds(src, (dgs_lds_void*)(Mb + wid * 1024), 16, 0, 0);
        else __builtin_amdgcn_global_load_lds(src, (dgs_lds_void*)(Mb + wid * 256), 4, 0, 0);
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
  float s1[TN][4], s2[TN][4], s3[TN][4];
#pragma unroll
  for (int ni = 0; ni < TN; ++ni)
#pragma unroll
    for (int j = 0; j < 4; ++j) { s1[ni][j] = 0.f; s2[ni][j] = 0.f; s3[ni][j] = 0.f; }

  const int cg = tid % ECH, rg = tid / ECH;   // row-store phase: ECH threads per row

  // one tile; Ac / Rc / Zc / Mc: this tile's operands, An / Rn / Zn / Mn: the next tile's (prefetched)
  auto tile = [&](int mt, const char* Ac, char* An, const char* Rc, char* Zc, const char* Mc, char* Rn, char* Zn,
                  char* Mn) {
    char* Ot = Z ? Zc : Os;   // output staging tile
    // this tile's A / epilogue operands: the only younger vector-memory operations of this wave are
    // the previous tile's NSTORE stores, which stay in flight (before the first tile: none)
    __builtin_amdgcn_s_waitcnt(dgs_vmcnt(NSTORE));
    dgs_barrier();   // this tile's A / epilogue operands landed in every wave; last tile's reads done
    if constexpr (ADB) issue_a(mt + a.G, An);

    f32x4 acc[TM][TN];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi)
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const char* A = Ac + ks * BM * 128;
      const char* B = Ws + ks * WROWS * 128;
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
    dgs_barrier();       // every wave is done reading this tile's A
    issue_e(mt + a.G, Rn, Zn, Mn);
    if constexpr (!ADB) issue_a(mt + a.G, An);   // the next tile's A streams in under this epilogue

    // epilogue on the D^T fragments: lane (fr, fg) holds row wm*WM + 16 mi + fr, channels
    // wn*WN + 16 ni + 4 fg + [0, 4)
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const int row = wm * WM + mi * 16 + fr;
      const float keep = mt * BM + row < a.M ? 1.f : 0.f;
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int col = wn * WN + ni * 16 + 4 * fg;
        const int eo = dgs_eoff<BN>(row, col);
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
            const uint32_t b = (uint32_t)(uint8_t)Mc[row * MBR + (col >> 3)] >> (col & 4);
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
          if constexpr (Z2) {
            const u32x2 q2 = *reinterpret_cast<const u32x2*>(Zc + (EZ2_OFF - EZ_OFF) + eo);
            const f32x4 z2{__uint_as_float(q2[0] << 16), __uint_as_float(q2[0] & 0xffff0000u),
                           __uint_as_float(q2[1] << 16), __uint_as_float(q2[1] & 0xffff0000u)};
#pragma unroll
            for (int j = 0; j < 4; ++j) s3[ni][j] += bf2f(f2bf(v[j])) * keep * z2[j];
          }
        }
        *reinterpret_cast<u32x2*>(Ot + eo) = u32x2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
      }
    }
    dgs_barrier();
#pragma unroll
    for (int i = 0; i < NSTORE; ++i) {
      const int row = rg + EP * i;
      const u32x4 q = *reinterpret_cast<const u32x4*>(Ot + row * ERB + ((cg ^ dgs_sw<BN>(row)) << 4));
      const int m = mt * BM + row;
      const uint32_t off0 = (uint32_t)(m * a.ldy + a.yoff + n0 + cg * 8) * 2u;   // 32-bit: host-checked
      __builtin_amdgcn_raw_buffer_store_b128(q, yr, m < a.M ? off0 : 0x80000000u, 0, 0);
    }
  };

  char* const A1p = ADB ? A1 : A0;
  int mt = g;
  if (mt < a.mtiles) {
    issue_a(mt, A0);
    issue_e(mt, E0, E0 + EZ_OFF, E0 + EM_OFF);
  }
  __builtin_amdgcn_s_waitcnt(dgs_vmcnt(0));
  for (; mt < a.mtiles;) {
    tile(mt, A0, A1p, E0, E0 + EZ_OFF, E0 + EM_OFF, E1, E1 + EZ_OFF, E1 + EM_OFF);
    mt += a.G;
    if (mt >= a.mtiles) break;
    tile(mt, A1p, A0, E1, E1 + EZ_OFF, E1 + EM_OFF, E0, E0 + EZ_OFF, E0 + EM_OFF);
    mt += a.G;
  }
  __builtin_amdgcn_s_waitcnt(dgs_vmcnt(0));   // no LDS-DMA in flight when the block retires

  if constexpr (Z) {
    // per-lane sums -> [WGM * 16][BN] (one statistic at a time, in the now free weight tile) -> one
    // row per block, summed in a fixed order
    constexpr int RR = WGM * 16;
    static_assert(RR * BN * 4 <= W_BYTES, "statistics combine fits the weight tile");
    float* red = reinterpret_cast<float*>(Ws);
    float* st = a.stats + (int64_t)g * NS * a.Kout + n0 + tid;
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      __syncthreads();
#pragma unroll
      for (int ni = 0; ni < TN; ++ni)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          red[(wm * 16 + fr) * BN + wn * WN + ni * 16 + 4 * fg + j] = k == 0 ? s1[ni][j] : (k == 1 ? s2[ni][j] : s3[ni][j]);
      __syncthreads();
      if (tid < BN && n0 + tid < a.Kout) {
        float t = 0.f;
        for (int q = 0; q < RR; ++q) t += red[q * BN + tid];
        st[k * a.Kout] = t;
      }
    }
  }
}

}  // namespace dlmpi

using namespace dlmpi;

// set_dgrad_stream(0|1) overrides the plan (tests; 2: also the
// opt-in tile variants)
static int g_dgs_override = -1;
extern "C" void dlmpi_set_dgrad_stream(int mode) { g_dgs_override = mode; }
// grid-size budget (blocks) set by the communicator that owns the CUs RCCL takes (parallel/comm.py
// rccl_channel_budget); <= 0: DLMPI_DGS_BLOCKS or one block per CU
static int g_dgs_blocks = 0;
extern "C" void dlmpi_set_dgs_blocks(int n) { g_dgs_blocks = n; }
extern "C" int dlmpi_dgs_blocks() {
  static const int env = [] {
    const char* e = getenv("DLMPI_DGS_BLOCKS");
    return e ? atoi(e) : 256;
  }();
  return g_dgs_blocks > 0 ? g_dgs_blocks : env;
}

// Tile plan: BM rows per tile and G blocks per 128-channel column (one block per CU over the chip),
// or 0 if the kernel does not apply to this shape.
// Grid size target: dlmpi_dgs_blocks() (default 256 = one block per CU; fewer with an RCCL
// communicator whose channels hold CUs).
extern "C" int dlmpi_dgrad_stream_plan(int64_t M, int K, int Kout, int mask_mode, int z2, int has_res, int* bm, int* bn,
                                       int* G) {
  const int blocks = dlmpi_dgs_blocks();
  const int on = g_dgs_override != 0;
  if (!on || M <= 0 || mask_mode < 0 || mask_mode > 2 || (z2 && mask_mode == 0)) return 0;
  // LDS per block (one block per CU): weights KS x BN x 128 B resident + A + 2 x epilogue operands
  if (K == 128 && Kout % 128 == 0) { *bm = 64; *bn = 128; }          // 98-146 KB
  else if (K == 256 && Kout % 128 == 0) {   // 48 rows: 6 waves (3 x 2), 135-149 KB; 32 with z2
    *bm = z2 ? 32 : 48;
    *bn = 128;
  }
  else if (K == 512 && Kout % 64 == 0) {
    // 64 x 64 tiles, 8 waves (136-144 KB) for the z-mask-only dual conv3 gradient; with a residual /
    // mask bits / z2: 32 x 64, 4 waves (113-121 KB)
    *bn = 64;
    *bm = (has_res || z2 || mask_mode == 1) ? 32 : 64;
    // 32 x 64 tiles measured slower than the general kernel (layer3.0 conv1 dual 2x256 -> 512: 359 vs
    // 289 us; layer4 conv1 77 vs 69 us -- eight 64-wide columns re-read A, 4 waves per CU; ResNet-50
    // 12,802 / 12,803 vs 12,837 / 12,968 img/s, profiles/r3_dgrad_stream/v4)
    if (g_dgs_override != 2 && *bm == 32) return 0;
  }
  else return 0;
  const int ntiles = Kout / *bn;
  const int64_t mtiles = (M + *bm - 1) / *bm;
  int target = blocks / ntiles;
  if (target < 8) target = 8;
  *G = (int)(mtiles < target ? mtiles : target);
  return 1;
}

extern "C" hipError_t dlmpi_conv1x1_dgrad_stream(const DgradStreamArgs* a, int bm, int bn, int mask_mode, hipStream_t s) {
  const dim3 grid((unsigned)(a->ntiles * a->G));
#define LAUNCH_DGS(BM_, BN_, KS_, NW_, WGM_, ADB_)                                                                   \
  do {                                                                                                       \
    const dim3 blk(64 * NW_);                                                                                \
    if (a->z2) {                                                                                             \
      if (mask_mode == 1) hipLaunchKernelGGL((conv1x1_dgrad_stream_kernel<BM_, BN_, KS_, NW_, WGM_, 1, true, ADB_>), grid, blk, 0, s, *a); \
      else hipLaunchKernelGGL((conv1x1_dgrad_stream_kernel<BM_, BN_, KS_, NW_, WGM_, 2, true, ADB_>), grid, blk, 0, s, *a); \
    } else if (mask_mode == 1) hipLaunchKernelGGL((conv1x1_dgrad_stream_kernel<BM_, BN_, KS_, NW_, WGM_, 1, false, ADB_>), grid, blk, 0, s, *a); \
    else if (mask_mode == 2) hipLaunchKernelGGL((conv1x1_dgrad_stream_kernel<BM_, BN_, KS_, NW_, WGM_, 2, false, ADB_>), grid, blk, 0, s, *a); \
    else hipLaunchKernelGGL((conv1x1_dgrad_stream_kernel<BM_, BN_, KS_, NW_, WGM_, 0, false, ADB_>), grid, blk, 0, s, *a); \
  } while (0)
  if (bm == 64 && bn == 128 && a->K == 128) LAUNCH_DGS(64, 128, 2, 8, 2, false);
  else if (bm == 48 && bn == 128 && a->K == 256 && !a->z2) {
    if (mask_mode == 1) hipLaunchKernelGGL((conv1x1_dgrad_stream_kernel<48, 128, 4, 6, 3, 1, false, false>), grid, dim3(384), 0, s, *a);
    else if (mask_mode == 2) hipLaunchKernelGGL((conv1x1_dgrad_stream_kernel<48, 128, 4, 6, 3, 2, false, false>), grid, dim3(384), 0, s, *a);
    else hipLaunchKernelGGL((conv1x1_dgrad_stream_kernel<48, 128, 4, 6, 3, 0, false, false>), grid, dim3(384), 0, s, *a);
  } else if (bm == 32 && bn == 128 && a->K == 256) {   // z2 (174 KB at 48 rows), or the 4-wave A/B variant
    if (a->z2) {
      if (mask_mode == 1) hipLaunchKernelGGL((conv1x1_dgrad_stream_kernel<32, 128, 4, 4, 2, 1, true, false>), grid, dim3(256), 0, s, *a);
      else hipLaunchKernelGGL((conv1x1_dgrad_stream_kernel<32, 128, 4, 4, 2, 2, true, false>), grid, dim3(256), 0, s, *a);
    } else if (mask_mode == 1) hipLaunchKernelGGL((conv1x1_dgrad_stream_kernel<32, 128, 4, 4, 2, 1, false, false>), grid, dim3(256), 0, s, *a);
    else if (mask_mode == 2) hipLaunchKernelGGL((conv1x1_dgrad_stream_kernel<32, 128, 4, 4, 2, 2, false, false>), grid, dim3(256), 0, s, *a);
    else hipLaunchKernelGGL((conv1x1_dgrad_stream_kernel<32, 128, 4, 4, 2, 0, false, false>), grid, dim3(256), 0, s, *a);
  }
  else if (bm == 32 && bn == 64 && a->K == 512) LAUNCH_DGS(32, 64, 8, 4, 2, false);
  else if (bm == 64 && bn == 64 && a->K == 512 && !a->z2 && !a->res) {   // z-mask / plain only
    if (mask_mode == 2) hipLaunchKernelGGL((conv1x1_dgrad_stream_kernel<64, 64, 8, 8, 2, 2, false, false>), grid, dim3(512), 0, s, *a);
    else if (mask_mode == 0) hipLaunchKernelGGL((conv1x1_dgrad_stream_kernel<64, 64, 8, 8, 2, 0, false, false>), grid, dim3(512), 0, s, *a);
    else return hipErrorInvalidValue;
  }
  else return hipErrorInvalidValue;
#undef LAUNCH_DGS
  return hipGetLastError();
}
