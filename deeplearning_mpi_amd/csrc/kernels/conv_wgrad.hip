// Convolution weight gradient on CDNA4 MFMA:  dW[ko][t][c] = sum_pix dY[pix][ko] * X[gather(pix,t)][c].
// Replaces cuDNN wgrad / cuBLAS Linear weight-grad of the reference.
//
// Both operands arrive pixel-major (NHWC: the reduction index is the SLOW axis), so they are
// staged row-major [64 pixels][cols] into LDS and fed to v_mfma_f32_16x16x32_bf16 through the
// gfx950 hardware-transposing read ds_read_b64_tr_b16 (cdna_hip_programming.md T10), with the
// XOR swizzle that makes those reads conflict-free.  The pixel axis is split across workgroups
// (split-K); every split writes its fp32 slice of a [splits][Ko][TC] workspace, and two reduction
// kernels sum the slices in a fixed order (bit-reproducible, no float atomics) into the flat fp32
// gradient buffer, undoing the compute-layout channel padding on the way.  (A last-arriver
// reduction inside this kernel measured slower at every split count, profiles/r3_wgrad_inlaunch_off.)
//
// Also used for ConvTranspose2d(k2,s2) weight-grad (roles of X and dY swapped, stride 2) and for
// Linear weight-grad (1x1 "conv" on a 1x1 image).
#include <cstdlib>

#include "common.h"

namespace dlmpi {

typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

// Byte offset of 16-B chunk `ch` of LDS row `row` in a tile with 256-B rows (16 chunks) or 128-B
// rows (8 chunks).  Both XORs make the 8 rows x 32 bytes touched by one half-wave of transposed
// reads land on 16 distinct 16-byte bank slots.
// 512-B rows (32 chunks): one transposed read touches rows k0 + 8g + q (+4), g, q in 0..3, chunks
// 2cb + {0,1}; XOR-ing the chunk pair index with (q | g << 2) spreads the 16 rows over all 32
// chunk slots = both 256-B bank rows exactly once each.
template <int ROW_BYTES>
__device__ __forceinline__ int tr_swz(int row) {
  if constexpr (ROW_BYTES == 512) return (((row & 3) | (((row >> 3) & 3) << 2)) << 1);
  else if constexpr (ROW_BYTES == 256) return ((row & 3) << 2) | ((row >> 2) & 3);
  else return (((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2);
}

template <int ROW_BYTES>
__device__ __forceinline__ int tr_off(int row, int ch) {
  return row * ROW_BYTES + ((ch ^ tr_swz<ROW_BYTES>(row)) << 4);
}

// 16x32 MFMA operand (16 columns starting at column 16*cb, 32 reduction rows starting at k0)
// from a row-major [k][col] LDS tile: lane (g, i) gets column i, rows k0+8g .. k0+8g+7.
template <int ROW_BYTES>
__device__ __forceinline__ bf16x8 tr_frag(const char* tile, int k0, int cb, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int row = k0 + 8 * g + q;
  const int ch = 2 * cb + (p >> 1);
  const int byte = (p & 1) * 8;
  const char* a0 = tile + tr_off<ROW_BYTES>(row, ch) + byte;
  const char* a1 = tile + tr_off<ROW_BYTES>(row + 4, ch) + byte;
  i16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(a0));
  i16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(a1));
  typedef short i16x8 __attribute__((ext_vector_type(8)));
  i16x8 r = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, r);
}

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void glds16(const void* g, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, (lds_void*)lds_wave_base, 16, 0, 0);
}

// Inverse of tr_off within a row: the chunk that lives at 16-B slot `pos` of row `row`.
template <int ROW_BYTES>
__device__ __forceinline__ int tr_chunk(int row, int pos) {
  return pos ^ tr_swz<ROW_BYTES>(row);
}

// Operands are staged global -> LDS with global_load_lds (no VGPR round trip): piece i of thread
// tid fills the 16-B LDS slot 16*(256 i + tid), i.e. each wave writes 1 KB contiguously, and the
// lane fetches whichever (pixel row, 16-B chunk) the swizzled layout puts there.  Single stage,
// two barriers per K-step, 32 KB LDS at BM = 128 -> several blocks per CU hide the load latency of
// one another.  (A double-buffered form with the DMA issued through glds16_raw ran the 1x1 weight
// gradients 5-13 % faster in isolation but cost ResNet-50 0.6-0.8 % in the step: 64 KB of LDS per
// block keep the data-gradient chain's streaming blocks off the CU, profiles/r5_wgrad.)
// PA = 2: the dy operand is a deferred BN-backward apply (dz = k1 dy + k2 Z + k3, Z staged beside
// dy); PB = 1: the x operand is a deferred BN-apply + ReLU (relu(x * scale + shift)).  Both are
// rewritten in LDS once a stage has landed, in-range pieces only (padding / tails stay zero), with
// the arithmetic of the standalone kernels they replace (bit-identical results).
// WR: wave-grid rows (WR x 4/WR waves).  64 x 256 (Ko <= 64 layers: the whole Ko by 256 columns)
// runs 1 x 4 waves of 64 x 64: 16 transposed-read pairs per 16 MFMAs instead of the 64 x 128 tile's
// 12 per 8, and every dy row is staged once per 256 instead of per 128 columns.
template <int BM, int BN, bool DIRECT, int PA = 0, int PB = 0, int WR = 2>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BN == 128 ? 3 : 2, 8)))
void conv_wgrad_kernel(const WgradArgs a) {
  constexpr int BK = 64;
  constexpr int WC = 4 / WR;                               // wave-grid columns
  constexpr int WM = BM / WR, WN = BN / WC, TM = WM / 16, TN = WN / 16;
  constexpr int A_ROW = BM * 2, B_ROW = BN * 2;          // bytes per LDS row
  constexpr int AL = BK * A_ROW / 4096, BL = BK * B_ROW / 4096;   // 16-B pieces per thread
  constexpr int A_BYTES = BK * A_ROW, B_BYTES = BK * B_ROW;
  constexpr int Z_BYTES = PA == 2 ? A_BYTES : 0;
  constexpr int SB = A_BYTES + B_BYTES + Z_BYTES;        // per stage: [A | B | Z]
  __shared__ __attribute__((aligned(16))) char smem[SB];

  const uint32_t ntile = (uint32_t)a.mtiles * a.ntiles;
  const uint32_t nwg = ntile * a.splits;
  const uint32_t bid = xcd_remap(blockIdx.x, nwg);
  const int z = bid / ntile;
  const int tile = bid - z * ntile;
  const int mt = tile / a.ntiles, nt = tile - mt * a.ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int pbeg = z * a.pix_per_split;
  const int pend = min(a.npix, pbeg + a.pix_per_split);
  const int nk = pend > pbeg ? (pend - pbeg + BK - 1) / BK : 0;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WC, wn = wid % WC;
  const int PQ = a.P * a.Q;
  const char* zp = reinterpret_cast<const char*>(g_zero_page);

  // Piece i of this lane: 16-B LDS slot o = 256 i + tid -> (pixel row, swizzled chunk).  Rows and
  // chunks are recomputed from (i, tid) (a few bit ops); only the gather tap of B is kept.
  auto piece = [&](int i, int ROW, int& row, int& ch) {
    const int o = 256 * i + tid;
    row = (o * 16) / ROW;
    const int pos = (o * 16 % ROW) / 16;
    ch = ROW == 512 ? tr_chunk<512>(row, pos) : ROW == 256 ? tr_chunk<256>(row, pos) : tr_chunk<128>(row, pos);
  };
  // B column chunk = (tap, channel): packed cch | (dh + 64) << 16 | (dw + 64) << 24, -1 = outside
  int b_pack[BL];
#pragma unroll
  for (int i = 0; i < BL; ++i) {
    int row, ch;
    piece(i, B_ROW, row, ch);
    const int col = n0 + 8 * ch;
    if (col < a.TC) {
      const int t = (int)fdiv((uint32_t)col, a.fdC);
      const int cch = col - t * a.C;
      const int tr = (int)fdiv((uint32_t)t, a.fdS);
      const int ts = t - tr * a.S;
      b_pack[i] = cch | ((tr - a.pad_h + 64) << 16) | ((ts - a.pad_w + 64) << 24);   // < 2^31
    } else {
      b_pack[i] = -1;
    }
  }
  const uint16_t* dyb = static_cast<const uint16_t*>(a.dy) + a.dyoff;
  const uint16_t* xb = static_cast<const uint16_t*>(a.x) + a.xoff;

  // Branch-free staging: every address is computed unconditionally (no dereference happens for
  // invalid pieces) and the zero page is selected with v_cndmask, so the glds issue is not split
  // into exec-masked regions.
  auto pick = [&](bool ok, const uint16_t* p) -> const char* {
    const uintptr_t a0 = reinterpret_cast<uintptr_t>(p), z = reinterpret_cast<uintptr_t>(zp);
    return reinterpret_cast<const char*>(ok ? a0 : z);
  };
  const uint16_t* zb = PA == 2 ? a.pz + a.pzoff : nullptr;

  // Fast staging for K-steps whose 64 pixel rows all lie inside the split, when every column piece
  // of the tile exists (wave-uniform, from a ballot): a per-K-step base in SGPRs (pix0 * ld) plus a
  // loop-invariant 32-bit byte offset per piece, so no DMA address costs vector arithmetic or a
  // select.  dy rows always qualify; x rows only for DIRECT (the gather decodes its pixel).  Not in
  // the prologue forms: their extra offsets push the 128 x 128 tile past 168 VGPRs (spills).
  constexpr bool FAST = PA == 0 && PB == 0;
  uint32_t a_lane[AL], z_lane[PA == 2 ? AL : 1], b_lane[DIRECT ? BL : 1];
  bool lane_ok = true;
#pragma unroll
  for (int i = 0; i < AL; ++i) {
    int row, ch;
    piece(i, A_ROW, row, ch);
    const int col = m0 + 8 * ch;
    lane_ok = lane_ok && col < a.Ko;
    a_lane[i] = 2u * ((uint32_t)row * (uint32_t)a.ldy + (uint32_t)col);
    if constexpr (PA == 2) z_lane[i] = 2u * ((uint32_t)row * (uint32_t)a.ldpz + (uint32_t)col);
  }
  if constexpr (DIRECT) {
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      int row, ch;
      piece(i, B_ROW, row, ch);
      lane_ok = lane_ok && b_pack[i] >= 0;
      b_lane[i] = 2u * ((uint32_t)row * (uint32_t)a.ldx + (uint32_t)(b_pack[i] & 0xffff));
    }
  }
  const bool cols_all = FAST && a.fast && __builtin_amdgcn_readfirstlane(__builtin_amdgcn_ballot_w64(!lane_ok) == 0);

  auto issue = [&](int buf, int pix0) {
    char* As = smem + buf * SB;
    char* Bs = As + A_BYTES;
    if (cols_all && pix0 + BK <= pend) {
      const char* ab = reinterpret_cast<const char*>(dyb + (int64_t)pix0 * a.ldy);
#pragma unroll
      for (int i = 0; i < AL; ++i) {
        glds16(ab + a_lane[i], As + 16 * (256 * i + 64 * wid));
        if constexpr (PA == 2)
          glds16(reinterpret_cast<const char*>(zb + (int64_t)pix0 * a.ldpz) + z_lane[i],
                 As + A_BYTES + B_BYTES + 16 * (256 * i + 64 * wid));
      }
      if constexpr (DIRECT) {
        const char* bb = reinterpret_cast<const char*>(xb + (int64_t)pix0 * a.ldx);
#pragma unroll
        for (int i = 0; i < BL; ++i) glds16(bb + b_lane[i], Bs + 16 * (256 * i + 64 * wid));
        return;
      }
    } else {
#pragma unroll
      for (int i = 0; i < AL; ++i) {
        int row, ch;
        piece(i, A_ROW, row, ch);
        const int pix = pix0 + row, col = m0 + 8 * ch;
        glds16(pick(pix < pend && col < a.Ko, dyb + (int64_t)pix * a.ldy + col), As + 16 * (256 * i + 64 * wid));
        if constexpr (PA == 2)
          glds16(pick(pix < pend && col < a.Ko, zb + (int64_t)pix * a.ldpz + col),
                 As + A_BYTES + B_BYTES + 16 * (256 * i + 64 * wid));
      }
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      int row, ch;
      piece(i, B_ROW, row, ch);
      const int pix = pix0 + row;
      const int bp = b_pack[i];
      const bool ok = pix < pend && bp >= 0;
      if constexpr (DIRECT) {   // 1x1, stride 1, no padding: the input pixel IS the output pixel
        glds16(pick(ok, xb + (int64_t)pix * a.ldx + (bp & 0xffff)), Bs + 16 * (256 * i + 64 * wid));
      } else {
        const uint32_t pp = ok ? (uint32_t)pix : 0u;
        const uint32_t n_img = fdiv(pp, a.fdPQ);
        const uint32_t rem = pp - n_img * PQ;
        const uint32_t p = fdiv(rem, a.fdQ);
        const uint32_t q = rem - p * a.Q;
        const int ih = (int)p * a.stride_h + ((bp >> 16) & 255) - 64;
        const int iw = (int)q * a.stride_w + ((bp >> 24) & 255) - 64;
        const bool in = ok && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        const int64_t off = (((int64_t)n_img * a.H + ih) * a.W + iw) * a.ldx + (bp & 0xffff);
        glds16(pick(in, xb + off), Bs + 16 * (256 * i + 64 * wid));
      }
    }
  };

  // Prologue work split: thread t rewrites 16-B chunk t % 16 (BM = 64: t % 8) of tile rows
  // t / 16 + 16 j, so its channel chunk -- and the coefficients -- are fixed per thread.
  auto prologue = [&](int buf, int pix0) {
    if constexpr (PA != 0 || PB != 0) {
      char* As = smem + buf * SB;
      if constexpr (PA == 2) {
        constexpr int CH = BM / 8, RS = 256 / CH;
        const int cq = tid % CH, r0 = tid / CH;
        const int col = m0 + 8 * cq;
        if (col < a.Ko) {
          const f32x4 k0a = *reinterpret_cast<const f32x4*>(a.pcoef + col);
          const f32x4 k0b = *reinterpret_cast<const f32x4*>(a.pcoef + col + 4);
          const f32x4 k1a = *reinterpret_cast<const f32x4*>(a.pcoef + a.Ko + col);
          const f32x4 k1b = *reinterpret_cast<const f32x4*>(a.pcoef + a.Ko + col + 4);
          const f32x4 k2a = *reinterpret_cast<const f32x4*>(a.pcoef + 2 * a.Ko + col);
          const f32x4 k2b = *reinterpret_cast<const f32x4*>(a.pcoef + 2 * a.Ko + col + 4);
#pragma unroll
          for (int r = r0; r < BK; r += RS) {
            if (pix0 + r >= pend) break;
            const int off = tr_off<A_ROW>(r, cq);
            u32x4* pa = reinterpret_cast<u32x4*>(As + off);
            float v[8], zv[8];
            unpack8(*pa, v);
            unpack8(*reinterpret_cast<const u32x4*>(As + A_BYTES + B_BYTES + off), zv);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[e] = __builtin_fmaf(k0a[e], v[e], __builtin_fmaf(k1a[e], zv[e], k2a[e]));
              v[e + 4] = __builtin_fmaf(k0b[e], v[e + 4], __builtin_fmaf(k1b[e], zv[e + 4], k2b[e]));
            }
            *pa = pack8(v);
          }
        }
      }
      if constexpr (PB == 1) {
        constexpr int CH = BN / 8, RS = 256 / CH;
        const int cq = tid % CH, r0 = tid / CH;
        const int col = n0 + 8 * cq;
        if (col < a.TC) {
          const int t = (int)fdiv((uint32_t)col, a.fdC);
          const int cch = col - t * a.C;
          const int tr = (int)fdiv((uint32_t)t, a.fdS);
          const int dh = tr - a.pad_h, dw = (t - tr * a.S) - a.pad_w;
          const f32x4 s0 = *reinterpret_cast<const f32x4*>(a.pscale + cch);
          const f32x4 s1 = *reinterpret_cast<const f32x4*>(a.pscale + cch + 4);
          const f32x4 h0 = *reinterpret_cast<const f32x4*>(a.pshift + cch);
          const f32x4 h1 = *reinterpret_cast<const f32x4*>(a.pshift + cch + 4);
          char* Bs = As + A_BYTES;
#pragma unroll
          for (int r = r0; r < BK; r += RS) {
            const int pix = pix0 + r;
            if (pix >= pend) break;
            if constexpr (!DIRECT) {   // out-of-image taps were staged as zeros: leave them
              const uint32_t n_img = fdiv((uint32_t)pix, a.fdPQ);
              const uint32_t rem = (uint32_t)pix - n_img * (uint32_t)(a.P * a.Q);
              const uint32_t p = fdiv(rem, a.fdQ);
              const uint32_t q = rem - p * a.Q;
              const int ih = (int)p * a.stride_h + dh, iw = (int)q * a.stride_w + dw;
              if ((unsigned)ih >= (unsigned)a.H || (unsigned)iw >= (unsigned)a.W) continue;
            }
            u32x4* pb = reinterpret_cast<u32x4*>(Bs + tr_off<B_ROW>(r, cq));
            float v[8];
            unpack8(*pb, v);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[e] = fmaxf(__builtin_fmaf(v[e], s0[e], h0[e]), 0.f);
              v[e + 4] = fmaxf(__builtin_fmaf(v[e + 4], s1[e], h1[e]), 0.f);
            }
            *pb = pack8(v);
          }
        }
      }
      __syncthreads();
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int mi = 0; mi < TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    issue(0, pbeg);
    __syncthreads();
    prologue(0, pbeg);
  }
  for (int ks = 0; ks < nk; ++ks) {
    if (ks > 0) {
      issue(0, pbeg + ks * BK);
      __syncthreads();
      prologue(0, pbeg + ks * BK);
    }
    const char* As = smem;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) af[mi] = tr_frag<A_ROW>(As, kk * 32, (wm * WM) / 16 + mi, lane);
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) bfr[ni] = tr_frag<B_ROW>(Bs, kk * 32, (wn * WN) / 16 + ni, lane);
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
    }
    __syncthreads();
  }

  // D[row = ko][col = tc]: lane holds col (lane&15), rows 4*(lane>>4) + r.
  const int fr = lane & 15, fg = lane >> 4;
  float* wsz = a.ws + (int64_t)z * a.Ko * a.TC;
#pragma unroll
  for (int mi = 0; mi < TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) {
      const int cc = n0 + wn * WN + ni * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ko = m0 + wm * WM + mi * 16 + fg * 4 + r;
        if (ko < a.Ko && cc < a.TC) wsz[(int64_t)ko * a.TC + cc] = acc[mi][ni][r];
      }
    }
}

// fp32 precision path: the same weight gradient with v_mfma_f32_16x16x4_f32.  Tile 64 (Ko) x 64
// (R*S*C columns) x 32 pixels per K-step, 4 waves of 32 x 32; operands staged through registers
// into pixel-major LDS rows padded to 80 floats, so the 4-byte fragment reads of the four lane
// groups (4 consecutive pixel rows) fall on disjoint banks.  Split over pixels into fp32 slabs,
// reduced by wgrad_reduce_stage1/2 like the bf16 path.
template <bool DIRECT>
__global__ __launch_bounds__(256) void conv_wgrad_f32_kernel(const WgradArgs a) {
  constexpr int BM = 64, BN = 64, BK = 32, LDR = 80;
  __shared__ __attribute__((aligned(16))) float As[BK * LDR], Bs[BK * LDR];
  const uint32_t ntile = (uint32_t)a.mtiles * a.ntiles;
  const uint32_t bid = xcd_remap(blockIdx.x, ntile * a.splits);
  const int z = bid / ntile;
  const int tile = bid - z * ntile;
  const int mt = tile / a.ntiles, nt = tile - mt * a.ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int pbeg = z * a.pix_per_split;
  const int pend = min(a.npix, pbeg + a.pix_per_split);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int fr = lane & 15, fg = lane >> 4;
  const float* dyb = static_cast<const float*>(a.dy) + a.dyoff;
  const float* xb = static_cast<const float*>(a.x) + a.xoff;
  const int PQ = a.P * a.Q;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int p0 = pbeg; p0 < pend; p0 += BK) {
    // 2 x 16-B chunks of A and of B per thread: chunk c -> row c / 16, columns 4 (c % 16) .. +3
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = tid + 256 * h, row = c >> 4, col = (c & 15) * 4;
      const int pix = p0 + row;
      f32x4 va = f32x4{0.f, 0.f, 0.f, 0.f}, vb = f32x4{0.f, 0.f, 0.f, 0.f};
      if (pix < pend && m0 + col < a.Ko) va = *reinterpret_cast<const f32x4*>(dyb + (int64_t)pix * a.ldy + m0 + col);
      const int tc = n0 + col;
      if (pix < pend && tc < a.TC) {
        const int t = (int)fdiv((uint32_t)tc, a.fdC);
        const int cch = tc - t * a.C;
        if (DIRECT) {
          vb = *reinterpret_cast<const f32x4*>(xb + (int64_t)pix * a.ldx + cch);
        } else {
          const int tr = (int)fdiv((uint32_t)t, a.fdS);
          const int ts = t - tr * a.S;
          const uint32_t n_img = fdiv((uint32_t)pix, a.fdPQ);
          const uint32_t rem = (uint32_t)pix - n_img * PQ;
          const uint32_t pp = fdiv(rem, a.fdQ);
          const uint32_t qq = rem - pp * a.Q;
          const int ih = (int)pp * a.stride_h + tr - a.pad_h, iw = (int)qq * a.stride_w + ts - a.pad_w;
          if ((unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W)
            vb = *reinterpret_cast<const f32x4*>(xb + (((int64_t)n_img * a.H + ih) * a.W + iw) * a.ldx + cch);
        }
      }
      *reinterpret_cast<f32x4*>(As + row * LDR + col) = va;
      *reinterpret_cast<f32x4*>(Bs + row * LDR + col) = vb;
    }
    __syncthreads();
#pragma unroll
    for (int k0 = 0; k0 < BK; k0 += 4) {
      float af[2], bfv[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = As[(k0 + fg) * LDR + wm * 32 + i * 16 + fr];
#pragma unroll
      for (int j = 0; j < 2; ++j) bfv[j] = Bs[(k0 + fg) * LDR + wn * 32 + j * 16 + fr];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfv[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  // D[row = ko][col = tc]: lane holds col (lane & 15), rows 4 (lane >> 4) + r
  float* wsz = a.ws + (int64_t)z * a.Ko * a.TC;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int cc = n0 + wn * 32 + j * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ko = m0 + wm * 32 + i * 16 + fg * 4 + r;
        if (ko < a.Ko && cc < a.TC) wsz[(int64_t)ko * a.TC + cc] = acc[i][j][r];
      }
    }
}

// Split reduction, stage 1: grid (ceil(total/1024), G): block (x, g) sums split slabs
// [g*per, (g+1)*per) for 1024 consecutive outputs (4 per thread, 16-byte loads) -> ws2[g][idx].
__global__ __launch_bounds__(256) void wgrad_reduce_stage1(const float* __restrict__ ws, int splits, int64_t total,
                                                           float* __restrict__ ws2) {
  const int G = gridDim.y, g = blockIdx.y;
  const int per = (splits + G - 1) / G;
  const int z0 = g * per, z1 = min(splits, z0 + per);
  const int64_t i4 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) * 4;
  if (i4 >= total) return;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
  for (int z = z0; z < z1; ++z) s += *reinterpret_cast<const f32x4*>(ws + (int64_t)z * total + i4);
  *reinterpret_cast<f32x4*>(ws2 + (int64_t)g * total + i4) = s;
}

// Stage 2: out[ko][t][c] += sum_g src[g][ko][t][c] for c < Creal, ko < Ko_real (fixed order).
__global__ __launch_bounds__(256) void wgrad_reduce_stage2(const float* __restrict__ src, int G, int Ko, int T,
                                                           int Cpad, int Creal, int Ko_real, float* __restrict__ out) {
  const int64_t TC = (int64_t)T * Cpad;
  const int64_t total = (int64_t)Ko_real * TC;
  const int64_t gstride = (int64_t)Ko * TC;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t ko = idx / TC;
    const int64_t rem = idx - ko * TC;
    const int64_t tt = rem / Cpad;
    const int c = (int)(rem - tt * Cpad);
    if (c >= Creal) continue;
    float s = 0.f;
#pragma unroll 8
    for (int g = 0; g < G; ++g) s += src[g * gstride + idx];
    out[(ko * T + tt) * Creal + c] += s;
  }
}

// Stage-1 groups: 0 (no stage 1: stage 2 sums the splits itself) when the tensor alone gives stage 2
// >= 1024 blocks of parallelism (>= 256k floats: every ResNet-50 layer-3/4 weight) -- one launch and
// one slab round trip less; else enough groups for >= 1024 stage-1 blocks.
static inline int reduce_groups(int splits, int64_t total) {
  if (total >= (int64_t)1024 * 256) return 0;
  const int64_t xb = (total / 4 + 255) / 256;
  int64_t G = (1024 + xb - 1) / xb;   // aim at >= 1024 blocks in stage 1
  if (G > splits) G = splits;
  if (G > 64) G = 64;
  return (int)(G < 1 ? 1 : G);
}

// Batched split reduction (up to kWgradBatch weight gradients that became ready together; ops.cpp
// queues and flushes them): stage 1 -- a block per (entry with G > 0, 1024-float chunk, group g)
// writes the group sum to ws2[g]; stage 2 -- a block per (entry, chunk) sums the G group sums (or,
// G == 0, the splits themselves) in order and accumulates into the gradient.  The same sums in the
// same order as dlmpi_wgrad_reduce's two launches per gradient: bit-identical.  (A single launch with
// a last-arriver ticket per chunk was measured 5x slower: every block's agent-scope release / acquire
// fence writes back / invalidates its XCD's L2 -- and the L2 of the data-gradient kernel running
// beside it.)
__device__ __forceinline__ void reduce_store4(const WgradReduceEntry& e, int64_t i4, f32x4 v) {
  const int64_t TC = (int64_t)e.T * e.Cpad;
  const int64_t ko = i4 / TC;
  if (ko >= e.Ko_real) return;
  const int64_t rem = i4 - ko * TC;
  const int64_t tt = rem / e.Cpad;   // Cpad % 8 == 0: the 4 outputs share (ko, tt)
  const int c = (int)(rem - tt * e.Cpad);
  float* o = e.out + (ko * e.T + tt) * e.Creal;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (c + k < e.Creal) o[c + k] += v[k];
}

__global__ __launch_bounds__(256) void wgrad_reduce_batch_s1(const WgradReduceBatch b) {
  int k = 0;
  while (k + 1 < b.n && (int)blockIdx.x >= b.e[k + 1].block1) ++k;
  const WgradReduceEntry& e = b.e[k];
  const int local = (int)blockIdx.x - e.block1;
  const int G = e.G, g = local % G, chunk = local / G;
  const int per = (e.splits + G - 1) / G;
  const int z0 = g * per, z1 = min(e.splits, z0 + per);
  const int64_t i4 = ((int64_t)chunk * 256 + threadIdx.x) * 4;
  if (i4 >= e.total) return;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
  for (int z = z0; z < z1; ++z) s += *reinterpret_cast<const f32x4*>(e.ws + (int64_t)z * e.total + i4);
  *reinterpret_cast<f32x4*>(e.ws2 + (int64_t)g * e.total + i4) = s;
}

__global__ __launch_bounds__(256) void wgrad_reduce_batch_s2(const WgradReduceBatch b) {
  int k = 0;
  while (k + 1 < b.n && (int)blockIdx.x >= b.e[k + 1].block2) ++k;
  const WgradReduceEntry& e = b.e[k];
  const int64_t i4 = ((int64_t)((int)blockIdx.x - e.block2) * 256 + threadIdx.x) * 4;
  if (i4 >= e.total) return;
  const float* src = e.G > 0 ? e.ws2 : e.ws;
  const int n = e.G > 0 ? e.G : e.splits;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
  for (int z = 0; z < n; ++z) s += *reinterpret_cast<const f32x4*>(src + (int64_t)z * e.total + i4);
  reduce_store4(e, i4, s);
}

}  // namespace dlmpi

using namespace dlmpi;

// Prologue combinations built: either operand deferred for 1x1 (direct) gradients -- the dual data
// gradient's dz (PA 2), the UNet head's deferred BN-apply input (PB 1) --, the dy prologue for
// gathers; not both at once.  (The gather PB 1 forms spilled 5 VGPRs at 128 x 128 and had no caller:
// the backend stores such an operand first, ops/backend.py conv_wgrad.)
template <int BM, int BN, int WR>
static hipError_t launch_wg(const WgradArgs* a, dim3 g, hipStream_t s) {
  const bool d = a->direct != 0;
  const int m = (a->pro_a ? 2 : 0) | (a->pro_b ? 1 : 0);
#define WG(D_, PA_, PB_) hipLaunchKernelGGL((conv_wgrad_kernel<BM, BN, D_, PA_, PB_, WR>), g, dim3(256), 0, s, *a)
  if (d) {
    if (m == 0) WG(true, 0, 0);
    else if (m == 2) WG(true, 2, 0);
    else if (m == 1) WG(true, 0, 1);
    else return hipErrorInvalidValue;
  } else {
    if (m == 0) WG(false, 0, 0);
    else if (m == 2) WG(false, 2, 0);
    else return hipErrorInvalidValue;
  }
#undef WG
  return hipGetLastError();
}
// the prologue combination launch_wg builds for this gradient
extern "C" int dlmpi_wgrad_pro_ok(int direct, int pro_a, int pro_b) {
  return !(pro_a && pro_b) && (direct || !pro_b);
}

static int g_wgrad_fast = 1;
extern "C" void dlmpi_set_wgrad_fast(int on) { g_wgrad_fast = on; }

extern "C" hipError_t dlmpi_conv_wgrad(const WgradArgs* a0, int bm, int bn, hipStream_t s) {
  WgradArgs args = *a0;
  args.fast = g_wgrad_fast;
  const WgradArgs* a = &args;
  const unsigned nwg = (unsigned)(a->mtiles * a->ntiles * a->splits);
  if (nwg == 0) return hipSuccess;
  const dim3 g(nwg), b(256);
  if (a->f32) {
    if (bm != 64 || bn != 64 || a->ws == nullptr || a->pro_a || a->pro_b) return hipErrorInvalidValue;
    if (a->direct) hipLaunchKernelGGL(conv_wgrad_f32_kernel<true>, g, b, 0, s, *a);
    else hipLaunchKernelGGL(conv_wgrad_f32_kernel<false>, g, b, 0, s, *a);
    return hipGetLastError();
  }
  if ((a->pro_a != 0 && a->pro_a != 2) || (a->pro_b != 0 && a->pro_b != 1)) return hipErrorInvalidValue;
  // 64 x 256, 1 x 4 waves (Ko <= 64 layers)
  if (bm == 64 && bn == 256) {
    if (a->pro_b != 0) return hipErrorInvalidValue;
    return launch_wg<64, 256, 1>(a, g, s);
  }
  // (a 128 x 256 variant was measured 1.3-1.9x slower: 2 waves/SIMD and register spills)
  if (bn != 128 || (bm != 128 && bm != 64)) return hipErrorInvalidValue;
  if (bm == 128) return launch_wg<128, 128, 2>(a, g, s);
  return launch_wg<64, 128, 2>(a, g, s);
}

extern "C" int dlmpi_wgrad_reduce_groups(int splits, int64_t total) { return reduce_groups(splits, total); }

// ws2 must hold reduce_groups(splits, Ko*T*Cpad) * Ko*T*Cpad floats (total % 4 == 0 since Cpad % 8 == 0).
extern "C" hipError_t dlmpi_wgrad_reduce(const float* ws, int splits, int Ko, int T, int Cpad, int Creal, int Ko_real,
                                         float* out, float* ws2, int ws2_floats, hipStream_t s) {
  const int64_t total = (int64_t)Ko * T * Cpad;
  if (total == 0 || Ko_real == 0) return hipSuccess;
  const int G = reduce_groups(splits, total);
  const float* src = ws;
  int Gs = splits;
  if (splits > 1 && G > 0) {
    if ((int64_t)G * total > (int64_t)ws2_floats) return hipErrorInvalidValue;
    hipLaunchKernelGGL(wgrad_reduce_stage1, dim3((unsigned)((total / 4 + 255) / 256), G), dim3(256), 0, s, ws, splits,
                       total, ws2);
    src = ws2;
    Gs = G;
  }
  int64_t blocks = ((int64_t)Ko_real * T * Cpad + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(wgrad_reduce_stage2, dim3((unsigned)blocks), dim3(256), 0, s, src, Gs, Ko, T, Cpad, Creal, Ko_real,
                     out);
  return hipGetLastError();
}

extern "C" hipError_t dlmpi_wgrad_reduce_batch(WgradReduceBatch* b, hipStream_t s) {
  if (b->n <= 0) return hipSuccess;
  if (b->n > kWgradBatch) return hipErrorInvalidValue;
  int64_t blocks1 = 0, blocks2 = 0;
  for (int i = 0; i < b->n; ++i) {
    WgradReduceEntry& e = b->e[i];
    if (e.total % 4 != 0 || e.Cpad % 8 != 0) return hipErrorInvalidValue;
    e.G = e.splits > 1 ? reduce_groups(e.splits, e.total) : 0;
    if (e.G > 0 && e.ws2 == nullptr) return hipErrorInvalidValue;
    const int64_t chunks = (e.total + 1023) / 1024;
    e.block1 = (int)blocks1;
    e.block2 = (int)blocks2;
    if (e.G > 0) blocks1 += chunks * e.G;
    blocks2 += chunks;
  }
  if (blocks1 > INT32_MAX || blocks2 > INT32_MAX) return hipErrorInvalidValue;
  // entries without a stage 1 get block1 = the next entry's start (the lookup skips them)
  if (blocks1 > 0) hipLaunchKernelGGL(wgrad_reduce_batch_s1, dim3((unsigned)blocks1), dim3(256), 0, s, *b);
  if (blocks2 > 0) hipLaunchKernelGGL(wgrad_reduce_batch_s2, dim3((unsigned)blocks2), dim3(256), 0, s, *b);
  return hipGetLastError();
}
