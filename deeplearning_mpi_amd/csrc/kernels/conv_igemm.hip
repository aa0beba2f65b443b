// Implicit-GEMM convolution on CDNA4 MFMA (v_mfma_f32_16x16x32_bf16), NHWC bf16, fp32 accumulate.
//
// One GEMM formulation serves every "gather-A" GEMM of the framework:
//   * Conv2d forward (any R x S, stride, pad; ResNet stem 7x7/s2, 3x3, 1x1, UNet 3x3),
//   * Conv2d data-gradient (stride^2 sub-pixel phases, each a dense conv with its own tap list,
//     so a stride-2 3x3 dgrad does no zero MACs),
//   * ConvTranspose2d(k=2, s=2) forward (4 phases of a 1x1 GEMM written to strided pixels),
//   * Linear (a 1x1 conv on a 1x1 image).
// Replaces what the reference gets implicitly from cuDNN conv fwd/dgrad and cuBLAS
// (call sites /root/reference/pytorch/unet/model.py:9-14, resnet main.py:40-41).
//
// Two kernels share the staging scheme and the epilogue:
//
// conv_igemm_kernel -- 4 waves, single LDS stage, two barriers per K-step, 3-4 blocks per CU
//   (latency hidden across blocks).  Every operand class: small channel counts (stem, UNet input),
//   operand prologues (deferred BN-apply), 2-D halo tiles, split-K for small grids, fp32 storage.
//   Best on the short / memory-bound GEMMs, where a block's whole life is a few K-steps.
//
// conv_pipe_kernel -- 8 waves, one block per CU, an LDS ring of STAGES K-steps with STAGES - 1 in
//   flight and ONE barrier per K-step: the LDS-DMA of step k + STAGES - 1 is issued right after the
//   barrier of step k and retired by a counted `s_waitcnt vmcnt` just before the barrier of the step
//   that reads it, so the loads stay in flight across barriers while the MFMAs of the intermediate
//   steps run (cdna_hip_programming.md §5 "Pipelining across barriers").  Per-wave 128 x 64 / 64 x 64
//   output tiles (LDS read traffic per MFMA 25-50 % below the 4-wave 64 x 64 kernel).  For the
//   compute-bound long reductions (3x3 convs from 64 channels, 1x1 from 1024).
//
// Staging (both): global -> LDS directly with global_load_lds_dwordx4 (no VGPR round trip, no
// ds_write): each wave instruction fills 8 LDS rows of 128 B lane-linearly; the XOR swizzle that
// makes the ds_read_b128 fragment reads bank-conflict-free is applied on the per-lane SOURCE address
// (cdna_hip_programming.md §5.4 rule 21): chunk ch of row r sits at slot ch ^ (r & 7).  That is
// conflict-free for 16 consecutive rows starting at ANY row (benchmarks/lds_banks.py), which the
// halo tiles need -- their fragment rows start at a tap-dependent halo offset; the former
// ch ^ ((r >> 1) & 7) was 2-way conflicted at 3 of every 4 offsets (halo: SQ_LDS_BANK_CONFLICT 92 % of
// the LDS-active cycles, profiles/r4_lab).  Out-of-image im2col pieces read a zero page.  Channel
// counts >= 64: the tap (r, s) and channel base are wave-uniform scalars and the per-row source
// pointers are rebuilt only when the tap changes.  All LDS is ONE __shared__ array: with a second
// LDS object hipcc tracks the DMA targets and waits for every in-flight DMA before each fragment read.
// Epilogue: the fp32 tile is staged through LDS for 16-byte stores with fused bias / residual
// add / folded-BN affine / ReLU and the per-channel BatchNorm partial sums of the stored
// (bf16-rounded) values.
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace dlmpi {

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void glds16(const void* g, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, (lds_void*)lds_wave_base, 16, 0, 0);
}

// LDS bytes the epilogue needs: fp32 tile staging in NP passes of <= 64 rows, or the statistics combine
template <int BM, int BN, int NT, int WM>
struct EpiSmem {
  static constexpr int NP0 = BM < 128 ? 1 : (BM / 64 < WM / 16 ? BM / 64 : WM / 16);
  // a pass must take the same number of fragment rows from every wave (7-fragment waves: 7 passes)
  static constexpr int NP = (WM / 16) % NP0 == 0 ? NP0 : WM / 16;
  static constexpr int CS_LD = BN + 4;
  static constexpr int EPI = (BM / NP) * CS_LD * 4;
  static constexpr int RED = (NT / (BN / 8)) * 3 * BN * 4;
  static constexpr int bytes = EPI > RED ? EPI : RED;
};

// ---- split-K combine (cdna_hip_programming.md "In-launch split-K reduction") ---------------------
// Every slice stores its fp32 accumulators (fragment layout) to its slab, publishes with an
// agent-scope release + ticket; the tile's last arriver acquires and sums ALL slices' slabs in
// slice order (deterministic whichever block arrives last), then runs the normal epilogue.
// Returns false in the blocks that are not the last arriver (they exit).
template <int NT, int NF>
__device__ __forceinline__ bool splitk_combine(const ConvArgs& a, f32x4* acc, char* smem, int tid, int mt, int nt) {
  const int S = a.splitk;
  // unique over phases (blockIdx.z): ConvTranspose phases all have tile_base 0
  const int64_t tile = (int64_t)blockIdx.z * gridDim.x + (int64_t)mt * a.ntiles + nt;
  f32x4* slab = reinterpret_cast<f32x4*>(a.sk_slab) + (tile * S + blockIdx.y) * NF * NT + tid;
#pragma unroll
  for (int i = 0; i < NF; ++i) slab[(int64_t)i * NT] = acc[i];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = reinterpret_cast<int*>(smem);   // the one LDS array (no second __shared__ object)
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    flag[0] = __hip_atomic_fetch_add(a.sk_tk + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == S - 1;
  }
  __syncthreads();
  if (!flag[0]) return false;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(a.sk_tk + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const f32x4* base = reinterpret_cast<const f32x4*>(a.sk_slab) + tile * S * NF * NT + tid;
#pragma unroll
  for (int i = 0; i < NF; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int sp = 0; sp < S; ++sp)
#pragma unroll
    for (int i = 0; i < NF; ++i) acc[i] += base[((int64_t)sp * NF + i) * NT];
  __syncthreads();   // flag (LDS) is reused by the epilogue staging
  return true;
}

// ---- epilogue ------------------------------------------------------------------------------------
// acc: this wave's (BM/WGM) x (BN/WGN) output fragments (wave (wm, wn) of a WGM x WGN grid).  The
// tile is dumped to LDS in NP passes of BM/NP rows; every thread then owns 8 channels of a row:
// bias -> BN statistics (forward) -> folded-BN affine -> residual -> ReLU -> backward mask and
// BN-backward statistics -> 16-byte store.  Per-channel partial sums are combined over the row
// groups in LDS and written as one stats row per M-tile.
template <int BM, int BN, int NT, int WGM, int WGN, typename T, bool HALO>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, const ConvPhase& ph,
                                              f32x4 (&acc)[BM / WGM / 16][BN / WGN / 16], char* smem, int tid,
                                              int m0, int n0, int mt, int hn, int hh0, int hw0) {
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int NP = EpiSmem<BM, BN, NT, WM>::NP;
  constexpr int CS_LD = EpiSmem<BM, BN, NT, WM>::CS_LD;
  static_assert(WM % (16 * NP) == 0 || NP == 1, "epilogue pass must split every wave's rows evenly");
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WGN, wn = wid % WGN;
  const int fr = lane & 15, fg = lane >> 4;
  const int PQ = ph.P * ph.Q;
  const int M = a.Nimg * PQ;
  float* Cs = reinterpret_cast<float*>(smem);

  constexpr int CG = BN / 8;       // channel groups of 8
  constexpr int RG = NT / CG;      // row groups
  const int cg = tid % CG, rg = tid / CG;
  const int c0 = n0 + cg * 8;
  const bool cvalid = c0 < a.Kout;
  float bias[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bias[e] = 0.f;
  if (cvalid && a.bias) {
#pragma unroll
    for (int e = 0; e < 8; ++e) bias[e] = a.bias[c0 + e];
  }
  float s1[8], s2[8], s3[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; s3[e] = 0.f; }
  // gradient of a BN+ReLU output: mask, then {sum dy, sum dy*z}
  const bool bwd = a.mask != nullptr || a.mscale != nullptr || a.mbits != nullptr;

  // NP passes over row slices: in pass h every wave dumps its fragments mi in
  // [h*TM/NP, (h+1)*TM/NP), i.e. tile rows wm*WM + h*HM + [0, HM), into a BM/NP-row buffer.
  constexpr int HM = WM / NP, HT = TM / NP;
#pragma unroll
  for (int h = 0; h < NP; ++h) {
  if (h) __syncthreads();         // every thread is done with pass h - 1
#pragma unroll
  for (int mi = 0; mi < HT; ++mi)
#pragma unroll
    for (int ni = 0; ni < TN; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Cs[(wm * HM + mi * 16 + fg * 4 + r) * CS_LD + wn * WN + ni * 16 + fr] = acc[h * HT + mi][ni][r];
  __syncthreads();
  constexpr int EPI_UNROLL = BM >= 256 ? 1 : 2;   // two rows' loads in flight (memory-bound epilogues)
#pragma unroll EPI_UNROLL
  for (int rr = rg; rr < BM / NP; rr += RG) {
    const int r = (rr / HM) * WM + h * HM + (rr % HM);
    const int m = m0 + r;
    int64_t pix;
    if constexpr (HALO) {
      const int pr = (int)fdiv((uint32_t)r, a.fd_tw), pc = r - pr * a.tw;
      const int oh = hh0 + pr, ow = hw0 + pc;
      if (r >= a.th * a.tw || oh >= ph.P || ow >= ph.Q || !cvalid) continue;
      pix = ((int64_t)hn * a.OH + oh * a.so + ph.oh0) * a.OW + ow * a.so + ph.ow0;
    } else {
      if (m >= M || !cvalid) continue;
    }
    float v[8];
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(Cs + rr * CS_LD + cg * 8);
    const f32x4 v1 = *reinterpret_cast<const f32x4*>(Cs + rr * CS_LD + cg * 8 + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) { v[e] = v0[e] + bias[e]; v[e + 4] = v1[e] + bias[e + 4]; }
    if (a.stats && !bwd) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float rv = stored<T>(v[e]);
        s1[e] += rv;
        s2[e] += rv * rv;
      }
    }
    if (a.scale) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = v[e] * a.scale[c0 + e] + a.shift[c0 + e];
    }
    if constexpr (!HALO) {
      const uint32_t n_img = fdiv((uint32_t)m, ph.fdPQ);
      const uint32_t rem = (uint32_t)m - n_img * PQ;
      const uint32_t p = fdiv(rem, ph.fdQ);
      const uint32_t q = rem - p * ph.Q;
      pix = ((int64_t)n_img * a.OH + (int)p * a.so + ph.oh0) * a.OW + (int)q * a.so + ph.ow0;
    }
    if (a.res) {
      float rr8[8];
      load8(static_cast<const T*>(a.res) + pix * a.ldres + a.resoff + c0, rr8);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += rr8[e];
    }
    if (a.relu) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    if (bwd) {
      float zz[8];
      if (a.z) load8(static_cast<const T*>(a.z) + pix * a.ldz + a.zoff + c0, zz);
      if (a.mbits) {
        const uint32_t b = a.mbits[pix * (a.Kout >> 3) + (c0 >> 3)];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (b >> e) & 1u ? v[e] : 0.f;
      } else if (a.mask) {
        float yy[8];
        load8(static_cast<const T*>(a.mask) + pix * a.ldmask + a.maskoff + c0, yy);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = yy[e] > 0.f ? v[e] : 0.f;
      } else {   // same fma as the forward BN-apply -> same sign as y
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = zz[e] * a.mscale[c0 + e] + a.mshift[c0 + e] > 0.f ? v[e] : 0.f;
      }
      if (a.stats) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float rv = stored<T>(v[e]);   // statistics of the stored gradient
          s1[e] += rv;
          s2[e] += rv * zz[e];
        }
        if (a.z2) {
          load8(static_cast<const T*>(a.z2) + pix * a.ldz2 + a.z2off + c0, zz);
#pragma unroll
          for (int e = 0; e < 8; ++e) s3[e] += stored<T>(v[e]) * zz[e];
        }
      }
    }
    if (a.vec_store) {
      if (a.out_f32) {
        float* yp = reinterpret_cast<float*>(a.y) + pix * a.ldy + a.yoff + c0;
        *reinterpret_cast<f32x4*>(yp) = f32x4{v[0], v[1], v[2], v[3]};
        *reinterpret_cast<f32x4*>(yp + 4) = f32x4{v[4], v[5], v[6], v[7]};
      } else {
        uint16_t* yp = reinterpret_cast<uint16_t*>(a.y) + pix * a.ldy + a.yoff + c0;
        *reinterpret_cast<u32x4*>(yp) = pack8(v);
      }
    } else {   // narrow / unaligned output (e.g. the 1-channel UNet head written as fp32 [N,1,H,W])
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (c0 + e >= a.kvalid) break;
        if (a.out_f32) reinterpret_cast<float*>(a.y)[pix * a.ldy + a.yoff + c0 + e] = v[e];
        else reinterpret_cast<uint16_t*>(a.y)[pix * a.ldy + a.yoff + c0 + e] = f2bf(v[e]);
      }
    }
  }
  }

  if (a.stats) {
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);
    const int ns = a.nstat;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(rg * 3 + 0) * BN + cg * 8 + e] = s1[e];
      red[(rg * 3 + 1) * BN + cg * 8 + e] = s2[e];
      red[(rg * 3 + 2) * BN + cg * 8 + e] = s3[e];
    }
    __syncthreads();
    if (tid < BN && n0 + tid < a.Kout) {
      float t1 = 0.f, t2 = 0.f, t3 = 0.f;
      for (int g = 0; g < RG; ++g) {
        t1 += red[(g * 3 + 0) * BN + tid];
        t2 += red[(g * 3 + 1) * BN + tid];
        t3 += red[(g * 3 + 2) * BN + tid];
      }
      float* st = a.stats + (int64_t)(ph.tile_base + mt) * ns * a.Kout + n0 + tid;
      st[0] = t1;
      st[a.Kout] = t2;
      if (ns > 2) st[2 * a.Kout] = t3;
    }
  }
}

// ---- the single-stage 4-wave kernel --------------------------------------------------------------
// Tile: BM (pixels) x BN (channels) x BK (reduction), 256 threads = 4 waves in WGM x (4 / WGM), each
// wave (BM/WGM) x (BN/WGN) as 16x16 MFMA tiles.  The stage is issued, drained (vmcnt(0) +
// barrier), read, and released by a second barrier: occupancy (3-4 blocks per CU) hides latency.
// WGM = 4: the 256 x 64 tile of 64-channel layers (per-wave 64 x 64 instead of 64 x 32: a third
// less LDS traffic per MFMA).
// T: storage type of activations and weights -- uint16_t (bf16, v_mfma_f32_16x16x32_bf16) or float
// (the fp32 precision path: v_mfma_f32_16x16x4_f32, four per 16-byte fragment; the LDS tile keeps
// its 128-byte rows, i.e. 32 fp32 reduction elements per K-step instead of 64 bf16).
// HALO: 3x3 / stride-1 / pad-1 convolutions (forward and stride-1 data gradient) by 2-D output tiles
// of th x tw pixels (th * tw <= 128 = BM) of one image: the (th + 2) x (tw + 2) input halo of a
// 64-channel chunk is staged ONCE and the 9 taps are 9 K-steps over it (only the weight tile is
// staged per tap) -- the K order is chunk-major, tap-minor.  An out-of-image halo pixel is staged as
// zeros, which is the zero padding of every tap; no per-tap im2col decode exists.
template <int BM, int BN, bool SMALLC, int WGM, int PRO = 0, typename ET = uint16_t, bool HALO = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BM * BN <= 16384 ? 3 : 2, 8))) void conv_igemm_kernel(const ConvArgs a) {
  constexpr int NW = 4;
  constexpr int NT = 64 * NW;                 // threads
  constexpr int WGN = NW / WGM;               // wave grid WGM x WGN
  using T = ET;                               // element (storage) type
  constexpr int ES = sizeof(T);               // bytes per element
  constexpr int BK = 128 / ES;                // reduction elements per K-step (one 128-B LDS row)
  constexpr int CPC = 16 / ES;                // channels per 16-byte chunk
  static_assert(PRO == 0 || (PRO == 3 && ES == 2), "operand prologue: mode 3, bf16");
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int RP = NT / 8;                  // tile rows staged per pass (8 lanes per 128-B row)
  constexpr int AL = BM / RP, BL = BN / RP;   // 16-byte pieces per thread per tile
  // (th + 2) * (tw + 2) <= HALO_ROWS (host-checked): 128-pixel tiles (8 x 16 -> 10 x 18 = 180 rows),
  // 256-pixel tiles (16 x 16 -> 18 x 18 = 324 rows)
  constexpr int HALO_ROWS = BM == 256 ? 352 : 192;
  static_assert(!HALO || ((BM == 128 || BM == 256) && !SMALLC && PRO == 0 && sizeof(ET) == 2),
                "halo mode: 128- or 256-pixel bf16 tiles");
  constexpr int HL = HALO ? HALO_ROWS * 128 / (16 * 64 * NW) : 1;   // halo pieces per thread
  constexpr int A_BYTES = (HALO ? HALO_ROWS : BM) * 128, B_BYTES = BN * 128;
  static_assert(PRO == 0 || !SMALLC, "operand prologue: regular channels");
  constexpr int Z_BYTES = PRO == 3 ? A_BYTES : 0;   // the prologue's residual operand, staged like A
  constexpr int SB = A_BYTES + B_BYTES + Z_BYTES;   // bytes of the stage: [A | B | Z]
  constexpr int EPI_NEED = EpiSmem<BM, BN, NT, WM>::bytes;
  constexpr int SMEM = SB > EPI_NEED ? SB : EPI_NEED;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WGN, wn = wid % WGN;
  const int lrow = tid >> 3;                          // staging row (+RP i)
  const int jc = (tid & 7) ^ ((tid >> 3) & 7);        // swizzled 16-B chunk this lane fetches (row & 7)
  const char* zp = reinterpret_cast<const char*>(g_zero_page);

  const int zph = blockIdx.z;
  const uint32_t nwg0 = (uint32_t)a.ph[zph].mtiles * (uint32_t)a.ntiles;
  if (blockIdx.x >= nwg0) return;
  const uint32_t bid = xcd_remap(blockIdx.x, nwg0);
  const ConvPhase ph = a.ph[zph];
  const int mt = bid / a.ntiles, nt = bid - mt * a.ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  int hn = 0, hh0 = 0, hw0 = 0;                       // HALO: image and tile origin of this M-tile
  if constexpr (HALO) {
    hn = (int)fdiv((uint32_t)mt, a.fd_thw);
    const int rem = mt - hn * a.tiles_h * a.tiles_w;
    const int ti = (int)fdiv((uint32_t)rem, a.fd_tilesw);
    hh0 = ti * a.th;
    hw0 = (rem - ti * a.tiles_w) * a.tw;
  }
  const int PQ = ph.P * ph.Q;
  const int M = a.Nimg * PQ;

  // ---- per-thread row state (kept compact: the 256-row tile has 4 rows per thread) ----------
  int a_hw[AL], a_pix[AL];                            // (h << 16) | w of the row's input origin
  uint32_t a_okm = 0;                                 // bit i: GEMM row valid
#pragma unroll
  for (int i = 0; i < AL; ++i) {
    const int m = m0 + lrow + RP * i;
    if (m < M) a_okm |= 1u << i;
    const uint32_t mm = m < M ? (uint32_t)m : 0u;
    const uint32_t n_img = fdiv(mm, ph.fdPQ);
    const uint32_t rem = mm - n_img * PQ;
    const uint32_t p = fdiv(rem, ph.fdQ);
    const uint32_t q = rem - p * ph.Q;
    const int h = (int)p * a.sa, w = (int)q * a.sa;
    a_hw[i] = (h << 16) | w;
    a_pix[i] = ((int)n_img * a.H + h) * a.W + w;
  }
  const char* xlane = reinterpret_cast<const char*>(a.x) + ES * ((int64_t)a.xoff + CPC * jc);
  // B rows n0 + lrow + RP i: one base pointer + validity bits
  const char* b_base = reinterpret_cast<const char*>(a.w) + ES * ((int64_t)(n0 + lrow) * a.ldw + CPC * jc);
  const int64_t b_step = (int64_t)ES * RP * a.ldw;     // bytes between rows RP apart
  uint32_t b_okm = 0;
#pragma unroll
  for (int i = 0; i < BL; ++i)
    if (n0 + lrow + RP * i < a.Kout) b_okm |= 1u << i;

  const int C = a.C;
  const int NTAP = ph.Tr * ph.Ts;
  const int nk = ph.ksteps;
  const int ldx2 = a.ldx * ES;

  // ---- staging ------------------------------------------------------------------------------
  // Regular path (C % 64 == 0): the tap t and channel base c are wave-uniform.
  uint32_t a_off[AL];                                 // element offset of the row's input pixel
  uint32_t z_off[PRO == 3 ? AL : 1];                  // the same pixel in the prologue's Z
  uint32_t a_vm = 0;                                  // bit i: (row, tap) inside the image
  int t_cur = 0, c_cur = 0, wtC2 = 0;
  auto tap_setup = [&](int t) {
    const int tr = (int)fdiv((uint32_t)t, ph.fdTs);
    const int ts = t - tr * ph.Ts;
    const int dh = ph.dh0 + tr * ph.dhs, dw = ph.dw0 + ts * ph.dws;
    const int wt = (ph.wr0 + tr * ph.wrs) * a.S + (ph.ws0 + ts * ph.wss);
    wtC2 = wt * C * ES;
    const int doff = dh * a.W + dw;
    a_vm = 0;
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      const int ih = (a_hw[i] >> 16) + dh, iw = (a_hw[i] & 0xffff) + dw;
      const bool ok = ((a_okm >> i) & 1) && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      if (ok) a_vm |= 1u << i;
      a_off[i] = (uint32_t)(a_pix[i] + doff) * (uint32_t)a.ldx;
      if constexpr (PRO == 3) z_off[i] = (uint32_t)(a_pix[i] + doff) * (uint32_t)a.ldpz;
    }
  };
  const char* zlane = PRO == 3 ? reinterpret_cast<const char*>(a.pz) + ES * ((int64_t)a.pzoff + CPC * jc) : nullptr;

  // HALO staging: piece i of this lane = halo row lrow + RP i (chunk jc), i.e. halo pixel (line,
  // col) relative to the tile origin; rows past the halo read the zero page
  const int hwd = HALO ? a.tw + 2 : 1;                 // halo row length (pixels)
  int hl_dh[HL], hl_dw[HL];
  uint32_t hl_ok = 0;
  if constexpr (HALO) {
    const int nrows = (a.th + 2) * hwd;
#pragma unroll
    for (int i = 0; i < HL; ++i) {
      const int hr = lrow + RP * i;
      const int line = hr / hwd;
      hl_dh[i] = line - 1;
      hl_dw[i] = hr - line * hwd - 1;
      if (hr < nrows) hl_ok |= 1u << i;
    }
  }
  int toff = 0;                                        // HALO: halo-row offset of the current tap
  int ts_cur = 0;                                      // HALO: column of the current tap
  bool need_halo = true;
  auto tap_setup_halo = [&](int t) {
    const int tr = (int)fdiv((uint32_t)t, ph.fdTs);
    const int ts = t - tr * ph.Ts;
    const int dh = ph.dh0 + tr * ph.dhs, dw = ph.dw0 + ts * ph.dws;
    const int wt = (ph.wr0 + tr * ph.wrs) * a.S + (ph.ws0 + ts * ph.wss);
    wtC2 = wt * C * ES;
    toff = (dh + 1) * hwd + (dw + 1);
    ts_cur = ts;
  };

  auto issue = [&](int ks) {
    char* As = smem;
    char* Bs = As + A_BYTES;
    if constexpr (HALO) {
      if (need_halo) {
        const char* xb = reinterpret_cast<const char*>(a.x) + ES * ((int64_t)a.xoff + c_cur + CPC * jc);
#pragma unroll
        for (int i = 0; i < HL; ++i) {
          const int ih = hh0 + hl_dh[i], iw = hw0 + hl_dw[i];
          const bool ok = ((hl_ok >> i) & 1) && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
          const char* src = ok ? xb + (int64_t)ES * (((int64_t)hn * a.H + ih) * a.W + iw) * a.ldx : zp;
          glds16(src, As + (RP * i + 8 * wid) * 128);
        }
        need_halo = false;
      }
#pragma unroll
      for (int i = 0; i < BL; ++i) {
        const char* s = ((b_okm >> i) & 1) ? b_base + i * b_step + wtC2 + ES * c_cur : zp;
        glds16(s, Bs + (RP * i + 8 * wid) * 128);
      }
    } else if constexpr (!SMALLC) {
#pragma unroll
      for (int i = 0; i < AL; ++i) {
        const char* s = ((a_vm >> i) & 1) ? xlane + ES * ((uint64_t)a_off[i] + c_cur) : zp;
        glds16(s, As + (RP * i + 8 * wid) * 128);
      }
      if constexpr (PRO == 3) {
        char* Zs = Bs + B_BYTES;
#pragma unroll
        for (int i = 0; i < AL; ++i) {
          const char* s = ((a_vm >> i) & 1) ? zlane + ES * ((uint64_t)z_off[i] + c_cur) : zp;
          glds16(s, Zs + (RP * i + 8 * wid) * 128);
        }
      }
#pragma unroll
      for (int i = 0; i < BL; ++i) {
        const char* s = ((b_okm >> i) & 1) ? b_base + i * b_step + wtC2 + ES * c_cur : zp;
        glds16(s, Bs + (RP * i + 8 * wid) * 128);
      }
    } else {
      // small C (8/16/32; stem & first UNet layer): every 16-B piece is its own tap
      const int kk = ks * BK + CPC * jc;
      const int t = kk / C, c = kk - t * C;
      const bool tv = t < NTAP;
      const int tt = tv ? t : 0;
      const int tr = (int)fdiv((uint32_t)tt, ph.fdTs);
      const int ts = tt - tr * ph.Ts;
      const int dh = ph.dh0 + tr * ph.dhs, dw = ph.dw0 + ts * ph.dws;
      const int wt = (ph.wr0 + tr * ph.wrs) * a.S + (ph.ws0 + ts * ph.wss);
      const char* xs = reinterpret_cast<const char*>(a.x) + ES * ((int64_t)a.xoff + c);
#pragma unroll
      for (int i = 0; i < AL; ++i) {
        const int ih = (a_hw[i] >> 16) + dh, iw = (a_hw[i] & 0xffff) + dw;
        const bool ok = tv && ((a_okm >> i) & 1) && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        const char* s = ok ? xs + (int64_t)(a_pix[i] + dh * a.W + dw) * ldx2 : zp;
        glds16(s, As + (RP * i + 8 * wid) * 128);
      }
#pragma unroll
      for (int i = 0; i < BL; ++i) {
        const char* s = (tv && ((b_okm >> i) & 1)) ? b_base + i * b_step - 16 * jc + ES * (wt * C + c) : zp;
        glds16(s, Bs + (RP * i + 8 * wid) * 128);
      }
    }
  };

  // Operand prologue (PRO 3, 1x1 / stride-1 consumers): this lane's own staged A pieces (row
  // lrow + RP i, chunk jc = channels c_cur + 8 jc) are the producer block's BN input z; once the stage
  // has landed they are rewritten in place as y = relu(z * scale + shift + r) -- r the staged
  // residual Z, or Z * rscale + rshift for a BN-output residual -- with bn_apply_kernel's arithmetic
  // in the same order (bit-identical to the unfused schedule); the blocks of output tile column 0 also
  // store y and its ReLU mask bits.  Pieces of rows past M hold zeros and are left alone.
  auto prologue = [&]() {
    if constexpr (PRO == 3) {
      char* As = smem;
      const int c = c_cur + 8 * jc;
      const f32x4 k0a = *reinterpret_cast<const f32x4*>(a.pscale + c);
      const f32x4 k0b = *reinterpret_cast<const f32x4*>(a.pscale + c + 4);
      const f32x4 k1a = *reinterpret_cast<const f32x4*>(a.pshift + c);
      const f32x4 k1b = *reinterpret_cast<const f32x4*>(a.pshift + c + 4);
      f32x4 k2a, k2b, kra, krb;
      if (a.prscale) {
        k2a = *reinterpret_cast<const f32x4*>(a.prscale + c);
        k2b = *reinterpret_cast<const f32x4*>(a.prscale + c + 4);
        kra = *reinterpret_cast<const f32x4*>(a.prshift + c);
        krb = *reinterpret_cast<const f32x4*>(a.prshift + c + 4);
      }
#pragma unroll
      for (int i = 0; i < AL; ++i) {
        if (!((a_vm >> i) & 1)) continue;
        u32x4* pa = reinterpret_cast<u32x4*>(As + RP * i * 128 + tid * 16);
        float v[8], r[8];
        unpack8(*pa, v);
        unpack8(*reinterpret_cast<const u32x4*>(As + A_BYTES + B_BYTES + RP * i * 128 + tid * 16), r);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = __builtin_fmaf(v[e], k0a[e], k1a[e]);
          v[e + 4] = __builtin_fmaf(v[e + 4], k0b[e], k1b[e]);
        }
        if (a.prscale) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            r[e] = __builtin_fmaf(r[e], k2a[e], kra[e]);
            r[e + 4] = __builtin_fmaf(r[e + 4], k2b[e], krb[e]);
          }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e] + r[e], 0.f);
        const u32x4 pk = pack8(v);
        *pa = pk;
        if (nt == 0) {   // with several output tile columns every column's blocks rebuild y; one stores it
          const int64_t px = a_pix[i];   // 1x1 / stride 1 (host-checked): input pixel = tile row
          *reinterpret_cast<u32x4*>(a.py + px * a.ldpy + a.pyoff + c) = pk;
          uint32_t b = 0;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            b |= (uint32_t)((pk[k] & 0xffffu) != 0u && !(pk[k] & 0x8000u)) << (2 * k);
            b |= (uint32_t)((pk[k] >> 16) != 0u && !(pk[k] & 0x80000000u)) << (2 * k + 1);
          }
          a.pmbits[px * (C >> 3) + (c >> 3)] = (uint8_t)b;
        }
      }
      __syncthreads();   // every wave's pieces are rewritten before any fragment read
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int mi = 0; mi < TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fg = lane >> 4;
  // HALO: halo row of this lane's fragment pixel (tile pixel r = (r / tw, r % tw)) at tap offset 0;
  // pixels past th * tw (unused tile rows) read halo row 0 -- computed, never stored
  int hb[HALO ? TM : 1];
  if constexpr (HALO) {
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const int r = wm * WM + mi * 16 + fr;
      const int pr = (int)fdiv((uint32_t)r, a.fd_tw), pc = r - pr * a.tw;
      hb[mi] = r < a.th * a.tw ? pr * hwd + pc : 0;
    }
  }
  auto advance = [&]() {
    if constexpr (HALO) {   // chunk-major, tap-minor; the tap offsets advance by per-tap deltas
      if (++t_cur == NTAP) {
        t_cur = 0;
        c_cur += BK;
        need_halo = true;
        ts_cur = 0;
        toff = (ph.dh0 + 1) * hwd + (ph.dw0 + 1);
        wtC2 = (ph.wr0 * a.S + ph.ws0) * C * ES;
      } else if (++ts_cur == ph.Ts) {
        ts_cur = 0;
        toff += ph.dhs * hwd - (ph.Ts - 1) * ph.dws;
        wtC2 += (ph.wrs * a.S - (ph.Ts - 1) * ph.wss) * C * ES;
      } else {
        toff += ph.dws;
        wtC2 += ph.wss * C * ES;
      }
    } else if constexpr (!SMALLC) {
      c_cur += BK;
      if (c_cur >= C) {
        c_cur = 0;
        ++t_cur;
        tap_setup(t_cur);
      }
    }
  };
  // split-K (small grids): block y of a.splitk reduces K-steps [kbeg, kend)
  int kbeg = 0, kend = nk;
  if (a.splitk > 1) {
    const int per = (nk + a.splitk - 1) / a.splitk;
    kbeg = min(nk, (int)blockIdx.y * per);
    kend = min(nk, kbeg + per);
  }
  if (kend > kbeg) {
    if constexpr (HALO) {
      c_cur = (kbeg / NTAP) * BK;
      t_cur = kbeg - (kbeg / NTAP) * NTAP;
      tap_setup_halo(t_cur);
    } else if constexpr (!SMALLC) {
      const int cps = C / BK;   // K-steps per tap
      t_cur = kbeg / cps;
      c_cur = (kbeg - t_cur * cps) * BK;
      tap_setup(t_cur);
    }
    issue(kbeg);
    __syncthreads();
    prologue();
  }
  for (int ks = kbeg; ks < kend; ++ks) {
    if (ks > kbeg) {
      advance();
      issue(ks);
      __syncthreads();   // this stage landed (vmcnt(0) + barrier)
      prologue();
    }
    const char* As = smem;
    const char* Bs = As + A_BYTES;
    // HALO: this tap's A fragment addresses for K-half 0 (K-half 1 flips address bit 6:
    // (4 + fg) ^ s == (fg ^ s) ^ 4 for fg < 4)
    int a_addr[HALO ? TM : 1];
    if constexpr (HALO) {
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
        const int r = hb[mi] + toff;
        a_addr[mi] = r * 128 + ((fg ^ (r & 7)) << 4);
      }
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      typedef typename std::conditional<sizeof(T) == 2, bf16x8, f32x4>::type frag_t;
      frag_t af[TM], bfr[TN];
      const int ch = kk * 4 + fg;
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
        if constexpr (HALO) {
          af[mi] = *reinterpret_cast<const frag_t*>(As + (kk ? (a_addr[mi] ^ 64) : a_addr[mi]));
        } else {
          const int r = wm * WM + mi * 16 + fr;
          af[mi] = *reinterpret_cast<const frag_t*>(As + r * 128 + ((ch ^ (r & 7)) << 4));
        }
      }
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int r = wn * WN + ni * 16 + fr;
        bfr[ni] = *reinterpret_cast<const frag_t*>(Bs + r * 128 + ((ch ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) {
          if constexpr (sizeof(T) == 2) {
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
          } else {
            // the lane's 16-byte chunk holds reduction elements 4 fg + j (j < 4) of this half-step:
            // MFMA j reduces element j of every lane group -- a fixed permutation of the K order,
            // identical for A and B
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[mi][jj], bfr[ni][jj], acc[mi][ni], 0, 0, 0);
          }
        }
    }
    __syncthreads();   // every wave is done reading the stage before it is overwritten
  }

  if (a.splitk > 1 && !splitk_combine<NT, TM * TN>(a, &acc[0][0], smem, tid, mt, nt)) return;
  conv_epilogue<BM, BN, NT, WGM, WGN, T, HALO>(a, ph, acc, smem, tid, m0, n0, mt, hn, hh0, hw0);
}

// 8 KB of zeros: the pipelined kernel's out-of-image A pieces read here at the K-step's channel offset
// (2 C + 16 jc < 8 KB: C <= kPipeMaxC, checked at launch)
static __device__ u32x4 g_zero_run[512] = {};
constexpr int kPipeMaxC = 4032;

// ---- the pipelined 8-wave kernel -----------------------------------------------------------------
// BM x BN x 64 tiles, 512 threads = 8 waves in WGM x WGN, one block per CU, bf16, C % 64 == 0, one
// phase per blockIdx.z (forward convs, dgrad sub-pixel phases), no operand prologue, no split-K.
// K loop (STAGES LDS slots of one K-step each, slot of step k = k mod STAGES):
//     wait  until this wave's DMA of step k has landed (counted vmcnt: the STAGES - 2 younger steps'
//           DMAs stay in flight) and its fragment reads of step k - 1 have returned (lgkmcnt(0))
//     barrier  -> every wave's step-k DMA has landed: slot k is readable (RAW); every wave is done
//              reading slot k - 1 = slot (k + STAGES - 1) mod STAGES: it may be refilled (WAR)
//     issue the DMA of step k + STAGES - 1 into that slot
//     MFMAs of step k from slot k
// The raw s_barrier (not __syncthreads, whose workgroup fence drains vmcnt to 0 and with it the
// prefetch) is bracketed by "memory"-clobbering asm statements, so neither the fragment reads nor the
// DMA issue can be moved across it.
// VAR (issue placement, measured in benchmarks/conv_lab, profiles/r4_lab).  A K-step runs in 4 phases
// (K-half kk, half of the A fragments); the next step's DMA is issued at: 2 = A pieces at phase 0, B
// pieces at phase 2; 4 = A at phase 0 / B at phase 2 for the lower waves, A at 1 / B at 3 for the
// upper waves (the two waves of a SIMD then issue at different times).  Issuing everything at phase 0,
// staggering only by wave, and s_setprio around the MFMA clusters were 3-8 % slower and are gone.
// BM need not be a multiple of the staging pass (224 = 2 x 7 fragments): rows past BM stage zeros.
template <int BM, int BN, int WGM, int WGN, int STAGES, int VAR>
__global__ __launch_bounds__(64 * WGM * WGN) __attribute__((amdgpu_waves_per_eu(2, 2))) void conv_pipe_kernel(const ConvArgs a) {
  constexpr int NW = WGM * WGN;
  constexpr int NT = 64 * NW;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM = WM / 16, TN = WN / 16;
  static_assert(WM % 16 == 0 && WN % 16 == 0, "whole fragments");
  constexpr int RP = NT / 8;                  // tile rows staged per pass (8 lanes per 128-B row)
  static_assert(BN % RP == 0, "staging: whole passes");
  constexpr int AL = (BM + RP - 1) / RP, BL = BN / RP;   // 16-byte pieces per thread per K-step
  constexpr int NLD = AL + BL;                // DMA instructions per thread per K-step
  static_assert(STAGES == 2 || STAGES == 3, "2 or 3 slots");
  constexpr int A_BYTES = AL * RP * 128, B_BYTES = BN * 128;
  constexpr int SB = A_BYTES + B_BYTES;
  constexpr int EPI_NEED = EpiSmem<BM, BN, NT, WM>::bytes;
  constexpr int SMEM = STAGES * SB > EPI_NEED ? STAGES * SB : EPI_NEED;
  static_assert(SMEM <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WGN, wn = wid % WGN;
  const int lrow = tid >> 3;
  const int jc = (tid & 7) ^ ((tid >> 3) & 7);
  const char* zp = reinterpret_cast<const char*>(g_zero_page);

  const int zph = blockIdx.z;
  const uint32_t nwg0 = (uint32_t)a.ph[zph].mtiles * (uint32_t)a.ntiles;
  if (blockIdx.x >= nwg0) return;
  const uint32_t bid = xcd_remap(blockIdx.x, nwg0);
  const ConvPhase ph = a.ph[zph];
  const int mt = bid / a.ntiles, nt = bid - mt * a.ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int PQ = ph.P * ph.Q;
  const int M = a.Nimg * PQ;

  int a_hw[AL], a_pix[AL];
  uint32_t a_okm = 0;
#pragma unroll
  for (int i = 0; i < AL; ++i) {
    const int m = m0 + lrow + RP * i;
    if (m < M && lrow + RP * i < BM) a_okm |= 1u << i;
    const uint32_t mm = m < M ? (uint32_t)m : 0u;
    const uint32_t n_img = fdiv(mm, ph.fdPQ);
    const uint32_t rem = mm - n_img * PQ;
    const uint32_t p = fdiv(rem, ph.fdQ);
    const uint32_t q = rem - p * ph.Q;
    const int h = (int)p * a.sa, w = (int)q * a.sa;
    a_hw[i] = (h << 16) | w;
    a_pix[i] = ((int)n_img * a.H + h) * a.W + w;
  }
  const char* xlane = reinterpret_cast<const char*>(a.x) + 2 * ((int64_t)a.xoff + 8 * jc);
  const char* b_base = reinterpret_cast<const char*>(a.w) + 2 * ((int64_t)(n0 + lrow) * a.ldw + 8 * jc);
  const int64_t b_step = (int64_t)2 * RP * a.ldw;
  uint32_t b_okm = 0;
#pragma unroll
  for (int i = 0; i < BL; ++i)
    if (n0 + lrow + RP * i < a.Kout) b_okm |= 1u << i;

  const int C = a.C;
  const int nk = ph.ksteps;
  // A pieces: one pointer per piece per tap (set at the tap's first K-step), the channel offset of the
  // K-step added as a scalar.  An out-of-image / past-M piece points into an 8 KB zero run instead,
  // which every channel offset (2 C + 16 jc < 8 KB, host-checked) keeps inside: no per-K-step select.
  const char* zr = reinterpret_cast<const char*>(g_zero_run);
  const char* a_ptr[AL];
  int t_cur = 0, c_cur = 0, wtC2 = 0;
  auto tap_setup = [&](int t) {
    const int tr = (int)fdiv((uint32_t)t, ph.fdTs);
    const int ts = t - tr * ph.Ts;
    const int dh = ph.dh0 + tr * ph.dhs, dw = ph.dw0 + ts * ph.dws;
    const int wt = (ph.wr0 + tr * ph.wrs) * a.S + (ph.ws0 + ts * ph.wss);
    wtC2 = wt * C * 2;
    const int doff = dh * a.W + dw;
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      const int ih = (a_hw[i] >> 16) + dh, iw = (a_hw[i] & 0xffff) + dw;
      const bool ok = ((a_okm >> i) & 1) && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      a_ptr[i] = ok ? xlane + 2 * (uint64_t)((uint32_t)(a_pix[i] + doff) * (uint32_t)a.ldx) : zr + 16 * jc;
    }
  };
  auto advance = [&]() {
    c_cur += 64;
    if (c_cur >= C) {
      c_cur = 0;
      ++t_cur;
      tap_setup(t_cur);
    }
  };
  auto issue_a = [&](int slot) {
    char* As = smem + slot * SB;
    const int c2 = 2 * c_cur;
#pragma unroll
    for (int i = 0; i < AL; ++i) glds16(a_ptr[i] + c2, As + (RP * i + 8 * wid) * 128);
  };
  const bool b_all = b_okm == (1u << BL) - 1;   // every weight row of the tile exists (Kout % BN == 0)
  auto issue_b = [&](int slot) {
    char* Bs = smem + slot * SB + A_BYTES;
    const int64_t boff = (int64_t)wtC2 + 2 * c_cur;
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const char* s = (b_all || ((b_okm >> i) & 1)) ? b_base + i * b_step + boff : zp;
      glds16(s, Bs + (RP * i + 8 * wid) * 128);
    }
  };
  auto issue = [&](int slot) {
    issue_a(slot);
    issue_b(slot);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int mi = 0; mi < TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fg = lane >> 4;
  // per-lane fragment row byte offsets (A rows wm*WM + 16 mi + fr, B rows wn*WN + 16 ni + fr) and
  // the swizzle term of each: (r & 7) is the same for every mi (16 | row step)
  const int sw = fr & 7;
  const int a_row0 = (wm * WM + fr) * 128, b_row0 = A_BYTES + (wn * WN + fr) * 128;

  if (nk > 0) {
    tap_setup(0);
    issue(0);
    if constexpr (STAGES == 3) {
      if (nk > 1) {
        advance();
        issue(1);
      }
    }
  }
  // one K-step on slot RD (a constant: the loop below is unrolled by STAGES, so every fragment read
  // is a lane offset + an immediate)
  auto step = [&](int ks, auto RDc) {
    constexpr int rd = decltype(RDc)::value;
    if constexpr (STAGES == 3) {
      if (ks + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)" :: "n"(NLD) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const bool more = ks + STAGES - 1 < nk;
    constexpr int wr = (rd + STAGES - 1) % STAGES;
    if (more) advance();
    const char* As = smem + rd * SB;
    const bool up = wid >= NW / 2;   // wave-uniform: waves w and w + NW/2 share a SIMD
    constexpr int MH = (TM + 1) / 2;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int cb = ((kk * 4 + fg) ^ sw) << 4;
      bf16x8 bfr[TN];
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) bfr[ni] = *reinterpret_cast<const bf16x8*>(As + b_row0 + ni * 16 * 128 + cb);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        // DMA issue points: phase p = (kk, half of the A fragments)
        const int p = kk * 2 + h;
        static_assert(VAR == 2 || VAR == 4, "issue placement");
        bool doA, doB;
        if constexpr (VAR == 2) { doA = p == 0; doB = p == 2; }
        else { doA = p == (up ? 1 : 0); doB = p == (up ? 3 : 2); }
        if (more && (doA || doB)) {
          if (doA) issue_a(wr);
          if (doB) issue_b(wr);
          asm volatile("" ::: "memory");
        }
        bf16x8 af[MH];
#pragma unroll
        for (int q = 0; q < MH; ++q)
          if (h * MH + q < TM) af[q] = *reinterpret_cast<const bf16x8*>(As + a_row0 + (h * MH + q) * 16 * 128 + cb);
#pragma unroll
        for (int q = 0; q < MH; ++q)
#pragma unroll
          for (int ni = 0; ni < TN; ++ni)
            if (h * MH + q < TM)
              acc[h * MH + q][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[q], bfr[ni], acc[h * MH + q][ni], 0, 0, 0);
      }
    }
  };
  for (int ks = 0; ks < nk; ks += STAGES) {
    step(ks, std::integral_constant<int, 0>{});
    if (ks + 1 < nk) step(ks + 1, std::integral_constant<int, 1>{});
    if constexpr (STAGES == 3)
      if (ks + 2 < nk) step(ks + 2, std::integral_constant<int, 2>{});
  }
  __syncthreads();   // the last fragment reads are done before the epilogue reuses the LDS
  conv_epilogue<BM, BN, NT, WGM, WGN, uint16_t, false>(a, ph, acc, smem, tid, m0, n0, mt, 0, 0, 0);
}

// ---- 2-D halo tiles with the weight tile double-buffered ---------------------------------------------
// conv_halo_pipe_kernel: conv_igemm_kernel's HALO mode (3x3 / stride 1 / pad 1, the (th + 2) x (tw + 2)
// input halo of a 64-channel chunk staged once, the 9 taps 9 K-steps over it; same tile decode, same
// fragment addressing, same epilogue) with two LDS slots for the weight tile, so the single-stage
// kernel's exposed DMA latency per tap is gone: the DMA of tap k + 1 goes into the other slot while
// the MFMAs of tap k run, and a K-step has ONE barrier:
//     wait   this wave's DMA of step k landed (vmcnt(0): nothing younger is in flight) and its
//            fragment reads of step k - 1 returned (lgkmcnt(0))
//     barrier -> every wave's step-k DMA landed (RAW); every wave is done reading slot (k + 1) mod 2 (WAR)
//     issue the weight DMA of step k + 1 into slot (k + 1) mod 2 (after this step's first fragment reads)
//     MFMAs of step k
// The halo itself stays single-buffered (45 KB at 256-pixel tiles; two of them would leave one block
// per CU): at the last tap of a chunk the next chunk's halo and first weight tile are issued after a
// second barrier, once every wave is done with the old halo -- one exposed load per 9 K-steps.
// Same K order and per-element arithmetic as conv_igemm_kernel: bit-identical results.  No split-K
// (the launcher keeps the single-stage kernel for split grids).
template <int BM, int BN, int WGM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void conv_halo_pipe_kernel(const ConvArgs a) {
  constexpr int NW = 4, NT = 256, WGN = NW / WGM;
  constexpr int WM = BM / WGM, WN = BN / WGN, TM = WM / 16, TN = WN / 16;
  constexpr int RP = NT / 8;                  // 32 tile rows per staging pass
  constexpr int BL = BN / RP;                 // weight pieces per thread per K-step
  constexpr int HALO_ROWS = BM == 256 ? 352 : 192;
  constexpr int HL = HALO_ROWS / RP;          // halo pieces per thread per chunk
  constexpr int A_BYTES = HALO_ROWS * 128, B_BYTES = BN * 128;
  constexpr int SB = A_BYTES + 2 * B_BYTES;   // [halo | weight slot 0 | weight slot 1]
  constexpr int EPI_NEED = EpiSmem<BM, BN, NT, WM>::bytes;
  constexpr int SMEM = SB > EPI_NEED ? SB : EPI_NEED;
  static_assert(HALO_ROWS % RP == 0 && BN % RP == 0 && TM >= 1 && TN >= 1, "tile shape");
  static_assert(2 * SMEM <= 160 * 1024, "two blocks per CU");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WGN, wn = wid % WGN;
  const int lrow = tid >> 3;
  const int jc = (tid & 7) ^ ((tid >> 3) & 7);
  const char* zp = reinterpret_cast<const char*>(g_zero_page);

  const int zph = blockIdx.z;
  const uint32_t nwg0 = (uint32_t)a.ph[zph].mtiles * (uint32_t)a.ntiles;
  if (blockIdx.x >= nwg0) return;
  const uint32_t bid = xcd_remap(blockIdx.x, nwg0);
  const ConvPhase ph = a.ph[zph];
  const int mt = bid / a.ntiles, nt = bid - mt * a.ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int hn = (int)fdiv((uint32_t)mt, a.fd_thw);
  const int rem = mt - hn * a.tiles_h * a.tiles_w;
  const int ti = (int)fdiv((uint32_t)rem, a.fd_tilesw);
  const int hh0 = ti * a.th, hw0 = (rem - ti * a.tiles_w) * a.tw;

  // weight pieces: a wave-uniform base (tile column, tap, chunk) + a per-lane 32-bit offset, so the
  // DMA takes the scalar-base address form (no 64-bit vector arithmetic per piece)
  const char* w_col = reinterpret_cast<const char*>(a.w) + (int64_t)2 * n0 * a.ldw;
  const uint32_t b_lane = 2u * ((uint32_t)lrow * (uint32_t)a.ldw + 8u * (uint32_t)jc);
  const uint32_t b_step = 2u * RP * (uint32_t)a.ldw;
  uint32_t b_okm = 0;
#pragma unroll
  for (int i = 0; i < BL; ++i)
    if (n0 + lrow + RP * i < a.Kout) b_okm |= 1u << i;
  const bool b_all = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_ballot_w64(b_okm != (1u << BL) - 1) == 0);

  const int C = a.C;
  const int NTAP = ph.Tr * ph.Ts;
  const int nk = ph.ksteps;
  const int hwd = a.tw + 2;                   // halo row length (pixels)
  // halo piece i of this lane: halo row lrow + RP i -> (line, col) relative to the tile origin; the
  // global pixel offset is kept per piece (-1: outside the image or past the halo: the zero page)
  int64_t hl_off[HL];
  {
    const int nrows = (a.th + 2) * hwd;
#pragma unroll
    for (int i = 0; i < HL; ++i) {
      const int hr = lrow + RP * i;
      const int line = hr / hwd;
      const int ih = hh0 + line - 1, iw = hw0 + (hr - line * hwd) - 1;
      const bool ok = hr < nrows && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      hl_off[i] = ok ? (int64_t)2 * (((int64_t)hn * a.H + ih) * a.W + iw) * a.ldx : -1;
    }
  }
  const char* xlane = reinterpret_cast<const char*>(a.x) + 2 * ((int64_t)a.xoff + 8 * jc);

  // the tap walk (tap t = (tr, ts) of a Tr x Ts window, chunk-major): halo-row offset and weight-tap
  // byte offset advanced by per-tap deltas instead of recomputed from t
  const int toff0 = (ph.dh0 + 1) * hwd + (ph.dw0 + 1);
  const int wt0 = (ph.wr0 * a.S + ph.ws0) * C * 2;
  const int dto_s = ph.dws, dwt_s = ph.wss * C * 2;                       // next ts
  const int dto_r = ph.dhs * hwd - (ph.Ts - 1) * ph.dws;                  // next tr (ts back to 0)
  const int dwt_r = (ph.wrs * a.S - (ph.Ts - 1) * ph.wss) * C * 2;
  int t_cur = 0, ts_cur = 0, c_cur = 0, wtC2 = wt0, toff = toff0;
  auto tap_next = [&]() {   // (t_cur, ts_cur, toff, wtC2) -> the next K-step's tap
    if (++t_cur == NTAP) {
      t_cur = 0;
      ts_cur = 0;
      c_cur += 64;
      toff = toff0;
      wtC2 = wt0;
    } else if (++ts_cur == ph.Ts) {
      ts_cur = 0;
      toff += dto_r;
      wtC2 += dwt_r;
    } else {
      toff += dto_s;
      wtC2 += dwt_s;
    }
  };
  auto issue_halo = [&]() {
    const char* xb = xlane + 2 * c_cur;
#pragma unroll
    for (int i = 0; i < HL; ++i) glds16(hl_off[i] >= 0 ? xb + hl_off[i] : zp, smem + (RP * i + 8 * wid) * 128);
  };
  auto issue_b = [&](int slot) {
    char* Bs = smem + A_BYTES + slot * B_BYTES;
    const char* wb = w_col + wtC2 + 2 * c_cur;
    if (b_all) {
#pragma unroll
      for (int i = 0; i < BL; ++i) glds16(wb + (b_lane + i * b_step), Bs + (RP * i + 8 * wid) * 128);
    } else {
#pragma unroll
      for (int i = 0; i < BL; ++i)
        glds16(((b_okm >> i) & 1) ? wb + (b_lane + i * b_step) : zp, Bs + (RP * i + 8 * wid) * 128);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int mi = 0; mi < TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fg = lane >> 4;
  // halo row of this lane's fragment pixel at tap offset 0 (pixels past th * tw read row 0, never stored)
  int hb[TM];
#pragma unroll
  for (int mi = 0; mi < TM; ++mi) {
    const int r = wm * WM + mi * 16 + fr;
    const int pr = (int)fdiv((uint32_t)r, a.fd_tw), pc = r - pr * a.tw;
    hb[mi] = r < a.th * a.tw ? pr * hwd + pc : 0;
  }
  const int b_row0 = A_BYTES + (wn * WN + fr) * 128;
  const int sw = fr & 7;   // (r & 7) of every B fragment row of this lane

  if (nk > 0) {
    issue_halo();
    issue_b(0);
  }
  auto step = [&](int ks, auto SLc) {
    constexpr int sl = decltype(SLc)::value;
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // this tap's A fragment addresses for K-half 0; K-half 1 flips chunk bit 2 = address bit 6
    // ((4 + fg) ^ s == (fg ^ s) ^ 4 for fg < 4)
    int a_addr[TM];
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const int r = hb[mi] + toff;
      a_addr[mi] = r * 128 + ((fg ^ (r & 7)) << 4);
    }
    const bool more = ks + 1 < nk;
    const bool chunk_end = more && t_cur + 1 == NTAP;
    if (more) tap_next();   // the next K-step's tap (and chunk)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk * 4 + fg;
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int ni = 0; ni < TN; ++ni)
        bfr[ni] = *reinterpret_cast<const bf16x8*>(smem + b_row0 + sl * B_BYTES + ni * 16 * 128 + ((ch ^ sw) << 4));
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
        af[mi] = *reinterpret_cast<const bf16x8*>(smem + (kk ? (a_addr[mi] ^ 64) : a_addr[mi]));
      if (kk == 0 && more && !chunk_end) {
        issue_b(sl ^ 1);
        asm volatile("" ::: "memory");
      }
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
    }
    if (chunk_end) {   // every wave done with the old halo: stage the next chunk's and its first weights
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      issue_halo();
      issue_b(sl ^ 1);
    }
  };
  for (int ks = 0; ks < nk; ks += 2) {
    step(ks, std::integral_constant<int, 0>{});
    if (ks + 1 < nk) step(ks + 1, std::integral_constant<int, 1>{});
  }
  __syncthreads();   // the last fragment reads are done before the epilogue reuses the LDS
  conv_epilogue<BM, BN, NT, WGM, WGN, uint16_t, true>(a, ph, acc, smem, tid, m0, n0, mt, hn, hh0, hw0);
}

// ---- the producer's BN-apply fused into a 1x1 consumer, register-staged ----------------------------
// conv1x1_apply_kernel: pro-3 launches (ConvArgs::pro 3: x = the producer BN's input z, pz its
// residual) of a 1x1 / stride-1 conv whose Kout (64 / 128 / 256) is ONE output tile column, so every
// input element is applied exactly once.  The single-stage pro-3 path of conv_igemm_kernel stages z
// and the residual by LDS-DMA, rewrites them in LDS after a barrier and only then runs the MFMAs: a
// memory-bound GEMM with no load in flight while it computes (ResNet-50 28^2 512->128: 215 us vs
// 115 + 58 us for the apply pass and the plain conv).  Here every K-step (64 channels) goes
//   global z / residual / weight pieces -> VGPRs (issued one K-step ahead, under the MFMAs)
//   -> y = relu(z * scale + shift + r) in registers (bn_apply_kernel's fma order: bit-identical y)
//   -> y and its ReLU mask bits to global, y and the weights into the LDS stage of the next K-step
// with two LDS stages and ONE barrier per K-step (the stage written at step k was last read at
// step k - 1, before the previous barrier).  128-row tiles, 8 waves, conv_epilogue (statistics, bias).
template <int BM, int BN, int WGM, int WGN>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(BN <= 128 ? 4 : 2, 8)))
void conv1x1_apply_kernel(const ConvArgs a) {
  constexpr int NT = 512;
  static_assert(WGM * WGN == 8, "8 waves");
  constexpr int WM = BM / WGM, WN = BN / WGN, TM = WM / 16, TN = WN / 16;
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128, SB = A_BYTES + B_BYTES;
  constexpr int MAXC = 4 * BN;                // the apply's per-channel vectors live in LDS (C <= MAXC)
  constexpr int PRM_BYTES = 4 * MAXC * 4;     // scale, shift, residual scale, residual shift
  constexpr int EPI_NEED = EpiSmem<BM, BN, NT, WM>::bytes;
  constexpr int SMEM = 2 * SB + PRM_BYTES > EPI_NEED ? 2 * SB + PRM_BYTES : EPI_NEED;
  constexpr int RP = NT / 8;                  // 64 tile rows per pass (8 lanes per 128-B row)
  constexpr int AL = BM / RP, BL = BN / RP;   // pieces per thread per K-step
  static_assert(AL >= 1 && BL >= 1, "tile shape");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WGN, wn = wid % WGN;
  const int lrow = tid >> 3, jc = tid & 7;    // row lrow + RP i, 16-B chunk jc (channels 8 jc ..)
  const ConvPhase& ph = a.ph[0];
  const int M = a.Nimg * ph.P * ph.Q;
  const uint32_t mt = xcd_remap(blockIdx.x, (uint32_t)ph.mtiles);
  const int m0 = (int)mt * BM;
  const int C = a.C, nk = C / 64;
  const bool rbn = a.prscale != nullptr;

  // per-channel vectors -> LDS once (read back per piece: no global loads in the K loop besides the
  // operands, and 16 fewer VGPRs than holding them)
  float* prm = reinterpret_cast<float*>(smem + 2 * SB);
  for (int i = tid; i < C; i += NT) {
    prm[i] = a.pscale[i];
    prm[MAXC + i] = a.pshift[i];
    if (rbn) {
      prm[2 * MAXC + i] = a.prscale[i];
      prm[3 * MAXC + i] = a.prshift[i];
    }
  }

  // 32-bit element offsets of this thread's rows (< 2^31: host-checked); 1x1 / stride 1 / pad 0:
  // the input pixel is the tile row
  const uint16_t* xb = static_cast<const uint16_t*>(a.x);
  const uint16_t* rb = static_cast<const uint16_t*>(a.pz);
  uint32_t zo[AL], ro[AL], yo[AL], bo[AL];
  uint32_t okm = 0;
#pragma unroll
  for (int i = 0; i < AL; ++i) {
    const int m = m0 + lrow + RP * i;
    if (m < M) okm |= 1u << i;
    const uint32_t mm = m < M ? (uint32_t)m : 0u;
    zo[i] = mm * (uint32_t)a.ldx + (uint32_t)a.xoff + 8 * jc;
    ro[i] = mm * (uint32_t)a.ldpz + (uint32_t)a.pzoff + 8 * jc;
    yo[i] = mm * (uint32_t)a.ldpy + (uint32_t)a.pyoff + 8 * jc;
    bo[i] = mm * (uint32_t)(C >> 3) + jc;
  }
  const uint16_t* wb = static_cast<const uint16_t*>(a.w) + (int64_t)lrow * a.ldw + 8 * jc;   // Kout == BN
  const int64_t wstep = (int64_t)RP * a.ldw;

  u32x4 zv[AL], rv[AL], wv[BL];
  auto load = [&](int k) {
    const int c = 64 * k;
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      zv[i] = *reinterpret_cast<const u32x4*>(xb + zo[i] + c);
      rv[i] = *reinterpret_cast<const u32x4*>(rb + ro[i] + c);
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) wv[i] = *reinterpret_cast<const u32x4*>(wb + i * wstep + c);
  };
  // y of the loaded pieces -> global (+ mask bits) and the LDS stage `buf`; weights -> the stage
  auto commit = [&](int k, int buf) {
    char* As = smem + buf * SB;
    char* Bs = As + A_BYTES;
    const int cc = 64 * k + 8 * jc;
    const f32x4 s0 = *reinterpret_cast<const f32x4*>(prm + cc), s1 = *reinterpret_cast<const f32x4*>(prm + cc + 4);
    const f32x4 h0 = *reinterpret_cast<const f32x4*>(prm + MAXC + cc);
    const f32x4 h1 = *reinterpret_cast<const f32x4*>(prm + MAXC + cc + 4);
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      const int r = lrow + RP * i;
      u32x4 pk = u32x4{0u, 0u, 0u, 0u};   // rows past M: zeros (their outputs are dropped)
      if ((okm >> i) & 1) {
        float v[8], q[8];
        unpack8(zv[i], v);
        unpack8(rv[i], q);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = __builtin_fmaf(v[e], s0[e], h0[e]);
          v[e + 4] = __builtin_fmaf(v[e + 4], s1[e], h1[e]);
        }
        if (rbn) {
          const f32x4 a0 = *reinterpret_cast<const f32x4*>(prm + 2 * MAXC + cc);
          const f32x4 a1 = *reinterpret_cast<const f32x4*>(prm + 2 * MAXC + cc + 4);
          const f32x4 b0 = *reinterpret_cast<const f32x4*>(prm + 3 * MAXC + cc);
          const f32x4 b1 = *reinterpret_cast<const f32x4*>(prm + 3 * MAXC + cc + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            q[e] = __builtin_fmaf(q[e], a0[e], b0[e]);
            q[e + 4] = __builtin_fmaf(q[e + 4], a1[e], b1[e]);
          }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e] + q[e], 0.f);
        pk = pack8(v);
        *reinterpret_cast<u32x4*>(a.py + yo[i] + 64 * k) = pk;
        uint32_t b = 0;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          b |= (uint32_t)((pk[t] & 0xffffu) != 0u && !(pk[t] & 0x8000u)) << (2 * t);
          b |= (uint32_t)((pk[t] >> 16) != 0u && !(pk[t] & 0x80000000u)) << (2 * t + 1);
        }
        a.pmbits[bo[i] + 8 * k] = (uint8_t)b;
      }
      *reinterpret_cast<u32x4*>(As + r * 128 + ((jc ^ (r & 7)) << 4)) = pk;
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const int r = lrow + RP * i;
      *reinterpret_cast<u32x4*>(Bs + r * 128 + ((jc ^ (r & 7)) << 4)) = wv[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int mi = 0; mi < TM; ++mi)
#pragma unroll
    for (int ni = 0; ni < TN; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fg = lane >> 4;

  load(0);
  __syncthreads();   // the per-channel vectors are in LDS
  commit(0, 0);
  __syncthreads();
  for (int k = 0; k < nk; ++k) {
    if (k + 1 < nk) load(k + 1);   // in flight under this step's MFMAs
    const char* As = smem + (k & 1) * SB;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[TM], bfr[TN];
      const int ch = kk * 4 + fg;
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
        const int r = wm * WM + mi * 16 + fr;
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
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
    }
    if (k + 1 < nk) commit(k + 1, (k + 1) & 1);   // the stage read at step k - 1 (before the last barrier)
    __syncthreads();
  }
  conv_epilogue<BM, BN, NT, WGM, WGN, uint16_t, false>(a, ph, acc, smem, tid, m0, 0, (int)mt, 0, 0, 0);
}

}  // namespace dlmpi

using namespace dlmpi;

// The operand prologue (pro 3) is built for the 128 x 64 tile only (the host's kPro3Bm x kPro3Bn; the
// 256 x 128 / 128 x 128 / 256 x 64 pro-3 instances spilled 40 / 17 / 0 VGPRs and 24 / 3 / 29 SGPRs).
template <int BM, int BN>
static hipError_t launch_tile(const ConvArgs* a, dim3 grid, hipStream_t s) {
  if (a->pro == 3) {
    if constexpr (BM == 128 && BN == 64) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, false, 2, 3>), grid, dim3(256), 0, s, *a);
    else return hipErrorInvalidValue;
  } else if (a->C < 64) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, true, 2>), grid, dim3(256), 0, s, *a);
  else hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, false, 2>), grid, dim3(256), 0, s, *a);
  return hipSuccess;
}

// Split-K plan for small grids (ResNet-18 on 32x32 CIFAR: layer4 is 1x1 pixels, 8 tiles x 72
// K-steps): slices so that tiles x slices reaches ~256 blocks, >= 4 K-steps per slice, <= 8 slices.
// Slabs (fp32) and tickets come per stream role (bn.hip), so the
// main and the branch stream can run split convolutions concurrently.
static int splitk_plan(int tiles, int nk) {
  if (tiles >= 256 || nk < 8) return 1;
  int S = (256 + tiles - 1) / tiles;
  S = S < nk / 4 ? S : nk / 4;
  S = S < 8 ? S : 8;
  return S < 2 ? 1 : S;
}

// fp32 precision path: single-stage 4-wave tiles up to 128 x 128 (the f32 MFMA is 1/16 of the
// bf16 rate, so the wider bf16 tiles buy nothing here)
static hipError_t launch_f32(const ConvArgs* a, int bm, int bn, dim3 grid, hipStream_t s) {
  if (a->pro != 0) return hipErrorInvalidValue;
  // the regular staging walks whole 32-channel K-steps per tap; anything else stages per 16-B piece
  const bool small = a->C < 32 || a->C % 32 != 0;
#define LAUNCH_F32(BM_, BN_)                                                                                   \
  do {                                                                                                       \
    if (small) hipLaunchKernelGGL((conv_igemm_kernel<BM_, BN_, true, 2, 0, float>), grid, dim3(256), 0, s, *a); \
    else hipLaunchKernelGGL((conv_igemm_kernel<BM_, BN_, false, 2, 0, float>), grid, dim3(256), 0, s, *a);     \
  } while (0)
  if (bm == 128 && bn == 128) LAUNCH_F32(128, 128);
  else if (bm == 128 && bn == 64) LAUNCH_F32(128, 64);
  else if (bm == 64 && bn == 128) LAUNCH_F32(64, 128);
  else if (bm == 64 && bn == 64) LAUNCH_F32(64, 64);
  else return hipErrorInvalidValue;
#undef LAUNCH_F32
  return hipGetLastError();
}

// Pipelined 8-wave tiles (conv_pipe_kernel): (bm, bn) -> instance.  Returns hipErrorInvalidValue
// when the launch does not fit the kernel (channels, prologue, split, fp32).
static hipError_t launch_pipe(const ConvArgs* a, int bm, int bn, int var, dim3 grid, hipStream_t s) {
  if (a->f32 || a->pro != 0 || a->C % 64 != 0 || a->C > kPipeMaxC || a->halo || grid.y != 1) return hipErrorInvalidValue;
  // the measured issue placement of each tile (profiles/r4_lab): VAR 2 for the 256 / 224 / 512-row
  // tiles, VAR 4 for 128 x 256; the other placements are gone (var must name the tile's own)
  if (var != (bm == 128 ? 4 : 2)) return hipErrorInvalidValue;
  if (bm == 256 && bn == 256) hipLaunchKernelGGL((conv_pipe_kernel<256, 256, 2, 4, 2, 2>), grid, dim3(512), 0, s, *a);
  else if (bm == 224 && bn == 256) hipLaunchKernelGGL((conv_pipe_kernel<224, 256, 2, 4, 2, 2>), grid, dim3(512), 0, s, *a);
  else if (bm == 256 && bn == 128) hipLaunchKernelGGL((conv_pipe_kernel<256, 128, 4, 2, 3, 2>), grid, dim3(512), 0, s, *a);
  else if (bm == 128 && bn == 256) hipLaunchKernelGGL((conv_pipe_kernel<128, 256, 2, 4, 3, 4>), grid, dim3(512), 0, s, *a);
  else if (bm == 512 && bn == 64) hipLaunchKernelGGL((conv_pipe_kernel<512, 64, 8, 1, 2, 2>), grid, dim3(512), 0, s, *a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// The fused apply + 1x1 kernel applies (shape only; the launch checks the rest)
extern "C" int dlmpi_conv1x1_apply_ok(int C, int K) {
  return C % 64 == 0 && C <= 4 * K && (K == 64 || K == 128 || K == 256);   // C <= 4 K: the LDS vectors
}

extern "C" hipError_t dlmpi_conv1x1_apply(const ConvArgs* a, int bm, hipStream_t s) {
  if (a->pro != 3 || a->f32 || a->halo || a->nphase != 1 || a->ntiles != 1 || !a->vec_store || a->res ||
      a->scale || a->relu || a->mask || a->mscale || a->mbits || a->z || a->splitk_req > 1 ||
      !dlmpi_conv1x1_apply_ok(a->C, a->Kout) || a->ph[0].Tr != 1 || a->ph[0].Ts != 1 || a->sa != 1 ||
      a->ph[0].mtiles != (a->Nimg * a->ph[0].P * a->ph[0].Q + bm - 1) / bm || a->ldw != a->C ||
      (int64_t)a->Nimg * a->H * a->W * (a->ldx > a->ldpz ? (a->ldx > a->ldpy ? a->ldx : a->ldpy)
                                                          : (a->ldpz > a->ldpy ? a->ldpz : a->ldpy)) >= (1ll << 31))
    return hipErrorInvalidValue;
  const dim3 grid((unsigned)a->ph[0].mtiles);
  if (grid.x == 0) return hipSuccess;
  if (bm == 128 && a->Kout == 64) hipLaunchKernelGGL((conv1x1_apply_kernel<128, 64, 8, 1>), grid, dim3(512), 0, s, *a);
  else if (bm == 128 && a->Kout == 128) hipLaunchKernelGGL((conv1x1_apply_kernel<128, 128, 4, 2>), grid, dim3(512), 0, s, *a);
  else if (bm == 128 && a->Kout == 256) hipLaunchKernelGGL((conv1x1_apply_kernel<128, 256, 2, 4>), grid, dim3(512), 0, s, *a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// 256 x 128 halo tiles on conv_halo_pipe_kernel (dlmpi_set_halo_pipe(0): the single-stage kernel, A/B).
// The 128 x 128 / 256 x 64 halo tiles stay single-stage: on the pipelined kernel (2 blocks per CU instead
// of 3) they measured 8 % slower (profiles/r6_halo_pipe/lab_small.log).
static int g_halo_pipe = 1;
extern "C" void dlmpi_set_halo_pipe(int on) { g_halo_pipe = on; }

// pipe != 0: the launch runs the pipelined kernel (tile bm x bn must be one of launch_pipe's)
extern "C" hipError_t dlmpi_conv_igemm_ex(const ConvArgs* a_in, int bm, int bn, int pipe, hipStream_t s) {
  int maxt = 0, tiles = 0, maxk = 0;
  for (int i = 0; i < a_in->nphase; ++i) {
    maxt = a_in->ph[i].mtiles > maxt ? a_in->ph[i].mtiles : maxt;
    tiles += a_in->ph[i].mtiles * a_in->ntiles;
    maxk = a_in->ph[i].ksteps > maxk ? a_in->ph[i].ksteps : maxk;
  }
  ConvArgs ab = *a_in;
  const ConvArgs* a = &ab;
  ab.splitk = 1;
  if (pipe) {
    const dim3 grid((unsigned)(maxt * a->ntiles), 1, (unsigned)a->nphase);
    if (grid.x == 0) return hipSuccess;
    return launch_pipe(a, bm, bn, pipe - 1, grid, s);
  }
  int S = a_in->splitk_req > 0 ? a_in->splitk_req : splitk_plan(tiles, maxk);
  if (S > maxk) S = maxk > 0 ? maxk : 1;
  if (S > 1) {
    const int ntile_ids = maxt * a_in->ntiles * a_in->nphase;   // kernel: z * gridDim.x + mt * ntiles + nt
    float* slab = dlmpi_splitk_slab(s, (size_t)ntile_ids * S * bm * bn);
    int* tk = dlmpi_splitk_tickets(s, ntile_ids);
    if (slab && tk) {
      ab.splitk = S;
      ab.sk_slab = slab;
      ab.sk_tk = tk;
    }
  }
  dim3 grid((unsigned)(maxt * a->ntiles), (unsigned)ab.splitk, (unsigned)a->nphase);
  if (grid.x == 0) return hipSuccess;
  if (a->f32) return launch_f32(a, bm, bn, grid, s);
  if (a->halo) {   // 3x3 / stride 1 / pad 1 by 2-D tiles with a staged halo (host-planned)
    if (a->pro != 0 || a->C % 64 != 0) return hipErrorInvalidValue;
    if (bm == 128 && bn == 128) hipLaunchKernelGGL((conv_igemm_kernel<128, 128, false, 2, 0, uint16_t, true>), grid, dim3(256), 0, s, *a);
    else if (bm == 128 && bn == 64) hipLaunchKernelGGL((conv_igemm_kernel<128, 64, false, 2, 0, uint16_t, true>), grid, dim3(256), 0, s, *a);
    // 256-pixel tiles: per-wave 64 x 64 (4 x 1 waves) / 128 x 64 (2 x 2): half the LDS reads per MFMA
    else if (bm == 256 && bn == 64) hipLaunchKernelGGL((conv_igemm_kernel<256, 64, false, 4, 0, uint16_t, true>), grid, dim3(256), 0, s, *a);
    else if (bm == 256 && bn == 128) {
      if (g_halo_pipe && ab.splitk == 1) hipLaunchKernelGGL((conv_halo_pipe_kernel<256, 128, 2>), grid, dim3(256), 0, s, *a);
      else hipLaunchKernelGGL((conv_igemm_kernel<256, 128, false, 2, 0, uint16_t, true>), grid, dim3(256), 0, s, *a);
    } else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (a->pro != 0 && (a->pro != 3 || a->C < 64 || a->C % 64 != 0)) return hipErrorInvalidValue;
  hipError_t e = hipSuccess;
  if (bm == 256 && bn == 64) {   // 64-channel layers: 4 x 1 waves of 64 x 64
    if (a->pro == 3) return hipErrorInvalidValue;
    if (a->C < 64) hipLaunchKernelGGL((conv_igemm_kernel<256, 64, true, 4>), grid, dim3(256), 0, s, *a);
    else hipLaunchKernelGGL((conv_igemm_kernel<256, 64, false, 4>), grid, dim3(256), 0, s, *a);
  } else if (bm == 256 && bn == 128) e = launch_tile<256, 128>(a, grid, s);
  else if (bm == 128 && bn == 128) e = launch_tile<128, 128>(a, grid, s);
  else if (bm == 128 && bn == 64) e = launch_tile<128, 64>(a, grid, s);
  else if (bm == 64 && bn == 128) e = launch_tile<64, 128>(a, grid, s);
  else if (bm == 64 && bn == 64) e = launch_tile<64, 64>(a, grid, s);
  else return hipErrorInvalidValue;
  return e != hipSuccess ? e : hipGetLastError();
}

extern "C" hipError_t dlmpi_conv_igemm(const ConvArgs* a, int bm, int bn, hipStream_t s) {
  return dlmpi_conv_igemm_ex(a, bm, bn, 0, s);
}
