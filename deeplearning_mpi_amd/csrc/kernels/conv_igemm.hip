// Implicit-GEMM convolution on CDNA4 MFMA (v_mfma_f32_16x16x32_bf16), NHWC bf16, fp32 accumulate.
//
// One kernel serves every "gather-A" GEMM of the framework:
//   * Conv2d forward (any R x S, stride, pad; ResNet stem 7x7/s2, 3x3, 1x1, UNet 3x3),
//   * Conv2d data-gradient (stride^2 sub-pixel phases, each a dense conv with its own tap list,
//     so a stride-2 3x3 dgrad does no zero MACs),
//   * ConvTranspose2d(k=2, s=2) forward (4 phases of a 1x1 GEMM written to strided pixels),
//   * Linear (a 1x1 conv on a 1x1 image).
// Replaces what the reference gets implicitly from cuDNN conv fwd/dgrad and cuBLAS
// (call sites /root/reference/pytorch/unet/model.py:9-14, resnet main.py:40-41).
//
// Tile: BM (pixels) x BN (channels) x 64 (reduction), 256 threads = 4 waves in 2x2, each wave
// (BM/2) x (BN/2) as (BM/32) x (BN/32) MFMA 16x16 tiles.
// Staging: global -> LDS directly with global_load_lds_dwordx4 (no VGPR round trip, no ds_write):
// each wave instruction fills 8 LDS rows of 128 B lane-linearly; the XOR swizzle that makes the
// ds_read_b128 fragment reads bank-conflict-free is applied on the per-lane SOURCE address
// (cdna_hip_programming.md §5.4 rule 21).  Out-of-image im2col pieces read a zero page.  The
// next K-tile's loads are issued before the current tile's MFMAs into the other LDS buffer
// (one barrier per K-step).  Channel counts >= 64: the tap (r, s) and channel base are
// wave-uniform scalars and the per-row source pointers are rebuilt only when the tap changes.
// Epilogue: the fp32 tile is staged through LDS for 16-byte stores with fused bias / residual
// add / folded-BN affine / ReLU and the per-channel BatchNorm partial sums of the stored
// (bf16-rounded) values.
#include <cstdlib>
#include <type_traits>

#ifndef DLMPI_W128   // waves/SIMD target of the 128x128 / 256x64 tiles (A/B builds)
#define DLMPI_W128 3
#endif

#include "common.h"
#include "bnfin.h"

namespace dlmpi {

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void glds16(const void* g, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(g, (lds_void*)lds_wave_base, 16, 0, 0);
}

// STAGES = 2: double-buffered K loop (one barrier per K-step, 2 blocks/CU at 128x128);
// STAGES = 1: single buffer, two barriers per K-step, 34 KB of LDS -> 4 blocks/CU (latency hidden
// across blocks instead of inside one).  The epilogue stages the fp32 tile through LDS in two
// row halves so it never needs more LDS than one stage.
// NW = 8 (512 threads, waves 2 x 4, per-wave 128 x 64 at 256 x 256): 25 % less LDS traffic per
// MFMA than 64 x 64 per wave, double-buffered (128 KB LDS, one block per CU) so that a whole
// K-step of MFMA work (2048 SIMD cycles) covers the next step's loads.
// WGM = wave rows (WGM x NW/WGM wave grid): 4 x 1 for the 256 x 64 tile of 64-channel layers
// (per-wave 64 x 64 instead of 64 x 32: a third less LDS traffic per MFMA).
// T: storage type of activations and weights -- uint16_t (bf16, v_mfma_f32_16x16x32_bf16) or float
// (the fp32 precision path: v_mfma_f32_16x16x4_f32, four per 16-byte fragment; the LDS tile keeps
// its 128-byte rows, i.e. 32 fp32 reduction elements per K-step instead of 64 bf16).
// SKM: stream-K work decomposition (ConvArgs::sk_*): a persistent grid walks the flattened
// (phase, tile, K-step) iterations; tiles split between blocks are summed by their last-arriving
// contributor in a fixed block order (deterministic), exactly like the split-K combine.
// HALO: 3x3 / stride-1 / pad-1 convolutions (forward and stride-1 data gradient) by 2-D output tiles
// of th x tw pixels (th * tw <= 128 = BM) of one image: the (th + 2) x (tw + 2) input halo of a
// 64-channel chunk is staged ONCE and the 9 taps are 9 K-steps over it (only the weight tile is
// staged per tap) -- the K order is chunk-major, tap-minor.  An out-of-image halo pixel is staged as
// zeros, which is the zero padding of every tap; no per-tap im2col decode exists.
template <int BM, int BN, bool SMALLC, int STAGES, int NW, int WGM, int PRO = 0, typename ET = uint16_t,
          bool SKM = false, bool REPI = false, bool HALO = false>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(STAGES == 1 && BM * BN <= 16384 ? (BM * BN == 16384 ? DLMPI_W128 : 3) : 2, 8))) void conv_igemm_kernel(const ConvArgs a) {
  constexpr int NT = 64 * NW;                 // threads
  constexpr int WGN = NW / WGM;               // wave grid WGM x WGN
  using T = ET;                               // element (storage) type
  constexpr int ES = sizeof(T);               // bytes per element
  constexpr int BK = 128 / ES;                // reduction elements per K-step (one 128-B LDS row)
  constexpr int CPC = 16 / ES;                // channels per 16-byte chunk
  static_assert(PRO == 0 || ES == 2, "operand prologues: bf16 only");
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int RP = NT / 8;                  // tile rows staged per pass (8 lanes per 128-B row)
  constexpr int AL = BM / RP, BL = BN / RP;   // 16-byte pieces per thread per tile
  constexpr int HALO_ROWS = 192;              // (th + 2) * (tw + 2) <= 192 (host-checked)
  static_assert(!HALO || (BM == 128 && NW == 4 && !SMALLC && STAGES == 1 && PRO == 0 && !SKM && !REPI &&
                          sizeof(ET) == 2), "halo mode: 128-pixel bf16 single-stage tiles");
  constexpr int HL = HALO ? HALO_ROWS * 128 / (16 * 64 * NW) : 1;   // halo pieces per thread
  constexpr int A_BYTES = (HALO ? HALO_ROWS : BM) * 128, B_BYTES = BN * 128;
  static_assert(PRO == 0 || (!SMALLC && STAGES == 1), "operand prologue: regular channels, single stage");
  constexpr int Z_BYTES = PRO >= 2 ? A_BYTES : 0;   // the second prologue operand, staged like A
  constexpr int SB = A_BYTES + B_BYTES + Z_BYTES;   // bytes per stage: [A | B | Z]
  constexpr int STAGE_BYTES = STAGES * SB;
  constexpr int CS_LD = BN + 4;
  constexpr int NP = BM >= 128 ? BM / 64 : 1;            // epilogue passes of <= 64 tile rows
  static_assert(WM % (16 * NP) == 0 || NP == 1, "epilogue pass must split every wave's rows evenly");
  constexpr int EPI_BYTES = (BM / NP) * CS_LD * 4;
  constexpr int RED_BYTES = (NT / (BN / 8)) * 3 * BN * 4;    // stats combine
  // REPI: no fp32 tile staging; [WGM][3][BN] floats of statistics, or the in-launch finalize's
  // 2 x NT doubles + flag
  constexpr int REPI_BYTES = (WGM * 3 * BN * 4 > 2 * NT * 8 + 16) ? WGM * 3 * BN * 4 : 2 * NT * 8 + 16;
  constexpr int EPI_NEED = REPI ? REPI_BYTES : (EPI_BYTES > RED_BYTES ? EPI_BYTES : RED_BYTES);
  constexpr int SMEM = STAGE_BYTES > EPI_NEED ? STAGE_BYTES : EPI_NEED;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WGN, wn = wid % WGN;
  const int lrow = tid >> 3;                          // staging row (+RP i)
  const int jc = (tid & 7) ^ ((tid >> 4) & 7);        // swizzled 16-B chunk this lane fetches
  const char* zp = reinterpret_cast<const char*>(g_zero_page);

  // stream-K: this block's iteration range (XCD-remapped so one XCD walks a contiguous range)
  int sk_lb = 0, sk_it = 0, sk_end = 0;
  if constexpr (SKM) {
    sk_lb = (int)xcd_remap(blockIdx.x, gridDim.x);
    sk_it = sk_lb * a.sk_per;
    sk_end = min(a.sk_total, sk_it + a.sk_per);
  }
  for (;;) {   // SKM: one pass per tile segment of the range; otherwise exactly one pass
  int zph, seg_k0 = 0, seg_k1 = 0, seg_start = 0;
  uint32_t bid;
  if constexpr (SKM) {
    if (sk_it >= sk_end) break;
    zph = 0;
    while (zph + 1 < a.nphase && sk_it >= a.sk_base[zph + 1]) ++zph;
    const int nkz = a.ph[zph].ksteps;
    const int loc = sk_it - a.sk_base[zph];
    const int tl = loc / nkz;
    seg_k0 = loc - tl * nkz;
    seg_k1 = min(nkz, seg_k0 + (sk_end - sk_it));
    seg_start = sk_it;
    sk_it += seg_k1 - seg_k0;
    bid = (uint32_t)tl;
  } else {
    zph = blockIdx.z;
    const uint32_t nwg0 = (uint32_t)a.ph[zph].mtiles * (uint32_t)a.ntiles;
    if (blockIdx.x >= nwg0) return;
    bid = xcd_remap(blockIdx.x, nwg0);
  }
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

  // ---- per-thread row state (kept compact: the 256-row tile has 8 rows per thread) ----------
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
  uint32_t z_off[PRO >= 2 ? AL : 1];                  // the same pixel in the prologue's Z
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
      if constexpr (PRO >= 2) z_off[i] = (uint32_t)(a_pix[i] + doff) * (uint32_t)a.ldpz;
    }
  };
  const char* zlane = PRO >= 2 ? reinterpret_cast<const char*>(a.pz) + ES * ((int64_t)a.pzoff + CPC * jc) : nullptr;

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
  bool need_halo = true;
  auto tap_setup_halo = [&](int t) {
    const int tr = (int)fdiv((uint32_t)t, ph.fdTs);
    const int ts = t - tr * ph.Ts;
    const int dh = ph.dh0 + tr * ph.dhs, dw = ph.dw0 + ts * ph.dws;
    const int wt = (ph.wr0 + tr * ph.wrs) * a.S + (ph.ws0 + ts * ph.wss);
    wtC2 = wt * C * ES;
    toff = (dh + 1) * hwd + (dw + 1);
  };

  auto issue = [&](int buf, int ks) {
    char* As = smem + buf * SB;
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
      if constexpr (PRO >= 2) {
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

  // Operand prologue: this lane's own staged A pieces (row lrow + RP i, chunk jc = channels
  // c_cur + 8 jc of the current tap) are rewritten in place once the stage has landed; pieces of
  // out-of-image taps / rows past M hold zeros and are left alone.  Same fma order and bf16
  // rounding as the standalone kernels it replaces (bn_apply_kernel / bn_bwd_apply_kernel), so the
  // fused and the unfused schedules are bit-identical.
  auto prologue = [&](int buf) {
    if constexpr (PRO != 0) {
      char* As = smem + buf * SB;
      const int c = c_cur + 8 * jc;
      f32x4 k0a, k0b, k1a, k1b, k2a, k2b, kra, krb;
      if constexpr (PRO == 1 || PRO == 3) {
        k0a = *reinterpret_cast<const f32x4*>(a.pscale + c);
        k0b = *reinterpret_cast<const f32x4*>(a.pscale + c + 4);
        k1a = *reinterpret_cast<const f32x4*>(a.pshift + c);
        k1b = *reinterpret_cast<const f32x4*>(a.pshift + c + 4);
        if constexpr (PRO == 3) {
          if (a.prscale) {
            k2a = *reinterpret_cast<const f32x4*>(a.prscale + c);
            k2b = *reinterpret_cast<const f32x4*>(a.prscale + c + 4);
            kra = *reinterpret_cast<const f32x4*>(a.prshift + c);
            krb = *reinterpret_cast<const f32x4*>(a.prshift + c + 4);
          }
        }
      } else {
        k0a = *reinterpret_cast<const f32x4*>(a.pcoef + c);
        k0b = *reinterpret_cast<const f32x4*>(a.pcoef + c + 4);
        k1a = *reinterpret_cast<const f32x4*>(a.pcoef + C + c);
        k1b = *reinterpret_cast<const f32x4*>(a.pcoef + C + c + 4);
        k2a = *reinterpret_cast<const f32x4*>(a.pcoef + 2 * C + c);
        k2b = *reinterpret_cast<const f32x4*>(a.pcoef + 2 * C + c + 4);
      }
#pragma unroll
      for (int i = 0; i < AL; ++i) {
        if (!((a_vm >> i) & 1)) continue;
        u32x4* pa = reinterpret_cast<u32x4*>(As + RP * i * 128 + tid * 16);
        float v[8];
        unpack8(*pa, v);
        if constexpr (PRO == 1) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = fmaxf(__builtin_fmaf(v[e], k0a[e], k1a[e]), 0.f);
            v[e + 4] = fmaxf(__builtin_fmaf(v[e + 4], k0b[e], k1b[e]), 0.f);
          }
        } else if constexpr (PRO == 3) {
          // the producer block's BN-apply + residual + ReLU (bn_apply_kernel's arithmetic, same
          // order), written back as the A operand AND stored: y and its ReLU mask bits
          float r[8];
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
          continue;
        } else {
          float zv[8];
          unpack8(*reinterpret_cast<const u32x4*>(As + A_BYTES + B_BYTES + RP * i * 128 + tid * 16), zv);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = __builtin_fmaf(k0a[e], v[e], __builtin_fmaf(k1a[e], zv[e], k2a[e]));
            v[e + 4] = __builtin_fmaf(k0b[e], v[e + 4], __builtin_fmaf(k1b[e], zv[e + 4], k2b[e]));
          }
        }
        *pa = pack8(v);
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
    if constexpr (HALO) {   // chunk-major, tap-minor
      if (++t_cur == NTAP) {
        t_cur = 0;
        c_cur += BK;
        need_halo = true;
      }
      tap_setup_halo(t_cur);
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
  if constexpr (SKM) {
    kbeg = seg_k0;
    kend = seg_k1;
  } else if (a.splitk > 1) {
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
    issue(0, kbeg);
    __syncthreads();
    prologue(0);
  }
  for (int ks = kbeg; ks < kend; ++ks) {
    int cur = 0;
    if constexpr (STAGES == 2) {
      cur = (ks - kbeg) & 1;
      if (ks + 1 < kend) {
        advance();
        issue(cur ^ 1, ks + 1);
      }
    } else if (ks > kbeg) {
      advance();
      issue(0, ks);
      __syncthreads();   // this stage landed (vmcnt(0) + barrier)
      prologue(0);
    }
    const char* As = smem + cur * SB;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      typedef typename std::conditional<sizeof(T) == 2, bf16x8, f32x4>::type frag_t;
      frag_t af[TM], bfr[TN];
      const int ch = kk * 4 + fg;
#pragma unroll
      for (int mi = 0; mi < TM; ++mi) {
        int r;
        if constexpr (HALO) r = hb[mi] + toff;
        else r = wm * WM + mi * 16 + fr;
        af[mi] = *reinterpret_cast<const frag_t*>(As + r * 128 + ((ch ^ ((r >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int r = wn * WN + ni * 16 + fr;
        bfr[ni] = *reinterpret_cast<const frag_t*>(Bs + r * 128 + ((ch ^ ((r >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int mi = 0; mi < TM; ++mi)
#pragma unroll
        for (int ni = 0; ni < TN; ++ni) {
          if constexpr (sizeof(T) == 2) {
            // REPI: D^T (rows = output channels, columns = pixels) -- the 16x16x32 operand layouts of
            // A and B are symmetric, so swapping them transposes the tile: every lane then holds 4
            // consecutive CHANNELS of one pixel, i.e. a contiguous 8-byte piece of an NHWC row
            if constexpr (REPI)
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[ni], af[mi], acc[mi][ni], 0, 0, 0);
            else
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
    // STAGES 2: waits for this wave's glds of tile ks+1, then all waves -> buffers swap;
    // STAGES 1: every wave is done reading the stage before it is overwritten
    __syncthreads();
  }

  // ---- split-K combine (cdna_hip_programming.md "In-launch split-K reduction") --------------
  // Every slice stores its fp32 accumulators (fragment layout) to its slab, publishes with an
  // agent-scope release + ticket; the tile's last arriver acquires and sums ALL slices' slabs in
  // slice order (deterministic whichever block arrives last), then runs the normal epilogue.
  if constexpr (SKM) {
    if (kbeg != 0 || kend != nk) {
      // partial tile: store this block's accumulators write-through (sc1) into its slab slot
      // (0: the range's first segment, 1: its last), take a ticket; the last contributor sums the
      // slots of every contributing block in block order (deterministic) and runs the epilogue
      constexpr int NF = TM * TN;
      const int slot = seg_start == sk_lb * a.sk_per ? 0 : 1;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          a.sk_slab + (int64_t)(sk_lb * 2 + slot) * NF * NT * 4, (short)0, NF * NT * 16, 0x00020000);
#pragma unroll
      for (int i = 0; i < NF; ++i)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i / TN][i % TN]), rs,
                                               (i * NT + tid) * 16, 0, 16 /* sc1 */);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const int s_it = a.sk_base[zph] + (int)bid * nk;       // the tile's iteration range [s_it, s_it + nk)
      const int b_lo = s_it / a.sk_per, b_hi = (s_it + nk - 1) / a.sk_per;
      const int gt = a.sk_tbase[zph] + (int)bid;
      int* flag = reinterpret_cast<int*>(smem);
      if (tid == 0)
        flag[0] = __hip_atomic_fetch_add(a.sk_tk + gt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == b_hi - b_lo;
      __syncthreads();
      if (!flag[0]) continue;
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(a.sk_tk + gt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < NF; ++i) acc[i / TN][i % TN] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int b = b_lo; b <= b_hi; ++b) {
        const int sl = b * a.sk_per >= s_it ? 0 : 1;
        const f32x4* src = reinterpret_cast<const f32x4*>(a.sk_slab) + (int64_t)(b * 2 + sl) * NF * NT + tid;
#pragma unroll
        for (int i = 0; i < NF; ++i) acc[i / TN][i % TN] += src[(int64_t)i * NT];
      }
      __syncthreads();   // flag (LDS) is reused by the epilogue staging
    }
  } else if (a.splitk > 1) {
    constexpr int NF = TM * TN;
    const int S = a.splitk;
    // unique over phases (blockIdx.z): ConvTranspose phases all have tile_base 0
    const int64_t tile = (int64_t)blockIdx.z * gridDim.x + (int64_t)mt * a.ntiles + nt;
    f32x4* slab = reinterpret_cast<f32x4*>(a.sk_slab) + (tile * S + blockIdx.y) * NF * NT + tid;
#pragma unroll
    for (int i = 0; i < NF; ++i) slab[(int64_t)i * NT] = acc[i / TN][i % TN];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(smem);   // the one LDS array (no second __shared__ object)
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      flag[0] = __hip_atomic_fetch_add(a.sk_tk + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == S - 1;
    }
    __syncthreads();
    if (!flag[0]) return;
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(a.sk_tk + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const f32x4* base = reinterpret_cast<const f32x4*>(a.sk_slab) + tile * S * NF * NT + tid;
#pragma unroll
    for (int i = 0; i < NF; ++i) acc[i / TN][i % TN] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int sp = 0; sp < S; ++sp)
#pragma unroll
      for (int i = 0; i < NF; ++i) acc[i / TN][i % TN] += base[((int64_t)sp * NF + i) * NT];
    __syncthreads();   // flag (LDS) is reused by the epilogue staging
  }

  // ---- register-direct epilogue (REPI) --------------------------------------------------------
  // No LDS staging of the fp32 tile: lane (fr, fg) holds, for pixel tile mi and channel tile ni,
  // output[pixel wm*WM + 16 mi + fr][channels wn*WN + 16 ni + 4 fg + 0..3] (D^T fragments), so the
  // epilogue math runs in registers and every lane stores / loads 8-byte channel quads directly.
  // BatchNorm partial sums: per lane over its pixels, then over the 16 lanes of a DPP row
  // (row_shr prefix chain, fixed order), then over the wave rows through a small LDS array.
  if constexpr (REPI) {
    static_assert(sizeof(T) == 2 && PRO == 0, "register epilogue: bf16, no operand prologue");
    const int fr = lane & 15, fg = lane >> 4;
    const bool bwd = a.mask != nullptr || a.mscale != nullptr || a.mbits != nullptr;
    const int ns = a.nstat;
    float s1[TN][4], s2[TN][4], s3[TN][4];
#pragma unroll
    for (int ni = 0; ni < TN; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) { s1[ni][r] = 0.f; s2[ni][r] = 0.f; s3[ni][r] = 0.f; }
    auto ld4 = [](const void* base, int64_t off) -> f32x4 {
      const u32x2 q = *reinterpret_cast<const u32x2*>(static_cast<const uint16_t*>(base) + off);
      return f32x4{__uint_as_float(q[0] << 16), __uint_as_float(q[0] & 0xffff0000u), __uint_as_float(q[1] << 16),
                   __uint_as_float(q[1] & 0xffff0000u)};
    };
#pragma unroll
    for (int mi = 0; mi < TM; ++mi) {
      const int m = m0 + wm * WM + mi * 16 + fr;
      if (m >= M) continue;
      const uint32_t n_img = fdiv((uint32_t)m, ph.fdPQ);
      const uint32_t rem = (uint32_t)m - n_img * PQ;
      const uint32_t p = fdiv(rem, ph.fdQ);
      const uint32_t q = rem - p * ph.Q;
      const int64_t pix = ((int64_t)n_img * a.OH + (int)p * a.so + ph.oh0) * a.OW + (int)q * a.so + ph.ow0;
#pragma unroll
      for (int ni = 0; ni < TN; ++ni) {
        const int c = n0 + wn * WN + ni * 16 + 4 * fg;
        if (c >= a.Kout) continue;   // Kout % 8 == 0: a quad is all in or all out
        f32x4 v = acc[mi][ni];
        if (a.bias) v += *reinterpret_cast<const f32x4*>(a.bias + c);
        if (a.stats && !bwd) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float rv = stored<T>(v[r]);
            s1[ni][r] += rv;
            s2[ni][r] += rv * rv;
          }
        }
        if (a.scale) v = v * *reinterpret_cast<const f32x4*>(a.scale + c) + *reinterpret_cast<const f32x4*>(a.shift + c);
        if (a.res) v += ld4(a.res, pix * a.ldres + a.resoff + c);
        if (a.relu) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
        }
        if (bwd) {
          f32x4 zz = f32x4{0.f, 0.f, 0.f, 0.f};
          if (a.z) zz = ld4(a.z, pix * a.ldz + a.zoff + c);
          if (a.mbits) {
            const uint32_t b = a.mbits[pix * (a.Kout >> 3) + (c >> 3)] >> (c & 7);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = (b >> r) & 1u ? v[r] : 0.f;
          } else if (a.mask) {
            const f32x4 yy = ld4(a.mask, pix * a.ldmask + a.maskoff + c);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = yy[r] > 0.f ? v[r] : 0.f;
          } else {   // same fma as the forward BN-apply -> same sign as y
            const f32x4 ms = *reinterpret_cast<const f32x4*>(a.mscale + c);
            const f32x4 mh = *reinterpret_cast<const f32x4*>(a.mshift + c);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = zz[r] * ms[r] + mh[r] > 0.f ? v[r] : 0.f;
          }
          if (a.stats) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float rv = stored<T>(v[r]);
              s1[ni][r] += rv;
              s2[ni][r] += rv * zz[r];
            }
            if (a.z2) {
              const f32x4 z2 = ld4(a.z2, pix * a.ldz2 + a.z2off + c);
#pragma unroll
              for (int r = 0; r < 4; ++r) s3[ni][r] += stored<T>(v[r]) * z2[r];
            }
          }
        }
        if (a.out_f32) {
          *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(a.y) + pix * a.ldy + a.yoff + c) = v;
        } else {
          const u32x2 pk = u32x2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
          u32x2* yp = reinterpret_cast<u32x2*>(reinterpret_cast<uint16_t*>(a.y) + pix * a.ldy + a.yoff + c);
          if (a.nt_store) __builtin_nontemporal_store(pk, yp);
          else *yp = pk;
        }
      }
    }
    if (a.stats) {
      // sum over the 16 pixel lanes of each DPP row: lane 15 of the row ends with the full sum
      auto row_sum = [](float v) {
        v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xf, 0xf, true));
        v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x112, 0xf, 0xf, true));
        v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x114, 0xf, 0xf, true));
        v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x118, 0xf, 0xf, true));
        return v;
      };
      float* red = reinterpret_cast<float*>(smem);   // [WGM][3][BN]
      __syncthreads();   // the K loop's last LDS reads are done
#pragma unroll
      for (int ni = 0; ni < TN; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float t1 = row_sum(s1[ni][r]), t2 = row_sum(s2[ni][r]);
          const float t3 = ns > 2 ? row_sum(s3[ni][r]) : 0.f;
          if (fr == 15) {
            const int cl = wn * WN + ni * 16 + 4 * fg + r;
            red[(wm * 3 + 0) * BN + cl] = t1;
            red[(wm * 3 + 1) * BN + cl] = t2;
            red[(wm * 3 + 2) * BN + cl] = t3;
          }
        }
      __syncthreads();
      const bool fin = !SKM && a.fin_on;
      if (tid < BN && n0 + tid < a.Kout) {
        float t1 = 0.f, t2 = 0.f, t3 = 0.f;
#pragma unroll
        for (int g = 0; g < WGM; ++g) {
          t1 += red[(g * 3 + 0) * BN + tid];
          t2 += red[(g * 3 + 1) * BN + tid];
          t3 += red[(g * 3 + 2) * BN + tid];
        }
        float* st = a.stats + (int64_t)(ph.tile_base + mt) * ns * a.Kout + n0 + tid;
        if (fin) {
          st_sc1(st, t1);
          st_sc1(st + a.Kout, t2);
          if (ns > 2) st_sc1(st + 2 * a.Kout, t3);
        } else {
          st[0] = t1;
          st[a.Kout] = t2;
          if (ns > 2) st[2 * a.Kout] = t3;
        }
      }
      if (fin) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        fin_in_launch<NT, BN>(a, a.stats, ns, ph.tile_base + mt, nt, n0, reinterpret_cast<double*>(smem),
                              reinterpret_cast<int*>(smem + 2 * NT * sizeof(double)));
      }
    }
  } else {
  // ---- epilogue ------------------------------------------------------------------------------
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
  if (h) __syncthreads();         // every thread is done with pass 0
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
      float rr[8];
      load8(static_cast<const T*>(a.res) + pix * a.ldres + a.resoff + c0, rr);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += rr[e];
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
        if (a.nt_store) __builtin_nontemporal_store(pack8(v), reinterpret_cast<u32x4*>(yp));
        else *reinterpret_cast<u32x4*>(yp) = pack8(v);
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
    const bool fin = !SKM && a.fin_on;
    if (tid < BN && n0 + tid < a.Kout) {
      float t1 = 0.f, t2 = 0.f, t3 = 0.f;
      for (int g = 0; g < RG; ++g) {
        t1 += red[(g * 3 + 0) * BN + tid];
        t2 += red[(g * 3 + 1) * BN + tid];
        t3 += red[(g * 3 + 2) * BN + tid];
      }
      float* st = a.stats + (int64_t)(ph.tile_base + mt) * ns * a.Kout + n0 + tid;
      if (fin) {   // published write-through for the in-launch finalize (bnfin.h)
        st_sc1(st, t1);
        st_sc1(st + a.Kout, t2);
        if (ns > 2) st_sc1(st + 2 * a.Kout, t3);
      } else {
        st[0] = t1;
        st[a.Kout] = t2;
        if (ns > 2) st[2 * a.Kout] = t3;
      }
    }
    if (fin) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its row stores
      __syncthreads();                                   // (also: red is free again)
      fin_in_launch<NT, BN>(a, a.stats, ns, ph.tile_base + mt, nt, n0, reinterpret_cast<double*>(smem),
                            reinterpret_cast<int*>(smem + 2 * NT * sizeof(double)));
    }
  }
  }   // LDS epilogue
  if constexpr (!SKM) break;
  __syncthreads();   // LDS (epilogue staging / stats) is reused by the next segment's staging
  }   // segment loop
}

}  // namespace dlmpi

using namespace dlmpi;

static int stages_choice() {
  static int v = [] {
    const char* e = getenv("DLMPI_CONV_STAGES");
    return e ? atoi(e) : 1;
  }();
  return v;
}

// DLMPI_CONV_REPI: 1 = register-direct epilogue (D^T fragments, no LDS staging of the output tile)
// for bf16 launches without operand prologue and with full-width vector stores; 0 (default) = the
// LDS-staged epilogue.  Measured slower (profiles/r3_repi_rejected): per-network forward 4.86 vs
// 4.70 ms, the memory-bound expand 1x1s +9..15 % (8-byte lane pieces make each store instruction
// cover 16 rows x 32 B instead of 4 rows x 256 B), ResNet-50 step 10.8k vs 12.0k img/s (the masked
// data-gradient epilogues' 8-byte z / mask loads).
static int g_repi_override = -1;
static bool repi_on(const ConvArgs* a) {
  static const int v = [] {
    const char* e = getenv("DLMPI_CONV_REPI");
    return e ? atoi(e) : 0;
  }();
  const int m = g_repi_override >= 0 ? g_repi_override : v;
  return m != 0 && !a->f32 && a->pro == 0 && a->vec_store && a->kvalid == a->Kout && a->Kout % 8 == 0;
}
extern "C" void dlmpi_set_conv_repi(int mode) { g_repi_override = mode; }

template <int BM, int BN>
static void launch_tile(const ConvArgs* a, dim3 grid, hipStream_t s) {
  const bool one = stages_choice() == 1;
  if (one && repi_on(a)) {
    if (a->C < 64) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, true, 1, 4, 2, 0, uint16_t, false, true>), grid, dim3(256), 0, s, *a);
    else hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, false, 1, 4, 2, 0, uint16_t, false, true>), grid, dim3(256), 0, s, *a);
    return;
  }
  if (a->pro == 1) {
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, false, 1, 4, 2, 1>), grid, dim3(256), 0, s, *a);
    return;
  }
  if (a->pro == 2) {
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, false, 1, 4, 2, 2>), grid, dim3(256), 0, s, *a);
    return;
  }
  if (a->pro == 3) {
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, false, 1, 4, 2, 3>), grid, dim3(256), 0, s, *a);
    return;
  }
  if (a->C < 64) {
    if (one) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, true, 1, 4, 2>), grid, dim3(256), 0, s, *a);
    else hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, true, 2, 4, 2>), grid, dim3(256), 0, s, *a);
  } else {
    if (one) hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, false, 1, 4, 2>), grid, dim3(256), 0, s, *a);
    else hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, false, 2, 4, 2>), grid, dim3(256), 0, s, *a);
  }
}

// Split-K plan for small grids (ResNet-18 on 32x32 CIFAR: layer4 is 1x1 pixels, 8 tiles x 72
// K-steps): slices so that tiles x slices reaches ~256 blocks, >= 4 K-steps per slice, <= 8 slices.
// DLMPI_CONV_SPLITK=0 disables.  Slabs (fp32) and tickets come per stream role (bn.hip), so the
// main and the branch stream can run split convolutions concurrently.
static int splitk_plan(int tiles, int nk) {
  static const int on = [] {
    const char* e = getenv("DLMPI_CONV_SPLITK");
    return e ? atoi(e) : 1;
  }();
  if (!on || tiles >= 256 || nk < 8) return 1;
  int S = (256 + tiles - 1) / tiles;
  S = S < nk / 4 ? S : nk / 4;
  S = S < 8 ? S : 8;
  return S < 2 ? 1 : S;
}

// ---- stream-K planning --------------------------------------------------------------------------
// A launch of T tiles on a chip holding `slots` resident blocks takes ceil(T / slots) tile-times; at
// ResNet-50 bs 256 many layers sit just above a multiple (784 tiles of 14^2 x 256 channels on 768
// slots: 2 tile-times for 1.02 tiles of work each, measured +48 % vs 248 images).  Stream-K runs
// exactly `slots` persistent blocks over the flattened (tile, K-step) iterations instead; a tile cut
// between two blocks costs one slab round trip + a ticket (sk_time below: + 0.15 tile-times).
static int cu_count() {
  static const int n = [] {
    int d = 0, v = 0;
    if (hipGetDevice(&d) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess)
      v = 256;
    return v > 0 ? v : 256;
  }();
  return n;
}

template <int BM, int BN>
static int sk_occupancy() {   // resident blocks per CU of the stream-K instance
  static const int occ = [] {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, conv_igemm_kernel<BM, BN, false, 1, 4, 2, 0, uint16_t, true>,
                                                     256, 0) != hipSuccess || n < 1)
      n = 2;
    return n;
  }();
  return occ;
}

static int g_sk_override = -1;   // dlmpi_set_conv_sk (tests); -1: the environment decides
static int g_sk_last = 0;        // 1 if the last conv launch ran stream-K (tests)
// DLMPI_CONV_SK: 0 off (default), 1 auto, 2 whenever applicable (tests).  Measured slower on every
// targeted ResNet-50 shape (profiles/r2_streamk_rejected): with ~1 iteration range per tile almost
// every tile is cut, and the 64 KB fp32 partials per cut tile cost more than the wave tail saved.
static int sk_mode_env() {
  static const int v = [] {
    const char* e = getenv("DLMPI_CONV_SK");
    return e ? atoi(e) : 0;
  }();
  return g_sk_override >= 0 ? g_sk_override : v;
}

extern "C" void dlmpi_set_conv_sk(int mode) { g_sk_override = mode; }
extern "C" int dlmpi_conv_sk_last() { return g_sk_last; }

// fp32 precision path: single-stage 4-wave tiles up to 128 x 128 (the f32 MFMA is 1/16 of the
// bf16 rate, so the wider bf16 tiles buy nothing here)
static hipError_t launch_f32(const ConvArgs* a, int bm, int bn, dim3 grid, hipStream_t s) {
  if (a->pro != 0) return hipErrorInvalidValue;
  // the regular staging walks whole 32-channel K-steps per tap; anything else stages per 16-B piece
  const bool small = a->C < 32 || a->C % 32 != 0;
#define DLMPI_F32(BM_, BN_)                                                                                        \
  do {                                                                                                            \
    if (small) hipLaunchKernelGGL((conv_igemm_kernel<BM_, BN_, true, 1, 4, 2, 0, float>), grid, dim3(256), 0, s, *a); \
    else hipLaunchKernelGGL((conv_igemm_kernel<BM_, BN_, false, 1, 4, 2, 0, float>), grid, dim3(256), 0, s, *a);     \
  } while (0)
  if (bm == 128 && bn == 128) DLMPI_F32(128, 128);
  else if (bm == 128 && bn == 64) DLMPI_F32(128, 64);
  else if (bm == 64 && bn == 128) DLMPI_F32(64, 128);
  else if (bm == 64 && bn == 64) DLMPI_F32(64, 64);
  else return hipErrorInvalidValue;
#undef DLMPI_F32
  return hipGetLastError();
}

extern "C" hipError_t dlmpi_conv_igemm(const ConvArgs* a_in, int bm, int bn, hipStream_t s) {
  int maxt = 0, tiles = 0, maxk = 0;
  for (int i = 0; i < a_in->nphase; ++i) {
    maxt = a_in->ph[i].mtiles > maxt ? a_in->ph[i].mtiles : maxt;
    tiles += a_in->ph[i].mtiles * a_in->ntiles;
    maxk = a_in->ph[i].ksteps > maxk ? a_in->ph[i].ksteps : maxk;
  }
  ConvArgs ab = *a_in;
  const ConvArgs* a = &ab;
  ab.splitk = 1;
  g_sk_last = 0;
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
  // stream-K: regular channel counts, no prologue, the single-stage 4-wave tiles
  const int skm = sk_mode_env();
  const bool sk_tile = (bm == 128 && (bn == 128 || bn == 64)) || (bm == 64 && (bn == 128 || bn == 64)) ||
                       (bm == 256 && bn == 128);
  bool kzero = false;
  int iters = 0;
  for (int i = 0; i < a_in->nphase; ++i) {
    kzero |= a_in->ph[i].ksteps == 0;
    iters += a_in->ph[i].mtiles * a_in->ntiles * a_in->ph[i].ksteps;
  }
  if (skm && !a->fin_on && ab.splitk == 1 && sk_tile && a->pro == 0 && a->C >= 64 && stages_choice() == 1 && !kzero &&
      tiles <= 4096 && iters > 0) {
    int occ = 2;
    if (bm == 128 && bn == 128) occ = sk_occupancy<128, 128>();
    else if (bm == 128) occ = sk_occupancy<128, 64>();
    else if (bm == 64 && bn == 128) occ = sk_occupancy<64, 128>();
    else if (bm == 64) occ = sk_occupancy<64, 64>();
    else occ = sk_occupancy<256, 128>();
    const int slots = cu_count() * occ;
    const int G = tiles < slots ? (tiles * 2 < slots ? 0 : slots) : slots;   // < half a wave: leave it
    if (G > 0) {
      const int per = (iters + G - 1) / G;
      const double now = (double)((tiles + slots - 1) / slots);
      const double sk = (double)per * tiles / iters + 0.15;
      if (skm == 2 || sk < 0.85 * now) {
        const int Ge = (iters + per - 1) / per;
        float* slab = dlmpi_splitk_slab(s, (size_t)Ge * 2 * bm * bn);
        int* tk = dlmpi_splitk_tickets(s, tiles);
        if (slab && tk) {
          ab.sk_mode = 1;
          ab.sk_per = per;
          ab.sk_total = iters;
          ab.sk_slab = slab;
          ab.sk_tk = tk;
          int it = 0, tb = 0;
          for (int i = 0; i < a_in->nphase; ++i) {
            ab.sk_base[i] = it;
            ab.sk_tbase[i] = tb;
            it += a_in->ph[i].mtiles * a_in->ntiles * a_in->ph[i].ksteps;
            tb += a_in->ph[i].mtiles * a_in->ntiles;
          }
          ab.sk_base[a_in->nphase] = it;
          const dim3 g((unsigned)Ge, 1, 1);
#define DLMPI_SK(BM_, BN_) \
  hipLaunchKernelGGL((conv_igemm_kernel<BM_, BN_, false, 1, 4, 2, 0, uint16_t, true>), g, dim3(256), 0, s, *a)
          if (bm == 128 && bn == 128) DLMPI_SK(128, 128);
          else if (bm == 128) DLMPI_SK(128, 64);
          else if (bm == 64 && bn == 128) DLMPI_SK(64, 128);
          else if (bm == 64) DLMPI_SK(64, 64);
          else DLMPI_SK(256, 128);
#undef DLMPI_SK
          g_sk_last = 1;
          return hipGetLastError();
        }
      }
    }
  }
  if (a->halo) {   // 3x3 / stride 1 / pad 1 by 2-D tiles with a staged halo (host-planned)
    if (a->pro != 0 || bm != 128 || a->C % 64 != 0 || a->sk_mode) return hipErrorInvalidValue;
    if (bn == 128) hipLaunchKernelGGL((conv_igemm_kernel<128, 128, false, 1, 4, 2, 0, uint16_t, false, false, true>), grid, dim3(256), 0, s, *a);
    else if (bn == 64) hipLaunchKernelGGL((conv_igemm_kernel<128, 64, false, 1, 4, 2, 0, uint16_t, false, false, true>), grid, dim3(256), 0, s, *a);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (a->pro != 0 && (a->C < 64 || a->C % 64 != 0 || (bm == 256 && bn == 256))) return hipErrorInvalidValue;
  if (bm == 256 && bn == 256) {   // 8 waves, double-buffered; regular channel counts only
    if (a->C < 64) return hipErrorInvalidValue;
    if (repi_on(a)) hipLaunchKernelGGL((conv_igemm_kernel<256, 256, false, 2, 8, 2, 0, uint16_t, false, true>), grid, dim3(512), 0, s, *a);
    else hipLaunchKernelGGL((conv_igemm_kernel<256, 256, false, 2, 8, 2>), grid, dim3(512), 0, s, *a);
  } else if (bm == 256 && bn == 64) {   // 64-channel layers: 4 x 1 waves of 64 x 64
    if (a->pro == 0 && repi_on(a)) {
      if (a->C < 64) hipLaunchKernelGGL((conv_igemm_kernel<256, 64, true, 1, 4, 4, 0, uint16_t, false, true>), grid, dim3(256), 0, s, *a);
      else hipLaunchKernelGGL((conv_igemm_kernel<256, 64, false, 1, 4, 4, 0, uint16_t, false, true>), grid, dim3(256), 0, s, *a);
    } else if (a->pro == 1) hipLaunchKernelGGL((conv_igemm_kernel<256, 64, false, 1, 4, 4, 1>), grid, dim3(256), 0, s, *a);
    else if (a->pro == 2) hipLaunchKernelGGL((conv_igemm_kernel<256, 64, false, 1, 4, 4, 2>), grid, dim3(256), 0, s, *a);
    else if (a->pro == 3) hipLaunchKernelGGL((conv_igemm_kernel<256, 64, false, 1, 4, 4, 3>), grid, dim3(256), 0, s, *a);
    else if (a->C < 64) hipLaunchKernelGGL((conv_igemm_kernel<256, 64, true, 1, 4, 4>), grid, dim3(256), 0, s, *a);
    else hipLaunchKernelGGL((conv_igemm_kernel<256, 64, false, 1, 4, 4>), grid, dim3(256), 0, s, *a);
  } else if (bm == 128 && bn == 256) {   // short reductions, wide outputs: 8 waves (2 x 4 of 64 x 64)
    if (a->C < 64 || a->pro != 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL((conv_igemm_kernel<128, 256, false, 1, 8, 2>), grid, dim3(512), 0, s, *a);
  } else if (bm == 256 && bn == 128) launch_tile<256, 128>(a, grid, s);
  else if (bm == 128 && bn == 128) launch_tile<128, 128>(a, grid, s);
  else if (bm == 128 && bn == 64) launch_tile<128, 64>(a, grid, s);
  else if (bm == 64 && bn == 128) launch_tile<64, 128>(a, grid, s);
  else if (bm == 64 && bn == 64) launch_tile<64, 64>(a, grid, s);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}
