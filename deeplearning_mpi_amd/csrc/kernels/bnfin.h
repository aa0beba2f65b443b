// BatchNorm finalize bodies shared by the standalone colsum kernels (bn.hip) and the in-launch
// finalize of the implicit-GEMM conv epilogue (conv_igemm.hip).
//
// In-launch finalize (ConvArgs::fin_on): the conv epilogue's per-tile statistics rows
// [T][ns][Kout] are summed by the LAUNCH ITSELF instead of a separate colsum_fin launch between
// the conv and the BN-apply that needs scale / shift -- that launch and its kernel boundary sat on
// the critical path of every training BN (96 per ResNet-50 step, ~11 us each).  Two-level,
// deterministic last-arriver tree (no waiting, no float atomics):
//   level 1: the T stats tiles of a column block (N-tile) form groups of G consecutive tiles; the
//            block whose arrival ticket completes its group sums the group's G rows in tile order
//            and publishes the group sum (fp64);
//   level 2: the block that completes the last group of its N-tile sums the group sums in group
//            order and finalizes the N-tile's channels (fin_fwd / fin_bwd).
// Hand-off protocol (MI355X_MICROARCH.md "Valid forms", table row 1): every published byte is
// stored write-through (sc1, agent-scope relaxed atomic stores), every storing wave drains
// (s_waitcnt vmcnt(0)) before the workgroup barrier and ONE lane's agent-scope ticket add; the
// block whose add returned last reads the bytes with sc1 loads only.  No release/acquire fence:
// a release would write back the XCD L2's dirty lines, i.e. the megabytes of conv output the
// launch just produced.  Tickets self-reset (the last arriver zeroes its ticket).
#pragma once
#include "common.h"

namespace dlmpi {

__device__ __forceinline__ void fin_fwd(const FinArgs& f, int c, double s1, double s2) {
  const double mean = s1 / f.count;
  double var = s2 / f.count - mean * mean;
  if (var < 0.0) var = 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)f.eps));
  const float g = f.gamma ? f.gamma[c] : 1.f;
  const float b = f.beta ? f.beta[c] : 0.f;
  const float sc = g * invstd;
  f.scale[c] = sc;
  f.shift[c] = b - (float)mean * sc;
  if (f.save_mean) f.save_mean[c] = (float)mean;
  if (f.save_invstd) f.save_invstd[c] = invstd;
  if (f.running_mean) {
    const double unbiased = f.count > 1.0 ? var * f.count / (f.count - 1.0) : var;
    f.running_mean[c] = (1.f - f.momentum) * f.running_mean[c] + f.momentum * (float)mean;
    f.running_var[c] = (1.f - f.momentum) * f.running_var[c] + f.momentum * (float)unbiased;
  }
}

// coef[0..2][C] = (k1, k2, k3) with dx = k1*dyr + k2*x + k3; dgamma/dbeta accumulate.
__device__ __forceinline__ void fin_bwd(const FinArgs& f, int c, double s1, double s2, int C) {
  // raw_z: the second sum is sum dyr*z (BN input), not sum dyr*xhat
  if (f.raw_z) s2 = (double)f.invstd[c] * (s2 - (double)f.mean[c] * s1);
  if (f.dbeta) f.dbeta[c] += (float)s1;
  if (f.dgamma) f.dgamma[c] += (float)s2;
  if (f.coef) {
    const double is = f.invstd[c];
    const double k1 = (f.gamma ? (double)f.gamma[c] : 1.0) * is;
    const double k2 = -k1 * is * s2 / f.count;
    const double k3 = -k1 * s1 / f.count - k2 * (double)f.mean[c];
    f.coef[c] = (float)k1;
    f.coef[C + c] = (float)k2;
    f.coef[2 * C + c] = (float)k3;
  }
}

typedef __attribute__((address_space(1))) int fin_gi32_t;
typedef __attribute__((address_space(1))) unsigned long long fin_gu64_t;

__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store((fin_gi32_t*)p, __float_as_int(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __int_as_float(__hip_atomic_load((fin_gi32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store((fin_gu64_t*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load((fin_gu64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// Called by EVERY block of the launch that produced stats row `row` (global stats tile index) for
// channels [n0, n0 + BN) of N-tile `nt`, after the row was stored with st_sc1 and drained by every
// storing wave and a workgroup barrier.  NT threads; red: >= NT*2 doubles of LDS scratch, flag: an
// LDS int (both free to reuse).  Rows are [T][ns][Kout]; the two summed rows are 0 and k2.
template <int NT, int BN>
__device__ __forceinline__ void fin_in_launch(const ConvArgs& a, const float* stats, int ns, int row, int nt, int n0,
                                              double* red, int* flag) {
  static_assert(NT % BN == 0, "row lanes");
  constexpr int L = NT / BN;                       // row lanes per channel
  const int tid = threadIdx.x;
  const int cl = tid % BN, rl = tid / BN;
  const int c = n0 + cl;
  const int K = a.Kout;
  const int G = a.fin_group, NG = a.fin_ngroups;
  const int g = row / G;
  const int r0 = g * G, r1 = min(a.fin_T, r0 + G);
  int* gtk = a.fin_tk + nt * NG + g;
  int* ttk = a.fin_tk + a.ntiles * NG + nt;
  if (tid == 0) *flag = __hip_atomic_fetch_add((fin_gi32_t*)gtk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == r1 - r0 - 1;
  __syncthreads();
  if (!*flag) return;
  if (tid == 0) __hip_atomic_store((fin_gi32_t*)gtk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // level 1: this group's rows, lane rl takes rows r0 + rl, r0 + rl + L, ... (all loads issued first)
  double s1 = 0.0, s2 = 0.0;
  if (c < K) {
    const int k2 = a.fin_k2;
#pragma unroll 4
    for (int r = r0 + rl; r < r1; r += L) {
      const float* p = stats + (int64_t)r * ns * K + c;
      s1 += (double)ld_sc1(p);
      s2 += (double)ld_sc1(p + (int64_t)k2 * K);
    }
  }
  red[(0 * L + rl) * BN + cl] = s1;
  red[(1 * L + rl) * BN + cl] = s2;
  __syncthreads();
  if (rl == 0 && c < K) {
#pragma unroll
    for (int q = 1; q < L; ++q) {
      s1 += red[(0 * L + q) * BN + cl];
      s2 += red[(1 * L + q) * BN + cl];
    }
    st_sc1(a.fin_gsum + ((int64_t)g * 2 + 0) * K + c, s1);
    st_sc1(a.fin_gsum + ((int64_t)g * 2 + 1) * K + c, s2);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) *flag = __hip_atomic_fetch_add((fin_gi32_t*)ttk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == NG - 1;
  __syncthreads();
  if (!*flag) return;
  if (tid == 0) __hip_atomic_store((fin_gi32_t*)ttk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // level 2: every group's sum of these channels, in group order per lane, lanes combined in order
  s1 = 0.0;
  s2 = 0.0;
  if (c < K) {
#pragma unroll 4
    for (int q = rl; q < NG; q += L) {
      s1 += ld_sc1(a.fin_gsum + ((int64_t)q * 2 + 0) * K + c);
      s2 += ld_sc1(a.fin_gsum + ((int64_t)q * 2 + 1) * K + c);
    }
  }
  __syncthreads();   // red is reused
  red[(0 * L + rl) * BN + cl] = s1;
  red[(1 * L + rl) * BN + cl] = s2;
  __syncthreads();
  if (rl == 0 && c < K) {
#pragma unroll
    for (int q = 1; q < L; ++q) {
      s1 += red[(0 * L + q) * BN + cl];
      s2 += red[(1 * L + q) * BN + cl];
    }
    if (a.fin.mode == 0) fin_fwd(a.fin, c, s1, s2);
    else fin_bwd(a.fin, c, s1, s2, K);
  }
}

}  // namespace dlmpi
