// Shared device helpers for the gfx950 (CDNA4 / MI355X) kernels.
//
// Conventions used by every kernel in this directory:
//   * activations are NHWC, bf16 stored as uint16_t (or fp32 on the fp32 precision path: the
//     kernels are templated on the storage type), channel count a multiple of 8 so one vector
//     = 8 consecutive channels of one pixel;
//   * master weights / gradients / BN statistics are fp32;
//   * all launchers are `extern "C"` and take an explicit hipStream_t so they can be
//     captured into a hipGraph (no allocation, no synchronisation inside a launcher).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "dlmpi_kernels.h"

namespace dlmpi {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// Round-to-nearest-even f32 -> bf16 (hipcc lowers the cast to v_cvt_pk_bf16_f32, NaN-preserving).
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}

__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

// 8 bf16 packed in a u32x4 <-> 8 floats.
__device__ __forceinline__ void unpack8(const u32x4 v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ u32x4 pack8(const float* f) {
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = pack2bf(f[2 * i], f[2 * i + 1]);
  return r;
}

// Storage-type-generic access to 8 consecutive channels (activations are bf16 -- stored as
// uint16_t -- or, for the fp32 precision path, float).  The arithmetic is always fp32.
__device__ __forceinline__ void load8(const uint16_t* p, float* f) { unpack8(*reinterpret_cast<const u32x4*>(p), f); }
__device__ __forceinline__ void load8(const float* p, float* f) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
  for (int e = 0; e < 4; ++e) { f[e] = a[e]; f[e + 4] = b[e]; }
}
__device__ __forceinline__ void store8(uint16_t* p, const float* f) { *reinterpret_cast<u32x4*>(p) = pack8(f); }
__device__ __forceinline__ void store8(float* p, const float* f) {
  *reinterpret_cast<f32x4*>(p) = f32x4{f[0], f[1], f[2], f[3]};
  *reinterpret_cast<f32x4*>(p + 4) = f32x4{f[4], f[5], f[6], f[7]};
}
__device__ __forceinline__ void store1(uint16_t* p, float v) { *p = f2bf(v); }
__device__ __forceinline__ void store1(float* p, float v) { *p = v; }
__device__ __forceinline__ float load1(const uint16_t* p) { return bf2f(*p); }
__device__ __forceinline__ float load1(const float* p) { return *p; }
// Raw 8-channel vector of storage type T (kept packed while loads are in flight).
struct f32x4x2 {
  f32x4 a, b;
};
template <typename T> struct Vec8;
template <> struct Vec8<uint16_t> { typedef u32x4 type; };
template <> struct Vec8<float> { typedef f32x4x2 type; };
template <typename T>
__device__ __forceinline__ typename Vec8<T>::type raw8(const T* p) {
  return *reinterpret_cast<const typename Vec8<T>::type*>(p);
}
__device__ __forceinline__ void unpack8(const f32x4x2& v, float* f) {
#pragma unroll
  for (int e = 0; e < 4; ++e) { f[e] = v.a[e]; f[e + 4] = v.b[e]; }
}
// the value as stored in T (statistics are taken of stored values)
template <typename T>
__device__ __forceinline__ float stored(float v) {
  if constexpr (sizeof(T) == 2) return bf2f(f2bf(v));
  else return v;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (__umulhi(n, f.mul) + n) >> f.shr;
}

// Bijective XCD-aware block remap (cdna_hip_programming.md T1): blocks b and b+8 share an XCD
// (observed round-robin dispatch); give each XCD a contiguous range of logical tiles so that
// tiles sharing an operand panel share that XCD's L2.  Pure speed choice, never correctness.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t bid, uint32_t nwg) {
  if (nwg < 16) return bid;
  const uint32_t xcd = bid & 7, idx = bid >> 3;
  const uint32_t q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double warp_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// 16-byte LDS-DMA piece (global_load_lds_dwordx4) issued from inline asm, so the compiler does not
// know it is in flight.  With the builtin, hipcc puts `s_waitcnt vmcnt(0)` in front of every
// ds_read_b64_tr_b16 that follows a DMA issue (the transposing read carries no memory operand the
// waitcnt pass could disambiguate), which drains every prefetch before the first fragment read of
// the K-step: the weight-gradient kernels' double buffer hid no DMA latency at all.  Callers own
// the wait (`s_waitcnt vmcnt(N)` + barrier before the stage is read) and must not mix this with
// the builtin in one kernel (M0 is set here and nowhere tracked).  `lds` is the wave's 1 KB
// destination (wave-uniform); lane i writes lds + 16 i.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"   // m0 is reserved: the clobber documents, it does not save
__device__ __forceinline__ void glds16_raw(const void* g, const char* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)lds);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(l) : "memory", "m0");
}
#pragma clang diagnostic pop

// 4 KiB of zeros: out-of-bounds im2col / tile pieces load from here instead of branching
// around the load (keeps the staging loads unconditional).
static __device__ u32x4 g_zero_page[16] = {};

}  // namespace dlmpi
