// Small device utilities that keep the per-step glue of the training step on our own kernels
// (no ATen fill / index / cat / add launches between the engine's kernels):
//   * fill of an fp32 buffer (gradient-arena zeroing, scratch init),
//   * int64 add of a constant (every BatchNorm's num_batches_tracked in one launch),
//   * indexed gather dst[i] (+)= src[idx[i]] over 2- or 4-byte elements (weight re-layouts built
//     from the compute copies, e.g. the space-to-depth stem weight; gradient scatter-back of the
//     same layout as a gather, so no atomics).
#include "common.h"

namespace dlmpi {

__global__ __launch_bounds__(256) void fill_f32_kernel(float* __restrict__ p, int64_t n, float v) {
  const int64_t n4 = n >> 2;
  f32x4* p4 = reinterpret_cast<f32x4*>(p);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x)
    p4[i] = f32x4{v, v, v, v};
  const int64_t t = (n4 << 2) + blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t < n) p[t] = v;   // the < 4 tail (grid >= 1 block of 256 threads)
}

__global__ __launch_bounds__(256) void add_i64_kernel(int64_t* __restrict__ p, int64_t n, int64_t v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] += v;
}

template <typename T, bool ACC>
__global__ __launch_bounds__(256) void gather_kernel(T* __restrict__ dst, const T* __restrict__ src,
                                                     const int64_t* __restrict__ idx, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = idx[i];
    if constexpr (ACC) dst[i] += src[j];
    else dst[i] = j >= 0 ? src[j] : T(0);   // idx < 0: zero padding
  }
}

static inline unsigned grid_for(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (unsigned)b;
}

}  // namespace dlmpi

using namespace dlmpi;

extern "C" hipError_t dlmpi_fill_f32(float* p, int64_t n, float v, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (reinterpret_cast<uintptr_t>(p) & 15) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fill_f32_kernel, dim3(grid_for((n + 3) / 4)), dim3(256), 0, s, p, n, v);
  return hipGetLastError();
}

extern "C" hipError_t dlmpi_add_i64(int64_t* p, int64_t n, int64_t v, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(add_i64_kernel, dim3(grid_for(n)), dim3(256), 0, s, p, n, v);
  return hipGetLastError();
}

// esize: element bytes (2: bf16, 4: fp32); accumulate: fp32 only
extern "C" hipError_t dlmpi_gather(void* dst, const void* src, const int64_t* idx, int64_t n, int esize, int accumulate,
                                   hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const dim3 g(grid_for(n));
  if (esize == 4 && accumulate)
    hipLaunchKernelGGL((gather_kernel<float, true>), g, dim3(256), 0, s, (float*)dst, (const float*)src, idx, n);
  else if (esize == 4)
    hipLaunchKernelGGL((gather_kernel<float, false>), g, dim3(256), 0, s, (float*)dst, (const float*)src, idx, n);
  else if (esize == 2 && !accumulate)
    hipLaunchKernelGGL((gather_kernel<uint16_t, false>), g, dim3(256), 0, s, (uint16_t*)dst, (const uint16_t*)src, idx,
                       n);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

// Clock stamp (bench.py sclk): `blocks` one-wave blocks; block b writes {XCC id, shader-clock counter
// (s_memtime), 100 MHz reference counter (s_memrealtime)} to out[3 b ..].  Two stamps bracketing a
// region give its mean shader clock per XCD: d(memtime) / d(realtime) x 100 MHz (MI355X_MICROARCH.md
// DVFS item 6).  Blocks are dispatched round-robin over the 8 XCDs, so 32 blocks sample each a few
// times.  Lanes 0-2 store one value each (vector stores of per-lane data).
// One wave per block writes {XCC id, hardware id, s_memtime, s_memrealtime}.  The host pairs a start
// and a stop stamp taken on the same CU (XCC id + the SE / SH / CU fields of HW_ID, bits 8-15): the
// shader-clock counters of different CUs are not synchronised, so pairing by XCD alone mixes their
// offsets into short windows.
__global__ __launch_bounds__(64) void clock_stamp_kernel(unsigned long long* out) {
  const int l = threadIdx.x;
  const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (3 << 11)) & 15u;   // hwreg(HW_REG_XCC_ID, 0, 4)
  const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));         // hwreg(HW_REG_HW_ID, 0, 32)
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  const unsigned long long r = __builtin_amdgcn_s_memrealtime();
  const unsigned long long v = l == 0 ? (unsigned long long)xcc : (l == 1 ? (unsigned long long)hw : (l == 2 ? t : r));
  if (l < 4) out[4 * blockIdx.x + l] = v;
}

extern "C" hipError_t dlmpi_clock_stamp(unsigned long long* out, int blocks, hipStream_t s) {
  if (blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(clock_stamp_kernel, dim3(blocks), dim3(64), 0, s, out);
  return hipGetLastError();
}
