// Fault injection and communication-load rehearsal kernels.
//
// delay_kernel: for the failure-detection tests: keeps a stream busy for a given
// wall-clock time, so a collective queued behind it "hangs" long enough for the RCCL watchdog to
// fire.  One wave, s_memrealtime (100 MHz constant clock) polling with s_sleep; it ALWAYS
// terminates after `ms` milliseconds.
//
// comm_load_kernel: the one-GPU stand-in for what an N-rank RCCL all-reduce costs the compute
// streams.  An RCCL collective occupies one workgroup per
// channel for its whole duration and streams the bucket through HBM; here `channels` workgroups of
// 256 threads with `lds` bytes of LDS each copy their stripe of the bucket into a scratch buffer
// (2 (W-1)/W of the bucket's bytes per rank, the ring all-reduce's send volume) and then hold their
// CU until the modeled collective time has passed (wall clock, bounded).  The bucket itself is
// only read.
#include "common.h"

namespace dlmpi {

__global__ __launch_bounds__(64) void delay_kernel(uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

__global__ __launch_bounds__(256) void comm_load_kernel(const u32x4* __restrict__ src, int64_t n16, u32x4* __restrict__ dst,
                                                        int64_t copy16, uint64_t ticks) {
  extern __shared__ u32x4 lds_hold[];   // the channel's LDS footprint (allocated by the launch)
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) lds_hold[0] = u32x4{0u, 0u, 0u, 0u};
  // this workgroup's stripe of the modeled traffic: element i of the copy reads src[i mod n16]
  const int64_t per = (copy16 + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * per, hi = lo + per < copy16 ? lo + per : copy16;
  for (int64_t i = lo + threadIdx.x; i < hi; i += 256) {
    const int64_t j = i < n16 ? i : i % n16;
    dst[j] = src[j];
  }
  // hold the CU for the rest of the modeled collective time (bounded: 2^20 polls)
  for (int it = 0; it < (1 << 20) && __builtin_amdgcn_s_memrealtime() - t0 < ticks; ++it) __builtin_amdgcn_s_sleep(8);
}

}  // namespace dlmpi

extern "C" hipError_t dlmpi_delay(double ms, hipStream_t s) {
  if (ms <= 0) return hipSuccess;
  if (ms > 60000) ms = 60000;   // hard cap: never more than a minute
  const uint64_t ticks = (uint64_t)(ms * 1e5);   // 100 MHz
  hipLaunchKernelGGL(dlmpi::delay_kernel, dim3(1), dim3(64), 0, s, ticks);
  return hipGetLastError();
}

// bucket: bytes of the all-reduced buffer (16-byte multiple read, tail ignored); scratch: at least
// that many bytes; copy_bytes: modeled traffic; us: modeled duration (capped at 100 ms)
extern "C" hipError_t dlmpi_comm_load(const void* bucket, int64_t bytes, void* scratch, int64_t copy_bytes,
                                      int channels, int lds_bytes, double us, hipStream_t s) {
  if (channels <= 0 || bytes < 16) return hipSuccess;
  if (us > 1e5) us = 1e5;
  if (lds_bytes < 16) lds_bytes = 16;
  if (lds_bytes > 160 * 1024) return hipErrorInvalidValue;
  const uint64_t ticks = (uint64_t)(us * 100.0);   // 100 MHz
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(dlmpi::comm_load_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess && lds_bytes > 64 * 1024) return attr;
  hipLaunchKernelGGL(dlmpi::comm_load_kernel, dim3((unsigned)channels), dim3(256), (unsigned)lds_bytes, s,
                     static_cast<const dlmpi::u32x4*>(bucket), bytes / 16, static_cast<dlmpi::u32x4*>(scratch),
                     copy_bytes / 16, ticks);
  return hipGetLastError();
}
