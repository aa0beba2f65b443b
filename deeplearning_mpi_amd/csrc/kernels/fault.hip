// Fault injection for the failure-detection tests: a bounded delay kernel that
// keeps a stream busy for a given wall-clock time, so a collective queued behind it "hangs" long
// enough for the RCCL watchdog to fire.  One wave, s_memrealtime (100 MHz constant clock) polling
// with s_sleep; it ALWAYS terminates after `ms` milliseconds.
#include "common.h"

namespace dlmpi {

__global__ __launch_bounds__(64) void delay_kernel(uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

}  // namespace dlmpi

extern "C" hipError_t dlmpi_delay(double ms, hipStream_t s) {
  if (ms <= 0) return hipSuccess;
  if (ms > 60000) ms = 60000;   // hard cap: never more than a minute
  const uint64_t ticks = (uint64_t)(ms * 1e5);   // 100 MHz
  hipLaunchKernelGGL(dlmpi::delay_kernel, dim3(1), dim3(64), 0, s, ticks);
  return hipGetLastError();
}
