// Multi-tensor weight re-layout + cast: fp32 master parameters -> bf16 compute copies in the
// layouts the GEMM kernels consume (forward [K][R][S][Cpad], data-gradient [C][R][S][K],
// transposed-conv [Cout][2][2][Cin], ...), all tensors in ONE launch.  Each entry describes a
// 4-D destination (contiguous), per-dimension source strides and a zero-padding limit.
// Also: the flat buffer pack used by coalesced broadcasts.
#include "common.h"

namespace dlmpi {

__global__ __launch_bounds__(256) void cast_weights_kernel(const CastEntry* __restrict__ ent, int n, int64_t total) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {   // last entry with start <= i
      const int mid = (lo + hi + 1) >> 1;
      if (ent[mid].start <= i) lo = mid;
      else hi = mid - 1;
    }
    const CastEntry& e = ent[lo];
    int64_t r = i - e.start;
    const int i3 = (int)(r % e.d[3]);
    r /= e.d[3];
    const int i2 = (int)(r % e.d[2]);
    r /= e.d[2];
    const int i1 = (int)(r % e.d[1]);
    const int i0 = (int)(r / e.d[1]);
    float v = 0.f;
    if (i0 < e.valid[0] && i1 < e.valid[1] && i2 < e.valid[2] && i3 < e.valid[3])
      v = e.src[i0 * e.st[0] + i1 * e.st[1] + i2 * e.st[2] + i3 * e.st[3]];
    e.dst[i - e.start] = f2bf(v);
  }
}

__global__ void pack_kernel(const void* const* __restrict__ srcs, const int64_t* __restrict__ offs, int n,
                            int64_t total, char* __restrict__ dst) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (offs[mid] <= i) lo = mid;
      else hi = mid - 1;
    }
    dst[i] = reinterpret_cast<const char*>(srcs[lo])[i - offs[lo]];
  }
}

}  // namespace dlmpi

using namespace dlmpi;

extern "C" hipError_t dlmpi_cast_weights(const CastEntry* entries_dev, int n, int64_t total, hipStream_t s) {
  if (total == 0) return hipSuccess;
  int64_t b = (total + 255) / 256;
  if (b > 8192) b = 8192;
  hipLaunchKernelGGL(cast_weights_kernel, dim3((unsigned)b), dim3(256), 0, s, entries_dev, n, total);
  return hipGetLastError();
}

extern "C" hipError_t dlmpi_pack(const void* const* srcs, const int64_t* offs, int n, int64_t total_bytes, void* dst,
                                 hipStream_t s) {
  if (total_bytes == 0) return hipSuccess;
  int64_t b = (total_bytes + 255) / 256;
  if (b > 8192) b = 8192;
  hipLaunchKernelGGL(pack_kernel, dim3((unsigned)b), dim3(256), 0, s, srcs, offs, n, total_bytes, (char*)dst);
  return hipGetLastError();
}
