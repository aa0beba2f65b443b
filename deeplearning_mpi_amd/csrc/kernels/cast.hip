// Multi-tensor weight re-layout + cast: fp32 master parameters -> bf16 (or, on the fp32 precision
// path, fp32) compute copies in the
// layouts the GEMM kernels consume (forward [K][R][S][Cpad], data-gradient [C][R][S][K],
// transposed-conv [Cout][2][2][Cin], ...), all tensors in ONE launch.  Each entry describes a
// 4-D destination (contiguous), per-dimension source strides and a zero-padding limit.
// Also: the flat buffer pack used by coalesced broadcasts.
#include "common.h"

namespace dlmpi {

// Work distribution: block b handles entry map[b].x as slice map[b].y of map[b].z blocks; the host
// gives each entry ~1 block per 4096 destination elements (= one 64x64 transpose tile), so the
// large tensors are not left to a fixed handful of blocks while the small ones finish.  Two paths:
//  * transpose (source unit stride on destination dim 0, e.g. [K][R][S][C] -> [C][R][S][K] for the
//    data-gradient copy): 64x64 tiles through LDS, coalesced reads along d0 and writes along d3;
//  * direct (anything else, e.g. the forward copy whose innermost dim is contiguous in the source):
//    one destination element per thread, grid-stride over the entry.
template <typename T>
__global__ __launch_bounds__(256) void cast_weights_kernel(const CastEntry* __restrict__ ent,
                                                           const int4* __restrict__ map) {
  __shared__ float tile[64][65];
  const int4 mb = map[blockIdx.x];
  const CastEntry& e = ent[mb.x];
  T* const dst = static_cast<T*>(e.dst);
  const int sub = mb.y, nsub = mb.z;
  const int D0 = e.d[0], D1 = e.d[1], D2 = e.d[2], D3 = e.d[3];
  const int64_t n = (int64_t)D0 * D1 * D2 * D3;
  // Transpose path (source unit stride on d0, e.g. the KRSC -> CRSK data-gradient copy).
  if (e.st[0] == 1 && e.st[3] != 1 && D0 >= 16 && D3 >= 16) {
    const int M0 = D0, M1 = D1, M2 = D2;
    const int V0 = e.valid[0], V1 = e.valid[1], V2 = e.valid[2];
    const int64_t S0 = 1, S1 = e.st[1], S2 = e.st[2];
    const int t0n = (M0 + 63) / 64, t3n = (D3 + 63) / 64;
    const int64_t ntiles = (int64_t)M1 * M2 * t0n * t3n;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;   // 64 x 4
    for (int64_t t = sub; t < ntiles; t += nsub) {
      int64_t r = t;
      const int b3 = (int)(r % t3n); r /= t3n;
      const int b0 = (int)(r % t0n); r /= t0n;
      const int i2 = (int)(r % M2);
      const int i1 = (int)(r / M2);
      const bool v12 = i1 < V1 && i2 < V2;
      // read: i0 = b0*64 + tx (unit stride in the source), i3 = b3*64 + ty + 4k
      for (int k = 0; k < 16; ++k) {
        const int i0 = b0 * 64 + tx, i3 = b3 * 64 + ty + 4 * k;
        float v = 0.f;
        if (v12 && i0 < V0 && i3 < e.valid[3])
          v = e.src[i0 * S0 + i1 * S1 + i2 * S2 + i3 * e.st[3]];
        tile[ty + 4 * k][tx] = v;
      }
      __syncthreads();
      for (int k = 0; k < 16; ++k) {
        const int i3 = b3 * 64 + tx, i0 = b0 * 64 + ty + 4 * k;
        if (i0 < M0 && i3 < D3)
          store1(dst + (((int64_t)i0 * M1 + i1) * M2 + i2) * D3 + i3, tile[tx][ty + 4 * k]);
      }
      __syncthreads();
    }
    return;
  }
  // Identity layout (no padding, the source row-major in the destination's order: the forward copy of
  // every conv whose channels need no padding -- the masters are stored [K][R][S][C] already): a plain
  // vectorized cast, 8 elements per thread (two 16-B loads, one 16-B store for bf16).
  if (e.valid[0] == D0 && e.valid[1] == D1 && e.valid[2] == D2 && e.valid[3] == D3 && e.st[3] == 1 &&
      e.st[2] == D3 && e.st[1] == (int64_t)D2 * D3 && e.st[0] == (int64_t)D1 * D2 * D3 && (n & 7) == 0 &&
      ((uintptr_t)e.src & 15) == 0 && ((uintptr_t)dst & (8 * sizeof(T) - 1)) == 0) {
    const int64_t n8 = n >> 3;
    for (int64_t q = sub * (int64_t)blockDim.x + threadIdx.x; q < n8; q += (int64_t)nsub * blockDim.x) {
      const f32x4 a0 = reinterpret_cast<const f32x4*>(e.src)[2 * q], a1 = reinterpret_cast<const f32x4*>(e.src)[2 * q + 1];
      const float v[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
      store8(dst + 8 * q, v);
    }
    return;
  }
  // Direct path.  When the entry's destination and source extents fit 32-bit indices (every
  // conv / linear weight does) and rows are a multiple of 4 wide, each lane produces 4
  // consecutive destination elements with one 4-element store and one 32-bit index decomposition
  // (instead of three 64-bit divisions per element).
  const int64_t smax = (int64_t)(e.valid[0] - 1) * e.st[0] + (int64_t)(e.valid[1] - 1) * e.st[1] +
                       (int64_t)(e.valid[2] - 1) * e.st[2] + (int64_t)(e.valid[3] - 1) * e.st[3];
  if ((D3 & 3) == 0 && n < (1ll << 31) && smax < (1ll << 31) &&
      ((uintptr_t)dst & (4 * sizeof(T) - 1)) == 0) {
    const uint32_t nq = (uint32_t)(n >> 2);
    const int s0 = (int)e.st[0], s1 = (int)e.st[1], s2 = (int)e.st[2], s3 = (int)e.st[3];
    const uint32_t uD3 = D3, uD2 = D2, uD1 = D1;
    for (uint32_t q = sub * blockDim.x + threadIdx.x; q < nq; q += nsub * blockDim.x) {
      const uint32_t i = q * 4u;
      uint32_t r = i / uD3;
      const int i3 = (int)(i - r * uD3);
      const uint32_t r2 = r / uD2;
      const int i2 = (int)(r - r2 * uD2);
      const int i0 = (int)(r2 / uD1);
      const int i1 = (int)(r2 - (uint32_t)i0 * uD1);
      const bool v012 = i0 < e.valid[0] && i1 < e.valid[1] && i2 < e.valid[2];
      const int base = i0 * s0 + i1 * s1 + i2 * s2 + i3 * s3;
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = (v012 && i3 + j < e.valid[3]) ? e.src[base + j * s3] : 0.f;
      if constexpr (sizeof(T) == 2) *reinterpret_cast<u32x2*>(dst + i) = u32x2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
      else *reinterpret_cast<f32x4*>(dst + i) = f32x4{v[0], v[1], v[2], v[3]};
    }
    return;
  }
  for (int64_t i = sub * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)nsub * blockDim.x) {
    int64_t r = i;
    const int i3 = (int)(r % D3);
    r /= D3;
    const int i2 = (int)(r % D2);
    r /= D2;
    const int i1 = (int)(r % D1);
    const int i0 = (int)(r / D1);
    float v = 0.f;
    if (i0 < e.valid[0] && i1 < e.valid[1] && i2 < e.valid[2] && i3 < e.valid[3])
      v = e.src[i0 * e.st[0] + i1 * e.st[1] + i2 * e.st[2] + i3 * e.st[3]];
    store1(dst + i, v);
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

extern "C" hipError_t dlmpi_cast_weights(const CastEntry* entries_dev, const void* block_map_dev, int nblocks,
                                         int f32, hipStream_t s) {
  if (nblocks <= 0) return hipSuccess;
  // gaps between entries (alignment padding) are zeroed once at allocation and never written
  if (f32)
    hipLaunchKernelGGL(cast_weights_kernel<float>, dim3((unsigned)nblocks), dim3(256), 0, s, entries_dev,
                       reinterpret_cast<const int4*>(block_map_dev));
  else
    hipLaunchKernelGGL(cast_weights_kernel<uint16_t>, dim3((unsigned)nblocks), dim3(256), 0, s, entries_dev,
                       reinterpret_cast<const int4*>(block_map_dev));
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
