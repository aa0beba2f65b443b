// Store-bandwidth probe for the conv epilogue's output layout (standalone, not part of the library).
// Writes an [M rows][ld] bf16 matrix of 411 MB (ResNet-50 56^2 x 256 channels at batch 256) in
// tiles of BM rows x BN channels, one tile per block, 16 B per lane, in several patterns:
//   mode 0: tile rows of BN*2 bytes, 4 waves, each thread stores rows tid/CG + RG*i (current epilogue)
//   mode 1: same, but the block loops over tiles (persistent, grid = CUs*occ)
//   mode 2: whole-row tiles (BN = ld), 16 B per lane
// hipcc --offload-arch=gfx950 -O3 store_bw.hip -o store_bw && ./store_bw
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int BM, int BN>
__global__ __launch_bounds__(256) void tile_store(uint16_t* y, int M, int ld, int ntn, int tiles, int persistent) {
  constexpr int CG = BN / 8, RG = 256 / CG;
  const int cg = threadIdx.x % CG, rg = threadIdx.x / CG;
  for (int t = blockIdx.x; t < tiles; t += persistent ? gridDim.x : tiles) {
    const int mt = t / ntn, nt = t % ntn;
    const u32x4 v = u32x4{(uint32_t)t, (uint32_t)cg, 1u, 2u};
#pragma unroll 4
    for (int r = rg; r < BM; r += RG) {
      const int m = mt * BM + r;
      if (m < M) *reinterpret_cast<u32x4*>(y + (int64_t)m * ld + nt * BN + cg * 8) = v;
    }
  }
}

int main() {
  const int M = 256 * 56 * 56, ld = 256;
  uint16_t* y;
  hipMalloc(&y, (size_t)M * ld * 2);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto run = [&](const char* name, auto kern, int tiles, int grid, int ntn, int pers) {
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, y, M, ld, ntn, tiles, pers);
    hipEventRecord(a);
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, y, M, ld, ntn, tiles, pers);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double us = ms * 100.0;
    printf("%-40s %8.1f us  %6.2f TB/s\n", name, us, (double)M * ld * 2 / (us * 1e-6) / 1e12);
  };
  const int t128 = (M / 128) * 2;
  run("128x128 tiles, 1 per block", tile_store<128, 128>, t128, t128, 2, 0);
  run("128x128 tiles, persistent 1024", tile_store<128, 128>, t128, 1024, 2, 1);
  run("128x128 tiles, persistent 2048", tile_store<128, 128>, t128, 2048, 2, 1);
  const int t256 = M / 128;
  run("128x256 whole rows, 1 per block", tile_store<128, 256>, t256, t256, 1, 0);
  run("128x256 whole rows, persistent 2048", tile_store<128, 256>, t256, 2048, 1, 1);
  const int t64 = (M / 64) * 2;
  run("64x128 tiles, 1 per block", tile_store<64, 128>, t64, t64, 2, 0);
  hipFree(y);
  return 0;
}
