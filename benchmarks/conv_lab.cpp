// Standalone A/B harness for the implicit-GEMM conv kernels (no torch, no Python: a fresh GPU box
// runs it in seconds).  For each conv shape it times the single-stage 4-wave kernel (128x128, the
// 256-row and halo variants) and every pipelined 8-wave tile in interleaved rounds on the same
// random operands, and checks each pipelined output bit-for-bit against the 128x128 gather kernel
// (same K order -> same fp32 accumulation) and the BN statistics column sums to 1e-5.
//
// Build (CPU container):  python -m deeplearning_mpi_amd.build && hipcc --offload-arch=gfx950 -O3 -std=c++17 -c
//   benchmarks/conv_lab.cpp -o /tmp/conv_lab.o && hipcc --offload-arch=gfx950 /tmp/conv_lab.o <build/obj/*.o but binding_*> -o benchmarks/conv_lab
// Run:  benchmarks/conv_lab [rounds] [shape ...]   shape = N,H,W,C,K,R,stride,pad  (default: the
//   ResNet-50 / UNet compute-bound set)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../deeplearning_mpi_amd/csrc/kernels/dlmpi_kernels.h"

using namespace dlmpi;

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
      exit(1);                                                                               \
    }                                                                                        \
  } while (0)

__global__ void fill_bf16(uint16_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    const float f = ((h & 0xffffff) / 16777216.0f) * 2.f - 1.f;
    p[i] = (uint16_t)(__float_as_uint(f) >> 16);
  }
}

struct Shape {
  int N, H, W, C, K, R, stride, pad;
};

static int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

static void halo_geom(int P, int Q, int bm, int& th, int& tw, int& tiles_h, int& tiles_w) {
  int best = 1 << 30;
  const int rows = bm == 256 ? 352 : 192;
  for (int w = bm == 256 ? 32 : 16; w >= 4; --w) {
    const int h = std::min(bm / w, rows / (w + 2) - 2);
    if (h < 1) continue;
    const int t = cdiv(P, h) * cdiv(Q, w);
    if (t < best) { best = t; th = h; tw = w; }
  }
  tiles_h = cdiv(P, th);
  tiles_w = cdiv(Q, tw);
}

// forward-conv ConvArgs for tile bm x bn (halo: 2-D tiles, bm must be 128)
static ConvArgs make_args(const Shape& s, const uint16_t* x, const uint16_t* w, uint16_t* y, float* stats, int bm,
                          int bn, int halo) {
  const int P = (s.H + 2 * s.pad - s.R) / s.stride + 1, Q = (s.W + 2 * s.pad - s.R) / s.stride + 1;
  ConvArgs a{};
  a.x = x; a.H = s.H; a.W = s.W; a.C = s.C; a.ldx = s.C; a.xoff = 0;
  a.w = w; a.ldw = s.R * s.R * s.C; a.S = s.R;
  a.y = y; a.OH = P; a.OW = Q; a.ldy = s.K; a.yoff = 0;
  a.so = 1; a.sa = s.stride; a.out_f32 = 0; a.Nimg = s.N; a.Kout = s.K; a.kvalid = s.K; a.vec_store = 1;
  a.stats = stats; a.nstat = 2;
  a.cstep = 64; a.tstep = 0;
  a.ntiles = cdiv(s.K, bn);
  a.nphase = 1;
  ConvPhase& p = a.ph[0];
  p.P = P; p.Q = Q; p.Tr = s.R; p.Ts = s.R;
  p.dh0 = -s.pad; p.dhs = 1; p.dw0 = -s.pad; p.dws = 1;
  p.wr0 = 0; p.wrs = 1; p.ws0 = 0; p.wss = 1;
  p.oh0 = 0; p.ow0 = 0;
  p.mtiles = cdiv((int64_t)s.N * P * Q, bm);
  p.ksteps = cdiv((int64_t)s.R * s.R * s.C, 64);
  p.tile_base = 0;
  p.fdPQ = make_fastdiv((uint32_t)(P * Q));
  p.fdQ = make_fastdiv((uint32_t)Q);
  p.fdTs = make_fastdiv((uint32_t)s.R);
  if (halo) {
    int th = 8, tw = 16, tiles_h = 1, tiles_w = 1;
    halo_geom(P, Q, bm, th, tw, tiles_h, tiles_w);
    a.halo = halo; a.th = th; a.tw = tw; a.tiles_h = tiles_h; a.tiles_w = tiles_w;
    a.fd_tw = make_fastdiv((uint32_t)tw);
    a.fd_tilesw = make_fastdiv((uint32_t)tiles_w);
    a.fd_thw = make_fastdiv((uint32_t)(tiles_h * tiles_w));
    p.mtiles = s.N * tiles_h * tiles_w;
  }
  return a;
}

struct Variant {
  const char* name;
  int bm, bn, pipe, halo;
};

int main(int argc, char** argv) {
  // --only=NAME[,NAME...]: time only these variants and skip the correctness pass (profiler runs)
  std::string only;
  int argi = 1;
  if (argc > 1 && strncmp(argv[1], "--only=", 7) == 0) {
    only = std::string(",") + (argv[1] + 7) + ",";
    ++argi;
  }
  int rounds = argc > argi ? atoi(argv[argi]) : 5;
  std::vector<Shape> shapes;
  for (int i = argi + 1; i < argc; ++i) {
    Shape s;
    if (sscanf(argv[i], "%d,%d,%d,%d,%d,%d,%d,%d", &s.N, &s.H, &s.W, &s.C, &s.K, &s.R, &s.stride, &s.pad) == 8)
      shapes.push_back(s);
  }
  if (shapes.empty()) {
    shapes = {
        {256, 14, 14, 256, 256, 3, 1, 1},  {256, 28, 28, 128, 128, 3, 1, 1}, {256, 56, 56, 64, 64, 3, 1, 1},
        {256, 7, 7, 512, 512, 3, 1, 1},    {256, 14, 14, 1024, 256, 1, 1, 0}, {256, 7, 7, 2048, 512, 1, 1, 0},
        {256, 28, 28, 512, 128, 1, 1, 0},  {16, 64, 64, 512, 512, 3, 1, 1},   {16, 128, 128, 256, 256, 3, 1, 1},
        {16, 256, 256, 128, 128, 3, 1, 1}, {16, 512, 512, 64, 64, 3, 1, 1},   {16, 32, 32, 1024, 1024, 3, 1, 1},
        {16, 64, 64, 1536, 512, 3, 1, 1},
    };
  }
  const Variant vars[] = {
      {"old128x128", 128, 128, 0, 0}, {"old256x128", 256, 128, 0, 0}, {"old256x64", 256, 64, 0, 0},
      {"oldhalo128", 128, 128, 0, 1}, {"oldhalo64", 128, 64, 0, 1}, {"halo256x64", 256, 64, 0, 1},
      {"halo256x128", 256, 128, 0, 1},
      {"pipe256x256v2", 256, 256, 3, 0}, {"pipe224x256v2", 224, 256, 3, 0}, {"pipe256x128v2", 256, 128, 3, 0},
      {"pipe128x256v4", 128, 256, 5, 0}, {"pipe512x64v2", 512, 64, 3, 0},
  };
  const int NV = sizeof(vars) / sizeof(vars[0]);
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const Shape& s : shapes) {
    const int P = (s.H + 2 * s.pad - s.R) / s.stride + 1, Q = (s.W + 2 * s.pad - s.R) / s.stride + 1;
    const int64_t M = (int64_t)s.N * P * Q;
    const size_t nx = (size_t)s.N * s.H * s.W * s.C, nw = (size_t)s.K * s.R * s.R * s.C, ny = (size_t)M * s.K;
    const double flop = 2.0 * M * s.K * s.R * s.R * s.C;
    uint16_t *x, *w, *y, *yref;
    float *stats, *sref;
    const size_t nst = (size_t)cdiv(M, 64) * 2 * s.K + 1024 * 2 * s.K;
    CK(hipMalloc(&x, nx * 2));
    CK(hipMalloc(&w, nw * 2));
    CK(hipMalloc(&y, ny * 2));
    CK(hipMalloc(&yref, ny * 2));
    CK(hipMalloc(&stats, nst * 4));
    CK(hipMalloc(&sref, nst * 4));
    hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, st, x, nx, 0x1234u);
    hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, st, w, nw, 0x9876u);
    // reference: 128x128 gather kernel
    ConvArgs ar = make_args(s, x, w, yref, sref, 128, 128, false);
    if (only.empty()) CK(dlmpi_conv_igemm_ex(&ar, 128, 128, 0, st));
    CK(hipStreamSynchronize(st));
    std::vector<uint16_t> href(ny), hout(ny);
    CK(hipMemcpy(href.data(), yref, ny * 2, hipMemcpyDeviceToHost));
    auto colsum = [&](float* dst, int rows) {
      std::vector<float> h((size_t)rows * 2 * s.K);
      CK(hipMemcpy(h.data(), dst, h.size() * 4, hipMemcpyDeviceToHost));
      std::vector<double> c(2 * s.K, 0.0);
      for (int r = 0; r < rows; ++r)
        for (int j = 0; j < 2 * s.K; ++j) c[j] += h[(size_t)r * 2 * s.K + j];
      return c;
    };
    const std::vector<double> cref = colsum(sref, ar.ph[0].mtiles);
    std::vector<std::vector<double>> times(NV);
    std::vector<int> ok(NV, 1);
    std::vector<std::string> note(NV);
    for (int v = 0; v < NV; ++v) {
      const Variant& V = vars[v];
      if (V.halo && !(s.R == 3 && s.stride == 1 && s.pad == 1)) { ok[v] = -1; continue; }
      if (V.bn > 64 && s.K <= V.bn / 2) { ok[v] = -1; continue; }
      if (!only.empty()) {
        if (only.find(std::string(",") + V.name + ",") == std::string::npos) ok[v] = -1;
        continue;
      }
      ConvArgs a = make_args(s, x, w, y, stats, V.bm, V.bn, V.halo);
      CK(hipMemsetAsync(y, 0xff, ny * 2, st));
      if (dlmpi_conv_igemm_ex(&a, V.bm, V.bn, V.pipe, st) != hipSuccess) { ok[v] = -1; (void)hipGetLastError(); continue; }
      CK(hipStreamSynchronize(st));
      CK(hipMemcpy(hout.data(), y, ny * 2, hipMemcpyDeviceToHost));
      size_t bad = 0;
      double maxd = 0;
      for (size_t i = 0; i < ny; ++i) {
        if (hout[i] != href[i]) {
          ++bad;
          uint32_t ua = (uint32_t)hout[i] << 16, ub = (uint32_t)href[i] << 16;
          float fa, fb;
          memcpy(&fa, &ua, 4);
          memcpy(&fb, &ub, 4);
          maxd = std::max(maxd, (double)fabsf(fa - fb) / std::max(1.0f, fabsf(fb)));   // relative
        }
      }
      const std::vector<double> c = colsum(stats, a.ph[0].mtiles);
      double sd = 0;
      for (int j = 0; j < 2 * s.K; ++j) sd = std::max(sd, fabs(c[j] - cref[j]) / (1.0 + fabs(cref[j])));
      char buf[160];
      snprintf(buf, sizeof buf, "diff %zu/%zu (max rel %.3g) stats %.2g", bad, ny, maxd, sd);
      note[v] = buf;
      // halo tiles sum the taps in another order: bf16 rounding-level differences (<= 2 ulp) are
      // expected there, and the stats columns (near-zero-mean sums) move by their accumulated rounding
      if ((!V.halo && bad) || maxd > 1.0 / 64 || sd > (V.halo ? 0.05 : 1e-4)) ok[v] = 0;
    }
    const int iters = std::max(3, (int)std::min<double>(50, 2e12 / flop));
    for (int r = 0; r < rounds; ++r)
      for (int v = 0; v < NV; ++v) {
        if (ok[v] < 0) continue;
        const Variant& V = vars[v];
        ConvArgs a = make_args(s, x, w, y, stats, V.bm, V.bn, V.halo);
        CK(dlmpi_conv_igemm_ex(&a, V.bm, V.bn, V.pipe, st));
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < iters; ++i) CK(dlmpi_conv_igemm_ex(&a, V.bm, V.bn, V.pipe, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        times[v].push_back(ms * 1e3 / iters);
      }
    printf("shape N=%d %dx%d C=%d K=%d R=%d s=%d  M=%lld  %.1f GFLOP\n", s.N, s.H, s.W, s.C, s.K, s.R, s.stride,
           (long long)M, flop * 1e-9);
    for (int v = 0; v < NV; ++v) {
      if (ok[v] < 0) continue;
      std::vector<double> t = times[v];
      std::sort(t.begin(), t.end());
      const double med = t[t.size() / 2];
      printf("  %-12s %8.1f us (min %8.1f)  %7.1f TF/s  %s %s\n", vars[v].name, med, t[0], flop / med * 1e-6,
             ok[v] ? "OK " : "BAD", note[v].c_str());
    }
    fflush(stdout);
    CK(hipFree(x)); CK(hipFree(w)); CK(hipFree(y)); CK(hipFree(yref)); CK(hipFree(stats)); CK(hipFree(sref));
  }
  return 0;
}
