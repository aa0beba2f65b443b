// 1x1 convolution with at most 4 output channels -- the UNet head, Conv2d(64, n_classes, 1) with
// n_classes = 1 for the binary masks (/root/reference/pytorch/unet/model.py:68, train.py:160) --
// as a streaming dot product:  y[m][k] = sum_c x[m][c] * w[k][c] + b[k].
//
// Through the GEMM it was a 128 x 64 tile per 128 rows with 63 of 64 output columns discarded
// (244 us for the 16 x 512^2 x 64 input = 2.2 TB/s).  Here L = C / 8 lanes share a row (16 B each,
// so one wave instruction reads 64 / L whole rows = 1 KB contiguous), each lane forms its 8-channel
// partial dot for every output channel in fp32 (weights in registers), and the L partials are
// combined by a fixed xor-shuffle tree; the first lane of the row adds the bias and stores.  Four
// row groups per wave are in flight per iteration.  The result differs from the MFMA path only in
// the fp32 summation order.
// psc / psh (optional): the input is a deferred BN-apply + ReLU of x -- bf16(relu(fma(x, psc, psh))),
// bn_apply_kernel's arithmetic, so identical to reading the stored BN output -- computed on the fly.
#include "common.h"

namespace dlmpi {

template <int L, int KV, typename TO>
__global__ __launch_bounds__(256) void head1x1_kernel(const uint16_t* __restrict__ x, int ldx, int xoff, int64_t M,
                                                      const uint16_t* __restrict__ w, int ldw,
                                                      const float* __restrict__ bias, TO* __restrict__ y, int ldy,
                                                      int yoff, const float* __restrict__ psc,
                                                      const float* __restrict__ psh) {
  constexpr int RPW = 64 / L;   // rows per wave instruction
  constexpr int U = 4;          // row groups in flight per wave
  const int lane = threadIdx.x & 63;
  const int sub = lane % L, rw = lane / L;
  float wv[KV][8], b[KV];
#pragma unroll
  for (int k = 0; k < KV; ++k) {
    load8(w + (int64_t)k * ldw + sub * 8, wv[k]);
    b[k] = bias ? bias[k] : 0.f;
  }
  float ps[8], ph[8];
  if (psc)
#pragma unroll
    for (int e = 0; e < 8; ++e) { ps[e] = psc[sub * 8 + e]; ph[e] = psh[sub * 8 + e]; }
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t step = (int64_t)gridDim.x * 4 * RPW * U;
  for (int64_t base = wave * RPW * U; base < M; base += step) {
    float v[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t row = base + u * RPW + rw;
      if (row < M) load8(x + row * ldx + xoff + sub * 8, v[u]);
      else
#pragma unroll
        for (int e = 0; e < 8; ++e) v[u][e] = 0.f;
      if (psc)
#pragma unroll
        for (int e = 0; e < 8; ++e) v[u][e] = bf2f(f2bf(fmaxf(__builtin_fmaf(v[u][e], ps[e], ph[e]), 0.f)));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t row = base + u * RPW + rw;
#pragma unroll
      for (int k = 0; k < KV; ++k) {
        float s = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) s = __builtin_fmaf(v[u][e], wv[k][e], s);
#pragma unroll
        for (int o = L / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        if (sub == 0 && row < M) store1(y + row * ldy + yoff + k, s + b[k]);
      }
    }
  }
}

}  // namespace dlmpi

using namespace dlmpi;

extern "C" int dlmpi_head1x1_ok(int C, int kv) {
  return kv >= 1 && kv <= 4 && (C == 16 || C == 32 || C == 64 || C == 128 || C == 256 || C == 512);
}

extern "C" hipError_t dlmpi_head1x1(const void* x, int ldx, int xoff, int64_t M, int C, const void* w, int ldw,
                                    const float* bias, void* y, int ldy, int yoff, int kv, int y_f32,
                                    const float* psc, const float* psh, hipStream_t s) {
  if ((psc == nullptr) != (psh == nullptr)) return hipErrorInvalidValue;
  if (!dlmpi_head1x1_ok(C, kv) || M <= 0 || ldx % 8 || xoff % 8 || ldw % 8) return hipErrorInvalidValue;
  const int L = C / 8;
  const int64_t rows_per_block = 4LL * (64 / L) * 4;
  const unsigned nblk = (unsigned)std::min<int64_t>((M + rows_per_block - 1) / rows_per_block, 4096);
  const uint16_t* xp = static_cast<const uint16_t*>(x);
  const uint16_t* wp = static_cast<const uint16_t*>(w);
#define HEAD_KV(L_, KV_)                                                                                       \
  do {                                                                                                         \
    if (y_f32)                                                                                                 \
      hipLaunchKernelGGL((head1x1_kernel<L_, KV_, float>), dim3(nblk), dim3(256), 0, s, xp, ldx, xoff, M, wp,   \
                         ldw, bias, static_cast<float*>(y), ldy, yoff, psc, psh);                              \
    else                                                                                                       \
      hipLaunchKernelGGL((head1x1_kernel<L_, KV_, uint16_t>), dim3(nblk), dim3(256), 0, s, xp, ldx, xoff, M,    \
                         wp, ldw, bias, static_cast<uint16_t*>(y), ldy, yoff, psc, psh);                       \
  } while (0)
#define HEAD_L(L_)                        \
  do {                                    \
    if (kv == 1) HEAD_KV(L_, 1);          \
    else if (kv == 2) HEAD_KV(L_, 2);     \
    else if (kv == 3) HEAD_KV(L_, 3);     \
    else HEAD_KV(L_, 4);                  \
  } while (0)
  switch (L) {
    case 2: HEAD_L(2); break;
    case 4: HEAD_L(4); break;
    case 8: HEAD_L(8); break;
    case 16: HEAD_L(16); break;
    case 32: HEAD_L(32); break;
    default: HEAD_L(64); break;
  }
#undef HEAD_L
#undef HEAD_KV
  return hipGetLastError();
}
