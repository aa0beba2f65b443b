// Fused losses and eval reductions.
//   softmax cross-entropy (ResNet: /root/reference/pytorch/resnet/main.py:113,129),
//   BCE-with-logits mean (UNet: /root/reference/pytorch/unet/train.py:162,183),
//   top-1 correct count (main.py:65-71) and per-sample sigmoid-threshold Dice (train.py:121-137).
// All reductions are two-stage with a fixed order: bit-reproducible, no float atomics.
#include "common.h"

namespace dlmpi {

__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = warp_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  float r = 0.f;
  const int nw = blockDim.x >> 6;
  for (int i = 0; i < nw; ++i) r += sh[i];
  return r;
}
__device__ __forceinline__ float block_max(float v, float* sh) {
  v = warp_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  float r = -INFINITY;
  const int nw = blockDim.x >> 6;
  for (int i = 0; i < nw; ++i) r = fmaxf(r, sh[i]);
  return r;
}

// one block per row: loss_rows[n] = logsumexp(x) - x[label]; lse[n] saved for the backward
__global__ __launch_bounds__(256) void softmax_ce_fwd_kernel(const float* __restrict__ logits, int ldl,
                                                             const int64_t* __restrict__ labels, int K,
                                                             float* __restrict__ loss_rows, float* __restrict__ lse) {
  __shared__ float sh[8];
  const int n = blockIdx.x;
  const float* x = logits + (int64_t)n * ldl;
  float m = -INFINITY;
  for (int k = threadIdx.x; k < K; k += blockDim.x) m = fmaxf(m, x[k]);
  m = block_max(m, sh);
  float s = 0.f;
  for (int k = threadIdx.x; k < K; k += blockDim.x) s += __expf(x[k] - m);
  s = block_sum(s, sh);
  if (threadIdx.x == 0) {
    const float l = m + __logf(s);
    lse[n] = l;
    const int64_t lab = labels[n];
    loss_rows[n] = (lab >= 0 && lab < K) ? l - x[lab] : 0.f;
  }
}

// dlogits[n][k] = (softmax - onehot) * (*go) * scale (fp32); padded columns K..ldd-1 are zeroed
__global__ __launch_bounds__(256) void softmax_ce_bwd_kernel(const float* __restrict__ logits, int ldl,
                                                             const int64_t* __restrict__ labels,
                                                             const float* __restrict__ lse, int K, int ldd,
                                                             const float* __restrict__ go, float scale,
                                                             float* __restrict__ dlogits) {
  const int n = blockIdx.x;
  const float g = (go ? *go : 1.f) * scale;
  const float l = lse[n];
  const int64_t lab = labels[n];
  for (int k = threadIdx.x; k < ldd; k += blockDim.x) {
    float d = 0.f;
    if (k < K) d = (__expf(logits[(int64_t)n * ldl + k] - l) - (k == lab ? 1.f : 0.f)) * g;
    dlogits[(int64_t)n * ldd + k] = d;
  }
}

__global__ __launch_bounds__(256) void sum_kernel(const float* __restrict__ x, int64_t n, float* __restrict__ out,
                                                  float scale) {
  __shared__ float sh[8];
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) s += x[i];
  s = block_sum(s, sh);
  if (threadIdx.x == 0) *out = s * scale;
}

__device__ __forceinline__ float bce_elem(float x, float t) {
  return fmaxf(x, 0.f) - x * t + log1pf(__expf(-fabsf(x)));
}

__global__ __launch_bounds__(256) void bce_fwd_kernel(const float* __restrict__ logits, int ldl,
                                                      const float* __restrict__ target, int64_t M,
                                                      float* __restrict__ partial) {
  __shared__ float sh[8];
  float s = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < M; i += (int64_t)gridDim.x * blockDim.x)
    s += bce_elem(logits[i * ldl], target[i]);
  s = block_sum(s, sh);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

// dlogits[i] = (sigmoid(x) - t) * go * scale  (fp32, contiguous)
__global__ __launch_bounds__(256) void bce_bwd_kernel(const float* __restrict__ logits, int ldl,
                                                      const float* __restrict__ target, int64_t M,
                                                      const float* __restrict__ go, float scale,
                                                      float* __restrict__ dlogits) {
  const float g = (go ? *go : 1.f) * scale;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < M; i += (int64_t)gridDim.x * blockDim.x) {
    const float x = logits[i * ldl];
    const float sg = 1.f / (1.f + __expf(-x));
    dlogits[i] = (sg - target[i]) * g;
  }
}

__global__ __launch_bounds__(256) void argmax_correct_kernel(const float* __restrict__ logits, int ldl,
                                                             const int64_t* __restrict__ labels, int K,
                                                             int* __restrict__ correct) {
  __shared__ float shv[4];
  __shared__ int shi[4];
  const int n = blockIdx.x;
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    const float v = logits[(int64_t)n * ldl + k];
    if (v > bv) { bv = v; bi = k; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { shv[w] = bv; shi[w] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i)
      if (shv[i] > bv || (shv[i] == bv && shi[i] < bi)) { bv = shv[i]; bi = shi[i]; }
    if ((int64_t)bi == labels[n]) atomicAdd(correct, 1);
  }
}

__global__ __launch_bounds__(256) void dice_kernel(const float* __restrict__ logits, int ldl,
                                                   const float* __restrict__ target, int64_t HW,
                                                   float* __restrict__ dice) {
  __shared__ float sh[8];
  const int n = blockIdx.x;
  float inter = 0.f, sp = 0.f, st = 0.f;
  for (int64_t i = threadIdx.x; i < HW; i += blockDim.x) {
    const float p = logits[((int64_t)n * HW + i) * ldl] > 0.f ? 1.f : 0.f;   // sigmoid(x) > 0.5
    const float t = target[(int64_t)n * HW + i];
    inter += p * t;
    sp += p;
    st += t;
  }
  inter = block_sum(inter, sh);
  sp = block_sum(sp, sh);
  st = block_sum(st, sh);
  if (threadIdx.x == 0) {
    const float uni = sp + st;
    dice[n] = uni > 0.f ? (2.f * inter + 1e-8f) / (uni + 1e-8f) : 1.f;
  }
}

}  // namespace dlmpi

using namespace dlmpi;

extern "C" hipError_t dlmpi_softmax_ce_fwd(const float* logits, int ldl, const int64_t* labels, int N, int K,
                                           float* loss_rows, float* lse, hipStream_t s) {
  hipLaunchKernelGGL(softmax_ce_fwd_kernel, dim3(N), dim3(256), 0, s, logits, ldl, labels, K, loss_rows, lse);
  return hipGetLastError();
}
extern "C" hipError_t dlmpi_softmax_ce_bwd(const float* logits, int ldl, const int64_t* labels, const float* lse,
                                           int N, int K, int ldd, const float* go, float scale, float* dlogits,
                                           hipStream_t s) {
  hipLaunchKernelGGL(softmax_ce_bwd_kernel, dim3(N), dim3(256), 0, s, logits, ldl, labels, lse, K, ldd, go, scale,
                     dlogits);
  return hipGetLastError();
}
extern "C" hipError_t dlmpi_sum_f32(const float* x, int64_t n, float* out, float scale, hipStream_t s) {
  hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(256), 0, s, x, n, out, scale);
  return hipGetLastError();
}
extern "C" hipError_t dlmpi_bce_fwd(const float* logits, int ldl, const float* target, int64_t M, float* partial,
                                    int nblk, hipStream_t s) {
  hipLaunchKernelGGL(bce_fwd_kernel, dim3(nblk), dim3(256), 0, s, logits, ldl, target, M, partial);
  return hipGetLastError();
}
extern "C" hipError_t dlmpi_bce_bwd(const float* logits, int ldl, const float* target, int64_t M, const float* go,
                                    float scale, float* dlogits, hipStream_t s) {
  int64_t b = (M + 255) / 256;
  if (b > 8192) b = 8192;
  hipLaunchKernelGGL(bce_bwd_kernel, dim3((unsigned)b), dim3(256), 0, s, logits, ldl, target, M, go, scale, dlogits);
  return hipGetLastError();
}
extern "C" hipError_t dlmpi_argmax_correct(const float* logits, int ldl, const int64_t* labels, int N, int K,
                                           int* correct, hipStream_t s) {
  hipLaunchKernelGGL(argmax_correct_kernel, dim3(N), dim3(256), 0, s, logits, ldl, labels, K, correct);
  return hipGetLastError();
}
extern "C" hipError_t dlmpi_dice(const float* logits, int ldl, const float* target, int N, int64_t HW, float* dice,
                                 hipStream_t s) {
  hipLaunchKernelGGL(dice_kernel, dim3(N), dim3(256), 0, s, logits, ldl, target, HW, dice);
  return hipGetLastError();
}
