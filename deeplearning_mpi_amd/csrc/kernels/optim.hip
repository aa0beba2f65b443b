// Fused optimizers over the flat fp32 parameter / gradient / state buffers of a ParamArena:
// one launch updates every parameter of the model (replaces the foreach SGD/Adam kernels and
// clip_grad_norm_ of the reference: /root/reference/pytorch/resnet/main.py:114,132,
// /root/reference/pytorch/unet/train.py:160-161,194,196).  Semantics follow torch.optim
// (SGD momentum/dampening/nesterov/L2 weight decay, Adam/AdamW with bias correction).
// `skip_flag` (device scalar, non-zero = skip) lets all ranks skip a step collectively when the
// all-reduced gradient is non-finite, without a host synchronisation.
#include "common.h"

namespace dlmpi {

__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                  float* __restrict__ m, int64_t n, float lr, float momentum,
                                                  float dampening, float wd, int nesterov, int first,
                                                  const float* __restrict__ skip_flag) {
  if (skip_flag && *skip_flag != 0.f) return;
  // 16-byte accesses when every buffer allows them (the arena's do), else the element loop below
  const bool vec = (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m) & 15) == 0;
  const int64_t n4 = vec ? n >> 2 : 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
    f32x4 pv = reinterpret_cast<f32x4*>(p)[i];
    f32x4 gv = reinterpret_cast<const f32x4*>(g)[i];
    if (wd != 0.f) gv += wd * pv;
    if (momentum != 0.f) {
      f32x4 mv = first ? gv : momentum * reinterpret_cast<f32x4*>(m)[i] + (1.f - dampening) * gv;
      reinterpret_cast<f32x4*>(m)[i] = mv;
      gv = nesterov ? gv + momentum * mv : mv;
    }
    reinterpret_cast<f32x4*>(p)[i] = pv - lr * gv;
  }
  // tail (or everything, unaligned)
  for (int64_t t = (n4 << 2) + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n; t += stride) {
    float pv = p[t], gv = g[t];
    if (wd != 0.f) gv += wd * pv;
    if (momentum != 0.f) {
      const float mv = first ? gv : momentum * m[t] + (1.f - dampening) * gv;
      m[t] = mv;
      gv = nesterov ? gv + momentum * mv : mv;
    }
    p[t] = pv - lr * gv;
  }
}

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float lr, float b1, float b2,
                                          float eps, float wd, int adamw, float bc1, float bc2, float coef) {
  g *= coef;
  if (wd != 0.f) {
    if (adamw) p *= (1.f - lr * wd);
    else g += wd * p;
  }
  m += (g - m) * (1.f - b1);             // torch: exp_avg.lerp_(grad, 1 - beta1)
  v = v * b2 + (1.f - b2) * g * g;
  const float denom = sqrtf(v) / sqrtf(bc2) + eps;
  p -= (lr / bc1) * m / denom;
}

// clip_coef = {scale, nonfinite}: the update uses g * scale.  wb (clip_grad_norm_ handed the scaling
// to the optimizer instead of a separate pass over the gradients): g * scale is also stored back into
// g when scale != 1, so the gradients read afterwards are the clipped ones, as after torch's in-place
// clip -- the same product the separate pass stored (bit-identical update and gradients).
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, int64_t n, float lr,
                                                   float b1, float b2, float eps, float wd, int adamw, float bc1,
                                                   float bc2, const float* __restrict__ clip_coef,
                                                   const float* __restrict__ tstep, int wb) {
  // tstep = number of updates applied so far (device scalar): this update is number tstep + 1
  const float coef = clip_coef ? clip_coef[0] : 1.f;
  if (clip_coef && clip_coef[1] != 0.f) return;   // non-finite gradient norm: collective skip
  const bool store_g = wb && coef != 1.f;
  if (tstep) {   // step count on the device: bias corrections stay correct under hipGraph replay
    const float t = *tstep + 1.f;
    bc1 = 1.f - powf(b1, t);
    bc2 = 1.f - powf(b2, t);
  }
  // 16-byte accesses when every state array is aligned (the flat arenas are), scalar tail; the
  // per-element arithmetic is unchanged (bit-identical)
  const bool vec = (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0;
  const int64_t n4 = vec ? n / 4 : 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
    f32x4 pv = reinterpret_cast<f32x4*>(p)[i], mv = reinterpret_cast<f32x4*>(m)[i];
    f32x4 vv = reinterpret_cast<f32x4*>(v)[i];
    const f32x4 gv = reinterpret_cast<const f32x4*>(g)[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float pe = pv[e], me = mv[e], ve = vv[e];
      adam_elem(pe, gv[e], me, ve, lr, b1, b2, eps, wd, adamw, bc1, bc2, coef);
      pv[e] = pe;
      mv[e] = me;
      vv[e] = ve;
    }
    reinterpret_cast<f32x4*>(p)[i] = pv;
    reinterpret_cast<f32x4*>(m)[i] = mv;
    reinterpret_cast<f32x4*>(v)[i] = vv;
    if (store_g) reinterpret_cast<f32x4*>(g)[i] = gv * coef;
  }
  for (int64_t i = 4 * n4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    float pv = p[i], mv = m[i], vv = v[i];
    const float gi = g[i];
    adam_elem(pv, gi, mv, vv, lr, b1, b2, eps, wd, adamw, bc1, bc2, coef);
    p[i] = pv;
    m[i] = mv;
    v[i] = vv;
    if (store_g) g[i] = gi * coef;
  }
}

// After adam_kernel: count the update only if it was applied, so a collectively skipped step
// (non-finite gradient norm) leaves every later bias correction exactly as if it never happened.
__global__ void adam_step_advance_kernel(float* __restrict__ tstep, const float* __restrict__ clip_coef) {
  if (threadIdx.x == 0 && !(clip_coef && clip_coef[1] != 0.f)) *tstep += 1.f;
}

// 16-byte loads, four independent sums per thread, four loads in flight per iteration (the scalar
// grid-stride loop ran at 1.1 TB/s: 110 us for the 31 M UNet gradients), scalar tail
__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ x, int64_t n,
                                                    float* __restrict__ partial) {
  __shared__ float sh[4];
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  const int64_t n4 = ((uintptr_t)x & 15) == 0 ? n / 4 : 0;
  const f32x4* x4 = reinterpret_cast<const f32x4*>(x);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n4; i += 4 * stride) {
    f32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = x4[i + u * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      s0 = __builtin_fmaf(v[u][0], v[u][0], s0);
      s1 = __builtin_fmaf(v[u][1], v[u][1], s1);
      s2 = __builtin_fmaf(v[u][2], v[u][2], s2);
      s3 = __builtin_fmaf(v[u][3], v[u][3], s3);
    }
  }
  for (; i < n4; i += stride) {
    const f32x4 v = x4[i];
    s0 = __builtin_fmaf(v[0], v[0], s0);
    s1 = __builtin_fmaf(v[1], v[1], s1);
    s2 = __builtin_fmaf(v[2], v[2], s2);
    s3 = __builtin_fmaf(v[3], v[3], s3);
  }
  for (int64_t j = 4 * n4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n; j += stride) s0 += x[j] * x[j];
  float s = (s0 + s1) + (s2 + s3);
  s = warp_sum(s);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}

// norm = sqrt(sum partial); coef_out[0] = min(1, max_norm / (norm + 1e-6)); coef_out[1] = !isfinite(norm);
// ncoef 4: also coef_out[2..3] = {1, !isfinite(norm)} -- the optimizer's (scale, skip) pair once the
// gradients are scaled in place (no copy + fill per step)
__global__ __launch_bounds__(256) void clip_coef_kernel(const float* __restrict__ partial, int nblk, float max_norm,
                                                        float* __restrict__ norm_out, float* __restrict__ coef_out,
                                                        int ncoef) {
  __shared__ double sh[4];
  double s = 0.0;
  for (int i = threadIdx.x; i < nblk; i += blockDim.x) s += (double)partial[i];
  s = warp_sum_d(s);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double tot = sh[0] + sh[1] + sh[2] + sh[3];
    const float norm = (float)sqrt(tot);
    if (norm_out) *norm_out = norm;
    if (coef_out) {
      const float c = max_norm / (norm + 1e-6f);
      coef_out[0] = c < 1.f ? c : 1.f;
      coef_out[1] = isfinite(norm) ? 0.f : 1.f;
      if (ncoef >= 4) {
        coef_out[2] = 1.f;
        coef_out[3] = coef_out[1];
      }
    }
  }
}

__global__ __launch_bounds__(256) void scale_kernel(float* __restrict__ x, int64_t n, const float* __restrict__ coef) {
  const float c = coef[0];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[i] *= c;
}

static inline unsigned blocks_for(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (unsigned)b;
}

}  // namespace dlmpi

using namespace dlmpi;

extern "C" hipError_t dlmpi_sgd(float* p, const float* g, float* m, int64_t n, float lr, float momentum,
                                float dampening, float wd, int nesterov, int first, const float* skip_flag,
                                hipStream_t s) {
  hipLaunchKernelGGL(sgd_kernel, dim3(blocks_for(n / 4 + 1)), dim3(256), 0, s, p, g, m, n, lr, momentum, dampening,
                     wd, nesterov, first, skip_flag);
  return hipGetLastError();
}
extern "C" hipError_t dlmpi_adam(float* p, float* g, float* m, float* v, int64_t n, float lr, float b1, float b2,
                                 float eps, float wd, int adamw, float bc1, float bc2, const float* clip_coef,
                                 float* tstep, int wb, hipStream_t s) {
  hipLaunchKernelGGL(adam_kernel, dim3(blocks_for(n / 4 + 1)), dim3(256), 0, s, p, g, m, v, n, lr, b1, b2, eps, wd, adamw,
                     bc1, bc2, clip_coef, tstep, wb);
  if (tstep) hipLaunchKernelGGL(adam_step_advance_kernel, dim3(1), dim3(64), 0, s, tstep, clip_coef);
  return hipGetLastError();
}
extern "C" hipError_t dlmpi_sumsq(const float* x, int64_t n, float* partial, int nblk, hipStream_t s) {
  hipLaunchKernelGGL(sumsq_kernel, dim3(nblk), dim3(256), 0, s, x, n, partial);
  return hipGetLastError();
}
extern "C" hipError_t dlmpi_clip_coef(const float* partial, int nblk, float max_norm, float* norm_out,
                                      float* coef_out, int ncoef, hipStream_t s) {
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(256), 0, s, partial, nblk, max_norm, norm_out, coef_out, ncoef);
  return hipGetLastError();
}
extern "C" hipError_t dlmpi_scale_f32(float* x, int64_t n, const float* coef, hipStream_t s) {
  hipLaunchKernelGGL(scale_kernel, dim3(blocks_for(n)), dim3(256), 0, s, x, n, coef);
  return hipGetLastError();
}
