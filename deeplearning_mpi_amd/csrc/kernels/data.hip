// Device-resident input pipeline (data/device.py): the whole training set lives in HBM (CIFAR-10
// is 150 MB of uint8; 288 GB per MI355X) and every batch is assembled by ONE kernel from a device
// index vector -- gather + RandomCrop(32, padding=4) + RandomHorizontalFlip + ToTensor + Normalize
// of the reference's CIFAR transform (/root/reference/pytorch/resnet/main.py:82-87) -- instead of
// per-sample host transforms in DataLoader worker processes and a host->device copy per step.
//
// Augmentation randomness is a counter-based hash of (seed, epoch, dataset index): reproducible,
// independent of batch size, rank layout and worker count, and identical in the torch reference
// (data/device.py:_aug_params).
#include "common.h"

namespace dlmpi {

__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

// One thread per output pixel (b, y, x), all C channels.  data: [Nds][H][W][C] uint8 (HWC);
// out: [B][C][H][W] fp32 normalised; out_labels[b] = labels[idx[b]].
__global__ __launch_bounds__(256) void image_batch_kernel(const uint8_t* __restrict__ data,
                                                          const int64_t* __restrict__ labels,
                                                          const int64_t* __restrict__ idx, int B, int H, int W,
                                                          int C, int pad, int augment, uint32_t seed, uint32_t epoch,
                                                          float m0, float m1, float m2, float s0, float s1, float s2,
                                                          float* __restrict__ out, int64_t* __restrict__ out_labels) {
  const int64_t total = (int64_t)B * H * W;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(i % W);
    const int64_t t = i / W;
    const int y = (int)(t % H);
    const int b = (int)(t / H);
    const int64_t d = idx[b];
    int oi = pad, oj = pad, flip = 0;
    if (augment) {
      const uint32_t h = fmix32(seed * 0x9E3779B1u + epoch * 0x85EBCA77u + (uint32_t)d);
      const uint32_t span = 2u * (uint32_t)pad + 1u;
      oi = (int)(h % span);
      oj = (int)((h >> 8) % span);
      flip = (int)((h >> 16) & 1u);
    }
    // RandomCrop of the zero-padded image at (oi, oj), then the horizontal flip of the crop
    const int sy = y + oi - pad;
    const int sx = (flip ? W - 1 - x : x) + oj - pad;
    const bool in = (unsigned)sy < (unsigned)H && (unsigned)sx < (unsigned)W;
    const uint8_t* px = data + ((d * H + (in ? sy : 0)) * W + (in ? sx : 0)) * C;
    const float mean[3] = {m0, m1, m2}, sd[3] = {s0, s1, s2};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      if (c >= C) break;
      const float v = in ? (float)px[c] / 255.f : 0.f;
      out[(((int64_t)b * C + c) * H + y) * W + x] = (v - mean[c]) / sd[c];
    }
    if (x == 0 && y == 0 && out_labels) out_labels[b] = labels[d];
  }
}

}  // namespace dlmpi

using namespace dlmpi;

extern "C" hipError_t dlmpi_image_batch(const uint8_t* data, const int64_t* labels, const int64_t* idx, int B, int H,
                                        int W, int C, int pad, int augment, uint32_t seed, uint32_t epoch,
                                        const float* mean3, const float* std3, float* out, int64_t* out_labels,
                                        hipStream_t s) {
  if (C < 1 || C > 3 || B <= 0) return B == 0 ? hipSuccess : hipErrorInvalidValue;
  int64_t blocks = ((int64_t)B * H * W + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(image_batch_kernel, dim3((unsigned)blocks), dim3(256), 0, s, data, labels, idx, B, H, W, C, pad,
                     augment, seed, epoch, mean3[0], mean3[1], mean3[2], std3[0], std3[1], std3[2], out, out_labels);
  return hipGetLastError();
}
