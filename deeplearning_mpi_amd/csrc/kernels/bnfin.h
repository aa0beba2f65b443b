// BatchNorm finalize bodies shared by the column-reduce + finalize kernels of bn.hip (forward:
// scale / shift / saved and running statistics; backward: dgamma / dbeta and the apply coefficients).
// An in-launch finalize inside the conv epilogue was measured and removed (every conv block paid a
// drained store + ticket before retiring: ResNet-50 -0.7 %, profiles/r3_fin_in_launch_rejected).
#pragma once
#include "common.h"

namespace dlmpi {

__device__ __forceinline__ void fin_fwd(const FinArgs& f, int c, double s1, double s2) {
  const double mean = s1 / f.count;
  double var = s2 / f.count - mean * mean;
  if (var < 0.0) var = 0.0;
  const float invstd = (float)(1.0 / sqrt(var + (double)f.eps));
  const float g = f.gamma ? f.gamma[c] : 1.f;
  const float b = f.beta ? f.beta[c] : 0.f;
  const float sc = g * invstd;
  f.scale[c] = sc;
  f.shift[c] = b - (float)mean * sc;
  if (f.save_mean) f.save_mean[c] = (float)mean;
  if (f.save_invstd) f.save_invstd[c] = invstd;
  if (f.running_mean) {
    const double unbiased = f.count > 1.0 ? var * f.count / (f.count - 1.0) : var;
    f.running_mean[c] = (1.f - f.momentum) * f.running_mean[c] + f.momentum * (float)mean;
    f.running_var[c] = (1.f - f.momentum) * f.running_var[c] + f.momentum * (float)unbiased;
  }
}

// coef[0..2][C] = (k1, k2, k3) with dx = k1*dyr + k2*x + k3; dgamma/dbeta accumulate.
__device__ __forceinline__ void fin_bwd(const FinArgs& f, int c, double s1, double s2, int C) {
  // raw_z: the second sum is sum dyr*z (BN input), not sum dyr*xhat
  if (f.raw_z) s2 = (double)f.invstd[c] * (s2 - (double)f.mean[c] * s1);
  if (f.dbeta) f.dbeta[c] += (float)s1;
  if (f.dgamma) f.dgamma[c] += (float)s2;
  if (f.coef) {
    const double is = f.invstd[c];
    const double k1 = (f.gamma ? (double)f.gamma[c] : 1.0) * is;
    const double k2 = -k1 * is * s2 / f.count;
    const double k3 = -k1 * s1 / f.count - k2 * (double)f.mean[c];
    f.coef[c] = (float)k1;
    f.coef[C + c] = (float)k2;
    f.coef[2 * C + c] = (float)k3;
  }
}

}  // namespace dlmpi
