// Per-channel training-BatchNorm coefficients from the accumulated [2C]
// (sum, sum of squares) of its input, shared by every kernel that applies a
// channels-last BN (bn_nhwc.hip, and the BN applied on load by the stem
// max-pool, pool_nhwc.hip): one copy of the arithmetic, with explicit fmas so
// every inlined instance rounds the same way (the fused paths are tested
// BITWISE against the BN's own apply).
#pragma once
#include "dl_common.h"

namespace dl {

__device__ __forceinline__ float bn_var_of(const float* __restrict__ acc, int C, int i, float invM, float m) {
  return fmaxf(fmaf(-m, m, acc[C + i] * invM), 0.f);
}

__device__ __forceinline__ void bn_stats8(const float* __restrict__ acc, int C, int c, float invM, float eps,
                                          float* mean, float* invstd) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float m = acc[c + k] * invM;
    mean[k] = m;
    invstd[k] = rsqrtf(bn_var_of(acc, C, c + k, invM, m) + eps);
  }
}

// scale / shift of 8 channels c.. (y = x * sc + sh); `publish`: also write the
// saved mean / invstd and update the running statistics (one thread per channel)
__device__ __forceinline__ void bn_coef8(const float* __restrict__ acc, const float* __restrict__ w,
                                         const float* __restrict__ b, int C, int c, int64_t M, float eps,
                                         float momentum, bool publish, float* __restrict__ save,
                                         float* __restrict__ run_mean, float* __restrict__ run_var, float* sc,
                                         float* sh) {
  const float invM = 1.f / (float)M;
  float mean[8], invstd[8];
  bn_stats8(acc, C, c, invM, eps, mean, invstd);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sc[k] = w[c + k] * invstd[k];
    sh[k] = fmaf(-mean[k], sc[k], b[c + k]);
  }
  if (publish) {
    const float unbias = M > 1 ? (float)M / (float)(M - 1) : 1.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      save[c + k] = mean[k];
      save[C + c + k] = invstd[k];
      if (run_mean != nullptr) {
        const float var = bn_var_of(acc, C, c + k, invM, mean[k]);
        const float keep_m = (1.f - momentum) * run_mean[c + k], keep_v = (1.f - momentum) * run_var[c + k];
        run_mean[c + k] = fmaf(momentum, mean[k], keep_m);
        run_var[c + k] = fmaf(momentum, var * unbias, keep_v);
      }
    }
  }
}

}  // namespace dl
