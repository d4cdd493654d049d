// Train-mode BatchNorm coefficients derived in the CONSUMER kernel from the
// atomically accumulated per-channel totals (reduction mode 1, see
// conv_igemm.hip g_red_atomic): sums = [2][C] (sum, sum of squares) of the M
// bf16 conv outputs.  Every thread derives the scale/shift of the channels it
// touches (a few flops), and block 0 publishes the full coefficient table
// coef [4][C] (mean, invstd, scale, shift -- what the backward kernels read)
// and updates the running statistics: the bn_finalize launch is gone.
// Identical arithmetic to bn_finalize_kernel, so both modes give the same
// coefficients for the same totals.
#pragma once
#include "dl_common.h"

namespace dl {

struct BnFin {
  const float* sums;  // [2][C]; nullptr: coefficients are read from coef (mode 0 / eval)
  const float* gamma;
  const float* beta;
  const float* bias;  // conv bias (running mean bookkeeping), may be null
  float* rmean;
  float* rvar;
  float* coef;        // [4][C] written by block 0
  int64_t M;
  float eps, momentum;
};

__device__ __forceinline__ void bn_fin_channel(const BnFin& f, int C, int c, float& mean, float& var, float& invstd,
                                               float& sc, float& sh) {
  const float t1 = f.sums[c], t2 = f.sums[C + c];
  mean = t1 / (float)f.M;
  var = fmaxf(t2 / (float)f.M - mean * mean, 0.f);
  invstd = rsqrtf(var + f.eps);
  sc = f.gamma[c] * invstd;
  sh = f.beta[c] - mean * sc;
}

// scale / shift of channels c0..c0+7
__device__ __forceinline__ void bn_fin_coef8(const BnFin& f, int C, int c0, float* sc, float* sh) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float mean, var, invstd;
    bn_fin_channel(f, C, c0 + k, mean, var, invstd, sc[k], sh[k]);
  }
}

// block 0: coefficient table + running statistics
__device__ __forceinline__ void bn_fin_publish(const BnFin& f, int C) {
  if (blockIdx.x != 0) return;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float mean, var, invstd, sc, sh;
    bn_fin_channel(f, C, c, mean, var, invstd, sc, sh);
    f.coef[c] = mean;
    f.coef[C + c] = invstd;
    f.coef[2 * C + c] = sc;
    f.coef[3 * C + c] = sh;
    if (f.rmean != nullptr) {
      const float unbiased = f.M > 1 ? var * (float)f.M / (float)(f.M - 1) : var;
      f.rmean[c] = (1.f - f.momentum) * f.rmean[c] + f.momentum * (mean + (f.bias ? f.bias[c] : 0.f));
      f.rvar[c] = (1.f - f.momentum) * f.rvar[c] + f.momentum * unbiased;
    }
  }
}

inline BnFin make_bn_fin(uintptr_t sums, int64_t M, uintptr_t gamma, uintptr_t beta, uintptr_t bias, uintptr_t rmean,
                         uintptr_t rvar, float eps, float momentum, uintptr_t coef) {
  return BnFin{(const float*)sums, (const float*)gamma, (const float*)beta, (const float*)bias, (float*)rmean,
               (float*)rvar, (float*)coef, M, eps, momentum};
}

}  // namespace dl
