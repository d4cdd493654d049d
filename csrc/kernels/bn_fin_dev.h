// Train-mode BatchNorm coefficients derived in the CONSUMER kernel from the
// atomically accumulated per-channel totals (atomic reduction modes, see
// conv_igemm.hip g_red_atomic): sums = R rows of [2][C] (sum, sum of squares)
// of the M bf16 conv outputs, summed here in a fixed order.  Every block
// derives the scale/shift of all channels into LDS (a few flops), and block 0
// publishes the full coefficient table coef [4][C] (mean, invstd, scale, shift
// -- what the backward kernels read) and updates the running statistics: the
// bn_finalize launch is gone.
// Identical arithmetic to bn_finalize_kernel, so both modes give the same
// coefficients for the same totals.
#pragma once
#include "dl_common.h"

namespace dl {

struct BnFin {
  const float* sums;  // [R][2][C]; nullptr: coefficients are read from coef (mode 0 / eval)
  const float* gamma;
  const float* beta;
  const float* bias;  // conv bias (running mean bookkeeping), may be null
  float* rmean;
  float* rvar;
  float* coef;        // [4][C] written by block 0
  int64_t M;
  float eps, momentum;
  int R;              // accumulated rows in sums
};

__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  f[0] = lo_bf16(v.x); f[1] = hi_bf16(v.x); f[2] = lo_bf16(v.y); f[3] = hi_bf16(v.y);
  f[4] = lo_bf16(v.z); f[5] = hi_bf16(v.z); f[6] = lo_bf16(v.w); f[7] = hi_bf16(v.w);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  return make_uint4(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]), pack_bf16x2(f[4], f[5]),
                    pack_bf16x2(f[6], f[7]));
}

// The forward BN -> ReLU -> 2x2 max-pool of 8 channels: max over the window
// v0..v3 of relu(sc*y + sh) (bf16 in / out).  Shared by the BN consumer
// kernel (bn_pool.hip) and the conv that pools its input on load
// (conv_igemm.hip, region kernel PL), so both produce the same bits.
// sc_ / sh_: 8 consecutive LDS floats, 16-byte aligned, read as two 16-byte
// vectors each (8 scalar pairs measured 6.06 vs 5.95 us per fwd-fin launch)
__device__ __forceinline__ uint4 bn_relu_pool8(const uint4& v0, const uint4& v1, const uint4& v2, const uint4& v3,
                                               const float* sc_, const float* sh_) {
  float sc[8], sh[8], f[8], mx[8];
  const float4 a0 = reinterpret_cast<const float4*>(sc_)[0], a1 = reinterpret_cast<const float4*>(sc_)[1];
  const float4 b0 = reinterpret_cast<const float4*>(sh_)[0], b1 = reinterpret_cast<const float4*>(sh_)[1];
  sc[0] = a0.x; sc[1] = a0.y; sc[2] = a0.z; sc[3] = a0.w; sc[4] = a1.x; sc[5] = a1.y; sc[6] = a1.z; sc[7] = a1.w;
  sh[0] = b0.x; sh[1] = b0.y; sh[2] = b0.z; sh[3] = b0.w; sh[4] = b1.x; sh[5] = b1.y; sh[6] = b1.z; sh[7] = b1.w;
  unpack8(v0, f);
#pragma unroll
  for (int k = 0; k < 8; ++k) mx[k] = fmaf(sc[k], f[k], sh[k]);
  unpack8(v1, f);
#pragma unroll
  for (int k = 0; k < 8; ++k) mx[k] = fmaxf(mx[k], fmaf(sc[k], f[k], sh[k]));
  unpack8(v2, f);
#pragma unroll
  for (int k = 0; k < 8; ++k) mx[k] = fmaxf(mx[k], fmaf(sc[k], f[k], sh[k]));
  unpack8(v3, f);
#pragma unroll
  for (int k = 0; k < 8; ++k) mx[k] = fmaxf(fmaxf(mx[k], fmaf(sc[k], f[k], sh[k])), 0.f);
  return pack8(mx);
}

constexpr int kFinMaxC = 1024;  // channels of the block-cooperative (LDS) coefficient tables
constexpr int kMaxRows = 32;    // accumulated rows (set_reduce_atomic caps R at 64; the executors use <= 32)

// t1 = sum_r p[r*stride], t2 = sum_r p[r*stride + off2] over r < R, in row
// order.  Every load is issued before the first add (straight-line code per
// row count): the rows were just written by memory-side atomics, so each
// load is a full memory round trip, and a dependent chain of R of them cost
// ~0.5 us per row (measured: 4-8 us per consumer kernel at R = 16).
template <int RR>
__device__ __forceinline__ void sum_rows2_t(const float* __restrict__ p, int stride, int off2, float& t1, float& t2) {
  float a[RR], b[RR];
#pragma unroll
  for (int r = 0; r < RR; ++r) {
    a[r] = p[(int64_t)r * stride];
    b[r] = p[(int64_t)r * stride + off2];
  }
  t1 = 0.f;
  t2 = 0.f;
#pragma unroll
  for (int r = 0; r < RR; ++r) { t1 += a[r]; t2 += b[r]; }
}

__device__ __forceinline__ void sum_rows2(const float* __restrict__ p, int stride, int off2, int R, float& t1,
                                          float& t2) {
  switch (R) {  // wave-uniform; R is a power of two <= kMaxRows (host-checked)
    case 1: sum_rows2_t<1>(p, stride, off2, t1, t2); break;
    case 2: sum_rows2_t<2>(p, stride, off2, t1, t2); break;
    case 4: sum_rows2_t<4>(p, stride, off2, t1, t2); break;
    case 8: sum_rows2_t<8>(p, stride, off2, t1, t2); break;
    case 16: sum_rows2_t<16>(p, stride, off2, t1, t2); break;
    default: {
      // R = 32 as two 16-row passes: a 32-deep instance held 64 loads in flight
      // and set the register budget of every kernel that includes this switch
      // (the row-summing consumers then ran at 2-3 blocks per CU)
      t1 = t2 = 0.f;
#pragma unroll 1
      for (int h = 0; h < R; h += 16) {
        float u1, u2;
        sum_rows2_t<16>(p + (int64_t)h * stride, stride, off2, u1, u2);
        t1 += u1;
        t2 += u2;
      }
      break;
    }
  }
}

__device__ __forceinline__ void bn_fin_from_sums(const BnFin& f, float gam, float bet, float t1, float t2, float& mean,
                                                 float& var, float& invstd, float& sc, float& sh) {
  mean = t1 / (float)f.M;
  var = fmaxf(t2 / (float)f.M - mean * mean, 0.f);
  invstd = rsqrtf(var + f.eps);
  sc = gam * invstd;
  sh = bet - mean * sc;
}

__device__ __forceinline__ void bn_fin_channel(const BnFin& f, int C, int c, float& mean, float& var, float& invstd,
                                               float& sc, float& sh) {
  const float gam = f.gamma[c], bet = f.beta[c];  // issued with (not after) the row loads
  float t1, t2;
  sum_rows2(f.sums + c, 2 * C, C, f.R, t1, t2);
  bn_fin_from_sums(f, gam, bet, t1, t2, mean, var, invstd, sc, sh);
}

// Two channels per thread (c and c + off) with all 4R row loads in flight at
// once: the C = 2 x blockDim case (the head's 512 channels over 256 threads),
// which as two loop iterations paid two dependent memory round trips.
template <int RR>
__device__ __forceinline__ void sum_rows2x2_t(const float* __restrict__ p, int off, int stride, int off2, float (&t)[4]) {
  float a[RR], b[RR], c[RR], d[RR];
#pragma unroll
  for (int r = 0; r < RR; ++r) {
    a[r] = p[(int64_t)r * stride];
    b[r] = p[(int64_t)r * stride + off2];
    c[r] = p[(int64_t)r * stride + off];
    d[r] = p[(int64_t)r * stride + off + off2];
  }
  t[0] = t[1] = t[2] = t[3] = 0.f;
#pragma unroll
  for (int r = 0; r < RR; ++r) { t[0] += a[r]; t[1] += b[r]; t[2] += c[r]; t[3] += d[r]; }
}

__device__ __forceinline__ void sum_rows2x2(const float* __restrict__ p, int off, int stride, int off2, int R,
                                            float (&t)[4]) {
  switch (R) {
    case 1: sum_rows2x2_t<1>(p, off, stride, off2, t); break;
    case 2: sum_rows2x2_t<2>(p, off, stride, off2, t); break;
    case 4: sum_rows2x2_t<4>(p, off, stride, off2, t); break;
    case 8: sum_rows2x2_t<8>(p, off, stride, off2, t); break;
    case 16: sum_rows2x2_t<16>(p, off, stride, off2, t); break;
    default: {  // R = 32: two 16-row passes (see sum_rows2)
      t[0] = t[1] = t[2] = t[3] = 0.f;
#pragma unroll 1
      for (int h = 0; h < R; h += 16) {
        float u[4];
        sum_rows2x2_t<16>(p + (int64_t)h * stride, off, stride, off2, u);
        t[0] += u[0]; t[1] += u[1]; t[2] += u[2]; t[3] += u[3];
      }
      break;
    }
  }
}

// LDS-only block barrier: global loads issued before it stay in flight (a
// consumer issues its first item's loads, then derives the coefficients, so
// the two memory round trips overlap instead of adding up).
__device__ __forceinline__ static void fin_block_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Block-cooperative: scale / shift of ALL C channels into LDS (ssc, ssh [C]),
// each channel's rows summed once per block instead of once per thread;
// block 0 also publishes coef + running statistics.  Ends with an LDS barrier.
// smu / sis (optional): also the mean and invstd per channel.
__device__ __forceinline__ void bn_fin_publish(const BnFin& f, int C, int c, float mean, float var, float invstd, float sc,
                                               float sh, float* ssc, float* ssh, float* smu, float* sis) {
  ssc[c] = sc;
  ssh[c] = sh;
  if (smu != nullptr) {
    smu[c] = mean;
    sis[c] = invstd;
  }
  if (blockIdx.x == 0) {
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

__device__ __forceinline__ void bn_fin_block(const BnFin& f, int C, float* ssc, float* ssh, float* smu = nullptr,
                                             float* sis = nullptr) {
  if (C == 2 * (int)blockDim.x) {  // block-uniform: both channels' rows in one memory round trip
    const int c0 = threadIdx.x, c1 = c0 + blockDim.x;
    const float g0 = f.gamma[c0], b0 = f.beta[c0], g1 = f.gamma[c1], b1 = f.beta[c1];
    float t[4];
    sum_rows2x2(f.sums + c0, blockDim.x, 2 * C, C, f.R, t);
    float mean, var, invstd, sc, sh;
    bn_fin_from_sums(f, g0, b0, t[0], t[1], mean, var, invstd, sc, sh);
    bn_fin_publish(f, C, c0, mean, var, invstd, sc, sh, ssc, ssh, smu, sis);
    bn_fin_from_sums(f, g1, b1, t[2], t[3], mean, var, invstd, sc, sh);
    bn_fin_publish(f, C, c1, mean, var, invstd, sc, sh, ssc, ssh, smu, sis);
    fin_block_sync();
    return;
  }
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float mean, var, invstd, sc, sh;
    bn_fin_channel(f, C, c, mean, var, invstd, sc, sh);
    ssc[c] = sc;
    ssh[c] = sh;
    if (smu != nullptr) {
      smu[c] = mean;
      sis[c] = invstd;
    }
    if (blockIdx.x == 0) {
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
  fin_block_sync();
}

inline BnFin make_bn_fin(uintptr_t sums, int64_t M, uintptr_t gamma, uintptr_t beta, uintptr_t bias, uintptr_t rmean,
                         uintptr_t rvar, float eps, float momentum, uintptr_t coef, int R) {
  return BnFin{(const float*)sums, (const float*)gamma, (const float*)beta, (const float*)bias, (float*)rmean,
               (float*)rvar, (float*)coef, M, eps, momentum, R};
}

}  // namespace dl
