// Channels-last (NHWC) training BatchNorm for the ResNet-50 path, fused with
// the activation and the residual add of a bottleneck:
//
//   forward   y  = act(x * scale + shift [+ res])        scale = w * invstd
//   backward  g  = dy * (y > 0)            (relu; dres = g when fused with +res)
//             dx = w * invstd * (g - mean(g) - xhat * mean(g * xhat))
//
// bf16 activations, fp32 statistics.  Replaces MIOpen's BN (+ torch's separate
// ReLU / add / ReLU-backward passes, each a full HBM round trip of the
// activation): measured in the ResNet-50 profile at 34 % (BN) + 19 %
// (elementwise) of the step (profiles/r1_resnet50_kernels.txt).
//
// Layout: x is [M, C] (M = N*H*W rows), each thread owns 8 consecutive
// channels (one 16-byte load per row).  A block covers CVB channel vectors
// (<= 256 channels) and RPI = 256 / CVB rows per iteration; the grid is
// (row blocks, channel groups).  Per-channel sums are reduced in LDS inside a
// block and across blocks with one fp32 global atomic per channel per block
// (vector-memory atomics; acc is zeroed by the host before each reduce).
// The apply kernels recompute mean / invstd from the sums; block (0, g) writes
// the saved statistics (and running stats / weight gradients) of its channels.
#include "dl_common.h"
#include "bn_coef_dev.h"
#include "dl_ops.h"

namespace dl {

namespace {

constexpr int kThreads = 256;

struct BnGeom {
  int64_t M;
  int C;
  int CVB;             // channel vectors (of 8) per block
  int RPI;             // rows per block iteration (= 256 / CVB)
  int64_t rows_per_block;
  // padded OUTPUT layout (apply kernels' y / dx): row m = (n, h, w) of an H x W
  // image is stored at pixel (n, h + opad, w + opad) of [N][H+2opad][W+2opad];
  // opad 0 = the input's row order.  The consumer is a 3x3 convolution that
  // reads its zero-bordered input directly (ops/conv.py Conv3x3).
  int H, W, opad;
  float inv_HW, inv_W;
};

// output row of input row `row` (see BnGeom); float-reciprocal division with
// one correction step (rows < 2^24, checked on the host)
__device__ __forceinline__ int64_t out_row(const BnGeom& g, int64_t row) {
  if (g.opad == 0) return row;
  const int HW = g.H * g.W, m = (int)row;
  int n = (int)((float)m * g.inv_HW), rem = m - n * HW;
  if (rem < 0) { --n; rem += HW; } else if (rem >= HW) { ++n; rem -= HW; }
  int h = (int)((float)rem * g.inv_W), w = rem - h * g.W;
  if (w < 0) { --h; w += g.W; } else if (w >= g.W) { ++h; w -= g.W; }
  const int Hp = g.H + 2 * g.opad, Wp = g.W + 2 * g.opad;
  return ((int64_t)n * Hp + h + g.opad) * Wp + w + g.opad;
}

__device__ __forceinline__ void unpack8(u32x4 v, float* f) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    f[2 * k] = __uint_as_float(v[k] << 16);
    f[2 * k + 1] = __uint_as_float(v[k] & 0xffff0000u);
  }
}

__device__ __forceinline__ u32x4 pack8(const float* f) {
  u32x4 v;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    v[k] = (uint32_t)f32_to_bf16(f[2 * k]) | ((uint32_t)f32_to_bf16(f[2 * k + 1]) << 16);
  return v;
}

// Sum a[8] and b[8] of every thread over the RPI row lanes of the block; add
// the block totals of its channels to acc[c] / acc[C + c].
template <int NT>
__device__ __forceinline__ void block_reduce_atomic(const float* a, const float* b, const BnGeom& g, int c0,
                                                    float* __restrict__ acc) {
  __shared__ float red[NT * 16];
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[t * 16 + k] = a[k];
    red[t * 16 + 8 + k] = b[k];
  }
  __syncthreads();
  const int nch = g.CVB * 8;
  for (int j = t; j < 2 * nch; j += NT) {
    const int which = j / nch, ch = j - which * nch;
    const int cv = ch >> 3, k = ch & 7;
    float s = 0.f;
    for (int r = 0; r < g.RPI; ++r) s += red[(r * g.CVB + cv) * 16 + which * 8 + k];
    atomicAdd(&acc[which * g.C + c0 + ch], s);
  }
}

template <int NT>
__global__ void __launch_bounds__(NT) bn_nhwc_stats_kernel(const bf16_t* __restrict__ x, BnGeom g,
                                                             float* __restrict__ acc) {
  const int t = threadIdx.x, cv = t % g.CVB, r = t / g.CVB;
  const int c0 = blockIdx.y * g.CVB * 8;
  const int c = c0 + cv * 8;
  const int64_t row0 = (int64_t)blockIdx.x * g.rows_per_block;
  const int64_t row1 = min(g.M, row0 + g.rows_per_block);
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int64_t row = row0 + r;
  // four rows per iteration: four independent 16-byte loads in flight per thread
  for (; row + 3 * g.RPI < row1; row += 4 * g.RPI) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *(const u32x4*)(x + (row + u * g.RPI) * g.C + c);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float f[8];
      unpack8(v[u], f);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s[k] += f[k];
        q[k] = fmaf(f[k], f[k], q[k]);
      }
    }
  }
  for (; row < row1; row += g.RPI) {
    float f[8];
    unpack8(*(const u32x4*)(x + row * g.C + c), f);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s[k] += f[k];
      q[k] = fmaf(f[k], f[k], q[k]);
    }
  }
  block_reduce_atomic<NT>(s, q, g, c0, acc);
}

// bit k = bf16 output channel k is nonzero (relu output >= 0: > 0 <=> nonzero,
// the mask relu mode 1 derives from y)
__device__ __forceinline__ uint8_t mask_byte(const u32x4& o) {
  const uint32_t w[4] = {o[0], o[1], o[2], o[3]};
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    m |= (w[k] & 0x7fffu) ? (1u << (2 * k)) : 0u;
    m |= (w[k] & 0x7fff0000u) ? (1u << (2 * k + 1)) : 0u;
  }
  return (uint8_t)m;
}

// The BatchNorm of the residual branch applied on load (ResBn; the ResNet-50
// downsample BN feeding a block's b3): `res` is then that BN's INPUT, the
// residual added is bf16(res * rsc + rsh) -- bitwise what its own apply launch
// would have written -- and block 0 publishes its saved mean / invstd and
// running statistics.  Its apply launch and the write + read of its output go.
struct ResBn {
  const float* acc;  // [2C] sum, sum of squares of the residual BN's input (null: plain residual)
  const float* w;
  const float* b;
  float* save;  // [2C] mean, invstd (its backward's)
  float* run_mean;
  float* run_var;
  float eps, momentum;
};

template <int U>
__global__ void __launch_bounds__(kThreads) bn_nhwc_fwd_apply_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ res, bf16_t* __restrict__ y,
    const float* __restrict__ acc, const float* __restrict__ w, const float* __restrict__ b, BnGeom g, float eps,
    int relu, float* __restrict__ save, float* __restrict__ run_mean, float* __restrict__ run_var, float momentum,
    uint8_t* __restrict__ mbits, const ResBn rbn) {
  const int t = threadIdx.x, cv = t % g.CVB, r = t / g.CVB;
  const int c0 = blockIdx.y * g.CVB * 8;
  const int c = c0 + cv * 8;
  const bool publish = blockIdx.x == 0 && r == 0;
  float sc[8], sh[8], rsc[8], rsh[8];
  bn_coef8(acc, w, b, g.C, c, g.M, eps, momentum, publish, save, run_mean, run_var, sc, sh);
  const bool rbn_on = rbn.acc != nullptr;
  if (rbn_on)
    bn_coef8(rbn.acc, rbn.w, rbn.b, g.C, c, g.M, rbn.eps, rbn.momentum, publish, rbn.save, rbn.run_mean,
             rbn.run_var, rsc, rsh);
  const int64_t row0 = (int64_t)blockIdx.x * g.rows_per_block;
  const int64_t row1 = min(g.M, row0 + g.rows_per_block);
  const u32x4 z = {0u, 0u, 0u, 0u};
  auto apply = [&](int64_t off, int64_t row, const u32x4& xr, const u32x4& rr) {
    float f[8];
    unpack8(xr, f);
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] = fmaf(f[k], sc[k], sh[k]);
    if (res != nullptr) {
      float q[8];
      unpack8(rr, q);
      if (rbn_on) {  // the residual BN's output as its own apply would store it (bf16)
#pragma unroll
        for (int k = 0; k < 8; ++k) q[k] = __uint_as_float((uint32_t)f32_to_bf16(fmaf(q[k], rsc[k], rsh[k])) << 16);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] += q[k];
    }
    if (relu) {
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = fmaxf(f[k], 0.f);
    }
    const u32x4 o = pack8(f);
    *(u32x4*)(y + off) = o;
    if (mbits != nullptr) mbits[row * (g.C >> 3) + (c >> 3)] = mask_byte(o);  // relu mode 3
  };
  int64_t row = row0 + r;
  for (; row + (U - 1) * g.RPI < row1; row += U * g.RPI) {  // U rows' loads in flight
    u32x4 xv[U], rv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t o = (row + u * g.RPI) * g.C + c;
      xv[u] = *(const u32x4*)(x + o);
      rv[u] = res != nullptr ? *(const u32x4*)(res + o) : z;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) apply(out_row(g, row + u * g.RPI) * g.C + c, row + u * g.RPI, xv[u], rv[u]);
  }
  for (; row < row1; row += g.RPI) {
    const int64_t o0 = row * g.C + c;
    apply(out_row(g, row) * g.C + c, row, *(const u32x4*)(x + o0), res != nullptr ? *(const u32x4*)(res + o0) : z);
  }
}

// g = dy * relu'(.): relu 0 = identity, 1 = mask from the saved output y (BN
// fused with a residual add), 2 = mask recomputed from x (x * sc + sh > 0,
// bitwise the forward's pre-activation: same fp32 operands and fma), which
// saves reading y in both backward passes, 3 = mask bits written by the forward
// apply (BN + residual: one byte per 8 channels per row instead of re-reading
// the 16 bytes of y in each backward pass; bit k = output channel k nonzero,
// the same mask as mode 1) -- applied inline by the two kernels below, after
// all of an iteration's loads are issued.
// The backward of the residual branch's BatchNorm fused into the BN + residual
// + ReLU's backward (ResNet-50 downsample blocks): the residual's gradient IS
// g = dy * mask, so the reduce also sums g * xhat_r over the residual BN's
// input x_r (its sum(g) is the same as ours), and the apply writes that BN's
// input gradient a_r (g - mean g - xhat_r mean(g xhat_r)) where it would have
// written g -- the residual BN's own reduce and apply passes, and the write +
// two reads of g, go.
struct ResBnBwd {
  const bf16_t* x;   // the residual BN's input (null: plain residual gradient)
  const float* save;  // its [2C] mean, invstd
  const float* w;
  float* acc;         // its [2C] backward sums (zeroed), filled by the reduce
  float* dw;
  float* db;
};

template <int NT>
__global__ void __launch_bounds__(NT) bn_nhwc_bwd_reduce_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y, const bf16_t* __restrict__ x,
    const float* __restrict__ save, const float* __restrict__ w, const float* __restrict__ b, BnGeom g, int relu,
    float* __restrict__ acc, const uint8_t* __restrict__ mbits, const ResBnBwd rb) {
  const int t = threadIdx.x, cv = t % g.CVB, r = t / g.CVB;
  const int c0 = blockIdx.y * g.CVB * 8;
  const int c = c0 + cv * 8;
  float mean[8], invstd[8], sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mean[k] = save[c + k];
    invstd[k] = save[g.C + c + k];
    sc[k] = w[c + k] * invstd[k];
    sh[k] = fmaf(-mean[k], sc[k], b[c + k]);
  }
  const bool fr = rb.x != nullptr;
  float rmean[8], rinv[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    rmean[k] = fr ? rb.save[c + k] : 0.f;
    rinv[k] = fr ? rb.save[g.C + c + k] : 0.f;
  }
  float sg[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sgx[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sgr[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int64_t row0 = (int64_t)blockIdx.x * g.rows_per_block;
  const int64_t row1 = min(g.M, row0 + g.rows_per_block);
  auto accum = [&](const u32x4& xr, const u32x4& dr, const u32x4& yr, unsigned mb, const u32x4& rr) {
    float gv[8], xv[8];
    unpack8(xr, xv);
    unpack8(dr, gv);
    if (relu == 3) {
#pragma unroll
      for (int k = 0; k < 8; ++k) gv[k] = (mb >> k) & 1u ? gv[k] : 0.f;
    } else if (relu == 2) {
#pragma unroll
      for (int k = 0; k < 8; ++k) gv[k] = fmaf(xv[k], sc[k], sh[k]) > 0.f ? gv[k] : 0.f;
    } else if (relu) {
      float yy[8];
      unpack8(yr, yy);
#pragma unroll
      for (int k = 0; k < 8; ++k) gv[k] = yy[k] > 0.f ? gv[k] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sg[k] += gv[k];
      sgx[k] = fmaf(gv[k], (xv[k] - mean[k]) * invstd[k], sgx[k]);
    }
    if (fr) {
      float xrv[8];
      unpack8(rr, xrv);
#pragma unroll
      for (int k = 0; k < 8; ++k) sgr[k] = fmaf(gv[k], (xrv[k] - rmean[k]) * rinv[k], sgr[k]);
    }
  };
  // four rows per iteration: every load of the group is issued before any is
  // consumed (8-12 16-byte loads in flight per lane; the single-row loop ran at
  // ~2 TB/s on the ResNet-50 shapes, profiles/r2_pmc_hotpath.txt)
  constexpr int U = 4;
  int64_t row = row0 + r;
  const u32x4 z = {0u, 0u, 0u, 0u};
  for (; row + (U - 1) * g.RPI < row1; row += U * g.RPI) {
    u32x4 xr[U], dr[U], yr[U], rr[U];
    unsigned mb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t off = (row + u * g.RPI) * g.C + c;
      xr[u] = *(const u32x4*)(x + off);
      dr[u] = *(const u32x4*)(dy + off);
      yr[u] = relu == 1 ? *(const u32x4*)(y + off) : z;
      mb[u] = relu == 3 ? mbits[(row + u * g.RPI) * (g.C >> 3) + (c >> 3)] : 0u;
      rr[u] = fr ? *(const u32x4*)(rb.x + off) : z;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) accum(xr[u], dr[u], yr[u], mb[u], rr[u]);
  }
  for (; row < row1; row += g.RPI) {
    const int64_t off = row * g.C + c;
    accum(*(const u32x4*)(x + off), *(const u32x4*)(dy + off), relu == 1 ? *(const u32x4*)(y + off) : z,
          relu == 3 ? mbits[row * (g.C >> 3) + (c >> 3)] : 0u, fr ? *(const u32x4*)(rb.x + off) : z);
  }
  block_reduce_atomic<NT>(sg, sgx, g, c0, acc);
  if (fr) {
    __syncthreads();  // (block_reduce_atomic's LDS is reused)
    block_reduce_atomic<NT>(sg, sgr, g, c0, rb.acc);
  }
}

template <int U>
__global__ void __launch_bounds__(kThreads) bn_nhwc_bwd_apply_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y, const bf16_t* __restrict__ x,
    const float* __restrict__ save, const float* __restrict__ w, const float* __restrict__ b,
    const float* __restrict__ acc, BnGeom g, int relu, bf16_t* __restrict__ dx, bf16_t* __restrict__ dres, float* __restrict__ dw, float* __restrict__ db,
    const uint8_t* __restrict__ mbits, const ResBnBwd rb) {
  const int t = threadIdx.x, cv = t % g.CVB, r = t / g.CVB;
  const int c0 = blockIdx.y * g.CVB * 8;
  const int c = c0 + cv * 8;
  const float invM = 1.f / (float)g.M;
  float mean[8], invstd[8], a[8], sh[8], mg[8], mgx[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mean[k] = save[c + k];
    invstd[k] = save[g.C + c + k];
    a[k] = w[c + k] * invstd[k];
    sh[k] = fmaf(-mean[k], a[k], b[c + k]);
    mg[k] = acc[c + k] * invM;
    mgx[k] = acc[g.C + c + k] * invM;
  }
  // the residual BN's coefficients (ResBnBwd): dres <- its input gradient
  const bool fr = rb.x != nullptr;
  float rmean[8], rinv[8], ra[8], rmg[8], rmgx[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    rmean[k] = fr ? rb.save[c + k] : 0.f;
    rinv[k] = fr ? rb.save[g.C + c + k] : 0.f;
    ra[k] = fr ? rb.w[c + k] * rinv[k] : 0.f;
    rmg[k] = fr ? rb.acc[c + k] * invM : 0.f;
    rmgx[k] = fr ? rb.acc[g.C + c + k] * invM : 0.f;
  }
  if (blockIdx.x == 0 && r == 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      db[c + k] = acc[c + k];
      dw[c + k] = acc[g.C + c + k];
      if (fr) {
        rb.db[c + k] = rb.acc[c + k];
        rb.dw[c + k] = rb.acc[g.C + c + k];
      }
    }
  }
  const int64_t row0 = (int64_t)blockIdx.x * g.rows_per_block;
  const int64_t row1 = min(g.M, row0 + g.rows_per_block);
  const u32x4 z = {0u, 0u, 0u, 0u};
  auto apply = [&](int64_t off, int64_t doff, const u32x4& xr, const u32x4& dr, const u32x4& yr, unsigned mb,
                   const u32x4& rr) {
    float gv[8], xv[8], o[8];
    unpack8(xr, xv);
    unpack8(dr, gv);
    if (relu == 3) {
#pragma unroll
      for (int k = 0; k < 8; ++k) gv[k] = (mb >> k) & 1u ? gv[k] : 0.f;
    } else if (relu == 2) {
#pragma unroll
      for (int k = 0; k < 8; ++k) gv[k] = fmaf(xv[k], a[k], sh[k]) > 0.f ? gv[k] : 0.f;
    } else if (relu) {
      float yy[8];
      unpack8(yr, yy);
#pragma unroll
      for (int k = 0; k < 8; ++k) gv[k] = yy[k] > 0.f ? gv[k] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float xh = (xv[k] - mean[k]) * invstd[k];
      o[k] = a[k] * (gv[k] - mg[k] - xh * mgx[k]);
    }
    *(u32x4*)(dx + doff) = pack8(o);
    if (fr) {  // the residual BN's input gradient in place of g
      float xrv[8], orr[8];
      unpack8(rr, xrv);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float xh = (xrv[k] - rmean[k]) * rinv[k];
        orr[k] = ra[k] * (gv[k] - rmg[k] - xh * rmgx[k]);
      }
      *(u32x4*)(dres + off) = pack8(orr);
    } else if (dres != nullptr) {
      *(u32x4*)(dres + off) = pack8(gv);
    }
  };
  int64_t row = row0 + r;
  for (; row + (U - 1) * g.RPI < row1; row += U * g.RPI) {  // U rows' loads in flight
    u32x4 xv[U], dv[U], yv[U], rv[U];
    unsigned mb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t o = (row + u * g.RPI) * g.C + c;
      xv[u] = *(const u32x4*)(x + o);
      dv[u] = *(const u32x4*)(dy + o);
      yv[u] = relu == 1 ? *(const u32x4*)(y + o) : z;
      mb[u] = relu == 3 ? mbits[(row + u * g.RPI) * (g.C >> 3) + (c >> 3)] : 0u;
      rv[u] = fr ? *(const u32x4*)(rb.x + o) : z;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      apply((row + u * g.RPI) * g.C + c, out_row(g, row + u * g.RPI) * g.C + c, xv[u], dv[u], yv[u], mb[u], rv[u]);
  }
  for (; row < row1; row += g.RPI) {
    const int64_t o0 = row * g.C + c;
    apply(o0, out_row(g, row) * g.C + c, *(const u32x4*)(x + o0), *(const u32x4*)(dy + o0),
          relu == 1 ? *(const u32x4*)(y + o0) : z, relu == 3 ? mbits[row * (g.C >> 3) + (c >> 3)] : 0u,
          fr ? *(const u32x4*)(rb.x + o0) : z);
  }
}

// max_rb: cap on the row blocks.  The statistics / backward-reduce kernels end
// with one fp32 atomic per channel per block, and same-address atomics from
// thousands of blocks serialise (the C = 64 statistics pass ran at ~2 TB/s with
// 2048 blocks): they use g_reduce_blocks, the apply kernels the default.  Swept
// on the ResNet-50 shapes (scripts/bench_bn.py BN_RB=..., profiles/r2_bn_reduce_blocks.txt):
// sum of statistics + backward times 2831 / 2450 / 2527 / 2626 us for 128 / 256 / 512 / 1024.
static int64_t g_reduce_blocks = 256;
// rows in flight per thread in the apply kernels (2 or 4) and the block size
// of the statistics / backward-reduce kernels (256, 512 or 1024): with the
// grid capped at g_reduce_blocks, the block size sets the waves per CU
static int g_apply_rows = 4;
static int g_reduce_threads = 256;

BnGeom make_geom(int64_t M, int C, dim3* grid, int64_t max_rb = 2048, int nt = kThreads) {
  if (M <= 0 || C <= 0 || C % 8 != 0 || (nt % (C / 8 < 32 ? C / 8 : 32)) != 0 ||
      (C / 8 > 32 && (C / 8) % 32 != 0))
    throw std::runtime_error("bn_nhwc: C must be a multiple of 8 dividing 256*8 or a multiple of 256 (got " +
                             std::to_string(C) + ")");
  BnGeom g;
  g.M = M;
  g.C = C;
  g.CVB = C / 8 < 32 ? C / 8 : 32;
  g.RPI = nt / g.CVB;
  const int groups = (C / 8) / g.CVB;
  int64_t cap = 262144 / C;
  if (cap < 64) cap = 64;
  if (cap > max_rb) cap = max_rb;
  int64_t rb = (M + (int64_t)g.RPI * 16 - 1) / ((int64_t)g.RPI * 16);
  if (rb > cap) rb = cap;
  if (rb < 1) rb = 1;
  int64_t rpb = (M + rb - 1) / rb;
  rpb = (rpb + g.RPI - 1) / g.RPI * g.RPI;
  rb = (M + rpb - 1) / rpb;
  g.rows_per_block = rpb;
  g.H = g.W = 1;
  g.opad = 0;
  g.inv_HW = g.inv_W = 1.f;
  *grid = dim3((unsigned)rb, (unsigned)groups);
  return g;
}

// set the padded output layout of the apply kernels (BnGeom)
void set_out_pad(BnGeom& g, int H, int W, int opad) {
  if (opad == 0) return;
  if (opad < 0 || H <= 0 || W <= 0 || g.M % ((int64_t)H * W) != 0 || g.M >= (1 << 24))
    throw std::runtime_error("bn_nhwc: bad padded-output geometry");
  g.H = H;
  g.W = W;
  g.opad = opad;
  g.inv_HW = 1.f / (float)(H * W);
  g.inv_W = 1.f / (float)W;
}

// zero the border ring of a [N][H+2p][W+2p][C] bf16 buffer (its interior is
// written by an apply kernel with the padded output layout)
// Items enumerate only the border pixels (top p rows, the p left + p right
// pixels of the H interior rows, bottom p rows; 6.8 % of a 58x58 image): the
// first version swept the whole buffer and skipped the interior (9.8 us per
// call on the 56x56x64 ResNet-50 buffers, 32 calls per step).
__global__ void __launch_bounds__(kThreads) zero_border_kernel(bf16_t* __restrict__ buf, int N, int H, int W, int C,
                                                               int p) {
  const int Hp = H + 2 * p, Wp = W + 2 * p, C8 = C >> 3;
  const int per_img = Hp * Wp - H * W;
  const int64_t total = (int64_t)N * per_img * C8;
  const u32x4 z = {0u, 0u, 0u, 0u};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % C8);
    const int64_t t = i / C8;
    const int64_t n = t / per_img;
    int b = (int)(t - n * per_img), h, w;
    if (b < p * Wp) {  // top rows
      h = b / Wp;
      w = b - h * Wp;
    } else if ((b -= p * Wp) < H * 2 * p) {  // left / right columns of the interior rows
      const int r = b / (2 * p), k = b - r * 2 * p;
      h = p + r;
      w = k < p ? k : W + k;
    } else {  // bottom rows
      b -= H * 2 * p;
      h = p + H + b / Wp;
      w = b % Wp;
    }
    *(u32x4*)(buf + ((n * Hp + h) * Wp + w) * C + c8 * 8) = z;
  }
}

}  // namespace

// Column sums of a convolution epilogue's deterministic per-M-tile partial
// rows [T][2][C] (sum, sum of squares) into acc [2C] (one block per channel,
// fixed order): the BatchNorm statistics of a 1x1 conv output for T*2C reads
// instead of a pass over the M*C activation (ops/conv.py).
// acc[c] += sum_t rows[t][0][c], acc[C + c] += sum_t rows[t][1][c] (acc zeroed by
// the caller: the per-step BatchNorm arena).  Grid (C/64 channel groups, S row
// chunks), block = 64 consecutive channels x 4 row lanes: every row read is a
// coalesced 256-B segment (one block per channel read one float per 64-B line,
// 16x the bytes), 4 rows of loads in flight per thread, one atomic per channel
// per block.
__global__ void __launch_bounds__(kThreads) bn_rows_reduce_kernel(const float* __restrict__ rows, int T, int C,
                                                                  float* __restrict__ acc, int rows_per_chunk) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), ly = threadIdx.x >> 6;
  const int t0 = blockIdx.y * rows_per_chunk, t1 = min(T, t0 + rows_per_chunk);
  float s1 = 0.f, s2 = 0.f;
  if (c < C) {
    int t = t0 + ly;
    for (; t + 12 < t1; t += 16) {
      float a[4], b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[u] = rows[(int64_t)(t + 4 * u) * 2 * C + c];
        b[u] = rows[(int64_t)(t + 4 * u) * 2 * C + C + c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) { s1 += a[u]; s2 += b[u]; }
    }
    for (; t < t1; t += 4) {
      s1 += rows[(int64_t)t * 2 * C + c];
      s2 += rows[(int64_t)t * 2 * C + C + c];
    }
  }
  __shared__ float red[2][4][64];
  red[0][ly][threadIdx.x & 63] = s1;
  red[1][ly][threadIdx.x & 63] = s2;
  __syncthreads();
  if (ly == 0 && c < C) {
    const int i = threadIdx.x & 63;
    atomicAdd(acc + c, red[0][0][i] + red[0][1][i] + red[0][2][i] + red[0][3][i]);
    atomicAdd(acc + C + c, red[1][0][i] + red[1][1][i] + red[1][2][i] + red[1][3][i]);
  }
}

void set_bn_reduce_blocks(int n) { g_reduce_blocks = n < 64 ? 64 : n; }

void set_bn_tuning(int apply_rows, int reduce_threads) {
  if ((apply_rows != 2 && apply_rows != 4) ||
      (reduce_threads != 256 && reduce_threads != 512 && reduce_threads != 1024))
    throw std::runtime_error("set_bn_tuning: apply_rows 2|4, reduce_threads 256|512|1024");
  g_apply_rows = apply_rows;
  g_reduce_threads = reduce_threads;
}

void bn_rows_reduce(uintptr_t rows, int T, int C, uintptr_t acc, uintptr_t stream) {
  if (T <= 0 || C <= 0) throw std::runtime_error("bn_rows_reduce: empty");
  const int cg = (C + 63) / 64;
  const int chunks = std::max(1, std::min((T + 63) / 64, (256 + cg - 1) / cg));  // ~256 blocks, >= 64 rows each
  const int rpc = (T + chunks - 1) / chunks;
  bn_rows_reduce_kernel<<<dim3(cg, (T + rpc - 1) / rpc), kThreads, 0, as_stream(stream)>>>((const float*)rows, T, C,
                                                                                       (float*)acc, rpc);
  DL_HIP_CHECK(hipGetLastError());
}

// acc: fp32 [2C], zeroed by the caller.  have_stats: acc already holds the
// per-channel sum / sum of squares of x (emitted by the producing 1x1
// convolution's epilogue, ops/conv.py): the statistics pass is skipped.
void bn_nhwc_fwd(uintptr_t x, uintptr_t res, uintptr_t y, uintptr_t acc, uintptr_t w, uintptr_t b, uintptr_t save,
                 uintptr_t run_mean, uintptr_t run_var, int64_t M, int C, double eps, double momentum, int relu,
                 int have_stats, uintptr_t stream) {
  bn_nhwc_fwd_pad(x, res, y, acc, w, b, save, run_mean, run_var, M, C, eps, momentum, relu, have_stats, 1, 1, 0,
                  stream, 0);
}

// y in the padded layout [N][H+2opad][W+2opad][C] (interior only; see zero_border_nhwc)
// rbn_acc != 0: `res` is the input of the residual branch's BatchNorm, applied
// on load (ResBn: rbn_acc = its [2C] sums, complete; rbn_w / rbn_b its affine
// parameters; rbn_save / rbn_rm / rbn_rv what its own apply would write)
void bn_nhwc_fwd_pad(uintptr_t x, uintptr_t res, uintptr_t y, uintptr_t acc, uintptr_t w, uintptr_t b,
                     uintptr_t save, uintptr_t run_mean, uintptr_t run_var, int64_t M, int C, double eps,
                     double momentum, int relu, int have_stats, int H, int W, int opad, uintptr_t stream,
                     uintptr_t mbits, uintptr_t rbn_acc, uintptr_t rbn_w, uintptr_t rbn_b, uintptr_t rbn_save,
                     uintptr_t rbn_rm, uintptr_t rbn_rv, double rbn_eps, double rbn_momentum) {
  if (mbits && !relu) throw std::runtime_error("bn_nhwc_fwd: mask bits need the ReLU");
  if (rbn_acc && (!res || !rbn_w || !rbn_b || !rbn_save))
    throw std::runtime_error("bn_nhwc_fwd: the residual BN needs its input, affine parameters and save buffer");
  const ResBn rbn{(const float*)rbn_acc, (const float*)rbn_w, (const float*)rbn_b, (float*)rbn_save,
                  (float*)rbn_rm, (float*)rbn_rv, (float)rbn_eps, (float)rbn_momentum};
  dim3 grid, grid_r;
  BnGeom g = make_geom(M, C, &grid);
  set_out_pad(g, H, W, opad);
  hipStream_t s = as_stream(stream);
  if (!have_stats) {
    const int nt = g_reduce_threads;
    const BnGeom gr = make_geom(M, C, &grid_r, g_reduce_blocks, nt);
    if (nt == 1024)
      bn_nhwc_stats_kernel<1024><<<grid_r, 1024, 0, s>>>((const bf16_t*)x, gr, (float*)acc);
    else if (nt == 512)
      bn_nhwc_stats_kernel<512><<<grid_r, 512, 0, s>>>((const bf16_t*)x, gr, (float*)acc);
    else
      bn_nhwc_stats_kernel<256><<<grid_r, 256, 0, s>>>((const bf16_t*)x, gr, (float*)acc);
    DL_HIP_CHECK(hipGetLastError());
  }
  auto fk = g_apply_rows == 4 ? bn_nhwc_fwd_apply_kernel<4> : bn_nhwc_fwd_apply_kernel<2>;
  fk<<<grid, kThreads, 0, s>>>((const bf16_t*)x, (const bf16_t*)res, (bf16_t*)y, (const float*)acc,
                               (const float*)w, (const float*)b, g, (float)eps, relu, (float*)save,
                               (float*)run_mean, (float*)run_var, (float)momentum, (uint8_t*)mbits, rbn);
  DL_HIP_CHECK(hipGetLastError());
}

// acc: fp32 [2C], zeroed by the caller; dres may be 0 (no fused residual);
// relu: 0 none, 1 mask from y, 2 mask recomputed from x (y may be 0).
void bn_nhwc_bwd(uintptr_t dy, uintptr_t y, uintptr_t x, uintptr_t save, uintptr_t w, uintptr_t b, uintptr_t acc,
                 uintptr_t dx,
                 uintptr_t dres, uintptr_t dw, uintptr_t db, int64_t M, int C, int relu, uintptr_t stream) {
  bn_nhwc_bwd_pad(dy, y, x, save, w, b, acc, dx, dres, dw, db, M, C, relu, 1, 1, 0, stream, 0, 0, 0, 0, 0, 0, 0, 0);
}

// dx in the padded layout [N][H+2opad][W+2opad][C] (interior only).
// have_sums: acc already holds sum(g), sum(g*xhat) -- computed by the epilogue
// of the convolution that produced dy (conv_igemm.hip set_conv_bn_reduce,
// ops/conv.py): the reduce pass over dy and x is skipped.
// rbn_x != 0: dres receives the input gradient of the residual branch's
// BatchNorm (ResBnBwd: its input rbn_x, saved mean / invstd, gamma, zeroed
// [2C] backward sums and dgamma / dbeta outputs) instead of g.
void bn_nhwc_bwd_pad(uintptr_t dy, uintptr_t y, uintptr_t x, uintptr_t save, uintptr_t w, uintptr_t b,
                     uintptr_t acc, uintptr_t dx, uintptr_t dres, uintptr_t dw, uintptr_t db, int64_t M, int C,
                     int relu, int H, int W, int opad, uintptr_t stream, int have_sums, uintptr_t mbits,
                     uintptr_t rbn_x, uintptr_t rbn_save, uintptr_t rbn_w, uintptr_t rbn_acc, uintptr_t rbn_dw,
                     uintptr_t rbn_db) {
  if ((relu == 3) != (mbits != 0)) throw std::runtime_error("bn_nhwc_bwd: relu mode 3 reads the forward's mask bits");
  if (relu == 1 && !y) throw std::runtime_error("bn_nhwc_bwd: relu mode 1 reads y");
  if (rbn_x && (have_sums || !dres || !rbn_save || !rbn_w || !rbn_acc || !rbn_dw || !rbn_db))
    throw std::runtime_error("bn_nhwc_bwd: the fused residual BN needs this reduce pass, dres and all its operands");
  const ResBnBwd rb{(const bf16_t*)rbn_x, (const float*)rbn_save, (const float*)rbn_w, (float*)rbn_acc,
                    (float*)rbn_dw, (float*)rbn_db};
  dim3 grid, grid_r;
  BnGeom g = make_geom(M, C, &grid);
  set_out_pad(g, H, W, opad);
  hipStream_t s = as_stream(stream);
  if (!have_sums) {
    const int nt = g_reduce_threads;
    const BnGeom gr = make_geom(M, C, &grid_r, g_reduce_blocks, nt);
    auto rk = nt == 1024 ? bn_nhwc_bwd_reduce_kernel<1024>
              : nt == 512 ? bn_nhwc_bwd_reduce_kernel<512> : bn_nhwc_bwd_reduce_kernel<256>;
    rk<<<grid_r, nt, 0, s>>>((const bf16_t*)dy, (const bf16_t*)y, (const bf16_t*)x, (const float*)save,
                             (const float*)w, (const float*)b, gr, relu, (float*)acc, (const uint8_t*)mbits, rb);
    DL_HIP_CHECK(hipGetLastError());
  }
  auto ak = g_apply_rows == 4 ? bn_nhwc_bwd_apply_kernel<4> : bn_nhwc_bwd_apply_kernel<2>;
  ak<<<grid, kThreads, 0, s>>>((const bf16_t*)dy, (const bf16_t*)y, (const bf16_t*)x, (const float*)save,
                               (const float*)w, (const float*)b, (const float*)acc, g, relu, (bf16_t*)dx,
                               (bf16_t*)dres, (float*)dw, (float*)db, (const uint8_t*)mbits, rb);
  DL_HIP_CHECK(hipGetLastError());
}

void zero_border_nhwc(uintptr_t buf, int N, int H, int W, int C, int pad, uintptr_t stream) {
  if (C % 8 != 0 || pad <= 0) throw std::runtime_error("zero_border_nhwc: C % 8 and pad > 0 required");
  const int64_t total = (int64_t)N * ((int64_t)(H + 2 * pad) * (W + 2 * pad) - (int64_t)H * W) * (C / 8);
  zero_border_kernel<<<stream_grid(total), kThreads, 0, as_stream(stream)>>>((bf16_t*)buf, N, H, W, C, pad);
  DL_HIP_CHECK(hipGetLastError());
}

}  // namespace dl
