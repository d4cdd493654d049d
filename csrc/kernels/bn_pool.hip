// Train-mode BatchNorm + ReLU + 2x2/2 max-pool, forward and backward, on
// NHWC bf16 activations (gfx950).
//
// Reference ops: nn.SpatialBatchNormalization(C, 1e-3) -> nn.ReLU ->
// nn.SpatialMaxPooling(2,2,2,2) (examples/cifar10.lua:109-129; SURVEY §2.8
// K14/K15/K16).  Instead of five separate passes (BN stats, BN apply, ReLU,
// pool, and their backwards) the block is:
//
//   forward : conv epilogue emits per-tile channel sums  (conv_igemm.hip)
//             bn_finalize      -> mean, invstd, scale, shift (+ running stats)
//             bn_relu_pool_fwd -> pooled = maxpool(relu(scale*y + shift))   (1 read of y)
//   backward: bn_relu_pool_bwd_reduce -> per-channel sum(dz), sum(dz*xhat)  (recomputes
//             the pool argmax / ReLU mask from y: nothing is stored in forward)
//             bn_bwd_finalize  -> dgamma, dbeta (into the flat grad), apply coefficients
//             bn_relu_pool_bwd_apply -> dy = a*dz + b*xhat + c           (dense NHWC)
//
// Every thread handles 8 channels (one 16-byte vector) of one pooled pixel.
// All reductions are deterministic (fixed-order partial rows, no atomics).
// The conv bias is not added in the train forward: BatchNorm in train mode is
// invariant to a per-channel shift, so the output and every gradient are
// unchanged and d(bias) is exactly 0; the running mean is updated with
// mean + bias so eval mode (running statistics) is exact.
#include "dl_common.h"
#include "dl_ops.h"
#include "head_wgrad_dev.h"
#include "bn_fin_dev.h"
#include "slab_reduce_dev.h"

namespace dl {

// DL_BN_STAMPS builds only (diagnostics): s_memtime of thread 0 of every block
// of the fused fwd-fin / bwd-apply kernels -> [kernel (0 fwd, 1 bwd)][C/64 - 1][block][4]
__device__ unsigned long long* g_bn_stamps = nullptr;
#ifdef DL_BN_STAMPS
__device__ __forceinline__ unsigned long long bstamp() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
#define BN_STAMP(kind, C, k)                                                                              \
  do {                                                                                                    \
    if (threadIdx.x == 0 && g_bn_stamps && (C) <= 256)                                                   \
      g_bn_stamps[(((size_t)(kind) * 4 + ((C) >> 6) - 1) * 2048 + blockIdx.x) * 4 + (k)] = bstamp();     \
  } while (0)
#else
#define BN_STAMP(kind, C, k) do { } while (0)
#endif
void set_bn_stamps(uintptr_t buf) {
  unsigned long long* p = (unsigned long long*)buf;
  DL_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_bn_stamps), &p, sizeof(p)));
}

// reduction mode (conv_igemm.hip g_red_atomic; set together by set_reduce_atomic):
// R >= 1 = the backward reduce atomically adds its per-block totals into row
// (block & (R-1)) of R zeroed [dgamma (C) ; dbeta (C)] rows (R = 1: straight
// into the BN parameter gradients of the flat buffer), and the apply kernel
// sums the rows and derives its coefficients from them.
__device__ int g_red_atomic_bn = 0;
static int g_host_rows = 0;  // host mirror (BnFin::R of the launchers)
int reduce_rows() { return g_host_rows; }

// Grid cap of the consumer kernels that sum the R accumulated rows in a
// per-block prologue (bn_relu_pool_fwd_fin, bn_relu_pool_bwd_apply_sums):
// every block re-reads C x R x 2 floats, so fewer blocks with several items
// per thread (the next item's loads stay in flight) read fewer row bytes.
static int g_fin_grid = 2048;
void set_bn_fin_grid(int cap) { g_fin_grid = cap < 1 ? 1 : cap; }
static int fin_grid(int64_t total) { return std::min(stream_grid(total), g_fin_grid); }
// register cap of the row-summing BN consumers (bn_relu_pool_fwd_fin /
// bn_relu_pool_bwd_apply_sums): 1 = compiler's choice, 4 = >= 4 waves per SIMD
// (fwd_fin, bwd_apply).  fwd_fin capped: 107 VGPRs, no scratch, 0.3273-0.3285
// vs 0.3293-0.3328 ms/step uncapped.  bwd_apply: with the forward coefficients
// held in registers across the row sums the capped instance spilled 76 B/lane
// (0.3336-0.3351 vs 0.3290-0.3301 ms/step, profiles/r3_bn_minw_ab.txt); with
// them derived into LDS it needs 110-117 VGPRs either way
static int g_bn_minw_fwd = 4, g_bn_minw_bwd = 4;
void set_bn_minw(int fwd, int bwd) {
  if ((fwd != 1 && fwd != 4) || (bwd != 1 && bwd != 4)) throw std::runtime_error("set_bn_minw: 1 or 4");
  g_bn_minw_fwd = fwd;
  g_bn_minw_bwd = bwd;
}

// (unpack8 / pack8 / bn_relu_pool8: bn_fin_dev.h)

// Per-channel column sums of partial rows [T][2][C] (stat 0 at +0, stat 1 at
// +C), one block per channel: every thread issues the loads of 4 rows before
// their first use (the rows were just written by other CUs: each round trip
// is a cross-XCD miss), then a fixed-order wave butterfly and a 4-wave
// combine (one barrier instead of an 8-level LDS tree).  Deterministic.
// Thread 0 returns the totals.
__device__ __forceinline__ void column_sums(const float* __restrict__ partial, int T, int C, int c, float& tot1,
                                            float& tot2) {
  __shared__ float red[2][4];
  float s1 = 0.f, s2 = 0.f;
  int t = threadIdx.x;
  for (; t + 768 < T; t += 1024) {
    float a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a[u] = partial[(int64_t)(t + 256 * u) * 2 * C + c];
      b[u] = partial[(int64_t)(t + 256 * u) * 2 * C + C + c];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) { s1 += a[u]; s2 += b[u]; }
  }
  for (; t < T; t += 256) {
    s1 += partial[(int64_t)t * 2 * C + c];
    s2 += partial[(int64_t)t * 2 * C + C + c];
  }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { red[0][wid] = s1; red[1][wid] = s2; }
  __syncthreads();
  tot1 = red[0][0] + red[0][1] + red[0][2] + red[0][3];
  tot2 = red[1][0] + red[1][1] + red[1][2] + red[1][3];
}

// ---------------------------------------------------------------------------
// finalize (forward): partial rows [T][2][C] (sum, sumsq) -> coefficients
// mode 0 = train (batch statistics, update running stats), 1 = eval
// coef layout [4][C]: mean, invstd, scale, shift
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) bn_finalize_kernel(const float* __restrict__ partial, int T, int C, int64_t M,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta,
                                                          const float* __restrict__ bias, float* __restrict__ rmean,
                                                          float* __restrict__ rvar, float eps, float momentum,
                                                          int mode, float* __restrict__ coef) {
  const int c = blockIdx.x;
  float mean, var;
  if (mode == 0) {
    float t1, t2;
    column_sums(partial, T, C, c, t1, t2);
    mean = t1 / (float)M;
    var = fmaxf(t2 / (float)M - mean * mean, 0.f);
  } else {
    mean = rmean[c] - (bias ? bias[c] : 0.f);  // eval: conv output excludes the bias
    var = rvar[c];
  }
  if (threadIdx.x == 0) {
    const float invstd = rsqrtf(var + eps);
    const float sc = gamma[c] * invstd;
    coef[c] = mean;
    coef[C + c] = invstd;
    coef[2 * C + c] = sc;
    coef[3 * C + c] = beta[c] - mean * sc;
    if (mode == 0 && rmean != nullptr) {
      const float unbiased = M > 1 ? var * (float)M / (float)(M - 1) : var;
      rmean[c] = (1.f - momentum) * rmean[c] + momentum * (mean + (bias ? bias[c] : 0.f));
      rvar[c] = (1.f - momentum) * rvar[c] + momentum * unbiased;
    }
  }
}

// ---------------------------------------------------------------------------
// forward apply: pooled[b][oh][ow][c] = max_{2x2} relu(scale*y + shift)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) bn_relu_pool_fwd_kernel(const bf16_t* __restrict__ y,
                                                               const float* __restrict__ coef,
                                                               bf16_t* __restrict__ out, int B, int H, int W, int C,
                                                               int opad) {
  // out: pooled [B][Ho+2 opad][Wo+2 opad][C], written in the interior (the
  // zero border is the next convolution's spatial padding)
  const int C8 = C >> 3, Ho = H >> 1, Wo = W >> 1;
  const int Hop = Ho + 2 * opad, Wop = Wo + 2 * opad;
  const int64_t total = (int64_t)B * Ho * Wo * C8;
  const float* scale = coef + 2 * C;
  const float* shift = coef + 3 * C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % C8);
    const int64_t pix = i / C8;
    const int ow = (int)(pix % Wo);
    const int64_t t = pix / Wo;
    const int oh = (int)(t % Ho);
    const int64_t b = t / Ho;
    const int c0 = c8 * 8;
    float sc[8], sh[8], mx[8];
    *reinterpret_cast<float4*>(sc) = *reinterpret_cast<const float4*>(scale + c0);
    *reinterpret_cast<float4*>(sc + 4) = *reinterpret_cast<const float4*>(scale + c0 + 4);
    *reinterpret_cast<float4*>(sh) = *reinterpret_cast<const float4*>(shift + c0);
    *reinterpret_cast<float4*>(sh + 4) = *reinterpret_cast<const float4*>(shift + c0 + 4);
    const bf16_t* base = y + (((b * H + 2 * oh) * W) + 2 * ow) * (int64_t)C + c0;
    const uint4 v0 = *reinterpret_cast<const uint4*>(base);
    const uint4 v1 = *reinterpret_cast<const uint4*>(base + C);
    const uint4 v2 = *reinterpret_cast<const uint4*>(base + (int64_t)W * C);
    const uint4 v3 = *reinterpret_cast<const uint4*>(base + (int64_t)W * C + C);
    float f[8];
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
    *reinterpret_cast<uint4*>(out + ((b * Hop + oh + opad) * Wop + ow + opad) * (int64_t)C + c0) = pack8(mx);
  }
}

// Same, with the BN coefficients derived from the atomically accumulated
// statistics (bn_fin_dev.h); block 0 publishes coef + running statistics.
template <int MINW = 1>  // (see bn_relu_pool_bwd_apply_kernel: uncapped 160 VGPRs = 3 blocks per CU)
__global__ void __launch_bounds__(256, MINW) bn_relu_pool_fwd_fin_kernel(const bf16_t* __restrict__ y, const BnFin fin,
                                                                   bf16_t* __restrict__ out, int B, int H, int W, int C,
                                                                   int opad) {
  __shared__ __attribute__((aligned(16))) float ssc[kFinMaxC], ssh[kFinMaxC];  // (bn_relu_pool8: 16-byte reads)
  const int C8 = C >> 3, Ho = H >> 1, Wo = W >> 1;
  const int Hop = Ho + 2 * opad, Wop = Wo + 2 * opad;
  const int64_t total = (int64_t)B * Ho * Wo * C8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  auto item_base = [&](int64_t i, int& c0, int64_t& pix) {
    const int c8 = (int)(i % C8);
    pix = i / C8;
    c0 = c8 * 8;
    const int ow = (int)(pix % Wo);
    const int64_t t = pix / Wo;
    const int oh = (int)(t % Ho);
    const int64_t b = t / Ho;
    return y + (((b * H + 2 * oh) * W) + 2 * ow) * (int64_t)C + c0;
  };
  auto load4 = [&](const bf16_t* base, uint4 (&v)[4]) {
    v[0] = *reinterpret_cast<const uint4*>(base);
    v[1] = *reinterpret_cast<const uint4*>(base + C);
    v[2] = *reinterpret_cast<const uint4*>(base + (int64_t)W * C);
    v[3] = *reinterpret_cast<const uint4*>(base + (int64_t)W * C + C);
  };
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint4 v[4];
  int c0 = 0;
  int64_t pix = 0;
  BN_STAMP(0, C, 0);
  if (i < total) load4(item_base(i, c0, pix), v);  // in flight across the coefficient prologue
  bn_fin_block(fin, C, ssc, ssh);
  BN_STAMP(0, C, 1);
  for (; i < total;) {
    const uint4 pooled = bn_relu_pool8(v[0], v[1], v[2], v[3], ssc + c0, ssh + c0);
    const int ow = (int)(pix % Wo);
    const int64_t t = pix / Wo;
    const int oh = (int)(t % Ho);
    const int64_t b = t / Ho;
    bf16_t* o = out + ((b * Hop + oh + opad) * Wop + ow + opad) * (int64_t)C + c0;
    i += stride;
    if (i < total) load4(item_base(i, c0, pix), v);
    *reinterpret_cast<uint4*>(o) = pooled;
  }
  BN_STAMP(0, C, 2);
}

// Backward signal of one pooled pixel x 8 channels: dz[w][k] = dP[k] at the
// first (row-major) window position holding the max of relu(z) if that z > 0,
// else 0; xh[w][k] = (y - mean) * invstd.
struct BwdCtx {
  float sc[8], sh[8], mu[8], is[8];
};

__device__ __forceinline__ void load8(float* d, const float* s) {
  *reinterpret_cast<float4*>(d) = *reinterpret_cast<const float4*>(s);
  *reinterpret_cast<float4*>(d + 4) = *reinterpret_cast<const float4*>(s + 4);
}

// ---------------------------------------------------------------------------
// backward reduce: partial[blk][0][c] = sum dz, partial[blk][1][c] = sum dz*xhat
// ---------------------------------------------------------------------------
// Body of the reduce for block `bid` of `nblk` (the reduce part of the grid).
__device__ __forceinline__ void bwd_reduce_body(const bf16_t* __restrict__ y, const bf16_t* __restrict__ dP,
                                                const float* __restrict__ coef, float* __restrict__ partial, int B,
                                                int H, int W, int C, int bid, int nblk) {
  const int C8 = C >> 3, Ho = H >> 1, Wo = W >> 1;
  const int64_t total = (int64_t)B * Ho * Wo * C8;
  // grid-stride keeps the channel chunk fixed per thread (stride % C8 == 0)
  const int64_t stride = (int64_t)nblk * blockDim.x;
  const int64_t i0 = (int64_t)bid * blockDim.x + threadIdx.x;
  const int c8 = (int)(i0 % C8), c0 = c8 * 8;
  BwdCtx cx;
  load8(cx.mu, coef + c0);
  load8(cx.is, coef + C + c0);
  load8(cx.sc, coef + 2 * C + c0);
  load8(cx.sh, coef + 3 * C + c0);
  float s1[8], s2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { s1[k] = 0.f; s2[k] = 0.f; }
  // items in batches of U: every load of the batch is issued before the
  // first use (the per-item load->use chain was latency-bound); the
  // accumulation order is the same item order as a plain loop
  constexpr int U = 4;
  auto item_loads = [&](int64_t i, uint4 (&yw)[4], uint4& gv) {
    const int64_t pix = i / C8;
    const int ow = (int)(pix % Wo);
    const int64_t t = pix / Wo;
    const int oh = (int)(t % Ho);
    const int64_t b = t / Ho;
    const bf16_t* base = y + (((b * H + 2 * oh) * W) + 2 * ow) * (int64_t)C + c0;
    yw[0] = *reinterpret_cast<const uint4*>(base);
    yw[1] = *reinterpret_cast<const uint4*>(base + C);
    yw[2] = *reinterpret_cast<const uint4*>(base + (int64_t)W * C);
    yw[3] = *reinterpret_cast<const uint4*>(base + (int64_t)W * C + C);
    gv = *reinterpret_cast<const uint4*>(dP + (((b * Ho + oh) * Wo) + ow) * (int64_t)C + c0);
  };
  auto item_acc = [&](const uint4 (&yw)[4], const uint4& gv) {
    float yv[4][8], g[8];
#pragma unroll
    for (int w = 0; w < 4; ++w) unpack8(yw[w], yv[w]);
    unpack8(gv, g);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float best = -INFINITY;
      int arg = 0;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const float r = fmaxf(fmaf(cx.sc[k], yv[w][k], cx.sh[k]), 0.f);
        if (r > best) { best = r; arg = w; }
      }
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const float dz = (w == arg && best > 0.f) ? g[k] : 0.f;
        s1[k] += dz;
        s2[k] += dz * (yv[w][k] - cx.mu[k]) * cx.is[k];
      }
    }
  };
  int64_t i = i0;
  for (; i + (U - 1) * stride < total; i += U * stride) {
    uint4 yw[U][4], gv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) item_loads(i + u * stride, yw[u], gv[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) item_acc(yw[u], gv[u]);
  }
  for (; i < total; i += stride) {
    uint4 yw[4], gv;
    item_loads(i, yw, gv);
    item_acc(yw, gv);
  }
  // block reduction over threads that own the same channel chunk
  __shared__ float red[256][17];
#pragma unroll
  for (int k = 0; k < 8; ++k) { red[threadIdx.x][k] = s1[k]; red[threadIdx.x][8 + k] = s2[k]; }
  __syncthreads();
  // thread t < C: channel t (chunk t/8, lane k = t%8)
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const int ch = c >> 3, k = c & 7;
    // threads with (blockIdx.x*256 + tid) % C8 == ch
    const int first = (int)(((int64_t)ch - ((int64_t)bid * blockDim.x) % C8 + C8) % C8);
    float a = 0.f, bsum = 0.f;
    for (int t = first; t < (int)blockDim.x; t += C8) { a += red[t][k]; bsum += red[t][8 + k]; }
    if (const int R = g_red_atomic_bn) {  // rows of [dgamma ; dbeta] = [sum dz*xhat ; sum dz]
      float* p = partial + (int64_t)(bid & (R - 1)) * 2 * C;
      unsafeAtomicAdd(p + c, bsum);
      unsafeAtomicAdd(p + C + c, a);
    } else {
      partial[(int64_t)bid * 2 * C + c] = a;
      partial[(int64_t)bid * 2 * C + C + c] = bsum;
    }
  }
}

// Split-K combine of a dgrad (SPL fp32 slabs [SPL][M][C], M = B*Ho*Wo pooled
// pixels) fused with the BN backward reduce of the block below, in the
// combine's row-blocked layout (the fast one for the slab reads: each block
// owns rows [r0, r1), each thread one 8-channel chunk, splits summed in
// order in batches of 4 with all loads of a batch in flight): dP = bf16(sum),
// stored once, and the reduce's window loads of y issued beside the first
// batch.  One partial row per block (mode 0, `partial` needs gridDim.x rows)
// or striped atomics (mode 2).
template <int SPL>
__global__ void __launch_bounds__(256) combine_bwd_reduce_kernel(const float* __restrict__ slab,
                                                                 bf16_t* __restrict__ dP, const bf16_t* __restrict__ y,
                                                                 const float* __restrict__ coef,
                                                                 float* __restrict__ partial, int B, int H, int W,
                                                                 int C, int rows_per_block) {
  const int C8 = C >> 3, Ho = H >> 1, Wo = W >> 1;
  const int M = B * Ho * Wo;
  const int tpr = C8, rpi = 256 / tpr;
  const int c8 = threadIdx.x % tpr, rsub = threadIdx.x / tpr, c0 = c8 * 8;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  const int64_t MN = (int64_t)M * C;
  BwdCtx cx;
  load8(cx.mu, coef + c0);
  load8(cx.is, coef + C + c0);
  load8(cx.sc, coef + 2 * C + c0);
  load8(cx.sh, coef + 3 * C + c0);
  float s1[8], s2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { s1[k] = 0.f; s2[k] = 0.f; }
  if (rsub < rpi) {
    for (int m = r0 + rsub; m < r1; m += rpi) {
      const int ow = m % Wo, t = m / Wo, oh = t % Ho, b = t / Ho;
      const bf16_t* base = y + (((int64_t)(b * H + 2 * oh) * W) + 2 * ow) * C + c0;
      uint4 yw[4];
      yw[0] = *reinterpret_cast<const uint4*>(base);
      yw[1] = *reinterpret_cast<const uint4*>(base + C);
      yw[2] = *reinterpret_cast<const uint4*>(base + (int64_t)W * C);
      yw[3] = *reinterpret_cast<const uint4*>(base + (int64_t)W * C + C);
      const float* q = slab + (int64_t)m * C + c0;
      constexpr int BT = SPL < 4 ? SPL : 4;
      float v[8];
      {
        float4 a[BT], bb[BT];
#pragma unroll
        for (int u = 0; u < BT; ++u) {
          a[u] = *reinterpret_cast<const float4*>(q + u * MN);
          bb[u] = *reinterpret_cast<const float4*>(q + u * MN + 4);
        }
        v[0] = a[0].x; v[1] = a[0].y; v[2] = a[0].z; v[3] = a[0].w;
        v[4] = bb[0].x; v[5] = bb[0].y; v[6] = bb[0].z; v[7] = bb[0].w;
#pragma unroll
        for (int u = 1; u < BT; ++u) {
          v[0] += a[u].x; v[1] += a[u].y; v[2] += a[u].z; v[3] += a[u].w;
          v[4] += bb[u].x; v[5] += bb[u].y; v[6] += bb[u].z; v[7] += bb[u].w;
        }
      }
#pragma unroll
      for (int s0 = BT; s0 < SPL; s0 += 4) {
        float4 a[4], bb[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          a[u] = *reinterpret_cast<const float4*>(q + (s0 + u) * MN);
          bb[u] = *reinterpret_cast<const float4*>(q + (s0 + u) * MN + 4);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          v[0] += a[u].x; v[1] += a[u].y; v[2] += a[u].z; v[3] += a[u].w;
          v[4] += bb[u].x; v[5] += bb[u].y; v[6] += bb[u].z; v[7] += bb[u].w;
        }
      }
      uint4 gv;
      gv.x = pack_bf16x2(v[0], v[1]); gv.y = pack_bf16x2(v[2], v[3]);
      gv.z = pack_bf16x2(v[4], v[5]); gv.w = pack_bf16x2(v[6], v[7]);
      *reinterpret_cast<uint4*>(dP + (int64_t)m * C + c0) = gv;
      float yv[4][8], g[8];
#pragma unroll
      for (int w = 0; w < 4; ++w) unpack8(yw[w], yv[w]);
      unpack8(gv, g);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float best = -INFINITY;
        int arg = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const float r = fmaxf(fmaf(cx.sc[k], yv[w][k], cx.sh[k]), 0.f);
          if (r > best) { best = r; arg = w; }
        }
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const float dz = (w == arg && best > 0.f) ? g[k] : 0.f;
          s1[k] += dz;
          s2[k] += dz * (yv[w][k] - cx.mu[k]) * cx.is[k];
        }
      }
    }
  }
  __shared__ float red[256][17];
#pragma unroll
  for (int k = 0; k < 8; ++k) { red[threadIdx.x][k] = s1[k]; red[threadIdx.x][8 + k] = s2[k]; }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const int ch = c >> 3, k = c & 7;
    float a = 0.f, bsum = 0.f;
    for (int t = ch; t < rpi * tpr; t += tpr) { a += red[t][k]; bsum += red[t][8 + k]; }
    if (const int R = g_red_atomic_bn) {  // rows of [dgamma ; dbeta] = [sum dz*xhat ; sum dz]
      float* p = partial + (int64_t)(blockIdx.x & (R - 1)) * 2 * C;
      unsafeAtomicAdd(p + c, bsum);
      unsafeAtomicAdd(p + C + c, a);
    } else {
      partial[(int64_t)blockIdx.x * 2 * C + c] = a;
      partial[(int64_t)blockIdx.x * 2 * C + C + c] = bsum;
    }
  }
}

__global__ void __launch_bounds__(256) bn_relu_pool_bwd_reduce_kernel(const bf16_t* __restrict__ y,
                                                                      const bf16_t* __restrict__ dP,
                                                                      const float* __restrict__ coef,
                                                                      float* __restrict__ partial, int B, int H,
                                                                      int W, int C) {
  bwd_reduce_body(y, dP, coef, partial, B, H, W, C, (int)blockIdx.x, (int)gridDim.x);
}

// One launch for two independent jobs that both wait only for the head:
// blocks [0, G) = the last conv block's BN backward reduce, blocks [G, ...) =
// the classifier weight gradient (head_wgrad_body).  Saves a kernel boundary
// and runs the small head job beside the reduce instead of after it.
struct HeadWgradArgs {
  const bf16_t* h;
  const float* dlogits;
  const float* loss_b;
  int F, B;
  float *dw, *db, *loss, *slot;
  unsigned long long* step_ctr;
};

__global__ void __launch_bounds__(256) bwd_reduce_head_kernel(const bf16_t* __restrict__ y,
                                                              const bf16_t* __restrict__ dP,
                                                              const float* __restrict__ coef,
                                                              float* __restrict__ partial, int B, int H, int W, int C,
                                                              int G, const HeadWgradArgs ha) {
  if ((int)blockIdx.x < G)
    bwd_reduce_body(y, dP, coef, partial, B, H, W, C, (int)blockIdx.x, G);
  else
    head_wgrad_body<10>(ha.h, ha.dlogits, ha.loss_b, ha.F, ha.B, ha.dw, ha.db, ha.loss, ha.slot, ha.step_ctr,
                        (int)blockIdx.x - G);
}

// One launch for two independent jobs: blocks [0, G) = this block's BN
// backward reduce (waits for the dgrad that produced dP), blocks [G, ...) =
// the split-K slab reduction of the NEXT conv block's weight gradient (its
// wgrad finished two launches earlier).  Saves the stand-alone slab_reduce
// launch and its kernel boundary.
struct SlabArgs {
  const float* slabs;
  float* dst;
  int splits, Cout, taps, Cp, C;
};

template <int TPO>
__global__ void __launch_bounds__(256) bwd_reduce_slab_kernel(const bf16_t* __restrict__ y,
                                                              const bf16_t* __restrict__ dP,
                                                              const float* __restrict__ coef,
                                                              float* __restrict__ partial, int B, int H, int W, int C,
                                                              int G, const SlabArgs sa) {
  if ((int)blockIdx.x < G)
    bwd_reduce_body(y, dP, coef, partial, B, H, W, C, (int)blockIdx.x, G);
  else
    slab_reduce_body<TPO>(sa.slabs, sa.dst, sa.splits, sa.Cout, sa.taps, sa.Cp, sa.C, (int)blockIdx.x - G,
                          (int)gridDim.x - G);
}

// backward finalize: dgamma = sum(dz*xhat), dbeta = sum(dz);
// apply coefficients [3][C]: dy = a*dz + b*xhat + c
__global__ void __launch_bounds__(256) bn_bwd_finalize_kernel(const float* __restrict__ partial, int T, int C,
                                                              int64_t M, const float* __restrict__ gamma,
                                                              const float* __restrict__ coef,
                                                              float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                              float* __restrict__ acoef) {
  const int c = blockIdx.x;
  float sdz, sdzx;
  column_sums(partial, T, C, c, sdz, sdzx);
  if (threadIdx.x == 0) {
    if (dgamma) dgamma[c] = sdzx;
    if (dbeta) dbeta[c] = sdz;
    const float a = gamma[c] * coef[C + c];  // gamma * invstd
    acoef[c] = a;
    acoef[C + c] = -a * sdzx / (float)M;
    acoef[2 * C + c] = -a * sdz / (float)M;
  }
}

// SUMS: acoef holds R accumulated rows of [dgamma ; dbeta] (reduction mode
// R >= 1); every block sums them in a fixed order and derives the apply
// coefficients a = gamma*invstd, b = -a*dgamma/M, c = -a*dbeta/M in LDS
// (the first item's loads are already in flight); block 0 also writes the
// totals to dgamma_out / dbeta_out (R > 1: the flat gradient; R = 1
// accumulated there directly and passes null).
template <bool SUMS, bool TWO_CH = false>
__device__ __forceinline__ void bwd_apply_body(const bf16_t* __restrict__ y, const bf16_t* __restrict__ dP,
                                               const float* __restrict__ coef, const float* __restrict__ acoef,
                                               bf16_t* __restrict__ dy, int B, int H, int W, int C, int opad,
                                               const float* __restrict__ gamma, float inv_m, int R,
                                               float* __restrict__ dgamma_out, float* __restrict__ dbeta_out, int bid,
                                               int nblk) {
  // dy: [B][H+2 opad][W+2 opad][C], written in the interior (zero border =
  // the dgrad convolution's spatial padding)
  // SUMS: per-channel loop coefficients derived in the prologue into LDS:
  // ka, kbi, kc (below) and the forward mu, sc, sh -- nothing but the item's
  // loads is live in registers across the row sums (with the forward
  // coefficients held in 32 registers there the kernel needed 146 VGPRs, 3
  // blocks per CU)
  __shared__ float sk[SUMS ? 6 : 1][SUMS ? kFinMaxC : 1];
  const int C8 = C >> 3, Ho = H >> 1, Wo = W >> 1;
  const int Hp = H + 2 * opad, Wp = W + 2 * opad;
  const int64_t total = (int64_t)B * Ho * Wo * C8;
  const int64_t stride = (int64_t)nblk * blockDim.x;
  int c0 = 0, oh = 0, ow = 0;
  int64_t b = 0;
  uint4 yw[4], gv;
  auto item_loads = [&](int64_t i) {
    c0 = (int)(i % C8) * 8;
    const int64_t pix = i / C8;
    ow = (int)(pix % Wo);
    const int64_t t = pix / Wo;
    oh = (int)(t % Ho);
    b = t / Ho;
    const bf16_t* base = y + (((b * H + 2 * oh) * W) + 2 * ow) * (int64_t)C + c0;
    yw[0] = *reinterpret_cast<const uint4*>(base);
    yw[1] = *reinterpret_cast<const uint4*>(base + C);
    yw[2] = *reinterpret_cast<const uint4*>(base + (int64_t)W * C);
    yw[3] = *reinterpret_cast<const uint4*>(base + (int64_t)W * C + C);
    gv = *reinterpret_cast<const uint4*>(dP + (((b * Ho + oh) * Wo) + ow) * (int64_t)C + c0);
  };
  BN_STAMP(1, C, 0);
  int64_t i = (int64_t)bid * blockDim.x + threadIdx.x;
  if (i < total) item_loads(i);
  // stride % C8 == 0 (C8 | 256): a thread's channel chunk c0 is the same for
  // every item
  c0 = (int)(i % C8) * 8;
  // ka * dz + kb * xhat + kc with xhat = (y - mu) * is, as ka * dz + kbi * (y - mu) + kc
  // (kbi = kb * is): the loop keeps no per-window float copies of y and no is[]
  float ka[8], kbi[8], kc[8], mu[8], sc[8], sh[8];
  if constexpr (SUMS) {
    auto put = [&](int c, float gam, float istd, float m, float s, float h, float dg, float db) {
      const float a = gam * istd;
      sk[0][c] = a;
      sk[1][c] = -a * dg * inv_m * istd;
      sk[2][c] = -a * db * inv_m;
      sk[3][c] = m;
      sk[4][c] = s;
      sk[5][c] = h;
      if (bid == 0 && dgamma_out != nullptr) { dgamma_out[c] = dg; dbeta_out[c] = db; }
    };
    if (TWO_CH && C == 2 * (int)blockDim.x) {  // both channels' rows in one memory round trip (the last block, C = 512)
      const int c0 = threadIdx.x, c1 = c0 + blockDim.x;
      const float g0 = gamma[c0], i0 = coef[C + c0], g1 = gamma[c1], i1 = coef[C + c1];
      const float m0 = coef[c0], s0 = coef[2 * C + c0], h0 = coef[3 * C + c0];
      const float m1 = coef[c1], s1 = coef[2 * C + c1], h1 = coef[3 * C + c1];
      float t[4];
      sum_rows2x2(acoef + c0, blockDim.x, 2 * C, C, R, t);
      put(c0, g0, i0, m0, s0, h0, t[0], t[1]);
      put(c1, g1, i1, m1, s1, h1, t[2], t[3]);
    } else {
#pragma unroll 1
      for (int c = threadIdx.x; c < C; c += blockDim.x) {
        // issued with (not after) the row loads
        const float gam = gamma[c], istd = coef[C + c], m = coef[c], sv = coef[2 * C + c], hv = coef[3 * C + c];
        float dg, db;
        sum_rows2(acoef + c, 2 * C, C, R, dg, db);
        put(c, gam, istd, m, sv, hv, dg, db);
      }
    }
    fin_block_sync();
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      ka[k] = sk[0][c0 + k]; kbi[k] = sk[1][c0 + k]; kc[k] = sk[2][c0 + k];
      mu[k] = sk[3][c0 + k]; sc[k] = sk[4][c0 + k]; sh[k] = sk[5][c0 + k];
    }
  } else {
    float is[8];
    load8(mu, coef + c0);
    load8(is, coef + C + c0);
    load8(sc, coef + 2 * C + c0);
    load8(sh, coef + 3 * C + c0);
    load8(ka, acoef + c0);
    load8(kbi, acoef + C + c0);
    load8(kc, acoef + 2 * C + c0);
#pragma unroll
    for (int k = 0; k < 8; ++k) kbi[k] *= is[k];
  }
  BN_STAMP(1, C, 1);
  auto yk = [&](int w, int k) {  // element k of window position w
    const uint32_t u = k < 2 ? yw[w].x : k < 4 ? yw[w].y : k < 6 ? yw[w].z : yw[w].w;
    return (k & 1) ? hi_bf16(u) : lo_bf16(u);
  };
  for (; i < total;) {
    float g[8];
    unpack8(gv, g);
    int sel[8];  // window position of the pooled max (-1: the max is not > 0, no gradient)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float best = -INFINITY;
      int arg = 0;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const float r = fmaxf(fmaf(sc[k], yk(w, k), sh[k]), 0.f);
        if (r > best) { best = r; arg = w; }
      }
      sel[k] = best > 0.f ? arg : -1;
    }
    uint4 o4[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = ka[k] * (sel[k] == w ? g[k] : 0.f) + kbi[k] * (yk(w, k) - mu[k]) + kc[k];
      o4[w] = pack8(o);
    }
    bf16_t* base = dy + (((b * Hp + 2 * oh + opad) * Wp) + 2 * ow + opad) * (int64_t)C + c0;
    const int64_t offs[4] = {0, C, (int64_t)Wp * C, (int64_t)Wp * C + C};
#pragma unroll
    for (int w = 0; w < 4; ++w) *reinterpret_cast<uint4*>(base + offs[w]) = o4[w];
    // next item's loads after this item's stores (the stores' 16 registers are
    // free again; at the CIFAR shapes every thread has one item anyway)
    i += stride;
    if (i < total) item_loads(i);
  }
  BN_STAMP(1, C, 2);
}

// MINW: minimum waves per SIMD the compiler must allow (register cap: 4 ->
// <= 128 VGPRs, 4 blocks per CU, so CIFAR layer 1's 1024 blocks fit one round;
// uncapped the <true> instance took 206 VGPRs = 2 blocks per CU, two rounds)
template <bool SUMS, int MINW = 1>
__global__ void __launch_bounds__(256, MINW) bn_relu_pool_bwd_apply_kernel(const bf16_t* __restrict__ y,
                                                                     const bf16_t* __restrict__ dP,
                                                                     const float* __restrict__ coef,
                                                                     const float* __restrict__ acoef,
                                                                     bf16_t* __restrict__ dy, int B, int H, int W,
                                                                     int C, int opad, const float* __restrict__ gamma,
                                                                     float inv_m, int R, float* __restrict__ dgamma_out,
                                                                     float* __restrict__ dbeta_out) {
  bwd_apply_body<SUMS>(y, dP, coef, acoef, dy, B, H, W, C, opad, gamma, inv_m, R, dgamma_out, dbeta_out,
                       (int)blockIdx.x, (int)gridDim.x);
}

// One launch for two jobs that both wait only for the head kernel (which also
// did the last block's BN backward reduce, head.hip RED): blocks [0, Ga) =
// this block's BN backward apply (atomic-rows mode), blocks [Ga, ...) = the
// classifier weight gradient (head_wgrad_body).
struct HeadWgradArgs2 {
  const bf16_t* h;
  const float* dlogits;
  const float* loss_b;
  int F, B;
  float *dw, *db, *loss, *slot;
  unsigned long long* step_ctr;
};

__global__ void __launch_bounds__(256) bwd_apply_head_kernel(const bf16_t* __restrict__ y,
                                                             const bf16_t* __restrict__ dP,
                                                             const float* __restrict__ coef,
                                                             const float* __restrict__ acoef,
                                                             bf16_t* __restrict__ dy, int B, int H, int W, int C,
                                                             int opad, const float* __restrict__ gamma, float inv_m,
                                                             int R, float* __restrict__ dgamma_out,
                                                             float* __restrict__ dbeta_out, int Ga,
                                                             const HeadWgradArgs2 ha) {
  if ((int)blockIdx.x < Ga)
    bwd_apply_body<true, true>(y, dP, coef, acoef, dy, B, H, W, C, opad, gamma, inv_m, R, dgamma_out, dbeta_out,
                         (int)blockIdx.x, Ga);
  else
    head_wgrad_body<10>(ha.h, ha.dlogits, ha.loss_b, ha.F, ha.B, ha.dw, ha.db, ha.loss, ha.slot, ha.step_ctr,
                        (int)blockIdx.x - Ga);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static void check_c(int C) {
  if (C % 8 != 0) throw std::runtime_error("bn/pool: C must be a multiple of 8");
}
// the backward apply keeps a thread's channel chunk for all its items (grid stride % C/8 == 0)
static void check_c_apply(int C) {
  check_c(C);
  if (256 % (C / 8) != 0) throw std::runtime_error("bn backward apply: C/8 must divide 256");
}

void bn_finalize(uintptr_t partial, int T, int C, int64_t M, uintptr_t gamma, uintptr_t beta, uintptr_t bias,
                 uintptr_t rmean, uintptr_t rvar, float eps, float momentum, int mode, uintptr_t coef,
                 uintptr_t stream) {
  bn_finalize_kernel<<<C, 256, 0, as_stream(stream)>>>((const float*)partial, T, C, M, (const float*)gamma,
                                                       (const float*)beta, (const float*)bias, (float*)rmean,
                                                       (float*)rvar, eps, momentum, mode, (float*)coef);
  DL_HIP_CHECK(hipGetLastError());
}

void bn_relu_pool_fwd(uintptr_t y, uintptr_t coef, uintptr_t out, int B, int H, int W, int C, int opad,
                      uintptr_t stream) {
  check_c(C);
  const int64_t total = (int64_t)B * (H / 2) * (W / 2) * (C / 8);
  bn_relu_pool_fwd_kernel<<<stream_grid(total), 256, 0, as_stream(stream)>>>(
      (const bf16_t*)y, (const float*)coef, (bf16_t*)out, B, H, W, C, opad);
  DL_HIP_CHECK(hipGetLastError());
}

// Grid of the backward reduce: one partial row per block, so more blocks
// cost the finalize more rows.  n > 0: n pooled pixels per thread (default
// 2; measured per step: 4 -> 0.376 ms, 2 -> 0.365, 1 -> 0.368); 0: at least
// one block per CU (256) and at most 4 pixels per thread (0.367).
static int g_bwd_items = 2;
void set_bn_bwd_items(int n) { g_bwd_items = n < 0 ? 0 : n; }

int bn_bwd_blocks(int B, int H, int W, int C) {
  const int64_t total = (int64_t)B * (H / 2) * (W / 2) * (C / 8);
  int64_t g;
  if (g_bwd_items > 0) {
    const int64_t per = 256 * (int64_t)g_bwd_items;
    g = (total + per - 1) / per;
  } else {
    g = std::max<int64_t>(std::min<int64_t>(256, (total + 255) / 256), (total + 1023) / 1024);
  }
  if (g > 1024) g = 1024;
  if (g < 1) g = 1;
  return (int)g;
}

void bn_relu_pool_bwd_reduce(uintptr_t y, uintptr_t dP, uintptr_t coef, uintptr_t partial, int B, int H, int W, int C,
                             int blocks, uintptr_t stream) {
  check_c(C);
  if ((256 % (C / 8)) != 0) throw std::runtime_error("bn_relu_pool_bwd_reduce: C/8 must divide 256");
  bn_relu_pool_bwd_reduce_kernel<<<blocks, 256, 0, as_stream(stream)>>>(
      (const bf16_t*)y, (const bf16_t*)dP, (const float*)coef, (float*)partial, B, H, W, C);
  DL_HIP_CHECK(hipGetLastError());
}

// dP = bf16(sum of the `splits` fp32 slabs of its split-K dgrad) fused with
// the BN backward reduce over (y, dP) (conv_fwd was called with the
// keep-slabs bit, so it launched no combine of its own).
// rows per block / blocks of combine_bwd_reduce (~384 blocks of whole row iterations)
static int cbr_rows_per_block(int M, int C) {
  const int rpi = 256 / (C / 8);
  int rpb = (M + 383) / 384;
  rpb = ((rpb + rpi - 1) / rpi) * rpi;
  return rpb < rpi ? rpi : rpb;
}

int combine_bwd_reduce_blocks(int B, int H, int W, int C) {
  const int M = B * (H / 2) * (W / 2), rpb = cbr_rows_per_block(M, C);
  return (M + rpb - 1) / rpb;
}

// dP = bf16(sum of the `splits` fp32 slabs of its split-K dgrad) fused with
// the BN backward reduce over (y, dP) (conv_fwd was called with the
// keep-slabs bit, so it launched no combine of its own).  Returns the number
// of partial rows written (mode 0: `partial` must hold that many).
int combine_bwd_reduce(uintptr_t slab, int splits, uintptr_t dP, uintptr_t y, uintptr_t coef, uintptr_t partial, int B,
                       int H, int W, int C, uintptr_t stream) {
  check_c(C);
  if ((256 % (C / 8)) != 0) throw std::runtime_error("combine_bwd_reduce: C/8 must divide 256");
  const int M = B * (H / 2) * (W / 2), rpb = cbr_rows_per_block(M, C), nb = (M + rpb - 1) / rpb;
  auto s = as_stream(stream);
  const float* S = (const float*)slab;
  bf16_t* D = (bf16_t*)dP;
  const bf16_t* Y = (const bf16_t*)y;
  const float* K = (const float*)coef;
  float* P = (float*)partial;
  switch (splits) {
    case 2: combine_bwd_reduce_kernel<2><<<nb, 256, 0, s>>>(S, D, Y, K, P, B, H, W, C, rpb); break;
    case 4: combine_bwd_reduce_kernel<4><<<nb, 256, 0, s>>>(S, D, Y, K, P, B, H, W, C, rpb); break;
    case 8: combine_bwd_reduce_kernel<8><<<nb, 256, 0, s>>>(S, D, Y, K, P, B, H, W, C, rpb); break;
    case 16: combine_bwd_reduce_kernel<16><<<nb, 256, 0, s>>>(S, D, Y, K, P, B, H, W, C, rpb); break;
    default: throw std::runtime_error("combine_bwd_reduce: splits must be 2, 4, 8 or 16");
  }
  DL_HIP_CHECK(hipGetLastError());
  return nb;
}

void bn_bwd_reduce_head(uintptr_t y, uintptr_t dP, uintptr_t coef, uintptr_t partial, int B, int H, int W, int C,
                        int blocks, uintptr_t h, uintptr_t dlogits, uintptr_t loss_b, int F, int NC, uintptr_t dw,
                        uintptr_t db, uintptr_t loss, uintptr_t slot, uintptr_t step_ctr, uintptr_t stream) {
  check_c(C);
  if ((256 % (C / 8)) != 0) throw std::runtime_error("bn_bwd_reduce_head: C/8 must divide 256");
  if (NC != 10) throw std::runtime_error("bn_bwd_reduce_head: built for 10 classes");
  const HeadWgradArgs ha{(const bf16_t*)h, (const float*)dlogits, (const float*)loss_b, F, B, (float*)dw,
                         (float*)db, (float*)loss, (float*)slot, (unsigned long long*)step_ctr};
  const int head_blocks = (F + 31) / 32 + 1;
  bwd_reduce_head_kernel<<<blocks + head_blocks, 256, 0, as_stream(stream)>>>(
      (const bf16_t*)y, (const bf16_t*)dP, (const float*)coef, (float*)partial, B, H, W, C, blocks, ha);
  DL_HIP_CHECK(hipGetLastError());
}

void bn_bwd_reduce_slab(uintptr_t y, uintptr_t dP, uintptr_t coef, uintptr_t partial, int B, int H, int W, int C,
                        int blocks, uintptr_t slabs, uintptr_t dst, int splits, int Cout, int taps, int Cp, int Creal,
                        uintptr_t stream) {
  check_c(C);
  if ((256 % (C / 8)) != 0) throw std::runtime_error("bn_bwd_reduce_slab: C/8 must divide 256");
  if (!slabs || !dst || splits < 1 || Creal > Cp) throw std::runtime_error("bn_bwd_reduce_slab: bad slab arguments");
  const SlabArgs sa{(const float*)slabs, (float*)dst, splits, Cout, taps, Cp, Creal};
  const int g = blocks + slab_reduce_grid(splits, Cout, taps, Creal);
  const int tpo = slab_reduce_tpo(splits);
  auto s = as_stream(stream);
  if (tpo == 32)
    bwd_reduce_slab_kernel<32><<<g, 256, 0, s>>>((const bf16_t*)y, (const bf16_t*)dP, (const float*)coef,
                                                 (float*)partial, B, H, W, C, blocks, sa);
  else if (tpo == 8)
    bwd_reduce_slab_kernel<8><<<g, 256, 0, s>>>((const bf16_t*)y, (const bf16_t*)dP, (const float*)coef,
                                                (float*)partial, B, H, W, C, blocks, sa);
  else
    bwd_reduce_slab_kernel<1><<<g, 256, 0, s>>>((const bf16_t*)y, (const bf16_t*)dP, (const float*)coef,
                                                (float*)partial, B, H, W, C, blocks, sa);
  DL_HIP_CHECK(hipGetLastError());
}

void bn_bwd_finalize(uintptr_t partial, int T, int C, int64_t M, uintptr_t gamma, uintptr_t coef, uintptr_t dgamma,
                     uintptr_t dbeta, uintptr_t acoef, uintptr_t stream) {
  bn_bwd_finalize_kernel<<<C, 256, 0, as_stream(stream)>>>((const float*)partial, T, C, M, (const float*)gamma,
                                                           (const float*)coef, (float*)dgamma, (float*)dbeta,
                                                           (float*)acoef);
  DL_HIP_CHECK(hipGetLastError());
}

void bn_relu_pool_bwd_apply(uintptr_t y, uintptr_t dP, uintptr_t coef, uintptr_t acoef, uintptr_t dy, int B, int H,
                            int W, int C, int opad, uintptr_t stream) {
  check_c_apply(C);
  const int64_t total = (int64_t)B * (H / 2) * (W / 2) * (C / 8);
  bn_relu_pool_bwd_apply_kernel<false><<<stream_grid(total), 256, 0, as_stream(stream)>>>(
      (const bf16_t*)y, (const bf16_t*)dP, (const float*)coef, (const float*)acoef, (bf16_t*)dy, B, H, W, C, opad,
      nullptr, 0.f, 0, nullptr, nullptr);
  DL_HIP_CHECK(hipGetLastError());
}

// atomic modes: dgb = the reduce's g_host_rows accumulated rows of [dgamma ; dbeta]
// (no bn_bwd_finalize launch); dgamma_out / dbeta_out receive the totals (0: the
// single row already is the flat gradient)
void bn_relu_pool_bwd_apply_sums(uintptr_t y, uintptr_t dP, uintptr_t coef, uintptr_t dgb, uintptr_t gamma, int64_t M,
                                 uintptr_t dy, int B, int H, int W, int C, int opad, uintptr_t dgamma_out,
                                 uintptr_t dbeta_out, uintptr_t stream) {
  check_c_apply(C);
  if (C > kFinMaxC) throw std::runtime_error("bn_relu_pool_bwd_apply_sums: C too large");
  if (g_host_rows < 1 || g_host_rows > kMaxRows)
    throw std::runtime_error("bn_relu_pool_bwd_apply_sums: needs an atomic reduction mode with <= 32 rows");
  if ((dgamma_out == 0) != (dbeta_out == 0)) throw std::runtime_error("bn_relu_pool_bwd_apply_sums: dgamma/dbeta");
  const int64_t total = (int64_t)B * (H / 2) * (W / 2) * (C / 8);
  auto k = g_bn_minw_bwd == 4 ? bn_relu_pool_bwd_apply_kernel<true, 4> : bn_relu_pool_bwd_apply_kernel<true, 1>;
  k<<<fin_grid(total), 256, 0, as_stream(stream)>>>(
      (const bf16_t*)y, (const bf16_t*)dP, (const float*)coef, (const float*)dgb, (bf16_t*)dy, B, H, W, C, opad,
      (const float*)gamma, 1.0f / (float)M, g_host_rows, (float*)dgamma_out, (float*)dbeta_out);
  DL_HIP_CHECK(hipGetLastError());
}

// bn_relu_pool_bwd_apply_sums + the classifier weight gradient in one launch
void bn_bwd_apply_head(uintptr_t y, uintptr_t dP, uintptr_t coef, uintptr_t dgb, uintptr_t gamma, int64_t M,
                       uintptr_t dy, int B, int H, int W, int C, int opad, uintptr_t dgamma_out, uintptr_t dbeta_out,
                       uintptr_t h, uintptr_t dlogits, uintptr_t loss_b, int F, int NC, uintptr_t dw, uintptr_t db,
                       uintptr_t loss, uintptr_t slot, uintptr_t step_ctr, uintptr_t stream) {
  check_c_apply(C);
  if (C > kFinMaxC) throw std::runtime_error("bn_bwd_apply_head: C too large");
  if (g_host_rows < 1 || g_host_rows > kMaxRows)
    throw std::runtime_error("bn_bwd_apply_head: needs an atomic reduction mode with <= 32 rows");
  if (NC != 10) throw std::runtime_error("bn_bwd_apply_head: built for 10 classes");
  const int64_t total = (int64_t)B * (H / 2) * (W / 2) * (C / 8);
  const int Ga = fin_grid(total);
  const HeadWgradArgs2 ha{(const bf16_t*)h, (const float*)dlogits, (const float*)loss_b, F, B, (float*)dw,
                          (float*)db, (float*)loss, (float*)slot, (unsigned long long*)step_ctr};
  const int head_blocks = (F + 31) / 32 + 1;
  bwd_apply_head_kernel<<<Ga + head_blocks, 256, 0, as_stream(stream)>>>(
      (const bf16_t*)y, (const bf16_t*)dP, (const float*)coef, (const float*)dgb, (bf16_t*)dy, B, H, W, C, opad,
      (const float*)gamma, 1.0f / (float)M, g_host_rows, (float*)dgamma_out, (float*)dbeta_out, Ga, ha);
  DL_HIP_CHECK(hipGetLastError());
}

// mode 1 forward apply: coefficients from the accumulated statistics `sums` [2][C]
void bn_relu_pool_fwd_fin(uintptr_t y, uintptr_t sums, int64_t M, uintptr_t gamma, uintptr_t beta, uintptr_t bias,
                          uintptr_t rmean, uintptr_t rvar, float eps, float momentum, uintptr_t coef, uintptr_t out,
                          int B, int H, int W, int C, int opad, uintptr_t stream) {
  check_c(C);
  if (C > kFinMaxC) throw std::runtime_error("bn_relu_pool_fwd_fin: C too large");
  if (g_host_rows < 1 || g_host_rows > kMaxRows)
    throw std::runtime_error("bn_relu_pool_fwd_fin: needs an atomic reduction mode with <= 32 rows");
  const int64_t total = (int64_t)B * (H / 2) * (W / 2) * (C / 8);
  const BnFin fin = make_bn_fin(sums, M, gamma, beta, bias, rmean, rvar, eps, momentum, coef, g_host_rows);
  auto k = g_bn_minw_fwd == 4 ? bn_relu_pool_fwd_fin_kernel<4> : bn_relu_pool_fwd_fin_kernel<1>;
  k<<<fin_grid(total), 256, 0, as_stream(stream)>>>((const bf16_t*)y, fin,
                                                                                   (bf16_t*)out, B, H, W, C, opad);
  DL_HIP_CHECK(hipGetLastError());
}

void set_reduce_atomic_bn(int rows) {
  if (rows < 0 || rows > 64 || (rows & (rows - 1)) != 0)
    throw std::runtime_error("set_reduce_atomic: rows must be 0 or a power of two <= 64");
  const int v = rows;
  DL_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_red_atomic_bn), &v, sizeof(int)));
  g_host_rows = rows;
}

}  // namespace dl
