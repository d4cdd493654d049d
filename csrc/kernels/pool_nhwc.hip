// Channels-last max pooling (the ResNet-50 stem: 3x3, stride 2, pad 1) with
// the argmax kept as one byte per output element, forward and backward
// (gfx950).  The backward is a GATHER (every input pixel collects the <= 4
// windows that may have chosen it), so it needs no atomics and no zero fill;
// torch's NHWC max-pool backward scattered through a zeroed fp32 buffer and
// took 0.62 ms per ResNet-50 step (profiles/r2_resnet50_hip1x1_kernels.txt).
// Ties resolve to the first maximum in row-major window order (torch's rule).
#include "dl_common.h"
#include "bn_coef_dev.h"
#include "dl_ops.h"

namespace dl {

namespace {

__device__ __forceinline__ void unpack8p(const uint4& v, float* f) {
  f[0] = lo_bf16(v.x); f[1] = hi_bf16(v.x); f[2] = lo_bf16(v.y); f[3] = hi_bf16(v.y);
  f[4] = lo_bf16(v.z); f[5] = hi_bf16(v.z); f[6] = lo_bf16(v.w); f[7] = hi_bf16(v.w);
}
__device__ __forceinline__ uint4 pack8p(const float* f) {
  return make_uint4(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]), pack_bf16x2(f[4], f[5]),
                    pack_bf16x2(f[6], f[7]));
}

struct PoolGeom {
  int N, H, W, C, Ho, Wo, K, S, P;
};

// one thread = 8 channels of one output pixel
__global__ void __launch_bounds__(256) maxpool_nhwc_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                               uint8_t* __restrict__ idx, const PoolGeom g) {
  const int C8 = g.C >> 3;
  const int64_t total = (int64_t)g.N * g.Ho * g.Wo * C8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % C8);
    const int64_t pix = i / C8;
    const int ow = (int)(pix % g.Wo);
    const int64_t t = pix / g.Wo;
    const int oh = (int)(t % g.Ho);
    const int64_t n = t / g.Ho;
    float best[8];
    uint8_t arg[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { best[k] = -INFINITY; arg[k] = 0; }
    const int h0 = oh * g.S - g.P, w0 = ow * g.S - g.P;
    for (int u = 0; u < g.K; ++u) {
      const int h = h0 + u;
      if (h < 0 || h >= g.H) continue;
      for (int v = 0; v < g.K; ++v) {
        const int w = w0 + v;
        if (w < 0 || w >= g.W) continue;
        float f[8];
        unpack8p(*reinterpret_cast<const uint4*>(x + ((n * g.H + h) * g.W + w) * (int64_t)g.C + c8 * 8), f);
        const uint8_t pos = (uint8_t)(u * g.K + v);
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (f[k] > best[k]) { best[k] = f[k]; arg[k] = pos; }
      }
    }
    const int64_t o = pix * g.C + c8 * 8;
    *reinterpret_cast<uint4*>(y + o) = pack8p(best);
    uint2 a;
    a.x = (uint32_t)arg[0] | ((uint32_t)arg[1] << 8) | ((uint32_t)arg[2] << 16) | ((uint32_t)arg[3] << 24);
    a.y = (uint32_t)arg[4] | ((uint32_t)arg[5] << 8) | ((uint32_t)arg[6] << 16) | ((uint32_t)arg[7] << 24);
    *reinterpret_cast<uint2*>(idx + o) = a;
  }
}

// one thread = 8 channels of one INPUT pixel: dx = sum of dy over the windows whose argmax is this pixel
__global__ void __launch_bounds__(256) maxpool_nhwc_bwd_kernel(const bf16_t* __restrict__ dy,
                                                               const uint8_t* __restrict__ idx, bf16_t* __restrict__ dx,
                                                               const PoolGeom g) {
  const int C8 = g.C >> 3;
  const int64_t total = (int64_t)g.N * g.H * g.W * C8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % C8);
    const int64_t pix = i / C8;
    const int w = (int)(pix % g.W);
    const int64_t t = pix / g.W;
    const int h = (int)(t % g.H);
    const int64_t n = t / g.H;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // windows oh with oh*S - P <= h <= oh*S - P + K - 1
    const int oh_lo = max(0, (h + g.P - g.K + g.S) / g.S), oh_hi = min(g.Ho - 1, (h + g.P) / g.S);
    const int ow_lo = max(0, (w + g.P - g.K + g.S) / g.S), ow_hi = min(g.Wo - 1, (w + g.P) / g.S);
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int u = h - (oh * g.S - g.P);
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int v = w - (ow * g.S - g.P);
        const uint8_t pos = (uint8_t)(u * g.K + v);
        const int64_t o = ((n * g.Ho + oh) * g.Wo + ow) * (int64_t)g.C + c8 * 8;
        const uint2 a = *reinterpret_cast<const uint2*>(idx + o);
        float d[8];
        unpack8p(*reinterpret_cast<const uint4*>(dy + o), d);
        const uint32_t aw[2] = {a.x, a.y};
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (((aw[k >> 2] >> (8 * (k & 3))) & 0xffu) == pos) acc[k] += d[k];
      }
    }
    *reinterpret_cast<uint4*>(dx + pix * g.C + c8 * 8) = pack8p(acc);
  }
}

// The ResNet-50 stem window (3x3, stride 2, pad 1) with 32-bit indexing and
// every load of an item issued before its first use: the generic kernels above
// run a dependent load chain per window position with 64-bit divisions and
// measured 154 us (forward) / 256 us (backward) per batch-256 step, about
// 3.7 / 2.2 TB/s.  Out-of-image taps load a valid pixel and are masked.
// The training BatchNorm + ReLU that produced the pooled tensor, applied on
// load (PoolBn; the ResNet-50 stem BN): x is then the BN's INPUT, each window
// element is bf16(relu(x * sc + sh)) -- bitwise what the BN's own apply would
// have stored -- and the threads of workgroup 0 publish its saved mean /
// invstd and running statistics: the BN's apply launch and the write + read of
// its 112x112 output go.
struct PoolBn {
  const float* acc;  // [2C] sum, sum of squares of the BN input (null: plain pooling)
  const float* w;
  const float* b;
  float* save;
  float* run_mean;
  float* run_var;
  float eps, momentum;
};

__global__ void __launch_bounds__(256) maxpool3s2_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                             uint8_t* __restrict__ idx, const PoolGeom g,
                                                             const PoolBn pb) {
  const int C8 = g.C >> 3;
  const int total = g.N * g.Ho * g.Wo * C8;
  // (the grid stride is a multiple of C8: a thread keeps its 8 channels)
  float sc[8], sh[8];
  const bool bn = pb.acc != nullptr;
  if (bn) {
    const int i0 = blockIdx.x * blockDim.x + threadIdx.x;
    bn_coef8(pb.acc, pb.w, pb.b, g.C, (i0 % C8) * 8, (int64_t)g.N * g.H * g.W, pb.eps, pb.momentum,
             blockIdx.x == 0 && (int)threadIdx.x < C8, pb.save, pb.run_mean, pb.run_var, sc, sh);
  }
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c8 = i % C8, pix = i / C8;
    const int ow = pix % g.Wo, t = pix / g.Wo;
    const int oh = t % g.Ho, n = t / g.Ho;
    const int h0 = 2 * oh - 1, w0 = 2 * ow - 1;
    uint4 v[9];
    bool ok[9];
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int h = h0 + u, w = w0 + q;
        ok[u * 3 + q] = h >= 0 && h < g.H && w >= 0 && w < g.W;
        const int hh = ok[u * 3 + q] ? h : oh * 2, ww = ok[u * 3 + q] ? w : ow * 2;  // (2 oh, 2 ow) is inside
        v[u * 3 + q] = *reinterpret_cast<const uint4*>(x + ((int64_t)(n * g.H + hh) * g.W + ww) * g.C + c8 * 8);
      }
    float best[8];
    uint8_t arg[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { best[k] = -INFINITY; arg[k] = 0; }
#pragma unroll
    for (int p = 0; p < 9; ++p) {
      if (!ok[p]) continue;
      float f[8];
      unpack8p(v[p], f);
      if (bn) {  // the stored BN + ReLU output (bf16), as the apply would write it
#pragma unroll
        for (int k = 0; k < 8; ++k) f[k] = __uint_as_float((uint32_t)f32_to_bf16(fmaxf(fmaf(f[k], sc[k], sh[k]), 0.f)) << 16);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (f[k] > best[k]) { best[k] = f[k]; arg[k] = (uint8_t)p; }
    }
    const int64_t o = (int64_t)pix * g.C + c8 * 8;
    *reinterpret_cast<uint4*>(y + o) = pack8p(best);
    uint2 a;
    a.x = (uint32_t)arg[0] | ((uint32_t)arg[1] << 8) | ((uint32_t)arg[2] << 16) | ((uint32_t)arg[3] << 24);
    a.y = (uint32_t)arg[4] | ((uint32_t)arg[5] << 8) | ((uint32_t)arg[6] << 16) | ((uint32_t)arg[7] << 24);
    *reinterpret_cast<uint2*>(idx + o) = a;
  }
}

// input row h is covered by the windows oh = h/2 (and (h+1)/2 when h is odd)
__global__ void __launch_bounds__(256) maxpool3s2_bwd_kernel(const bf16_t* __restrict__ dy,
                                                             const uint8_t* __restrict__ idx, bf16_t* __restrict__ dx,
                                                             const PoolGeom g) {
  const int C8 = g.C >> 3;
  const int total = g.N * g.H * g.W * C8;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c8 = i % C8, pix = i / C8;
    const int w = pix % g.W, t = pix / g.W;
    const int h = t % g.H, n = t / g.H;
    const int ohs[2] = {h >> 1, min(g.Ho - 1, (h + 1) >> 1)};
    const int ows[2] = {w >> 1, min(g.Wo - 1, (w + 1) >> 1)};
    uint4 d[4];
    uint2 a[4];
    bool ok[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int oh = ohs[j >> 1], ow = ows[j & 1];
      ok[j] = (j < 2 || ohs[1] != ohs[0]) && ((j & 1) == 0 || ows[1] != ows[0]);
      const int64_t o = ((int64_t)(n * g.Ho + oh) * g.Wo + ow) * g.C + c8 * 8;
      d[j] = *reinterpret_cast<const uint4*>(dy + o);
      a[j] = *reinterpret_cast<const uint2*>(idx + o);
    }
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!ok[j]) continue;
      const int oh = ohs[j >> 1], ow = ows[j & 1];
      const uint32_t pos = (uint32_t)((h - (2 * oh - 1)) * 3 + (w - (2 * ow - 1)));
      float f[8];
      unpack8p(d[j], f);
      const uint32_t aw[2] = {a[j].x, a[j].y};
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (((aw[k >> 2] >> (8 * (k & 3))) & 0xffu) == pos) acc[k] += f[k];
    }
    *reinterpret_cast<uint4*>(dx + (int64_t)pix * g.C + c8 * 8) = pack8p(acc);
  }
}

// The stem max-pool backward fused with the backward of the BN + ReLU that
// produced its input (relu mode 2: mask recomputed from the BN input x): every
// input pixel gathers its dz (rounded to bf16, as the plain backward stores
// it), g = dz * (x * sc + sh > 0), and
//   PASS 0: per-channel sum(g), sum(g * xhat) -> acc (zeroed; one fp32 atomic
//           per channel per block, grid capped like bn_nhwc's reduce);
//   PASS 1: dx = w * invstd * (g - mean(g) - xhat * mean(g xhat)) and, block 0,
//           dgamma / dbeta -- bn_nhwc.hip's arithmetic (relu mode 2).
// The 112x112 dz is never written, and the BN's two passes re-read the small
// pooled gradient and argmax bytes instead of it.
template <int PASS>
__global__ void __launch_bounds__(256) maxpool3s2_bwd_bn_kernel(const bf16_t* __restrict__ dy,
                                                                const uint8_t* __restrict__ idx,
                                                                const bf16_t* __restrict__ x,
                                                                const float* __restrict__ save,
                                                                const float* __restrict__ w,
                                                                const float* __restrict__ b, float* __restrict__ acc,
                                                                bf16_t* __restrict__ dx, float* __restrict__ dw,
                                                                float* __restrict__ db, const PoolGeom g) {
  const int C8 = g.C >> 3;
  const int total = g.N * g.H * g.W * C8;
  const int t0 = blockIdx.x * blockDim.x + threadIdx.x;
  const int c0 = (t0 % C8) * 8;  // (the grid stride is a multiple of C8: fixed channels per thread)
  const float invM = 1.f / (float)((int64_t)g.N * g.H * g.W);
  float mean[8], invstd[8], sc[8], sh[8], mg[8], mgx[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mean[k] = save[c0 + k];
    invstd[k] = save[g.C + c0 + k];
    sc[k] = w[c0 + k] * invstd[k];
    sh[k] = fmaf(-mean[k], sc[k], b[c0 + k]);
    mg[k] = PASS == 1 ? acc[c0 + k] * invM : 0.f;
    mgx[k] = PASS == 1 ? acc[g.C + c0 + k] * invM : 0.f;
  }
  if (PASS == 1 && blockIdx.x == 0 && (int)threadIdx.x < C8) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      db[c0 + k] = acc[c0 + k];
      dw[c0 + k] = acc[g.C + c0 + k];
    }
  }
  float s1[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, s2[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int i = t0; i < total; i += gridDim.x * blockDim.x) {
    const int c8 = i % C8, pix = i / C8;
    const int ww = pix % g.W, t = pix / g.W;
    const int h = t % g.H, n = t / g.H;
    const int ohs[2] = {h >> 1, min(g.Ho - 1, (h + 1) >> 1)};
    const int ows[2] = {ww >> 1, min(g.Wo - 1, (ww + 1) >> 1)};
    uint4 d[4];
    uint2 a[4];
    bool ok[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int oh = ohs[j >> 1], ow = ows[j & 1];
      ok[j] = (j < 2 || ohs[1] != ohs[0]) && ((j & 1) == 0 || ows[1] != ows[0]);
      const int64_t o = ((int64_t)(n * g.Ho + oh) * g.Wo + ow) * g.C + c8 * 8;
      d[j] = *reinterpret_cast<const uint4*>(dy + o);
      a[j] = *reinterpret_cast<const uint2*>(idx + o);
    }
    const int64_t xo = (int64_t)pix * g.C + c8 * 8;
    const uint4 xr = *reinterpret_cast<const uint4*>(x + xo);
    float dz[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!ok[j]) continue;
      const int oh = ohs[j >> 1], ow = ows[j & 1];
      const uint32_t pos = (uint32_t)((h - (2 * oh - 1)) * 3 + (ww - (2 * ow - 1)));
      float f[8];
      unpack8p(d[j], f);
      const uint32_t aw[2] = {a[j].x, a[j].y};
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (((aw[k >> 2] >> (8 * (k & 3))) & 0xffu) == pos) dz[k] += f[k];
    }
    float xv[8], gv[8];
    unpack8p(pack8p(dz), gv);  // the stored dz's bf16 values
    unpack8p(xr, xv);
#pragma unroll
    for (int k = 0; k < 8; ++k) gv[k] = fmaf(xv[k], sc[k], sh[k]) > 0.f ? gv[k] : 0.f;
    if (PASS == 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s1[k] += gv[k];
        s2[k] = fmaf(gv[k], (xv[k] - mean[k]) * invstd[k], s2[k]);
      }
    } else {
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float xh = (xv[k] - mean[k]) * invstd[k];
        o[k] = sc[k] * (gv[k] - mg[k] - xh * mgx[k]);
      }
      *reinterpret_cast<uint4*>(dx + xo) = pack8p(o);
    }
  }
  if (PASS == 0) {  // threads t and t + C8, t + 2 C8, ... share channels: sum them, one atomic per channel
    __shared__ float red[256 * 16];
    const int tt = threadIdx.x;
#pragma unroll
    for (int k = 0; k < 8; ++k) { red[tt * 16 + k] = s1[k]; red[tt * 16 + 8 + k] = s2[k]; }
    __syncthreads();
    for (int j = tt; j < 2 * g.C; j += 256) {
      const int which = j / g.C, ch = j - which * g.C;
      float sum = 0.f;
      for (int r = ch >> 3; r < 256; r += C8) sum += red[r * 16 + which * 8 + (ch & 7)];
      atomicAdd(&acc[which * g.C + ch], sum);
    }
  }
}

static bool stem_window(const PoolGeom& g, int64_t in_items) {
  return g.K == 3 && g.S == 2 && g.P == 1 && in_items < (1ll << 31);
}

PoolGeom pool_geom(int N, int H, int W, int C, int K, int S, int P) {
  if (C % 8 != 0) throw std::runtime_error("maxpool_nhwc: C % 8 != 0");
  if (K * K > 255 || K <= 0 || S <= 0 || P < 0 || 2 * P > K) throw std::runtime_error("maxpool_nhwc: bad window");
  PoolGeom g{N, H, W, C, (H + 2 * P - K) / S + 1, (W + 2 * P - K) / S + 1, K, S, P};
  return g;
}

}  // namespace

// bn_acc != 0: x is the input of a training BatchNorm + ReLU applied on load
// (PoolBn: its complete [2C] sums, gamma / beta, and the save / running
// statistics its own apply would write); 3x3 / stride 2 / pad 1 only.
void maxpool_nhwc_fwd(uintptr_t x, uintptr_t y, uintptr_t idx, int N, int H, int W, int C, int K, int S, int P,
                      uintptr_t stream, uintptr_t bn_acc, uintptr_t bn_w, uintptr_t bn_b, uintptr_t bn_save,
                      uintptr_t bn_rm, uintptr_t bn_rv, double bn_eps, double bn_momentum) {
  const PoolGeom g = pool_geom(N, H, W, C, K, S, P);
  const int64_t total = (int64_t)N * g.Ho * g.Wo * (C / 8);
  const bool stem = stem_window(g, (int64_t)N * H * W * (C / 8));
  if (bn_acc && (!stem || !bn_w || !bn_b || !bn_save || 256 % (C / 8) != 0))
    throw std::runtime_error("maxpool_nhwc_fwd: BN on load needs the 3x3/2 window, its parameters and C/8 | 256");
  const PoolBn pb{(const float*)bn_acc, (const float*)bn_w, (const float*)bn_b, (float*)bn_save, (float*)bn_rm,
                  (float*)bn_rv, (float)bn_eps, (float)bn_momentum};
  if (stem)
    maxpool3s2_fwd_kernel<<<(int)std::min<int64_t>((total + 255) / 256, 8192), 256, 0, as_stream(stream)>>>(
        (const bf16_t*)x, (bf16_t*)y, (uint8_t*)idx, g, pb);
  else
    maxpool_nhwc_fwd_kernel<<<stream_grid(total), 256, 0, as_stream(stream)>>>((const bf16_t*)x, (bf16_t*)y,
                                                                                (uint8_t*)idx, g);
  DL_HIP_CHECK(hipGetLastError());
}

void maxpool_nhwc_bwd(uintptr_t dy, uintptr_t idx, uintptr_t dx, int N, int H, int W, int C, int K, int S, int P,
                      uintptr_t stream) {
  const PoolGeom g = pool_geom(N, H, W, C, K, S, P);
  const int64_t total = (int64_t)N * H * W * (C / 8);
  if (stem_window(g, total))
    maxpool3s2_bwd_kernel<<<(int)std::min<int64_t>((total + 255) / 256, 8192), 256, 0, as_stream(stream)>>>(
        (const bf16_t*)dy, (const uint8_t*)idx, (bf16_t*)dx, g);
  else
    maxpool_nhwc_bwd_kernel<<<stream_grid(total), 256, 0, as_stream(stream)>>>((const bf16_t*)dy, (const uint8_t*)idx,
                                                                                (bf16_t*)dx, g);
  DL_HIP_CHECK(hipGetLastError());
}

// The stem max-pool backward fused with its input BN + ReLU's backward
// (maxpool3s2_bwd_bn_kernel): dy / idx the pooled gradient and argmax bytes,
// x the BN input, save its [2C] mean / invstd, w / b its affine parameters,
// acc its [2C] backward sums (zeroed), dx the BN input gradient, dw / db its
// parameter gradients.
void maxpool_bn_bwd(uintptr_t dy, uintptr_t idx, uintptr_t x, uintptr_t save, uintptr_t w, uintptr_t b,
                    uintptr_t acc, uintptr_t dx, uintptr_t dw, uintptr_t db, int N, int H, int W, int C,
                    uintptr_t stream) {
  const PoolGeom g = pool_geom(N, H, W, C, 3, 2, 1);
  const int64_t total = (int64_t)N * H * W * (C / 8);
  if (!stem_window(g, total) || 256 % (C / 8) != 0)
    throw std::runtime_error("maxpool_bn_bwd: the 3x3/2 window, C/8 | 256");
  if (!dy || !idx || !x || !save || !w || !b || !acc || !dx || !dw || !db)
    throw std::runtime_error("maxpool_bn_bwd: null operand");
  hipStream_t s = as_stream(stream);
  // (the sums pass: 2048 blocks -- at 256, one 4-wave block per CU left its gather loads exposed: 456 us)
  maxpool3s2_bwd_bn_kernel<0><<<(int)std::min<int64_t>((total + 255) / 256, 2048), 256, 0, s>>>(
      (const bf16_t*)dy, (const uint8_t*)idx, (const bf16_t*)x, (const float*)save, (const float*)w,
      (const float*)b, (float*)acc, nullptr, nullptr, nullptr, g);
  DL_HIP_CHECK(hipGetLastError());
  maxpool3s2_bwd_bn_kernel<1><<<(int)std::min<int64_t>((total + 255) / 256, 8192), 256, 0, s>>>(
      (const bf16_t*)dy, (const uint8_t*)idx, (const bf16_t*)x, (const float*)save, (const float*)w,
      (const float*)b, (float*)acc, (bf16_t*)dx, (float*)dw, (float*)db, g);
  DL_HIP_CHECK(hipGetLastError());
}

}  // namespace dl
