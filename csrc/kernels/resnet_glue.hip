// ResNet-50 glue kernels (gfx950): the data re-layouts that let the strided
// convolutions, the stem and the classifier run on the MFMA implicit-GEMM
// kernels of conv_igemm.hip (conv_fwd_ex / conv_wgrad_ex / conv_fwd /
// conv_wgrad) instead of MIOpen / hipBLAS:
//
//  * stem (7x7 stride 2 over 3 channels): 2x2 space-to-depth of the padded
//    image (12 channels, padded to 16) turns it into a 4x4 stride-1 conv --
//    s2d_stem_input, stem_weight_pack (7x7x3 -> 4x4x16 bf16 weights, per
//    step from the bf16 shadow) and stem_wgrad_unpack (the 4x4x16 weight
//    gradient slabs back into the fp32 [64][3][7][7] gradient);
//  * stride-2 3x3 input gradient: one KH x KW phase conv per output parity
//    (phase_weights: the flipped/transposed weight's taps per phase);
//  * classifier: spatial mean (head_pool), log-softmax + NLL + dlogits from
//    the fp32 split-K logits slabs (head_softmax_nll), the per-step bf16
//    weight copies (head_weight_prep), the broadcast of dpooled over the
//    7x7 positions (head_broadcast) and the fc weight gradient reduce.
// All are memory-bound streaming kernels with 16-byte accesses where the
// layout allows.
#include "dl_common.h"
#include "dl_ops.h"

namespace dl {

// ---------------------------------------------------------------------------
// stem: S[n][i][j][(a*2+b)*3 + c] = x[n][2i+a-3][2j+b-3][c] (0 outside), i, j < Hs
// x: NHWC bf16 [N][H][W][3]; S: [N][Hs][Ws][16], channels 12..15 zero.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) s2d_stem_input_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ S,
                                                             int N, int H, int W, int Hs, int Ws, int pad) {
  const int64_t total = (int64_t)N * Hs * Ws;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(t % Ws);
    const int64_t r = t / Ws;
    const int i = (int)(r % Hs);
    const int64_t n = r / Hs;
    uint32_t v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    bf16_t h[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) h[k] = 0;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int yy = 2 * i + a - pad, xx = 2 * j + b - pad;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
          const bf16_t* p = x + ((n * H + yy) * W + xx) * 3;
#pragma unroll
          for (int c = 0; c < 3; ++c) h[(a * 2 + b) * 3 + c] = p[c];
        }
      }
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = (uint32_t)h[2 * k] | ((uint32_t)h[2 * k + 1] << 16);
    uint4* o = reinterpret_cast<uint4*>(S + t * 16);
    o[0] = make_uint4(v[0], v[1], v[2], v[3]);
    o[1] = make_uint4(v[4], v[5], v[6], v[7]);
  }
}

// W4[o][th][tw][(a*2+b)*3+c] = W7[o][c][2th+a][2tw+b] (bf16 shadow, OIHW 7x7); 0 outside
__global__ void __launch_bounds__(256) stem_weight_pack_kernel(const bf16_t* __restrict__ w7, bf16_t* __restrict__ w4,
                                                               int Cout) {
  const int total = Cout * 256;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int ch = t & 15, tw = (t >> 4) & 3, th = (t >> 6) & 3, o = t >> 8;
    bf16_t v = 0;
    if (ch < 12) {
      const int c = ch % 3, ab = ch / 3, a = ab >> 1, b = ab & 1;
      const int kh = 2 * th + a, kw = 2 * tw + b;
      if (kh < 7 && kw < 7) v = w7[((o * 3 + c) * 7 + kh) * 7 + kw];
    }
    w4[t] = v;
  }
}

// dW7[o][c][kh][kw] += sum_s slab[s][o][(kh/2*4 + kw/2)*16 + ((kh%2)*2 + kw%2)*3 + c]
__global__ void __launch_bounds__(256) stem_wgrad_unpack_kernel(const float* __restrict__ slab, float* __restrict__ dw7,
                                                                int splits, int Cout) {
  const int total = Cout * 3 * 49;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int kw = t % 7, kh = (t / 7) % 7, c = (t / 49) % 3, o = t / 147;
    const int k = ((kh >> 1) * 4 + (kw >> 1)) * 16 + ((kh & 1) * 2 + (kw & 1)) * 3 + c;
    float s = 0.f;
    for (int q = 0; q < splits; ++q) s += slab[((int64_t)q * Cout + o) * 256 + k];
    dw7[t] += s;
  }
}

// ---------------------------------------------------------------------------
// stride-2 3x3 dgrad phases.  wt: flipped/transposed weight [Cin][3][3][Cout]
// (weight_flip_transpose: wt[c][kh'][kw'][o] = W[o][2-kh'][2-kw'][c]).
// Input-gradient row parity r (ih = 2q + r - 1 + 1 ... see ops/conv.py
// Conv3x3S2): parity 0 uses flipped tap {1}, parity 1 uses flipped taps {0, 2}
// (t = 0 -> 0, t = 1 -> 2).  Phase p = rh*2 + rw gets [Cin][KHp][KWp][Cout]
// at arena offset off_p = Cin*Cout*(sum of the previous phases' taps).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int phase_tap(int r, int t) { return r == 0 ? 1 : 2 * t; }

__global__ void __launch_bounds__(256) phase_weights_kernel(const bf16_t* __restrict__ wt, bf16_t* __restrict__ out,
                                                            int Cin, int Cout) {
  const int C8 = Cout / 8;
  const int64_t total = (int64_t)Cin * 9 * C8;  // 1 + 2 + 2 + 4 = 9 taps over the 4 phases
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int o8 = (int)(t % C8);
    int64_t r = t / C8;
    int tap = (int)(r % 9);
    const int c = (int)(r / 9);
    // tap -> (phase, th, tw): phase 0 has 1 tap, phases 1 and 2 two, phase 3 four
    int p, th, tw, kh, kw, base;
    if (tap == 0) { p = 0; th = 0; tw = 0; base = 0; }
    else if (tap < 3) { p = 1; th = 0; tw = tap - 1; base = 1; }
    else if (tap < 5) { p = 2; th = tap - 3; tw = 0; base = 3; }
    else { p = 3; th = (tap - 5) >> 1; tw = (tap - 5) & 1; base = 5; }
    const int rh = p >> 1, rw = p & 1;
    const int KHp = rh ? 2 : 1, KWp = rw ? 2 : 1;
    kh = phase_tap(rh, th);
    kw = phase_tap(rw, tw);
    const uint4 v = *reinterpret_cast<const uint4*>(wt + (((int64_t)c * 3 + kh) * 3 + kw) * Cout + o8 * 8);
    bf16_t* dst = out + (int64_t)base * Cin * Cout + (((int64_t)c * KHp + th) * KWp + tw) * Cout + o8 * 8;
    *reinterpret_cast<uint4*>(dst) = v;
  }
}

// ---------------------------------------------------------------------------
// classifier head
// ---------------------------------------------------------------------------
// f[b][c] = bf16(mean_hw h[b][hw][c]); h bf16 [B][HW][C], 8 channels per thread;
// also zeroes the step's loss accumulator (head_softmax_nll adds into it)
__global__ void __launch_bounds__(256) head_pool_kernel(const bf16_t* __restrict__ h, bf16_t* __restrict__ f, int B,
                                                        int HW, int C, float* __restrict__ loss) {
  const int C8 = C / 8;
  if (loss && blockIdx.x == 0 && threadIdx.x == 0) loss[0] = 0.f;
  const int64_t total = (int64_t)B * C8;
  const float inv = 1.f / (float)HW;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(t % C8);
    const int64_t b = t / C8;
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const bf16_t* p = h + b * HW * C + c8 * 8;
    for (int q = 0; q < HW; ++q) {
      const uint4 v = *reinterpret_cast<const uint4*>(p + (int64_t)q * C);
      s[0] += lo_bf16(v.x); s[1] += hi_bf16(v.x); s[2] += lo_bf16(v.y); s[3] += hi_bf16(v.y);
      s[4] += lo_bf16(v.z); s[5] += hi_bf16(v.z); s[6] += lo_bf16(v.w); s[7] += hi_bf16(v.w);
    }
    *reinterpret_cast<uint4*>(f + b * C + c8 * 8) =
        make_uint4(pack_bf16x2(s[0] * inv, s[1] * inv), pack_bf16x2(s[2] * inv, s[3] * inv),
                   pack_bf16x2(s[4] * inv, s[5] * inv), pack_bf16x2(s[6] * inv, s[7] * inv));
  }
}

// One block per sample: logits[c] = sum_s slab[s][b][c] + bias[c] (c < NC of the
// NCp padded columns), logp = log-softmax, loss_b = -logp[label]; with labels:
// dl[b][c] = bf16((softmax - onehot) * dscale) (0 in the padded columns) and
// db[c] += (softmax - onehot) / B (fp32 atomics).  NC <= 4 * 256.
__global__ void __launch_bounds__(256) head_softmax_nll_kernel(const float* __restrict__ slab, int splits, int B,
                                                               int NC, int NCp, const float* __restrict__ bias,
                                                               const int64_t* __restrict__ labels,
                                                               float* __restrict__ logp, float* __restrict__ loss_b,
                                                               bf16_t* __restrict__ dl, float dscale,
                                                               float* __restrict__ db, float* __restrict__ loss) {
  const int b = blockIdx.x, tid = threadIdx.x;
  constexpr int PER = 4;
  float v[PER];
  float mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int c = tid + k * 256;
    float s = -INFINITY;
    if (c < NC) {
      s = bias[c];
      for (int q = 0; q < splits; ++q) s += slab[((int64_t)q * B + b) * NCp + c];
    }
    v[k] = s;
    mx = fmaxf(mx, s);
  }
  __shared__ float red[4];
  mx = wave_max(mx);
  if ((tid & 63) == 0) red[tid >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float se = 0.f;
#pragma unroll
  for (int k = 0; k < PER; ++k) se += (tid + k * 256 < NC) ? __expf(v[k] - mx) : 0.f;
  se = wave_sum(se);
  if ((tid & 63) == 0) red[tid >> 6] = se;
  __syncthreads();
  const float lse = mx + __logf(red[0] + red[1] + red[2] + red[3]);
  const int64_t y64 = labels ? labels[b] : -1;
  const int y = (int)y64;
  if (labels && tid == 0 && (y64 < 0 || y64 >= NC)) {
    // out-of-range label: this sample's loss (and the mean) become NaN rather
    // than silently leaving loss_b unwritten (the gradient row is label-free)
    loss_b[b] = __builtin_nanf("");
    if (loss) unsafeAtomicAdd(loss, __builtin_nanf(""));
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int c = tid + k * 256;
    if (c < NC) {
      const float lp = v[k] - lse;
      if (logp) logp[(int64_t)b * NC + c] = lp;
      if (labels) {
        const float g = __expf(lp) - (c == y ? 1.f : 0.f);
        dl[(int64_t)b * NCp + c] = f32_to_bf16(g * dscale);
        unsafeAtomicAdd(db + c, g / (float)B);
        if (c == y) {
          loss_b[b] = -lp;
          if (loss) unsafeAtomicAdd(loss, -lp / (float)B);
        }
      }
    } else if (labels && c < NCp) {
      dl[(int64_t)b * NCp + c] = 0;
    }
  }
}

// wb[n][c] = bf16(w[n][c]) (n < NC, 0 for NC <= n < NCp);  wbt[c][n] = wb[n][c]
__global__ void __launch_bounds__(256) head_weight_prep_kernel(const float* __restrict__ w, bf16_t* __restrict__ wb,
                                                               bf16_t* __restrict__ wbt, int NC, int NCp, int C) {
  __shared__ bf16_t tile[64][66];
  const int tilesC = C / 64;
  const int tn = blockIdx.x / tilesC, tc = blockIdx.x - tn * tilesC;
  const int n0 = tn * 64, c0 = tc * 64;
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int r = e >> 6, cc = e & 63;
    const int n = n0 + r;
    const bf16_t v = n < NC ? f32_to_bf16(w[(int64_t)n * C + c0 + cc]) : (bf16_t)0;
    wb[(int64_t)n * C + c0 + cc] = v;
    tile[r][cc] = v;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int r = e >> 6, nn = e & 63;
    wbt[(int64_t)(c0 + r) * NCp + n0 + nn] = tile[nn][r];
  }
}

// dh[b][q][c] = df[b][c] (bf16) for q < HW: the mean's backward (1/HW already
// folded into dlogits); 8 channels per thread
__global__ void __launch_bounds__(256) head_broadcast_kernel(const bf16_t* __restrict__ df, bf16_t* __restrict__ dh,
                                                             int B, int HW, int C) {
  const int C8 = C / 8;
  const int64_t total = (int64_t)B * HW * C8;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(t % C8);
    const int64_t b = t / ((int64_t)HW * C8);
    reinterpret_cast<uint4*>(dh)[t] = *reinterpret_cast<const uint4*>(df + b * C + c8 * 8);
  }
}

// dw[n][c] += scale * sum_s slab[s][n][c] for n < NC (the padded rows NC..NCp-1 dropped)
__global__ void __launch_bounds__(256) head_wgrad_reduce_kernel(const float* __restrict__ slab, float* __restrict__ dw,
                                                                int splits, int NC, int NCp, int C, float scale) {
  const int64_t total = (int64_t)NC * C / 4;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int q = 0; q < splits; ++q) {
      const float4 v = reinterpret_cast<const float4*>(slab + (int64_t)q * NCp * C)[t];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    float4 d = reinterpret_cast<float4*>(dw)[t];
    d.x += scale * a.x; d.y += scale * a.y; d.z += scale * a.z; d.w += scale * a.w;
    reinterpret_cast<float4*>(dw)[t] = d;
  }
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
void s2d_stem_input(uintptr_t x, uintptr_t S, int N, int H, int W, int Hs, int Ws, int pad, uintptr_t stream) {
  const int64_t total = (int64_t)N * Hs * Ws;
  s2d_stem_input_kernel<<<stream_grid(total), 256, 0, as_stream(stream)>>>((const bf16_t*)x, (bf16_t*)S, N, H, W, Hs,
                                                                          Ws, pad);
  DL_HIP_CHECK(hipGetLastError());
}

void stem_weight_pack(uintptr_t w7, uintptr_t w4, int Cout, uintptr_t stream) {
  stem_weight_pack_kernel<<<stream_grid((int64_t)Cout * 256), 256, 0, as_stream(stream)>>>((const bf16_t*)w7,
                                                                                           (bf16_t*)w4, Cout);
  DL_HIP_CHECK(hipGetLastError());
}

void stem_wgrad_unpack(uintptr_t slab, uintptr_t dw7, int splits, int Cout, uintptr_t stream) {
  stem_wgrad_unpack_kernel<<<stream_grid((int64_t)Cout * 147), 256, 0, as_stream(stream)>>>(
      (const float*)slab, (float*)dw7, splits, Cout);
  DL_HIP_CHECK(hipGetLastError());
}

void phase_weights(uintptr_t wt, uintptr_t out, int Cin, int Cout, uintptr_t stream) {
  if (Cout % 8 != 0) throw std::runtime_error("phase_weights: Cout % 8 != 0");
  phase_weights_kernel<<<stream_grid((int64_t)Cin * 9 * (Cout / 8)), 256, 0, as_stream(stream)>>>(
      (const bf16_t*)wt, (bf16_t*)out, Cin, Cout);
  DL_HIP_CHECK(hipGetLastError());
}

void head_pool(uintptr_t h, uintptr_t f, int B, int HW, int C, uintptr_t loss, uintptr_t stream) {
  if (C % 8 != 0) throw std::runtime_error("head_pool: C % 8 != 0");
  head_pool_kernel<<<stream_grid((int64_t)B * (C / 8)), 256, 0, as_stream(stream)>>>((const bf16_t*)h, (bf16_t*)f, B,
                                                                                      HW, C, (float*)loss);
  DL_HIP_CHECK(hipGetLastError());
}

void head_softmax_nll(uintptr_t slab, int splits, int B, int NC, int NCp, uintptr_t bias, uintptr_t labels,
                      uintptr_t logp, uintptr_t loss_b, uintptr_t dl, float dscale, uintptr_t db, uintptr_t loss,
                      uintptr_t stream) {
  if (NC > 1024 || NCp < NC) throw std::runtime_error("head_softmax_nll: NC <= 1024 <= NCp");
  head_softmax_nll_kernel<<<B, 256, 0, as_stream(stream)>>>((const float*)slab, splits, B, NC, NCp, (const float*)bias,
                                                            (const int64_t*)labels, (float*)logp, (float*)loss_b,
                                                            (bf16_t*)dl, dscale, (float*)db, (float*)loss);
  DL_HIP_CHECK(hipGetLastError());
}

void head_weight_prep(uintptr_t w, uintptr_t wb, uintptr_t wbt, int NC, int NCp, int C, uintptr_t stream) {
  if (NCp % 64 != 0 || C % 64 != 0) throw std::runtime_error("head_weight_prep: NCp, C multiples of 64");
  head_weight_prep_kernel<<<(NCp / 64) * (C / 64), 256, 0, as_stream(stream)>>>((const float*)w, (bf16_t*)wb,
                                                                                 (bf16_t*)wbt, NC, NCp, C);
  DL_HIP_CHECK(hipGetLastError());
}

void head_broadcast(uintptr_t df, uintptr_t dh, int B, int HW, int C, uintptr_t stream) {
  if (C % 8 != 0) throw std::runtime_error("head_broadcast: C % 8 != 0");
  head_broadcast_kernel<<<stream_grid((int64_t)B * HW * (C / 8)), 256, 0, as_stream(stream)>>>(
      (const bf16_t*)df, (bf16_t*)dh, B, HW, C);
  DL_HIP_CHECK(hipGetLastError());
}

void head_wgrad_reduce(uintptr_t slab, uintptr_t dw, int splits, int NC, int NCp, int C, float scale,
                       uintptr_t stream) {
  if (C % 4 != 0) throw std::runtime_error("head_wgrad_reduce: C % 4 != 0");
  head_wgrad_reduce_kernel<<<stream_grid((int64_t)NC * C / 4), 256, 0, as_stream(stream)>>>(
      (const float*)slab, (float*)dw, splits, NC, NCp, C, scale);
  DL_HIP_CHECK(hipGetLastError());
}

}  // namespace dl
