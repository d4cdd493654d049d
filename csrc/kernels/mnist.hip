// The reference MNIST convnet's whole training step (forward + backward) in
// FOUR small kernels, parallel over (channel x sample) workgroups (gfx950).
//
// Reference: examples/mnist.lua:53-88 (and mnist-ea.lua:41-57):
//   Reshape(1,32,32) -> SpatialConvolutionMM(1,16,5,5) -> Tanh -> SpatialMaxPooling(2,2,2,2)
//   -> SpatialConvolutionMM(16,16,5,5) -> Tanh -> SpatialMaxPooling(2,2,2,2)
//   -> Reshape(400) -> Linear(400,10) -> logSoftMax, loss = logMultinomialLoss
// at a per-node batch of 1 (mnist.lua:33): ~6 MFLOP per step, so the step is
// latency bound.  The first version did everything in ONE workgroup with all
// intermediates in LDS and took 177 us (one CU doing everything serially,
// profiles/r2_mnist_fused_v1_kernels.txt) -- slower than PyTorch's 35-kernel
// graph at 142 us.  This version splits every phase by channel so 16
// workgroups per sample run each phase, with the minimum of dependency
// boundaries:
//   K1 (c, b):  conv1 channel c -> tanh -> pool1 (keeps tanh + argmax bytes)
//   K2 (co, b): conv2 output channel co (reads all of pool1) -> tanh -> pool2
//   K3 (b):     linear -> log-softmax -> NLL -> dlogits -> linear backward
//               (dW/db atomics) -> pool2 / tanh backward -> dz2
//   K4 (ci, b): conv2 weight gradient slice [:, ci] + conv2 input gradient of
//               channel ci (branch-free over a zero-bordered dz2 in LDS) ->
//               pool1 / tanh backward -> conv1 weight gradient of channel ci
// Weight gradients of the B samples (and of the per-channel slices) are added
// with fp32 atomics into the zeroed flat gradient; the step is these kernels
// + the engine's zero fill + the fused SGD update, captured in one hipGraph.
// fp32 arithmetic throughout (the reference's precision).
#include "dl_common.h"
#include "dl_ops.h"

namespace dl {

namespace {

constexpr int kT = 256;
constexpr int IMG = 32, K5 = 5, C1 = 16, H1 = 28, P1 = 14, C2 = 16, H2 = 10, P2 = 5;
constexpr int NF = C2 * P2 * P2;  // 400
constexpr int NC = 10;
constexpr int PADW = H2 + 2 * (K5 - 1);  // 18: dz2 zero-bordered for the full convolution

// per-sample scratch (fp32 words; byte tensors at the end)
constexpr int S_A1 = 0;                      // 16x28x28 tanh(conv1)
constexpr int S_P1 = S_A1 + C1 * H1 * H1;    // 16x14x14 pool1
constexpr int S_A2 = S_P1 + C1 * P1 * P1;    // 16x10x10 tanh(conv2)
constexpr int S_P2 = S_A2 + C2 * H2 * H2;    // 400 features
constexpr int S_DZ2 = S_P2 + NF;             // 16x10x10 conv2 output gradient
constexpr int S_I1 = S_DZ2 + C2 * H2 * H2;   // bytes: 16x14x14 pool1 argmax
constexpr int S_I2 = S_I1 + C1 * P1 * P1 / 4;  // bytes: 400 pool2 argmax
constexpr int S_WORDS = (S_I2 + NF / 4 + 63) / 64 * 64;

// tanh(v) = 1 - 2 / (exp(2v) + 1) on the hardware exp (exact limits at +-inf)
__device__ __forceinline__ float tanh_f(float v) { return 1.f - 2.f / (__expf(2.f * v) + 1.f); }

template <bool BF16_IN>
__device__ __forceinline__ float load_x(const void* x, int64_t i) {
  if constexpr (BF16_IN) return bf16_to_f32(reinterpret_cast<const bf16_t*>(x)[i]);
  else return reinterpret_cast<const float*>(x)[i];
}

// K1: conv1 channel c of sample b -> tanh -> pool1 (+ argmax)
template <bool BF16_IN>
__global__ void __launch_bounds__(kT) mnist_k1(const void* __restrict__ xin, const float* __restrict__ w1,
                                               const float* __restrict__ b1, float* __restrict__ scratch) {
  __shared__ float sx[IMG * IMG];
  __shared__ float sa[H1 * H1];
  const int c = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  float* S = scratch + (int64_t)b * S_WORDS;
  for (int i = tid; i < IMG * IMG; i += kT) sx[i] = load_x<BF16_IN>(xin, (int64_t)b * IMG * IMG + i);
  float w[K5 * K5];
#pragma unroll
  for (int t = 0; t < K5 * K5; ++t) w[t] = w1[c * K5 * K5 + t];
  const float bias = b1[c];
  __syncthreads();
  for (int o = tid; o < H1 * H1; o += kT) {
    const int i = o / H1, j = o - i * H1;
    float z = bias;
#pragma unroll
    for (int u = 0; u < K5; ++u)
#pragma unroll
      for (int v = 0; v < K5; ++v) z = fmaf(w[u * K5 + v], sx[(i + u) * IMG + j + v], z);
    const float a = tanh_f(z);
    sa[o] = a;
    S[S_A1 + c * H1 * H1 + o] = a;
  }
  __syncthreads();
  uint8_t* i1 = reinterpret_cast<uint8_t*>(S + S_I1);
  for (int o = tid; o < P1 * P1; o += kT) {
    const int i = o / P1, j = o - i * P1;
    const float* base = sa + 2 * i * H1 + 2 * j;
    float m = base[0];
    int k = 0;
    if (base[1] > m) { m = base[1]; k = 1; }
    if (base[H1] > m) { m = base[H1]; k = 2; }
    if (base[H1 + 1] > m) { m = base[H1 + 1]; k = 3; }
    S[S_P1 + c * P1 * P1 + o] = m;
    i1[c * P1 * P1 + o] = (uint8_t)k;
  }
}

// K2: conv2 output channel co of sample b -> tanh -> pool2 (+ argmax)
__global__ void __launch_bounds__(kT) mnist_k2(const float* __restrict__ w2, const float* __restrict__ b2,
                                               float* __restrict__ scratch) {
  __shared__ float sp[C1 * P1 * P1];
  __shared__ float sw[C1 * K5 * K5];
  __shared__ float sa[H2 * H2];
  const int co = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  float* S = scratch + (int64_t)b * S_WORDS;
  for (int i = tid; i < C1 * P1 * P1; i += kT) sp[i] = S[S_P1 + i];
  for (int i = tid; i < C1 * K5 * K5; i += kT) sw[i] = w2[co * C1 * K5 * K5 + i];
  __syncthreads();
  // 100 outputs x 16 input channels: thread = (output, half of the input channels)
  float z = 0.f;
  const int o = tid % (H2 * H2), part = tid / (H2 * H2);
  const bool act = tid < 2 * H2 * H2;
  if (act) {
    const int i = o / H2, j = o - i * H2;
    for (int ci = part * 8; ci < part * 8 + 8; ++ci) {
      const float* wp = sw + ci * K5 * K5;
      const float* xp = sp + ci * P1 * P1 + i * P1 + j;
#pragma unroll
      for (int u = 0; u < K5; ++u)
#pragma unroll
        for (int v = 0; v < K5; ++v) z = fmaf(wp[u * K5 + v], xp[u * P1 + v], z);
    }
  }
  __shared__ float zp[2 * H2 * H2];
  if (act) zp[tid] = z;
  __syncthreads();
  if (tid < H2 * H2) {
    const float a = tanh_f(b2[co] + zp[tid] + zp[H2 * H2 + tid]);
    sa[tid] = a;
    S[S_A2 + co * H2 * H2 + tid] = a;
  }
  __syncthreads();
  if (tid < P2 * P2) {
    const int i = tid / P2, j = tid - i * P2;
    const float* base = sa + 2 * i * H2 + 2 * j;
    float m = base[0];
    int k = 0;
    if (base[1] > m) { m = base[1]; k = 1; }
    if (base[H2] > m) { m = base[H2]; k = 2; }
    if (base[H2 + 1] > m) { m = base[H2 + 1]; k = 3; }
    S[S_P2 + co * P2 * P2 + tid] = m;  // NCHW flatten order: c*25 + i*5 + j
    reinterpret_cast<uint8_t*>(S + S_I2)[co * P2 * P2 + tid] = (uint8_t)k;
  }
}

// K3: classifier + loss + dlogits + linear backward + pool2/tanh backward
__global__ void __launch_bounds__(kT) mnist_k3(const int64_t* __restrict__ labels, const float* __restrict__ wf,
                                               const float* __restrict__ bfc, float* __restrict__ gwf,
                                               float* __restrict__ gbf, float* __restrict__ logp_out,
                                               float* __restrict__ loss_b, float* __restrict__ scratch, int B) {
  __shared__ float sf[NF];
  __shared__ float red[kT / 64][16];
  __shared__ float dl[16];
  __shared__ float dp2[NF];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  float* S = scratch + (int64_t)b * S_WORDS;
  for (int i = tid; i < NF; i += kT) sf[i] = S[S_P2 + i];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    float s = 0.f;
    for (int f = tid; f < NF; f += kT) s = fmaf(wf[k * NF + f], sf[f], s);
    s = wave_sum(s);
    if (lane == 0) red[wid][k] = s;
  }
  __syncthreads();
  if (tid == 0) {
    float z[NC], mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      float t = bfc[k];
      for (int w = 0; w < kT / 64; ++w) t += red[w][k];
      z[k] = t;
      mx = fmaxf(mx, t);
    }
    float se = 0.f;
#pragma unroll
    for (int k = 0; k < NC; ++k) se += __expf(z[k] - mx);
    const float lse = mx + __logf(se);
    const int y = labels ? (int)labels[b] : -1;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const float lp = z[k] - lse;
      logp_out[(int64_t)b * NC + k] = lp;
      dl[k] = (__expf(lp) - (k == y ? 1.f : 0.f)) / (float)B;  // d(batch-mean NLL)/dlogits
    }
    if (loss_b) loss_b[b] = y >= 0 ? lse - z[y] : 0.f;
  }
  if (labels == nullptr) return;
  __syncthreads();
  for (int e = tid; e < NC * NF; e += kT) unsafeAtomicAdd(gwf + e, dl[e / NF] * sf[e % NF]);
  if (tid < NC) unsafeAtomicAdd(gbf + tid, dl[tid]);
  for (int f = tid; f < NF; f += kT) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NC; ++k) s = fmaf(wf[k * NF + f], dl[k], s);
    dp2[f] = s;
  }
  __syncthreads();
  const uint8_t* i2 = reinterpret_cast<const uint8_t*>(S + S_I2);
  for (int o = tid; o < C2 * H2 * H2; o += kT) {
    const int c = o / (H2 * H2), r = o - c * H2 * H2, i = r / H2, j = r - i * H2;
    const int q = c * P2 * P2 + (i >> 1) * P2 + (j >> 1);
    const float g = (i2[q] == (((i & 1) << 1) | (j & 1))) ? dp2[q] : 0.f;
    const float t = S[S_A2 + o];
    S[S_DZ2 + o] = g * (1.f - t * t);
  }
}

// K4: channel ci of sample b: conv2 weight-gradient slice dW2[:, ci], conv2
// input gradient of ci, pool1/tanh backward, conv1 weight gradient of ci
template <bool BF16_IN>
__global__ void __launch_bounds__(kT) mnist_k4(const void* __restrict__ xin, const float* __restrict__ w2,
                                               float* __restrict__ gw1, float* __restrict__ gb1,
                                               float* __restrict__ gw2, float* __restrict__ gb2,
                                               float* __restrict__ scratch) {
  __shared__ float dzp[C2 * PADW * PADW];  // zero-bordered dz2 (full convolution, branch free)
  __shared__ float sw[C2 * K5 * K5];       // W2[:, ci]
  __shared__ float sp[P1 * P1];            // pool1 channel ci
  __shared__ float sdz1[H1 * H1];          // dz1 channel ci
  __shared__ float sx[IMG * IMG];
  __shared__ float red[2][kT / 64];
  const int ci = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  float* S = scratch + (int64_t)b * S_WORDS;
  for (int i = tid; i < C2 * PADW * PADW; i += kT) {
    const int co = i / (PADW * PADW), r = i - co * PADW * PADW, y = r / PADW - (K5 - 1), x = r % PADW - (K5 - 1);
    dzp[i] = (y >= 0 && y < H2 && x >= 0 && x < H2) ? S[S_DZ2 + co * H2 * H2 + y * H2 + x] : 0.f;
  }
  for (int i = tid; i < C2 * K5 * K5; i += kT) {
    const int co = i / (K5 * K5), t = i - co * K5 * K5;
    sw[i] = w2[(co * C1 + ci) * K5 * K5 + t];
  }
  for (int i = tid; i < P1 * P1; i += kT) sp[i] = S[S_P1 + ci * P1 * P1 + i];
  for (int i = tid; i < IMG * IMG; i += kT) sx[i] = load_x<BF16_IN>(xin, (int64_t)b * IMG * IMG + i);
  __syncthreads();
  // conv2 weight gradient slice: dW2[co][ci][u][v] = sum_{i,j} dz2[co][i][j] p1[ci][i+u][j+v]
  for (int e = tid; e < C2 * K5 * K5; e += kT) {
    const int co = e / (K5 * K5), t = e - co * K5 * K5, u = t / K5, v = t - u * K5;
    const float* g = dzp + co * PADW * PADW + (K5 - 1) * PADW + (K5 - 1);
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < H2; ++i)
#pragma unroll
      for (int j = 0; j < H2; ++j) s = fmaf(g[i * PADW + j], sp[(i + u) * P1 + j + v], s);
    unsafeAtomicAdd(gw2 + (co * C1 + ci) * K5 * K5 + t, s);
  }
  if (ci == 0 && tid < C2) {  // conv2 bias gradient (once per sample)
    float s = 0.f;
    for (int i = 0; i < H2 * H2; ++i) s += S[S_DZ2 + tid * H2 * H2 + i];
    unsafeAtomicAdd(gb2 + tid, s);
  }
  // conv2 input gradient of channel ci, then pool1 / tanh backward -> dz1 (28x28)
  const uint8_t* i1 = reinterpret_cast<const uint8_t*>(S + S_I1) + ci * P1 * P1;
  for (int o = tid; o < H1 * H1; o += kT) sdz1[o] = 0.f;
  __syncthreads();
  for (int o = tid; o < P1 * P1; o += kT) {
    const int y = o / P1, x = o - y * P1;
    float s = 0.f;
    for (int co = 0; co < C2; ++co) {
      const float* wp = sw + co * K5 * K5;
      const float* g = dzp + co * PADW * PADW + y * PADW + x;  // dz2[y-u][x-v] at +(4-u, 4-v)
#pragma unroll
      for (int u = 0; u < K5; ++u)
#pragma unroll
        for (int v = 0; v < K5; ++v) s = fmaf(wp[u * K5 + v], g[(K5 - 1 - u) * PADW + (K5 - 1 - v)], s);
    }
    // route to the pooled position, times tanh'
    const int k = i1[o];
    const int hi = 2 * y + (k >> 1), wi = 2 * x + (k & 1);
    const float t = S[S_A1 + ci * H1 * H1 + hi * H1 + wi];
    sdz1[hi * H1 + wi] = s * (1.f - t * t);
  }
  __syncthreads();
  // conv1 weight gradient of channel ci: dW1[ci][u][v] = sum dz1[i][j] x[i+u][j+v]; bias = sum dz1
  // 25 taps x 8 row groups = 200 threads
  if (tid < K5 * K5 * 8) {
    const int t = tid % (K5 * K5), part = tid / (K5 * K5), u = t / K5, v = t - u * K5;
    float s = 0.f;
    for (int i = part; i < H1; i += 8)
#pragma unroll 4
      for (int j = 0; j < H1; ++j) s = fmaf(sdz1[i * H1 + j], sx[(i + u) * IMG + j + v], s);
    unsafeAtomicAdd(gw1 + ci * K5 * K5 + t, s);
  }
  float sb = 0.f;
  for (int o = tid; o < H1 * H1; o += kT) sb += sdz1[o];
  sb = wave_sum(sb);
  if (lane == 0) red[0][wid] = sb;
  __syncthreads();
  if (tid == 0) {
    float s = 0.f;
    for (int w = 0; w < kT / 64; ++w) s += red[0][w];
    unsafeAtomicAdd(gb1 + ci, s);
  }
}

}  // namespace

int64_t mnist_scratch_bytes(int B) { return (int64_t)B * S_WORDS * 4; }

void mnist_step(uintptr_t x, int x_bf16, uintptr_t labels, uintptr_t w1, uintptr_t b1, uintptr_t w2, uintptr_t b2,
                uintptr_t wf, uintptr_t bf, uintptr_t gw1, uintptr_t gb1, uintptr_t gw2, uintptr_t gb2, uintptr_t gwf,
                uintptr_t gbf, uintptr_t logp, uintptr_t loss_b, uintptr_t scratch, int B, uintptr_t stream) {
  if (B <= 0) return;
  if (B > 65535) throw std::runtime_error("mnist_step: batch too large");
  hipStream_t s = as_stream(stream);
  float* S = (float*)scratch;
  const dim3 gc(C1, B);
  if (x_bf16) mnist_k1<true><<<gc, kT, 0, s>>>((const void*)x, (const float*)w1, (const float*)b1, S);
  else mnist_k1<false><<<gc, kT, 0, s>>>((const void*)x, (const float*)w1, (const float*)b1, S);
  mnist_k2<<<dim3(C2, B), kT, 0, s>>>((const float*)w2, (const float*)b2, S);
  mnist_k3<<<B, kT, 0, s>>>((const int64_t*)labels, (const float*)wf, (const float*)bf, (float*)gwf, (float*)gbf,
                            (float*)logp, (float*)loss_b, S, B);
  if (labels) {
    if (x_bf16)
      mnist_k4<true><<<gc, kT, 0, s>>>((const void*)x, (const float*)w2, (float*)gw1, (float*)gb1, (float*)gw2,
                                       (float*)gb2, S);
    else
      mnist_k4<false><<<gc, kT, 0, s>>>((const void*)x, (const float*)w2, (float*)gw1, (float*)gb1, (float*)gw2,
                                        (float*)gb2, S);
  }
  DL_HIP_CHECK(hipGetLastError());
}

}  // namespace dl
