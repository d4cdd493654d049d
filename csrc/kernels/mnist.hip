// The reference MNIST convnet, forward AND backward of a whole training step
// in ONE kernel launch (gfx950).
//
// Reference: examples/mnist.lua:53-88 (and mnist-ea.lua:41-57):
//   Reshape(1,32,32) -> SpatialConvolutionMM(1,16,5,5) -> Tanh -> SpatialMaxPooling(2,2,2,2)
//   -> SpatialConvolutionMM(16,16,5,5) -> Tanh -> SpatialMaxPooling(2,2,2,2)
//   -> Reshape(400) -> Linear(400,10) -> logSoftMax, loss = logMultinomialLoss
// at a per-node batch of 1 (mnist.lua:33).  The model is 10,842 parameters and
// ~6 MFLOP per sample: every library-kernel version of the step is a chain of
// ~35 tiny launches, so the step is launch-latency bound.
// Here one workgroup owns one sample and keeps EVERYTHING in LDS -- the
// parameters (47 KB), the 16x28x28 conv1 activations, pooled maps, argmax
// indices and every backward intermediate (~135 KB of the CU's 160 KB):
// conv1 -> tanh -> pool -> conv2 -> tanh -> pool -> linear -> log-softmax ->
// NLL -> dlogits -> linear backward -> pool/tanh backward -> conv2 wgrad/dgrad
// -> pool/tanh backward -> conv1 wgrad.  Weight gradients of the B samples are
// accumulated with fp32 atomics into the (zeroed) flat gradient buffer, so the
// step is this kernel plus the fused SGD update (graph-captured by the engine).
// fp32 arithmetic throughout (the model is tiny; fp32 = the reference's
// precision).
#include "dl_common.h"
#include "dl_ops.h"

namespace dl {

namespace {

constexpr int kT = 1024;  // threads per workgroup (16 waves: 4 per SIMD hide the LDS latency)
constexpr int kNW = kT / 64;
constexpr int IMG = 32, K5 = 5, C1 = 16, H1 = 28, P1 = 14, C2 = 16, H2 = 10, P2 = 5;
constexpr int NF = C2 * P2 * P2;  // 400 features
constexpr int NC = 10;

// LDS layout (floats)
constexpr int L_X = 0;                         // 1024 input
constexpr int L_W1 = L_X + IMG * IMG;          // 400
constexpr int L_B1 = L_W1 + C1 * K5 * K5;      // 16
constexpr int L_W2 = L_B1 + C1;                // 6400
constexpr int L_B2 = L_W2 + C2 * C1 * K5 * K5; // 16
constexpr int L_WF = L_B2 + C2;                // 4000
constexpr int L_BF = L_WF + NC * NF;           // 10 (+6 pad)
constexpr int L_A1 = L_BF + 16;                // 12544 tanh(conv1), later dz1
constexpr int L_P1 = L_A1 + C1 * H1 * H1;      // 3136 pooled 1
constexpr int L_DP1 = L_P1 + C1 * P1 * P1;     // 3136 d pooled 1
constexpr int L_A2 = L_DP1 + C1 * P1 * P1;     // 1600 tanh(conv2), later dz2
constexpr int L_P2 = L_A2 + C2 * H2 * H2;      // 400 pooled 2 (features)
constexpr int L_DP2 = L_P2 + NF;               // 400 d features
constexpr int L_LG = L_DP2 + NF;               // 16 logits / dlogits
constexpr int L_RED = L_LG + 16;               // kNW x 16 wave partials
constexpr int L_END = L_RED + kNW * 16;
constexpr int L_IDX1 = L_END;                  // 3136 bytes of argmax (as floats: 784)
constexpr int L_IDX2 = L_IDX1 + C1 * P1 * P1 / 4;  // 400 bytes (100 floats)
constexpr int L_TOTAL = L_IDX2 + NF / 4;
constexpr size_t kLdsBytes = (size_t)L_TOTAL * 4;
static_assert(kLdsBytes <= 160 * 1024, "MNIST step does not fit in LDS");

// tanh(v) = 1 - 2 / (exp(2v) + 1): exact limits at +-inf, ~1 ulp-level error
// on the hardware exp (the reference's Tanh is fp32 too)
__device__ __forceinline__ float tanh_f(float v) { return 1.f - 2.f / (__expf(2.f * v) + 1.f); }

}  // namespace

// params (fp32, flat views): w1 [16][1][5][5], b1 [16], w2 [16][16][5][5], b2, wf [10][400], bf [10]
// grads: same shapes, ZEROED by the caller (the samples' contributions are atomically added)
template <bool BF16_IN>
__global__ void __launch_bounds__(kT) mnist_step_kernel(const void* __restrict__ xin, const int64_t* __restrict__ labels,
                                                        const float* __restrict__ w1, const float* __restrict__ b1,
                                                        const float* __restrict__ w2, const float* __restrict__ b2,
                                                        const float* __restrict__ wf, const float* __restrict__ bfc,
                                                        float* __restrict__ gw1, float* __restrict__ gb1,
                                                        float* __restrict__ gw2, float* __restrict__ gb2,
                                                        float* __restrict__ gwf, float* __restrict__ gbf,
                                                        float* __restrict__ logp_out, float* __restrict__ loss_b,
                                                        int B) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  float* sx = lds + L_X;
  float* sw1 = lds + L_W1;
  float* sb1 = lds + L_B1;
  float* sw2 = lds + L_W2;
  float* sb2 = lds + L_B2;
  float* swf = lds + L_WF;
  float* sbf = lds + L_BF;
  float* a1 = lds + L_A1;
  float* p1 = lds + L_P1;
  float* dp1 = lds + L_DP1;
  float* a2 = lds + L_A2;
  float* p2 = lds + L_P2;
  float* dp2 = lds + L_DP2;
  float* lg = lds + L_LG;
  float* red = lds + L_RED;
  uint8_t* idx1 = reinterpret_cast<uint8_t*>(lds + L_IDX1);
  uint8_t* idx2 = reinterpret_cast<uint8_t*>(lds + L_IDX2);

  // ---- stage the sample and the parameters ---------------------------------------
  for (int i = tid; i < IMG * IMG; i += kT) {
    if constexpr (BF16_IN)
      sx[i] = bf16_to_f32(reinterpret_cast<const bf16_t*>(xin)[(int64_t)b * IMG * IMG + i]);
    else
      sx[i] = reinterpret_cast<const float*>(xin)[(int64_t)b * IMG * IMG + i];
  }
  for (int i = tid; i < C1 * K5 * K5; i += kT) sw1[i] = w1[i];
  for (int i = tid; i < C2 * C1 * K5 * K5; i += kT) sw2[i] = w2[i];
  for (int i = tid; i < NC * NF; i += kT) swf[i] = wf[i];
  if (tid < C1) sb1[tid] = b1[tid];
  if (tid < C2) sb2[tid] = b2[tid];
  if (tid < NC) sbf[tid] = bfc[tid];
  __syncthreads();

  // ---- conv1 (valid 5x5) + tanh ----------------------------------------------------
  for (int o = tid; o < C1 * H1 * H1; o += kT) {
    const int c = o / (H1 * H1), r = o - c * H1 * H1, i = r / H1, j = r - i * H1;
    float z = sb1[c];
#pragma unroll
    for (int u = 0; u < K5; ++u)
#pragma unroll
      for (int v = 0; v < K5; ++v) z = fmaf(sw1[(c * K5 + u) * K5 + v], sx[(i + u) * IMG + j + v], z);
    a1[o] = tanh_f(z);
  }
  __syncthreads();
  // ---- pool1 (2x2/2, first max in row-major window order) ------------------------
  for (int o = tid; o < C1 * P1 * P1; o += kT) {
    const int c = o / (P1 * P1), r = o - c * P1 * P1, i = r / P1, j = r - i * P1;
    const float* base = a1 + c * H1 * H1 + 2 * i * H1 + 2 * j;
    float m = base[0];
    int k = 0;
    if (base[1] > m) { m = base[1]; k = 1; }
    if (base[H1] > m) { m = base[H1]; k = 2; }
    if (base[H1 + 1] > m) { m = base[H1 + 1]; k = 3; }
    p1[o] = m;
    idx1[o] = (uint8_t)k;
  }
  __syncthreads();
  // ---- conv2 (valid 5x5, 16 -> 16) + tanh ----------------------------------------
  for (int o = tid; o < C2 * H2 * H2; o += kT) {
    const int co = o / (H2 * H2), r = o - co * H2 * H2, i = r / H2, j = r - i * H2;
    float z = sb2[co];
    for (int ci = 0; ci < C1; ++ci) {
      const float* wp = sw2 + (co * C1 + ci) * K5 * K5;
      const float* xp = p1 + ci * P1 * P1 + i * P1 + j;
#pragma unroll
      for (int u = 0; u < K5; ++u)
#pragma unroll
        for (int v = 0; v < K5; ++v) z = fmaf(wp[u * K5 + v], xp[u * P1 + v], z);
    }
    a2[o] = tanh_f(z);
  }
  __syncthreads();
  // ---- pool2 -> 400 features (NCHW flatten order: c*25 + i*5 + j) -------------------
  for (int o = tid; o < NF; o += kT) {
    const int c = o / (P2 * P2), r = o - c * P2 * P2, i = r / P2, j = r - i * P2;
    const float* base = a2 + c * H2 * H2 + 2 * i * H2 + 2 * j;
    float m = base[0];
    int k = 0;
    if (base[1] > m) { m = base[1]; k = 1; }
    if (base[H2] > m) { m = base[H2]; k = 2; }
    if (base[H2 + 1] > m) { m = base[H2 + 1]; k = 3; }
    p2[o] = m;
    idx2[o] = (uint8_t)k;
  }
  __syncthreads();
  // ---- linear 400 -> 10 (fixed-order wave + 4-wave reduction) --------------------
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    float s = 0.f;
    for (int f = tid; f < NF; f += kT) s = fmaf(swf[k * NF + f], p2[f], s);
    s = wave_sum(s);
    if (lane == 0) red[wid * 16 + k] = s;
  }
  __syncthreads();
  if (tid == 0) {
    float z[NC], mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      float t = sbf[k];
      for (int w = 0; w < kNW; ++w) t += red[w * 16 + k];
      z[k] = t;
      mx = fmaxf(mx, z[k]);
    }
    float se = 0.f;
#pragma unroll
    for (int k = 0; k < NC; ++k) se += __expf(z[k] - mx);
    const float lse = mx + __logf(se);
    const int y = labels ? (int)labels[b] : -1;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const float lp = z[k] - lse;
      if (logp_out) logp_out[(int64_t)b * NC + k] = lp;
      lg[k] = (__expf(lp) - (k == y ? 1.f : 0.f)) / (float)B;  // dlogits of the batch-mean loss
    }
    if (loss_b) loss_b[b] = y >= 0 ? lse - z[y] : 0.f;
  }
  if (labels == nullptr) return;  // predict
  __syncthreads();

  // ================================ backward ======================================
  // linear: dWf += dl x features, dbf += dl, dfeatures = Wf^T dl
  for (int e = tid; e < NC * NF; e += kT) unsafeAtomicAdd(gwf + e, lg[e / NF] * p2[e % NF]);
  if (tid < NC) unsafeAtomicAdd(gbf + tid, lg[tid]);
  for (int f = tid; f < NF; f += kT) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NC; ++k) s = fmaf(swf[k * NF + f], lg[k], s);
    dp2[f] = s;
  }
  __syncthreads();
  // pool2 / tanh backward: dz2 = (routed dp2) * (1 - a2^2), in place of a2
  for (int o = tid; o < C2 * H2 * H2; o += kT) {
    const int c = o / (H2 * H2), r = o - c * H2 * H2, i = r / H2, j = r - i * H2;
    const int q = c * P2 * P2 + (i >> 1) * P2 + (j >> 1);
    const int pos = ((i & 1) << 1) | (j & 1);
    const float g = (idx2[q] == pos) ? dp2[q] : 0.f;
    const float t = a2[o];
    a2[o] = g * (1.f - t * t);
  }
  __syncthreads();
  float* dz2 = a2;
  // conv2 wgrad: dW2[co][ci][u][v] += sum_{i,j} dz2[co][i][j] p1[ci][i+u][j+v]; db2
  for (int e = tid; e < C2 * C1 * K5 * K5; e += kT) {
    const int co = e / (C1 * K5 * K5), r = e - co * C1 * K5 * K5, ci = r / (K5 * K5), t = r - ci * K5 * K5;
    const int u = t / K5, v = t - u * K5;
    const float* g = dz2 + co * H2 * H2;
    const float* xp = p1 + ci * P1 * P1 + u * P1 + v;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < H2; ++i)
#pragma unroll
      for (int j = 0; j < H2; ++j) s = fmaf(g[i * H2 + j], xp[i * P1 + j], s);
    unsafeAtomicAdd(gw2 + e, s);
  }
  if (tid < C2) {
    float s = 0.f;
    for (int i = 0; i < H2 * H2; ++i) s += dz2[tid * H2 * H2 + i];
    unsafeAtomicAdd(gb2 + tid, s);
  }
  // conv2 dgrad: dp1[ci][y][x] = sum_{co,u,v} W2[co][ci][u][v] dz2[co][y-u][x-v]
  for (int o = tid; o < C1 * P1 * P1; o += kT) {
    const int ci = o / (P1 * P1), r = o - ci * P1 * P1, y = r / P1, x = r - y * P1;
    float s = 0.f;
    for (int co = 0; co < C2; ++co) {
      const float* wp = sw2 + (co * C1 + ci) * K5 * K5;
      const float* g = dz2 + co * H2 * H2;
#pragma unroll
      for (int u = 0; u < K5; ++u) {
        const int i = y - u;
        if (i < 0 || i >= H2) continue;
#pragma unroll
        for (int v = 0; v < K5; ++v) {
          const int j = x - v;
          if (j >= 0 && j < H2) s = fmaf(wp[u * K5 + v], g[i * H2 + j], s);
        }
      }
    }
    dp1[o] = s;
  }
  __syncthreads();
  // pool1 / tanh backward: dz1 in place of a1
  for (int o = tid; o < C1 * H1 * H1; o += kT) {
    const int c = o / (H1 * H1), r = o - c * H1 * H1, i = r / H1, j = r - i * H1;
    const int q = c * P1 * P1 + (i >> 1) * P1 + (j >> 1);
    const int pos = ((i & 1) << 1) | (j & 1);
    const float g = (idx1[q] == pos) ? dp1[q] : 0.f;
    const float t = a1[o];
    a1[o] = g * (1.f - t * t);
  }
  __syncthreads();
  float* dz1 = a1;
  // conv1 wgrad: dW1[c][u][v] += sum_{i,j} dz1[c][i][j] x[i+u][j+v]  (4 partial sums per output)
  for (int e = tid; e < 4 * C1 * K5 * K5; e += kT) {
    const int part = e & 3, w = e >> 2;
    const int c = w / (K5 * K5), t = w - c * K5 * K5, u = t / K5, v = t - u * K5;
    const float* g = dz1 + c * H1 * H1;
    float s = 0.f;
    for (int i = part; i < H1; i += 4)
#pragma unroll 4
      for (int j = 0; j < H1; ++j) s = fmaf(g[i * H1 + j], sx[(i + u) * IMG + j + v], s);
    unsafeAtomicAdd(gw1 + w, s);
  }
  if (tid < C1 * 4) {
    const int c = tid >> 2, part = tid & 3;
    float s = 0.f;
    for (int i = part; i < H1 * H1; i += 4) s += dz1[c * H1 * H1 + i];
    unsafeAtomicAdd(gb1 + c, s);
  }
}

void mnist_step(uintptr_t x, int x_bf16, uintptr_t labels, uintptr_t w1, uintptr_t b1, uintptr_t w2, uintptr_t b2,
                uintptr_t wf, uintptr_t bf, uintptr_t gw1, uintptr_t gb1, uintptr_t gw2, uintptr_t gb2, uintptr_t gwf,
                uintptr_t gbf, uintptr_t logp, uintptr_t loss_b, int B, uintptr_t stream) {
  if (B <= 0) return;
  auto go = [&](auto kern) {
    static bool attr = false;
    if (!attr) {
      DL_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsBytes));
      attr = true;
    }
    kern<<<B, kT, kLdsBytes, as_stream(stream)>>>(
        (const void*)x, (const int64_t*)labels, (const float*)w1, (const float*)b1, (const float*)w2, (const float*)b2,
        (const float*)wf, (const float*)bf, (float*)gw1, (float*)gb1, (float*)gw2, (float*)gb2, (float*)gwf,
        (float*)gbf, (float*)logp, (float*)loss_b, B);
  };
  if (x_bf16) go(mnist_step_kernel<true>);
  else go(mnist_step_kernel<false>);
  DL_HIP_CHECK(hipGetLastError());
}

}  // namespace dl
