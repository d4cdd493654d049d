// Metrics + input-pipeline kernels (gfx950).
//
//  * K12 confusion-matrix accumulate: argmax(pred) -> histogram [C x C]
//    (reference: confusionMatrix:add(prediction[b], y[b]) per sample,
//     examples/cifar10.lua:194-196, examples/mnist.lua:119). One wave per
//    sample row, argmax by wave reduction, one 64-bit atomic per sample.
//  * batch gather: uint8 NHWC images selected by a sampler index list ->
//    normalised bf16 NHWC mini-batch (replaces the torch-dataset worker
//    threads + input:copy(res) of examples/cifar10.lua:53-71).
#include "dl_common.h"

namespace dl {

// pred: [B, C] (bf16 or f32), target: int64 [B] (0-based), mat: int64 [C, C]
// row = target, col = predicted (optim.ConfusionMatrix convention).
template <typename T>
__global__ void __launch_bounds__(256) confusion_kernel(const T* __restrict__ pred, const int64_t* __restrict__ target,
                                                        unsigned long long* __restrict__ mat, int B, int C) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (row >= B) return;
  float best = -INFINITY;
  int arg = 0x7fffffff;
  for (int c = lane; c < C; c += 64) {
    float v;
    if constexpr (sizeof(T) == 2) v = bf16_to_f32(((const bf16_t*)pred)[(int64_t)row * C + c]);
    else v = ((const float*)pred)[(int64_t)row * C + c];
    if (v > best) { best = v; arg = c; }
  }
  // wave argmax: larger value wins, ties -> smaller index (torch/Lua max semantics)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float ob = __shfl_xor(best, o, 64);
    int oa = __shfl_xor(arg, o, 64);
    if (ob > best || (ob == best && oa < arg)) { best = ob; arg = oa; }
  }
  if (lane == 0) {
    int64_t t = target[row];
    if (t >= 0 && t < C && arg < C) atomicAdd(&mat[t * C + arg], 1ull);
  }
}

void confusion_update(uintptr_t pred, int pred_is_bf16, uintptr_t target, uintptr_t mat, int B, int C,
                      uintptr_t stream) {
  if (B <= 0) return;
  dim3 grid((B + 3) / 4), block(256);
  if (pred_is_bf16)
    confusion_kernel<bf16_t><<<grid, block, 0, as_stream(stream)>>>((const bf16_t*)pred, (const int64_t*)target,
                                                                     (unsigned long long*)mat, B, C);
  else
    confusion_kernel<float><<<grid, block, 0, as_stream(stream)>>>((const float*)pred, (const int64_t*)target,
                                                                    (unsigned long long*)mat, B, C);
  DL_HIP_CHECK(hipGetLastError());
}

// images: uint8 [N, H, W, Cs] (Cs source channels), idx: int64 [B]
// out: bf16 [B, H, W, Cd] with Cd >= Cs (extra channels zero-padded),
// out = (x/255 - mean[c]) / std[c].  One thread per output pixel-channel group.
__global__ void __launch_bounds__(256) gather_normalize_kernel(const uint8_t* __restrict__ images,
                                                               const int64_t* __restrict__ idx,
                                                               bf16_t* __restrict__ out, int B, int HW, int Cs, int Cd,
                                                               float m0, float m1, float m2, float s0, float s1,
                                                               float s2) {
  const int64_t total = (int64_t)B * HW;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int b = (int)(t / HW);
    const int p = (int)(t - (int64_t)b * HW);
    const int64_t src = (idx[b] * HW + p) * Cs;
    bf16_t* o = out + t * Cd;
    for (int c = 0; c < Cd; ++c) {
      float v = 0.f;
      if (c < Cs) {
        float x = images[src + c] * (1.0f / 255.0f);
        float m = c == 0 ? m0 : (c == 1 ? m1 : m2);
        float s = c == 0 ? s0 : (c == 1 ? s1 : s2);
        v = (x - m) / s;
      }
      o[c] = f32_to_bf16(v);
    }
  }
}

void gather_normalize(uintptr_t images, uintptr_t idx, uintptr_t out, int B, int HW, int Cs, int Cd, float m0,
                      float m1, float m2, float s0, float s1, float s2, uintptr_t stream) {
  int64_t total = (int64_t)B * HW;
  if (total == 0) return;
  gather_normalize_kernel<<<stream_grid(total), 256, 0, as_stream(stream)>>>(
      (const uint8_t*)images, (const int64_t*)idx, (bf16_t*)out, B, HW, Cs, Cd, m0, m1, m2, s0, s1, s2);
  DL_HIP_CHECK(hipGetLastError());
}

}  // namespace dl
