// Common device/host helpers for the distlearn MI355X (gfx950) native library.
//
// Everything in csrc/ is written for CDNA4 directly: 64-lane wavefronts,
// 16-byte vector memory accesses, bf16 stored as raw 16-bit words.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdexcept>
#include <string>

#define DL_HIP_CHECK(expr)                                                          \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    if (_e != hipSuccess) {                                                         \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + \
                               " at " + __FILE__ + ":" + std::to_string(__LINE__)); \
    }                                                                               \
  } while (0)

namespace dl {

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

typedef uint16_t bf16_t;  // raw bf16 bits

using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x16 = __attribute__((ext_vector_type(16))) float;
using bf16x8 = __attribute__((ext_vector_type(8))) short;   // MFMA A/B fragment (4 VGPRs)
using bf16x4 = __attribute__((ext_vector_type(4))) short;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;
using u32x2 = __attribute__((ext_vector_type(2))) unsigned int;

__device__ __forceinline__ float bf16_to_f32(bf16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}

// Round-to-nearest-even, NaN preserving (hipcc lowers the __bf16 cast to
// v_cvt_pk_bf16_f32 on gfx950).
__device__ __forceinline__ bf16_t f32_to_bf16(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
}

__device__ __forceinline__ float lo_bf16(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi_bf16(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// First-layer packed weight index of element e of a [Cout][taps][C] weight.
// cp > 0: channel-padded [Cout][taps][cp].  cp = -KW (square KW x KW kernel,
// C <= 4): two horizontally adjacent taps per 16-byte chunk,
// [Cout][KW][ceil(KW/2)][2][4] -- the layout of the pair-packed first-layer
// forward (conv_fwd_c8_kernel<.., PAIR>); pads are never written.
__device__ __forceinline__ int64_t pack1_index(int64_t e, int C, int cp) {
  const int64_t px = e / C;
  const int c = (int)(e - px * C);
  if (cp > 0) return px * cp + c;
  const int kw = -cp, taps = kw * kw, cpr = (kw + 1) >> 1;
  const int64_t co = px / taps;
  const int tap = (int)(px - co * taps), kh = tap / kw, kx = tap - kh * kw;
  return ((co * kw + kh) * cpr + (kx >> 1)) * 8 + (kx & 1) * 4 + c;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Grid size for a grid-stride streaming kernel over `n_vec` vector items:
// enough blocks to fill 256 CUs x 8 blocks, never more work-items than items.
inline int stream_grid(int64_t n_vec, int block = 256) {
  int64_t g = (n_vec + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

inline hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace dl
