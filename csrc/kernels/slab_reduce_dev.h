// Split-K weight-gradient slab reduction body, shared by the stand-alone
// slab_reduce kernel (conv_igemm.hip) and the combined launch that runs it
// beside the previous layer's BatchNorm backward reduce (bn_pool.hip).
//   dst[co][tap][c] (= / +=) sum_sp slabs[sp][co][tap][c'], c < C <= Cp
// TPO lanes share one output (each sums a strided subset of the splits, then
// a fixed-order shuffle reduction): enough parallelism for 64-way slabs.
// ACC: dst += sum (gradient accumulation semantics) instead of dst = sum.
// OIHW: dst in [Cout][C][taps] order (a PyTorch conv weight) instead of [Cout][taps][C].
#pragma once
#include "dl_common.h"

namespace dl {

// The reduction itself: f(i, rest, c, s) is called by lane sub == 0 of each
// output i (rest = co*taps + tap) with its sum s.  Shared by the reduce
// kernels below and by the one-node SGD that consumes the slabs directly
// (flat_ops.hip), so both produce bitwise the same sums.
template <int TPO, class F>
__device__ __forceinline__ void slab_reduce_each(const float* __restrict__ slabs, int splits, int Cout, int taps,
                                                 int Cp, int C, int bid, int nblk, F&& f) {
  const int64_t total = (int64_t)Cout * taps * C;
  // Cp < 0: the pair-packed first layer (dl_common.h pack1_index, -Cp = kernel width)
  const int64_t slab = Cp > 0 ? (int64_t)Cout * taps * Cp : (int64_t)Cout * (-Cp) * ((1 - Cp) / 2) * 8;
  const int sub = threadIdx.x % TPO;
  const int64_t opb = 256 / TPO;  // outputs per block iteration
  for (int64_t i = (int64_t)bid * opb + threadIdx.x / TPO; i < total; i += (int64_t)nblk * opb) {
    const int c = (int)(i % C);
    const int64_t rest = i / C;  // co*taps + tap
    const int64_t src = Cp > 0 ? rest * Cp + c : pack1_index(i, C, Cp);
    // splits in batches of 4 loads in flight before the adds (a load->add chain
    // per split was latency-bound); the adds keep the split order
    float s = 0.f;
    int sp = sub;
    for (; sp + 3 * TPO < splits; sp += 4 * TPO) {
      float a[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] = slabs[(int64_t)(sp + u * TPO) * slab + src];
#pragma unroll
      for (int u = 0; u < 4; ++u) s += a[u];
    }
    for (; sp < splits; sp += TPO) s += slabs[(int64_t)sp * slab + src];
#pragma unroll
    for (int o = TPO / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (sub == 0) f(i, rest, c, s);
  }
}

template <int TPO, bool ACC = false, bool OIHW = false>
__device__ __forceinline__ void slab_reduce_body(const float* __restrict__ slabs, float* __restrict__ dst, int splits,
                                                 int Cout, int taps, int Cp, int C, int bid, int nblk) {
  slab_reduce_each<TPO>(slabs, splits, Cout, taps, Cp, C, bid, nblk, [&](int64_t i, int64_t rest, int c, float s) {
    int64_t o = i;
    if constexpr (OIHW) {
      const int64_t co = rest / taps;
      o = (co * C + c) * taps + (rest - co * taps);
    }
    dst[o] = ACC ? dst[o] + s : s;
  });
}

// Threads per output and grid of a slab reduction (the stand-alone launcher's rule).
inline int slab_reduce_tpo(int splits) { return splits >= 32 ? 32 : splits >= 8 ? 8 : 1; }
inline int slab_reduce_grid(int splits, int Cout, int taps, int C) {
  const int64_t total = (int64_t)Cout * taps * C;
  const int tpo = slab_reduce_tpo(splits);
  if (tpo == 1) return stream_grid(total);
  return (int)std::min<int64_t>((total * tpo + 255) / 256, 4096);
}

}  // namespace dl
