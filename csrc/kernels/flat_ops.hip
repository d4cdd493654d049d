// Flat-bucket optimizer / elastic-averaging / participation kernels (gfx950).
//
// These are the per-step hot path of the reference's algorithms, done over ONE
// persistent flat fp32 buffer instead of a walkTable loop of per-tensor ops:
//   * K3  grad:mul(1/n)                      lua/AllReduceSGD.lua:23-27
//   * K5  params:add(-lr, grads)             examples/cifar10.lua:187-191
//   * K8  delta=alpha(p-c); p-=delta         lua/AllReduceEA.lua:35-39
//   * K9  center += sum(delta)               lua/AllReduceEA.lua:43-45
//   * K10 fused drain step                   lua/AllReduceEA.lua:60-68
//   * K4/K11 fill / copy                     lua/AllReduceSGD.lua:37,44
// All kernels are grid-stride streaming kernels with 16-byte (float4) accesses;
// the participation count `n` is read on the device from the all-reduced slot,
// so the normalisation needs no host synchronisation (graph-capturable).
#include <vector>

#include "dl_common.h"
#include "slab_reduce_dev.h"

namespace dl {

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ float participation_scale(const float* slot) {
  if (slot == nullptr) return 1.0f;
  float n = *slot;
  return n > 1.0f ? 1.0f / n : 1.0f;  // reference: only divide when n > 1
}

// ---------------------------------------------------------------------------
// SGD (+ optional momentum / weight decay), fused with 1/n normalisation and
// the bf16 shadow-weight refresh used by the bf16 compute path.
// ---------------------------------------------------------------------------
// G16: the gradient is the bf16 all-reduced wire copy (grad_comm_dtype="bf16":
// half the xGMI bytes; read here directly, never widened back to fp32).
__device__ __forceinline__ float4 load_grad4(const float* g, int64_t i) {
  return reinterpret_cast<const float4*>(g)[i];
}
__device__ __forceinline__ float4 load_grad4(const bf16_t* g, int64_t i) {
  const uint2 u = reinterpret_cast<const uint2*>(g)[i];
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xffff0000u));
}

// One element of the fused update, with every rounding step explicit (fma
// contraction left to the compiler differs between the float4 and the scalar
// code paths; the slab-consuming update must match this kernel bit for bit).
template <bool kMomentum>
__device__ __forceinline__ float sgd_elem(float p, float g, float* m, float s, float wd, float lr, float momentum) {
  float gx = __builtin_fmaf(g, s, wd * p);
  if constexpr (kMomentum) {
    const float mv = __builtin_fmaf(momentum, *m, gx);
    *m = mv;
    gx = mv;
  }
  return __builtin_fmaf(-lr, gx, p);
}

template <bool kMomentum>
__device__ __forceinline__ float4 sgd_elem4(float4 p, const float4 g, float4& m, float s, float wd, float lr,
                                            float momentum) {
  p.x = sgd_elem<kMomentum>(p.x, g.x, &m.x, s, wd, lr, momentum);
  p.y = sgd_elem<kMomentum>(p.y, g.y, &m.y, s, wd, lr, momentum);
  p.z = sgd_elem<kMomentum>(p.z, g.z, &m.z, s, wd, lr, momentum);
  p.w = sgd_elem<kMomentum>(p.w, g.w, &m.w, s, wd, lr, momentum);
  return p;
}

template <bool kMomentum, bool kShadow, typename GT = float>
__global__ void __launch_bounds__(256) sgd_kernel(float* __restrict__ p, const GT* __restrict__ g,
                                                  float* __restrict__ mom, bf16_t* __restrict__ p16,
                                                  const float* __restrict__ slot, float lr, float momentum,
                                                  float wd, int64_t n4) {
  const float s = participation_scale(slot);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  auto update = [&](int64_t i, float4 pv, const float4 gv, float4 mv) {
    pv = sgd_elem4<kMomentum>(pv, gv, mv, s, wd, lr, momentum);
    if constexpr (kMomentum) reinterpret_cast<float4*>(mom)[i] = mv;
    reinterpret_cast<float4*>(p)[i] = pv;
    if constexpr (kShadow) {
      uint2 packed;
      packed.x = pack_bf16x2(pv.x, pv.y);
      packed.y = pack_bf16x2(pv.z, pv.w);
      reinterpret_cast<uint2*>(p16)[i] = packed;
    }
  };
  // two items per thread per trip, every load of both issued before the first
  // update (one memory round trip per trip instead of one per item: the
  // 2048-block grid gives ~2 items per thread on the CIFAR flat buffer)
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += 2 * stride) {
    const int64_t j = i + stride;
    const bool two = j < n4;
    const float4 pa = reinterpret_cast<const float4*>(p)[i];
    const float4 ga = load_grad4(g, i);
    float4 ma = z4, pb = z4, gb = z4, mb = z4;
    if constexpr (kMomentum) ma = reinterpret_cast<const float4*>(mom)[i];
    if (two) {
      pb = reinterpret_cast<const float4*>(p)[j];
      gb = load_grad4(g, j);
      if constexpr (kMomentum) mb = reinterpret_cast<const float4*>(mom)[j];
    }
    update(i, pa, ga, ma);
    if (two) update(j, pb, gb, mb);
  }
}

// ---------------------------------------------------------------------------
// SGD whose gradient for some ranges still lies in split-K weight-gradient
// slabs (one GPU, nothing to all-reduce: the conv executor skips the slab
// reduce launches and the update sums the slabs itself).  The sum per element
// is bitwise the one slab_reduce_body<TPO> computes (slab_reduce_dev.h):
// TPO lanes each add a strided subset of the splits in split order, then a
// xor-shuffle tree -- so deferring the reduce changes no bit of the update.
// ---------------------------------------------------------------------------
constexpr int kSlabRanges = 4;
constexpr int kSlabMaxSplits = 31;  // the stand-alone reduce uses 1 or 8 lanes per output up to here
struct SlabRanges {
  int n;
  int64_t lo4[kSlabRanges], hi4[kSlabRanges];  // float4 index range in the updated buffer
  const float* slab[kSlabRanges];               // [splits][len] fp32, len = (hi4 - lo4) * 4
  int64_t stride4[kSlabRanges];                 // float4s per split
  int splits[kSlabRanges], tpo[kSlabRanges];
  // one "tail" range whose slabs are channel-padded (Cp > C) or have >= 32
  // splits (the first conv layer: 3 -> 8 channels, 128 splits): reduced by
  // extra blocks of the same launch with the stand-alone reduce's lane split
  // (slab_reduce_each) and updated element by element
  int tail_nblk;  // 0: none
  int64_t tail_lo, tail_lo4, tail_hi4;  // element offset; float4 range the main blocks skip
  const float* tail_slab;
  int tail_splits, tail_cout, tail_taps, tail_cp, tail_c, tail_tpo;
};

template <int TPO>
__device__ __forceinline__ void add4(float4 (&part)[TPO], int t, const float4& v) {
  // t is a compile-time constant after unrolling (no dynamic register indexing)
  float4& q = part[t];
  q.x += v.x; q.y += v.y; q.z += v.z; q.w += v.w;
}

template <int TPO>
__device__ __forceinline__ float4 slab_sum4(const float4* __restrict__ s, int64_t stride4, int splits) {
  float4 part[TPO];
#pragma unroll
  for (int t = 0; t < TPO; ++t) part[t] = make_float4(0.f, 0.f, 0.f, 0.f);
  // chunks of 4 splits, the chunk's loads in flight before its adds; lane t of
  // the stand-alone reduce adds splits t, t+TPO, ... in order: same here
  for (int sp0 = 0; sp0 < splits; sp0 += 4) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (sp0 + u < splits) v[u] = s[(int64_t)(sp0 + u) * stride4];
    const bool hi = TPO == 8 && (sp0 & 4);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (sp0 + u >= splits) break;
      if constexpr (TPO == 1) add4<TPO>(part, 0, v[u]);
      else if (hi) add4<TPO>(part, 4 + u, v[u]);
      else add4<TPO>(part, u, v[u]);
    }
  }
#pragma unroll
  for (int o = TPO / 2; o > 0; o >>= 1) {
    float4 np[TPO];
#pragma unroll
    for (int t = 0; t < TPO; ++t) {
      const float4 a = part[t], b = part[t ^ o];
      np[t] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
    }
#pragma unroll
    for (int t = 0; t < TPO; ++t) part[t] = np[t];
  }
  return part[0];
}

__device__ __forceinline__ float4 grad4_or_slabs(const float* __restrict__ g, const SlabRanges& r, int64_t i) {
  for (int k = 0; k < r.n; ++k) {
    if (i >= r.lo4[k] && i < r.hi4[k]) {
      const float4* s = reinterpret_cast<const float4*>(r.slab[k]) + (i - r.lo4[k]);
      return r.tpo[k] == 8 ? slab_sum4<8>(s, r.stride4[k], r.splits[k]) : slab_sum4<1>(s, r.stride4[k], r.splits[k]);
    }
  }
  return load_grad4(g, i);
}

template <bool kMomentum, bool kShadow>
__global__ void __launch_bounds__(256) sgd_slabs_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                        float* __restrict__ mom, bf16_t* __restrict__ p16,
                                                        const float* __restrict__ slot, float lr, float momentum,
                                                        float wd, int64_t n4, const SlabRanges r) {
  const float s = participation_scale(slot);
  const int nmain = (int)gridDim.x - r.tail_nblk;
  if ((int)blockIdx.x >= nmain) {
    auto upd = [&](int64_t i, int64_t, int, float gs) {
      const int64_t e = r.tail_lo + i;  // KRSC weight: element i of the reduce's output order
      float mv = kMomentum ? mom[e] : 0.f;
      const float pv = sgd_elem<kMomentum>(p[e], gs, &mv, s, wd, lr, momentum);
      if constexpr (kMomentum) mom[e] = mv;
      p[e] = pv;
      if constexpr (kShadow) p16[e] = f32_to_bf16(pv);
    };
    const int bid = (int)blockIdx.x - nmain;
    if (r.tail_tpo == 32)
      slab_reduce_each<32>(r.tail_slab, r.tail_splits, r.tail_cout, r.tail_taps, r.tail_cp, r.tail_c, bid,
                           r.tail_nblk, upd);
    else if (r.tail_tpo == 8)
      slab_reduce_each<8>(r.tail_slab, r.tail_splits, r.tail_cout, r.tail_taps, r.tail_cp, r.tail_c, bid,
                          r.tail_nblk, upd);
    else
      slab_reduce_each<1>(r.tail_slab, r.tail_splits, r.tail_cout, r.tail_taps, r.tail_cp, r.tail_c, bid,
                          r.tail_nblk, upd);
    return;
  }
  const int64_t stride = (int64_t)nmain * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    if (i >= r.tail_lo4 && i < r.tail_hi4) continue;  // the tail blocks update these
    float4 pv = reinterpret_cast<const float4*>(p)[i];
    const float4 gv = grad4_or_slabs(g, r, i);
    float4 mv = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (kMomentum) mv = reinterpret_cast<const float4*>(mom)[i];
    pv = sgd_elem4<kMomentum>(pv, gv, mv, s, wd, lr, momentum);
    if constexpr (kMomentum) reinterpret_cast<float4*>(mom)[i] = mv;
    reinterpret_cast<float4*>(p)[i] = pv;
    if constexpr (kShadow) {
      uint2 packed;
      packed.x = pack_bf16x2(pv.x, pv.y);
      packed.y = pack_bf16x2(pv.z, pv.w);
      reinterpret_cast<uint2*>(p16)[i] = packed;
    }
  }
}

// x *= 1/n (n read from the all-reduced participation slot)
__global__ void __launch_bounds__(256) scale_by_count_kernel(float* __restrict__ x, const float* __restrict__ slot,
                                                             int64_t n4) {
  const float s = participation_scale(slot);
  if (s == 1.0f) return;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = reinterpret_cast<float4*>(x)[i];
    v.x *= s; v.y *= s; v.z *= s; v.w *= s;
    reinterpret_cast<float4*>(x)[i] = v;
  }
}

// Elastic step. If `pending` is non-null, first c += pending (the previous
// round's all-reduced sum of deltas: K9 fused into K8 = K10).
//   delta = alpha * (p - c);  p -= delta;  out = delta
template <bool kPending, bool kShadow>
__global__ void __launch_bounds__(256) elastic_kernel(float* __restrict__ p, float* __restrict__ c,
                                                      const float* __restrict__ pending, float* __restrict__ out,
                                                      bf16_t* __restrict__ p16, float alpha, int64_t n4) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pv = reinterpret_cast<float4*>(p)[i];
    float4 cv = reinterpret_cast<float4*>(c)[i];
    if constexpr (kPending) {
      float4 dv = reinterpret_cast<const float4*>(pending)[i];
      cv.x += dv.x; cv.y += dv.y; cv.z += dv.z; cv.w += dv.w;
      reinterpret_cast<float4*>(c)[i] = cv;
    }
    float4 d;
    d.x = alpha * (pv.x - cv.x); d.y = alpha * (pv.y - cv.y);
    d.z = alpha * (pv.z - cv.z); d.w = alpha * (pv.w - cv.w);
    pv.x -= d.x; pv.y -= d.y; pv.z -= d.z; pv.w -= d.w;
    reinterpret_cast<float4*>(p)[i] = pv;
    reinterpret_cast<float4*>(out)[i] = d;
    if constexpr (kShadow) {
      uint2 packed;
      packed.x = pack_bf16x2(pv.x, pv.y);
      packed.y = pack_bf16x2(pv.z, pv.w);
      reinterpret_cast<uint2*>(p16)[i] = packed;
    }
  }
}

// y += x
__global__ void __launch_bounds__(256) add_inplace_kernel(float* __restrict__ y, const float* __restrict__ x, int64_t n4) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 a = reinterpret_cast<float4*>(y)[i];
    float4 b = reinterpret_cast<const float4*>(x)[i];
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    reinterpret_cast<float4*>(y)[i] = a;
  }
}

// x[0:n] = v, and x[slot_index] = slot_value (slot_index < 0: none)
__global__ void __launch_bounds__(256) fill_kernel(float* __restrict__ x, float v, int64_t n4, int64_t slot_index,
                                                   float slot_value) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const float4 fv = make_float4(v, v, v, v);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 w = fv;
    if (slot_index >= 0 && (slot_index >> 2) == i) {
      switch (slot_index & 3) {
        case 0: w.x = slot_value; break;
        case 1: w.y = slot_value; break;
        case 2: w.z = slot_value; break;
        default: w.w = slot_value; break;
      }
    }
    reinterpret_cast<float4*>(x)[i] = w;
  }
}

__global__ void __launch_bounds__(256) cast_f32_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y,
                                                            int64_t n4) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = reinterpret_cast<const float4*>(x)[i];
    uint2 packed;
    packed.x = pack_bf16x2(v.x, v.y);
    packed.y = pack_bf16x2(v.z, v.w);
    reinterpret_cast<uint2*>(y)[i] = packed;
  }
}

// bf16 -> fp32 (the all-reduced bf16 wire copy back into the fp32 gradient)
__global__ void __launch_bounds__(256) cast_bf16_f32_kernel(const bf16_t* __restrict__ x, float* __restrict__ y,
                                                            int64_t n4) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride)
    reinterpret_cast<float4*>(y)[i] = load_grad4(x, i);
}

// ---------------------------------------------------------------------------
// Host launchers (C ABI-ish, raw pointers + stream handle)
// ---------------------------------------------------------------------------
static void check_vec4(int64_t n, const char* what) {
  if (n % 4 != 0) throw std::runtime_error(std::string(what) + ": element count must be a multiple of 4");
}

void sgd_update(uintptr_t p, uintptr_t g, uintptr_t mom, uintptr_t p16, uintptr_t slot, float lr, float momentum,
                float wd, int64_t n, uintptr_t stream) {
  check_vec4(n, "sgd_update");
  const int64_t n4 = n / 4;
  if (n4 == 0) return;
  dim3 grid(stream_grid(n4)), block(256);
  auto s = as_stream(stream);
  float* P = (float*)p; const float* G = (const float*)g; float* M = (float*)mom; bf16_t* P16 = (bf16_t*)p16;
  const float* S = (const float*)slot;
  if (mom && p16) sgd_kernel<true, true><<<grid, block, 0, s>>>(P, G, M, P16, S, lr, momentum, wd, n4);
  else if (mom) sgd_kernel<true, false><<<grid, block, 0, s>>>(P, G, M, P16, S, lr, momentum, wd, n4);
  else if (p16) sgd_kernel<false, true><<<grid, block, 0, s>>>(P, G, M, P16, S, lr, momentum, wd, n4);
  else sgd_kernel<false, false><<<grid, block, 0, s>>>(P, G, M, P16, S, lr, momentum, wd, n4);
  DL_HIP_CHECK(hipGetLastError());
}

void sgd_update_slabs(uintptr_t p, uintptr_t g, uintptr_t mom, uintptr_t p16, uintptr_t slot, float lr,
                      float momentum, float wd, int64_t n, std::vector<int64_t> offs, std::vector<int64_t> lens,
                      std::vector<uintptr_t> slabs, std::vector<int> splits, std::vector<int64_t> tail,
                      uintptr_t tail_slab, uintptr_t stream) {
  check_vec4(n, "sgd_update_slabs");
  const size_t k = offs.size();
  if (k > (size_t)kSlabRanges || lens.size() != k || slabs.size() != k || splits.size() != k)
    throw std::runtime_error("sgd_update_slabs: up to 4 consistent slab ranges");
  SlabRanges r{};
  r.n = (int)k;
  for (size_t j = 0; j < k; ++j) {
    if (offs[j] % 4 || lens[j] % 4 || offs[j] < 0 || offs[j] + lens[j] > n || slabs[j] % 16)
      throw std::runtime_error("sgd_update_slabs: ranges must be 16-byte aligned and inside the buffer");
    if (splits[j] < 1 || splits[j] > kSlabMaxSplits)
      throw std::runtime_error("sgd_update_slabs: 1..31 splits per range");
    if (j > 0 && offs[j] < offs[j - 1] + lens[j - 1]) throw std::runtime_error("sgd_update_slabs: ranges overlap");
    r.lo4[j] = offs[j] / 4;
    r.hi4[j] = (offs[j] + lens[j]) / 4;
    r.slab[j] = (const float*)slabs[j];
    r.stride4[j] = lens[j] / 4;
    r.splits[j] = splits[j];
    r.tpo[j] = slab_reduce_tpo(splits[j]) == 1 ? 1 : 8;  // the stand-alone slab_reduce's lane split
  }
  // tail = {offset, numel, splits, Cout, taps, Cp, C} or empty
  r.tail_lo4 = r.tail_hi4 = -1;
  if (!tail.empty()) {
    if (tail.size() != 7) throw std::runtime_error("sgd_update_slabs: tail = (offset, numel, splits, Cout, taps, Cp, C)");
    const int64_t off = tail[0], len = tail[1];
    r.tail_splits = (int)tail[2]; r.tail_cout = (int)tail[3]; r.tail_taps = (int)tail[4];
    r.tail_cp = (int)tail[5]; r.tail_c = (int)tail[6];
    if (off % 4 || len % 4 || off < 0 || off + len > n || len != (int64_t)r.tail_cout * r.tail_taps * r.tail_c ||
        r.tail_c > r.tail_cp || r.tail_splits < 1 || tail_slab == 0)
      throw std::runtime_error("sgd_update_slabs: inconsistent tail range");
    for (size_t j = 0; j < k; ++j)
      if (offs[j] < off + len && off < offs[j] + lens[j]) throw std::runtime_error("sgd_update_slabs: tail overlaps");
    r.tail_lo = off;
    r.tail_lo4 = off / 4;
    r.tail_hi4 = (off + len) / 4;
    r.tail_slab = (const float*)tail_slab;
    r.tail_tpo = slab_reduce_tpo(r.tail_splits);
    r.tail_nblk = slab_reduce_grid(r.tail_splits, r.tail_cout, r.tail_taps, r.tail_c);
  }
  const int64_t n4 = n / 4;
  if (n4 == 0) return;
  dim3 grid(stream_grid(n4) + r.tail_nblk), block(256);
  auto s = as_stream(stream);
  float* P = (float*)p; const float* G = (const float*)g; float* M = (float*)mom; bf16_t* P16 = (bf16_t*)p16;
  const float* S = (const float*)slot;
  if (mom && p16) sgd_slabs_kernel<true, true><<<grid, block, 0, s>>>(P, G, M, P16, S, lr, momentum, wd, n4, r);
  else if (mom) sgd_slabs_kernel<true, false><<<grid, block, 0, s>>>(P, G, M, P16, S, lr, momentum, wd, n4, r);
  else if (p16) sgd_slabs_kernel<false, true><<<grid, block, 0, s>>>(P, G, M, P16, S, lr, momentum, wd, n4, r);
  else sgd_slabs_kernel<false, false><<<grid, block, 0, s>>>(P, G, M, P16, S, lr, momentum, wd, n4, r);
  DL_HIP_CHECK(hipGetLastError());
}

void sgd_update_g16(uintptr_t p, uintptr_t g16, uintptr_t mom, uintptr_t p16, uintptr_t slot, float lr,
                    float momentum, float wd, int64_t n, uintptr_t stream) {
  check_vec4(n, "sgd_update_g16");
  const int64_t n4 = n / 4;
  if (n4 == 0) return;
  dim3 grid(stream_grid(n4)), block(256);
  auto s = as_stream(stream);
  float* P = (float*)p; const bf16_t* G = (const bf16_t*)g16; float* M = (float*)mom; bf16_t* P16 = (bf16_t*)p16;
  const float* S = (const float*)slot;
  if (mom && p16) sgd_kernel<true, true, bf16_t><<<grid, block, 0, s>>>(P, G, M, P16, S, lr, momentum, wd, n4);
  else if (mom) sgd_kernel<true, false, bf16_t><<<grid, block, 0, s>>>(P, G, M, P16, S, lr, momentum, wd, n4);
  else if (p16) sgd_kernel<false, true, bf16_t><<<grid, block, 0, s>>>(P, G, M, P16, S, lr, momentum, wd, n4);
  else sgd_kernel<false, false, bf16_t><<<grid, block, 0, s>>>(P, G, M, P16, S, lr, momentum, wd, n4);
  DL_HIP_CHECK(hipGetLastError());
}

void cast_bf16_f32(uintptr_t x, uintptr_t y, int64_t n, uintptr_t stream) {
  check_vec4(n, "cast_bf16_f32");
  const int64_t n4 = n / 4;
  if (n4 == 0) return;
  cast_bf16_f32_kernel<<<stream_grid(n4), 256, 0, as_stream(stream)>>>((const bf16_t*)x, (float*)y, n4);
  DL_HIP_CHECK(hipGetLastError());
}

void scale_by_count(uintptr_t x, uintptr_t slot, int64_t n, uintptr_t stream) {
  check_vec4(n, "scale_by_count");
  const int64_t n4 = n / 4;
  if (n4 == 0) return;
  scale_by_count_kernel<<<stream_grid(n4), 256, 0, as_stream(stream)>>>((float*)x, (const float*)slot, n4);
  DL_HIP_CHECK(hipGetLastError());
}

void elastic_step(uintptr_t p, uintptr_t c, uintptr_t pending, uintptr_t out, uintptr_t p16, float alpha, int64_t n,
                  uintptr_t stream) {
  check_vec4(n, "elastic_step");
  const int64_t n4 = n / 4;
  if (n4 == 0) return;
  dim3 grid(stream_grid(n4)), block(256);
  auto s = as_stream(stream);
  float* P = (float*)p; float* C = (float*)c; const float* D = (const float*)pending; float* O = (float*)out;
  bf16_t* P16 = (bf16_t*)p16;
  if (pending && p16) elastic_kernel<true, true><<<grid, block, 0, s>>>(P, C, D, O, P16, alpha, n4);
  else if (pending) elastic_kernel<true, false><<<grid, block, 0, s>>>(P, C, D, O, P16, alpha, n4);
  else if (p16) elastic_kernel<false, true><<<grid, block, 0, s>>>(P, C, D, O, P16, alpha, n4);
  else elastic_kernel<false, false><<<grid, block, 0, s>>>(P, C, D, O, P16, alpha, n4);
  DL_HIP_CHECK(hipGetLastError());
}

void add_inplace(uintptr_t y, uintptr_t x, int64_t n, uintptr_t stream) {
  check_vec4(n, "add_inplace");
  const int64_t n4 = n / 4;
  if (n4 == 0) return;
  add_inplace_kernel<<<stream_grid(n4), 256, 0, as_stream(stream)>>>((float*)y, (const float*)x, n4);
  DL_HIP_CHECK(hipGetLastError());
}

void fill_f32(uintptr_t x, float v, int64_t n, int64_t slot_index, float slot_value, uintptr_t stream) {
  check_vec4(n, "fill_f32");
  const int64_t n4 = n / 4;
  if (n4 == 0) return;
  fill_kernel<<<stream_grid(n4), 256, 0, as_stream(stream)>>>((float*)x, v, n4, slot_index, slot_value);
  DL_HIP_CHECK(hipGetLastError());
}

void cast_f32_bf16(uintptr_t x, uintptr_t y, int64_t n, uintptr_t stream) {
  check_vec4(n, "cast_f32_bf16");
  const int64_t n4 = n / 4;
  if (n4 == 0) return;
  cast_f32_bf16_kernel<<<stream_grid(n4), 256, 0, as_stream(stream)>>>((const float*)x, (bf16_t*)y, n4);
  DL_HIP_CHECK(hipGetLastError());
}

}  // namespace dl
