// Device side of the fused SGD update, shared by the flat-buffer update
// kernels (flat_ops.hip) and the conv kernels that carry part of the update
// as extra workgroups (conv_igemm.hip: "side" SGD on the CUs a backward conv
// leaves free).  Every path runs the same element arithmetic (explicit fma)
// and the same slab sums, so where an element is updated changes no bit.
#pragma once
#include <stdexcept>
#include <vector>

#include "dl_common.h"
#include "slab_reduce_dev.h"

namespace dl {

__device__ __forceinline__ float participation_scale(const float* slot) {
  if (slot == nullptr) return 1.0f;
  float n = *slot;
  return n > 1.0f ? 1.0f / n : 1.0f;  // reference: only divide when n > 1
}


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

#ifndef DL_SLAB_CHUNK
#define DL_SLAB_CHUNK 8
#endif
constexpr int kSlabChunk = DL_SLAB_CHUNK;  // splits' loads in flight per chunk (build A/B: -DDL_SLAB_CHUNK=16)

template <int TPO>
__device__ __forceinline__ float4 slab_sum4(const float4* __restrict__ s, int64_t stride4, int splits) {
  float4 part[TPO];
#pragma unroll
  for (int t = 0; t < TPO; ++t) part[t] = make_float4(0.f, 0.f, 0.f, 0.f);
  // chunks of kSlabChunk splits, the chunk's loads in flight before its adds
  // (a chain of dependent 4-load chunks left the 19-split sums latency-bound);
  // lane t of the stand-alone reduce adds splits t, t+TPO, ... in order: same
  // here (kSlabChunk is a multiple of TPO, so split sp0 + u lands in part[u % TPO])
  static_assert(kSlabChunk % 8 == 0, "chunk of whole 8-split groups");
  for (int sp0 = 0; sp0 < splits; sp0 += kSlabChunk) {
    float4 v[kSlabChunk];
#pragma unroll
    for (int u = 0; u < kSlabChunk; ++u)
      if (sp0 + u < splits) v[u] = s[(int64_t)(sp0 + u) * stride4];
#pragma unroll
    for (int u = 0; u < kSlabChunk; ++u) {
      if (sp0 + u >= splits) break;
      if constexpr (TPO == 1) add4<TPO>(part, 0, v[u]);
      else add4<TPO>(part, u % TPO, v[u]);
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

// One update job: p[lo4, hi4) (float4 indices of the updated buffer) minus
// the skip range, gradient from g or from the slab ranges of r (+ r's tail).
struct SgdJob {
  float* p;
  const float* g;
  float* mom;           // null: no momentum
  bf16_t* p16;          // null: no bf16 shadow
  const float* slot;    // participation count (null: 1)
  float lr, momentum, wd;
  int64_t lo4, hi4;     // float4 range
  int64_t skip_lo4, skip_hi4;  // updated elsewhere (another launch's side job); empty: -1, -1
  SlabRanges r;
  int nblk;             // side job: workgroups of the host launch that run it (0: none)
  // the tail's updated weights also go to this packed bf16 copy (pack1_index:
  // channel-padded, or pair-packed for cp < 0; pads untouched): the first conv layer's operand,
  // when the launch prepares the next step (flat_ops.hip, prep_dev.h)
  bf16_t* tail_pack;
  int tail_pack_cp;
  // ... or, when the first layer is not a tail range (its gradient was
  // all-reduced: no slabs), the updated elements [pack_lo4, pack_hi4) of the
  // main loop ([Cout][taps][pack_c] weights) go to tail_pack the same way
  int64_t pack_lo4, pack_hi4;
  int pack_c;
  // reduce-only job (red != null): no update -- the slab sums of the ranges
  // (and of the tail) are written to red (same indexing as p), bitwise the
  // stand-alone slab_reduce's: a multi-node step's weight gradients
  // materialised for the all-reduce in extra workgroups of another launch
  float* red;
};

// The first-layer pack of an element range the main loop updated (pack_c of
// 3: a float4 straddles two output channels' tap rows).
__device__ __forceinline__ void pack_range4(const SgdJob& j, int64_t i, const float4& pv) {
  const float v[4] = {pv.x, pv.y, pv.z, pv.w};
  const int64_t e0 = (i - j.pack_lo4) * 4;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t e = e0 + k;
    j.tail_pack[pack1_index(e, j.pack_c, j.tail_pack_cp)] = f32_to_bf16(v[k]);
  }
}

// The update of a job without slab ranges (a multi-node step: every gradient
// was all-reduced from the flat buffer): two items per thread per trip, every
// load of both issued before the first update (flat_ops.hip sgd_kernel's
// pattern) -- the per-item loop below pays one memory round trip per item.
template <bool kMomentum, bool kShadow>
__device__ __forceinline__ void sgd_plain_loop2(const SgdJob& j, int bid, int nblk) {
  const float s = participation_scale(j.slot);
  const int64_t stride = (int64_t)nblk * blockDim.x;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  auto live = [&](int64_t i) { return i < j.hi4 && !(i >= j.skip_lo4 && i < j.skip_hi4); };
  auto finish = [&](int64_t i, float4 pv, const float4 gv, float4 mv) {
    pv = sgd_elem4<kMomentum>(pv, gv, mv, s, j.wd, j.lr, j.momentum);
    if constexpr (kMomentum) reinterpret_cast<float4*>(j.mom)[i] = mv;
    reinterpret_cast<float4*>(j.p)[i] = pv;
    if constexpr (kShadow) {
      uint2 packed;
      packed.x = pack_bf16x2(pv.x, pv.y);
      packed.y = pack_bf16x2(pv.z, pv.w);
      reinterpret_cast<uint2*>(j.p16)[i] = packed;
    }
    if (i >= j.pack_lo4 && i < j.pack_hi4) pack_range4(j, i, pv);
  };
  for (int64_t i = j.lo4 + (int64_t)bid * blockDim.x + threadIdx.x; i < j.hi4; i += 2 * stride) {
    const int64_t i2 = i + stride;
    const bool a = live(i), b = live(i2);
    float4 pa = z4, ga = z4, ma = z4, pb = z4, gb = z4, mb = z4;
    if (a) {
      pa = reinterpret_cast<const float4*>(j.p)[i];
      ga = load_grad4(j.g, i);
      if constexpr (kMomentum) ma = reinterpret_cast<const float4*>(j.mom)[i];
    }
    if (b) {
      pb = reinterpret_cast<const float4*>(j.p)[i2];
      gb = load_grad4(j.g, i2);
      if constexpr (kMomentum) mb = reinterpret_cast<const float4*>(j.mom)[i2];
    }
    if (a) finish(i, pa, ga, ma);
    if (b) finish(i2, pb, gb, mb);
  }
}

template <bool kMomentum, bool kShadow>
__device__ __forceinline__ void sgd_range_loop(const SgdJob& j, int bid, int nblk) {
  const SlabRanges& r = j.r;
  if (r.n == 0 && r.tail_hi4 <= r.tail_lo4) {  // (wave-uniform)
    sgd_plain_loop2<kMomentum, kShadow>(j, bid, nblk);
    return;
  }
  const float s = participation_scale(j.slot);
  const int64_t stride = (int64_t)nblk * blockDim.x;
  for (int64_t i = j.lo4 + (int64_t)bid * blockDim.x + threadIdx.x; i < j.hi4; i += stride) {
    if (i >= r.tail_lo4 && i < r.tail_hi4) continue;  // the tail blocks update these
    if (i >= j.skip_lo4 && i < j.skip_hi4) continue;  // a side job updated these
    float4 pv = reinterpret_cast<const float4*>(j.p)[i];
    const float4 gv = grad4_or_slabs(j.g, r, i);
    float4 mv = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (kMomentum) mv = reinterpret_cast<const float4*>(j.mom)[i];
    pv = sgd_elem4<kMomentum>(pv, gv, mv, s, j.wd, j.lr, j.momentum);
    if constexpr (kMomentum) reinterpret_cast<float4*>(j.mom)[i] = mv;
    reinterpret_cast<float4*>(j.p)[i] = pv;
    if constexpr (kShadow) {
      uint2 packed;
      packed.x = pack_bf16x2(pv.x, pv.y);
      packed.y = pack_bf16x2(pv.z, pv.w);
      reinterpret_cast<uint2*>(j.p16)[i] = packed;
    }
    if (i >= j.pack_lo4 && i < j.pack_hi4) pack_range4(j, i, pv);
  }
}

// Reduce-only job: the slab sums of every in-place range into j.red.
__device__ __forceinline__ void slab_reduce_range_loop(const SgdJob& j, int bid, int nblk) {
  const SlabRanges& r = j.r;
  const int64_t stride = (int64_t)nblk * blockDim.x;
  for (int k = 0; k < r.n; ++k) {
    const float4* s0 = reinterpret_cast<const float4*>(r.slab[k]);
    for (int64_t i = r.lo4[k] + (int64_t)bid * blockDim.x + threadIdx.x; i < r.hi4[k]; i += stride) {
      const float4* s = s0 + (i - r.lo4[k]);
      reinterpret_cast<float4*>(j.red)[i] =
          r.tpo[k] == 8 ? slab_sum4<8>(s, r.stride4[k], r.splits[k]) : slab_sum4<1>(s, r.stride4[k], r.splits[k]);
    }
  }
}

template <bool kMomentum, bool kShadow>
__device__ __forceinline__ void sgd_tail_block(const SgdJob& j, int bid) {
  const float s = participation_scale(j.slot);
  const SlabRanges& r = j.r;
  auto upd = [&](int64_t i, int64_t, int, float gs) {
    const int64_t e = r.tail_lo + i;  // KRSC weight: element i of the reduce's output order
    if (j.red) {  // reduce-only job
      j.red[e] = gs;
      return;
    }
    float mv = kMomentum ? j.mom[e] : 0.f;
    const float pv = sgd_elem<kMomentum>(j.p[e], gs, &mv, s, j.wd, j.lr, j.momentum);
    if constexpr (kMomentum) j.mom[e] = mv;
    j.p[e] = pv;
    if constexpr (kShadow) j.p16[e] = f32_to_bf16(pv);
    if (j.tail_pack) j.tail_pack[pack1_index(i, r.tail_c, j.tail_pack_cp)] = f32_to_bf16(pv);
  };
  if (r.tail_tpo == 32)
    slab_reduce_each<32>(r.tail_slab, r.tail_splits, r.tail_cout, r.tail_taps, r.tail_cp, r.tail_c, bid, r.tail_nblk,
                         upd);
  else if (r.tail_tpo == 8)
    slab_reduce_each<8>(r.tail_slab, r.tail_splits, r.tail_cout, r.tail_taps, r.tail_cp, r.tail_c, bid, r.tail_nblk,
                        upd);
  else
    slab_reduce_each<1>(r.tail_slab, r.tail_splits, r.tail_cout, r.tail_taps, r.tail_cp, r.tail_c, bid, r.tail_nblk,
                        upd);
}

// Host: an update job over elements [lo, hi) of a buffer of n floats, with
// up to 4 in-place slab ranges (offs / lens / slabs / splits: elements of the
// buffer) and an optional channel-padded tail {offset, numel, splits, Cout,
// taps, Cp, C} over tail_slab.  Validates every range.
inline SgdJob make_sgd_job(uintptr_t p, uintptr_t g, uintptr_t mom, uintptr_t p16, uintptr_t slot, float lr,
                           float momentum, float wd, int64_t lo, int64_t hi, const std::vector<int64_t>& offs,
                           const std::vector<int64_t>& lens, const std::vector<uintptr_t>& slabs,
                           const std::vector<int>& splits, const std::vector<int64_t>& tail, uintptr_t tail_slab) {
  const size_t k = offs.size();
  if (k > (size_t)kSlabRanges || lens.size() != k || slabs.size() != k || splits.size() != k)
    throw std::runtime_error("sgd job: up to 4 consistent slab ranges");
  if (lo % 4 || hi % 4 || lo < 0 || hi < lo) throw std::runtime_error("sgd job: 16-byte aligned element range");
  SgdJob j{};
  j.p = (float*)p; j.g = (const float*)g; j.mom = (float*)mom; j.p16 = (bf16_t*)p16; j.slot = (const float*)slot;
  j.lr = lr; j.momentum = momentum; j.wd = wd;
  j.lo4 = lo / 4; j.hi4 = hi / 4;
  j.skip_lo4 = j.skip_hi4 = -1;
  SlabRanges& r = j.r;
  r.n = (int)k;
  for (size_t q = 0; q < k; ++q) {
    if (offs[q] % 4 || lens[q] % 4 || offs[q] < lo || offs[q] + lens[q] > hi || slabs[q] % 16)
      throw std::runtime_error("sgd job: slab ranges must be 16-byte aligned and inside the job");
    if (splits[q] < 1 || splits[q] > kSlabMaxSplits) throw std::runtime_error("sgd job: 1..31 splits per slab range");
    if (q > 0 && offs[q] < offs[q - 1] + lens[q - 1]) throw std::runtime_error("sgd job: slab ranges overlap");
    r.lo4[q] = offs[q] / 4;
    r.hi4[q] = (offs[q] + lens[q]) / 4;
    r.slab[q] = (const float*)slabs[q];
    r.stride4[q] = lens[q] / 4;
    r.splits[q] = splits[q];
    r.tpo[q] = slab_reduce_tpo(splits[q]) == 1 ? 1 : 8;  // the stand-alone slab_reduce's lane split
  }
  r.tail_lo4 = r.tail_hi4 = -1;
  if (!tail.empty()) {
    if (tail.size() != 7) throw std::runtime_error("sgd job: tail = (offset, numel, splits, Cout, taps, Cp, C)");
    const int64_t off = tail[0], len = tail[1];
    r.tail_splits = (int)tail[2]; r.tail_cout = (int)tail[3]; r.tail_taps = (int)tail[4];
    r.tail_cp = (int)tail[5]; r.tail_c = (int)tail[6];
    if (off % 4 || len % 4 || off < lo || off + len > hi || len != (int64_t)r.tail_cout * r.tail_taps * r.tail_c ||
        (r.tail_cp > 0 ? r.tail_c > r.tail_cp : (r.tail_c > 4 || r.tail_taps != r.tail_cp * r.tail_cp)) ||
        r.tail_splits < 1 || tail_slab == 0)
      throw std::runtime_error("sgd job: inconsistent tail range");
    for (size_t q = 0; q < k; ++q)
      if (offs[q] < off + len && off < offs[q] + lens[q]) throw std::runtime_error("sgd job: tail overlaps");
    r.tail_lo = off;
    r.tail_lo4 = off / 4;
    r.tail_hi4 = (off + len) / 4;
    r.tail_slab = (const float*)tail_slab;
    r.tail_tpo = slab_reduce_tpo(r.tail_splits);
    r.tail_nblk = slab_reduce_grid(r.tail_splits, r.tail_cout, r.tail_taps, r.tail_c);
  }
  return j;
}

// Host: a reduce-only job writing the slab sums of the ranges (and of the
// tail) into the gradient buffer g (float index space of the job).
inline SgdJob make_reduce_job(uintptr_t g, int64_t lo, int64_t hi, const std::vector<int64_t>& offs,
                              const std::vector<int64_t>& lens, const std::vector<uintptr_t>& slabs,
                              const std::vector<int>& splits, const std::vector<int64_t>& tail, uintptr_t tail_slab) {
  if (!g) throw std::runtime_error("reduce job: null gradient buffer");
  SgdJob j = make_sgd_job(g, g, 0, 0, 0, 0.f, 0.f, 0.f, lo, hi, offs, lens, slabs, splits, tail, tail_slab);
  j.red = (float*)g;
  return j;
}

// A side job run by workgroup `bid` of the job's nblk extra workgroups of a
// host launch (conv_fwd_kernel): no tail range, always a bf16 shadow (the
// conv executors' flat buffers have one; make_side_job checks), momentum at
// run time -- or a reduce-only job (red).
__device__ __forceinline__ void sgd_side_block(const SgdJob& j, int bid) {
  if (j.red) slab_reduce_range_loop(j, bid, j.nblk);
  else if (j.mom) sgd_range_loop<true, true>(j, bid, j.nblk);
  else sgd_range_loop<false, true>(j, bid, j.nblk);
}

}  // namespace dl
