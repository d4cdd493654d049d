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
#include "prep_dev.h"
#include "sgd_dev.h"

namespace dl {

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// SGD (+ optional momentum / weight decay), fused with 1/n normalisation and
// the bf16 shadow-weight refresh used by the bf16 compute path.
// ---------------------------------------------------------------------------
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

// Blocks: [next step's pad/gather | next step's zero job | update | tail].
// `next` (nb_pad = nb_zero = 0: none) prepares the following step of an
// unrolled graph in the same launch -- its input batch and zeroed
// accumulators; the tail writes the first layer's packed operand -- so that
// step runs without a prep launch of its own.
template <bool kMomentum, bool kShadow>
__global__ void __launch_bounds__(256) sgd_slabs_kernel(const SgdJob job, const PrepArgs next) {
  int blk = (int)blockIdx.x;
  if (blk < next.nb_pad) {
    prep_pad_block(next, blk);
    return;
  }
  blk -= next.nb_pad;
  if (blk < next.nb_zero) {
    prep_zero_block(next, blk);
    return;
  }
  blk -= next.nb_zero;
  const int nmain = (int)gridDim.x - next.nb_pad - next.nb_zero - job.r.tail_nblk;
  if (blk >= nmain) {
    sgd_tail_block<kMomentum, kShadow>(job, blk - nmain);
    return;
  }
  if (job.red) slab_reduce_range_loop(job, blk, nmain);  // reduce-only job (slab_reduce_multi)
  else sgd_range_loop<kMomentum, kShadow>(job, blk, nmain);
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

// Elastic step for AsyncEA's bf16 delta wire: delta = alpha * (p - c) rounded
// to bf16 (the wire copy out16), and p moves by the ROUNDED delta, so p + c is
// conserved exactly as with the fp32 wire; out = the rounded delta in fp32
// (what the server adds), p16 = the bf16 shadow.  One pass instead of the
// elastic step + cast + correction + shadow passes.
__global__ void __launch_bounds__(256) elastic_wire16_kernel(float* __restrict__ p, const float* __restrict__ c,
                                                             float* __restrict__ out, bf16_t* __restrict__ out16,
                                                             bf16_t* __restrict__ p16, float alpha, int64_t n4) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pv = reinterpret_cast<float4*>(p)[i];
    const float4 cv = reinterpret_cast<const float4*>(c)[i];
    uint2 w;
    w.x = pack_bf16x2(alpha * (pv.x - cv.x), alpha * (pv.y - cv.y));
    w.y = pack_bf16x2(alpha * (pv.z - cv.z), alpha * (pv.w - cv.w));
    const float4 d = make_float4(lo_bf16(w.x), hi_bf16(w.x), lo_bf16(w.y), hi_bf16(w.y));
    pv.x -= d.x; pv.y -= d.y; pv.z -= d.z; pv.w -= d.w;
    reinterpret_cast<float4*>(p)[i] = pv;
    reinterpret_cast<float4*>(out)[i] = d;
    reinterpret_cast<uint2*>(out16)[i] = w;
    if (p16) {
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

// Device timestamp (the constant-rate wall clock, hipDeviceAttributeWallClockRate)
// written by one lane with a vector store.  A captured graph re-runs it at every
// replay, so bucket timings read after a replay time the replayed schedule
// (engine.comm_profile(replay=True); HIP refuses external event-record nodes
// in a capture, scripts/probe_graph_events.py).
__global__ void __launch_bounds__(64) stamp_kernel(long long* __restrict__ slot) {
  if (threadIdx.x == 0) {
    const long long t = wall_clock64();
    __builtin_nontemporal_store(t, slot);
  }
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

// size the update grid to the elements left after a skipped suffix (A/B)
static bool g_sgd_trim = true;
void set_sgd_trim(bool on) { g_sgd_trim = on; }

// One-shot: the next sgd_update_slabs launch also prepares the next step
// (prep_dev.h jobs + the first layer's packed weights from its tail range).
static PrepArgs g_next_prep{};
static bool g_next_armed = false;
static bf16_t* g_next_pack = nullptr;
static int g_next_pack_cp = 0;
static int64_t g_next_pack_off = 0, g_next_pack_len = 0;  // the first layer's elements in the updated buffer

// pack_off / pack_len: the first conv layer's weight [Cout][taps][C] as an
// element range of the buffer the consuming update writes -- packed from the
// main loop when the layer is not the update's slab tail (its gradient was
// all-reduced at N > 1, so the update reads it from the flat gradient).
void arm_sgd_next_prep(uintptr_t img, uintptr_t order, uintptr_t lab_all, uintptr_t lab_out, uintptr_t ctr,
                       int n_order, int B, int C, std::vector<float> mean, std::vector<float> stdv, uintptr_t xp,
                       int Cp, int H, int W, int sp, std::vector<uintptr_t> zp, std::vector<int64_t> zn,
                       uintptr_t w1p, int w1_cp, int64_t pack_off, int64_t pack_len) {
  if (g_next_armed) throw std::runtime_error("arm_sgd_next_prep: already armed (no sgd_update_slabs consumed it)");
  if (!xp || !w1p || (w1_cp > 0 ? w1_cp < C : C > 4)) throw std::runtime_error("arm_sgd_next_prep: input buffer / packed weights");
  if (pack_off % 4 || pack_len % 4 || pack_off < 0 || pack_len <= 0 || pack_len % C)
    throw std::runtime_error("arm_sgd_next_prep: the first layer's element range must be 16-byte aligned");
  PrepArgs a{};
  a.xp = (bf16_t*)xp; a.C = C; a.Cp = Cp; a.H = H; a.W = W; a.sp = sp;
  prep_set_gather(a, img, order, lab_all, lab_out, ctr, n_order, B, C, mean, stdv);
  prep_set_pad(a, (int64_t)B * H * W);
  prep_set_zero(a, zp, zn);
  g_next_prep = a;
  g_next_pack = (bf16_t*)w1p;
  g_next_pack_cp = w1_cp;
  g_next_pack_off = pack_off;
  g_next_pack_len = pack_len;
  g_next_armed = true;
}

bool sgd_next_prep_armed() { return g_next_armed; }

void disarm_sgd_next_prep() { g_next_armed = false; }

void sgd_update_slabs(uintptr_t p, uintptr_t g, uintptr_t mom, uintptr_t p16, uintptr_t slot, float lr,
                      float momentum, float wd, int64_t n, std::vector<int64_t> offs, std::vector<int64_t> lens,
                      std::vector<uintptr_t> slabs, std::vector<int> splits, std::vector<int64_t> tail,
                      uintptr_t tail_slab, int64_t skip_lo, int64_t skip_hi, uintptr_t stream) {
  check_vec4(n, "sgd_update_slabs");
  SgdJob job = make_sgd_job(p, g, mom, p16, slot, lr, momentum, wd, 0, n, offs, lens, slabs, splits, tail, tail_slab);
  if (skip_hi > skip_lo) {
    if (skip_lo % 4 || skip_hi % 4 || skip_lo < 0 || skip_hi > n) throw std::runtime_error("sgd_update_slabs: bad skip");
    job.skip_lo4 = skip_lo / 4;
    job.skip_hi4 = skip_hi / 4;
    if (skip_hi == n && g_sgd_trim) {
      // a skipped suffix (the side job's range): the grid covers only the rest
      // (the tail blocks cover their own range)
      job.hi4 = std::max(job.lo4, job.skip_lo4);
    }
  }
  const int64_t n4 = n / 4;
  PrepArgs next{};
  if (g_next_armed) {
    g_next_armed = false;
    if (job.r.tail_nblk > 0) {  // the first layer is the slab tail: its blocks write the packed operand
      if (job.r.tail_c != g_next_prep.C || job.r.tail_lo != g_next_pack_off)
        throw std::runtime_error("sgd_update_slabs: the slab tail is not the first layer the next step packs");
    } else {  // the main loop packs the first layer's range
      const int64_t lo4 = g_next_pack_off / 4, hi4 = (g_next_pack_off + g_next_pack_len) / 4;
      if (lo4 < job.lo4 || hi4 > job.hi4 || (lo4 < job.skip_hi4 && job.skip_lo4 < hi4))
        throw std::runtime_error("sgd_update_slabs: the first layer is not updated by this launch's main loop");
      for (int k = 0; k < job.r.n; ++k)
        if (lo4 < job.r.hi4[k] && job.r.lo4[k] < hi4)
          throw std::runtime_error("sgd_update_slabs: the first layer overlaps a slab range");
      job.pack_lo4 = lo4;
      job.pack_hi4 = hi4;
      job.pack_c = g_next_prep.C;
    }
    next = g_next_prep;
    job.tail_pack = g_next_pack;
    job.tail_pack_cp = g_next_pack_cp;
  }
  if (n4 == 0) return;
  dim3 grid(stream_grid(job.hi4 - job.lo4) + job.r.tail_nblk + next.nb_pad + next.nb_zero), block(256);
  auto s = as_stream(stream);
  if (mom && p16) sgd_slabs_kernel<true, true><<<grid, block, 0, s>>>(job, next);
  else if (mom) sgd_slabs_kernel<true, false><<<grid, block, 0, s>>>(job, next);
  else if (p16) sgd_slabs_kernel<false, true><<<grid, block, 0, s>>>(job, next);
  else sgd_slabs_kernel<false, false><<<grid, block, 0, s>>>(job, next);
  DL_HIP_CHECK(hipGetLastError());
}

// Reduce-only launch (no update): the split-K weight-gradient slabs of up to
// 4 in-place ranges and one channel-padded tail summed into the gradient
// buffer g of n floats -- the weight gradients a multi-node step all-reduces,
// bitwise the stand-alone slab_reduce's, several layers per launch.
void slab_reduce_multi(uintptr_t g, int64_t n, std::vector<int64_t> offs, std::vector<int64_t> lens,
                       std::vector<uintptr_t> slabs, std::vector<int> splits, std::vector<int64_t> tail,
                       uintptr_t tail_slab, uintptr_t stream) {
  check_vec4(n, "slab_reduce_multi");
  SgdJob job = make_reduce_job(g, 0, n, offs, lens, slabs, splits, tail, tail_slab);
  int64_t n4 = 0;
  for (int k = 0; k < job.r.n; ++k) n4 = std::max(n4, job.r.hi4[k] - job.r.lo4[k]);
  if (job.r.n == 0 && job.r.tail_nblk == 0) return;
  const int nmain = job.r.n ? stream_grid(n4) : 0;
  sgd_slabs_kernel<false, false><<<nmain + job.r.tail_nblk, 256, 0, as_stream(stream)>>>(job, PrepArgs{});
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

void elastic_step_wire16(uintptr_t p, uintptr_t c, uintptr_t out, uintptr_t out16, uintptr_t p16, float alpha,
                         int64_t n, uintptr_t stream) {
  check_vec4(n, "elastic_step_wire16");
  const int64_t n4 = n / 4;
  if (n4 == 0) return;
  elastic_wire16_kernel<<<stream_grid(n4), 256, 0, as_stream(stream)>>>((float*)p, (const float*)c, (float*)out,
                                                                         (bf16_t*)out16, (bf16_t*)p16, alpha, n4);
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

void stamp_time(uintptr_t slot, uintptr_t stream) {
  stamp_kernel<<<1, 64, 0, as_stream(stream)>>>((long long*)slot);
  DL_HIP_CHECK(hipGetLastError());
}

int wall_clock_khz() {
  int dev = 0, khz = 0;
  DL_HIP_CHECK(hipGetDevice(&dev));
  DL_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
  return khz;
}

}  // namespace dl
