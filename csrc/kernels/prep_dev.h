// Device side of the per-step operand preparation (the input batch into the
// zero-bordered, channel-padded layer-1 buffer + zeroing the step's atomic
// accumulators), shared by the stand-alone prep launch (conv_igemm.hip
// prep_step_kernel) and the SGD launch that prepares the NEXT step of an
// unrolled graph in extra workgroups (flat_ops.hip sgd_slabs_kernel).
#pragma once
#include <algorithm>
#include <stdexcept>
#include <vector>

#include "dl_common.h"

namespace dl {

struct PrepArgs {
  const bf16_t* x; bf16_t* xp; int P; int C, Cp;                // input pad (channels + spatial)
  int H, W, sp;                                                 // image dims, spatial zero pad
  // device-side data path (img != nullptr): gather + normalise the step's
  // batch straight from the HBM-resident uint8 dataset
  const uint8_t* img; const int* order; const int64_t* lab_all; int64_t* lab_out;
  const unsigned long long* ctr;  // [0] = step counter (advanced by head_wgrad)
  int n_order, B;
  float mean[3], inv_std[3];
  const float* w1; bf16_t* w1p; int w1_cout, taps, w1_c, w1_cp;  // layer-1 pack
  int nt;                                                        // transposes
  const bf16_t* tw[4]; bf16_t* twt[4]; int tcout[4], tcin[4];
  int nb_pad, nb_pack, nb_t[4];
  int quad;  // fast gather/pad path: one block per image, 4 pixels per thread
  // zero job: the step's atomic accumulators (BN statistics, BN parameter
  // gradients, split-K weight gradients) -- float4 granularity
  int nz, nb_zero;
  float* zp[8];
  int zn4[8];
};

// Workgroup blk (< nb_pad) of the pad/gather job.
__device__ __forceinline__ void prep_pad_block(const PrepArgs& a, int blk) {
  if (a.quad) {
    // fast path (3 -> 8 channels, W % 4 == 0): block = one image, thread =
    // 4 consecutive pixels of one row; every load of a thread is issued
    // before the first use (one dependent round trip for the sample index,
    // one for the pixels) and the 4 padded pixels go out as 64 contiguous B
    const int HW = a.H * a.W, Hp = a.H + 2 * a.sp, Wp = a.W + 2 * a.sp;
    const int b = blk;
    int smp = 0;
    if (a.img) {
      const unsigned long long step = *a.ctr;  // advanced by head_wgrad later in the step
      const int pos = (int)((step * (unsigned long long)a.B + (unsigned long long)b) % (unsigned)a.n_order);
      smp = a.order[pos];
      if (threadIdx.x == 0) a.lab_out[b] = a.lab_all[smp];
    }
    for (int q4 = threadIdx.x; q4 < HW / 4; q4 += 256) {
      const int r = q4 * 4, h = r / a.W, w = r - h * a.W;
      float f[12];
      if (a.img) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(a.img + ((int64_t)smp * HW + r) * 3);
        const uint32_t d0 = src[0], d1 = src[1], d2 = src[2];
        const uint32_t d[3] = {d0, d1, d2};
#pragma unroll
        for (int k = 0; k < 12; ++k) {
          const float u = (float)((d[k >> 2] >> (8 * (k & 3))) & 0xffu);
          f[k] = (u * (1.0f / 255.0f) - a.mean[k % 3]) * a.inv_std[k % 3];
        }
      } else {
        const uint2* src = reinterpret_cast<const uint2*>(a.x + ((int64_t)b * HW + r) * 3);
        const uint2 e0 = src[0], e1 = src[1], e2 = src[2];
        const uint32_t d[6] = {e0.x, e0.y, e1.x, e1.y, e2.x, e2.y};
#pragma unroll
        for (int k = 0; k < 12; ++k) f[k] = (k & 1) ? hi_bf16(d[k >> 1]) : lo_bf16(d[k >> 1]);
      }
      if (a.Cp == 4) {  // 8-byte pixels (the pair-packed first layer: csrc conv_fwd_c8_kernel PAIR)
        uint2* dst = reinterpret_cast<uint2*>(a.xp + (((int64_t)b * Hp + h + a.sp) * Wp + w + a.sp) * 4);
#pragma unroll
        for (int px = 0; px < 4; ++px)
          dst[px] = make_uint2(pack_bf16x2(f[3 * px], f[3 * px + 1]), pack_bf16x2(f[3 * px + 2], 0.f));
      } else {
        uint4* dst = reinterpret_cast<uint4*>(a.xp + (((int64_t)b * Hp + h + a.sp) * Wp + w + a.sp) * 8);
#pragma unroll
        for (int px = 0; px < 4; ++px)
          dst[px] = make_uint4(pack_bf16x2(f[3 * px], f[3 * px + 1]), pack_bf16x2(f[3 * px + 2], 0.f), 0u, 0u);
      }
    }
    return;
  }
  const int HW = a.H * a.W, Hp = a.H + 2 * a.sp, Wp = a.W + 2 * a.sp;
  // step counter: advanced by head_wgrad later in the same step (stream order)
  const unsigned long long step = a.img ? *a.ctr : 0ull;
  for (int p = blk * 256 + threadIdx.x; p < a.P; p += a.nb_pad * 256) {
    const int b = p / HW;
    const int r = p - b * HW, h = r / a.W, w = r - h * a.W;
    bf16_t v[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) v[c] = 0;
    if (a.img) {
      // sample of this step = order[(step * B + b) mod n_order]
      const int pos = (int)((step * (unsigned long long)a.B + (unsigned long long)b) % (unsigned)a.n_order);
      const int smp = a.order[pos];
      const uint8_t* src = a.img + ((int64_t)smp * HW + r) * a.C;
      for (int c = 0; c < a.C && c < 3; ++c) v[c] = f32_to_bf16((src[c] * (1.0f / 255.0f) - a.mean[c]) * a.inv_std[c]);
      if (r == 0) a.lab_out[b] = a.lab_all[smp];
    } else {
      for (int c = 0; c < a.C; ++c) v[c] = a.x[(int64_t)p * a.C + c];
    }
    const int64_t q = ((int64_t)b * Hp + h + a.sp) * Wp + w + a.sp;  // interior of the zero-bordered buffer
    if (a.Cp == 4) {
      *reinterpret_cast<uint2*>(a.xp + q * 4) = *reinterpret_cast<const uint2*>(v);
    } else {
      for (int c = 0; c < a.Cp; c += 8)
        *reinterpret_cast<uint4*>(a.xp + q * a.Cp + c) = *reinterpret_cast<const uint4*>(v + c);
    }
  }
}

// Workgroup blk (< nb_zero) of the zero job.
__device__ __forceinline__ void prep_zero_block(const PrepArgs& a, int blk) {
  int64_t total = 0;
  for (int j = 0; j < a.nz; ++j) total += a.zn4[j];
  for (int64_t i = (int64_t)blk * 256 + threadIdx.x; i < total; i += (int64_t)a.nb_zero * 256) {
    int64_t r = i;
    int j = 0;
    while (r >= a.zn4[j]) { r -= a.zn4[j]; ++j; }
    reinterpret_cast<float4*>(a.zp[j])[r] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// Host: the zero job's ranges (16-byte aligned, multiples of 4 floats).
inline void prep_set_zero(PrepArgs& a, const std::vector<uintptr_t>& zp, const std::vector<int64_t>& zn) {
  if (zp.size() != zn.size() || zp.size() > 8) throw std::runtime_error("prep_step: up to 8 zero ranges");
  a.nz = (int)zp.size();
  int64_t z4 = 0;
  for (int j = 0; j < a.nz; ++j) {
    if (zn[j] % 4 != 0 || zp[j] % 16 != 0 || zn[j] <= 0 || zn[j] / 4 >= (1ll << 31))
      throw std::runtime_error("prep_step: zero ranges must be 16-byte aligned multiples of 4 floats");
    a.zp[j] = (float*)zp[j];
    a.zn4[j] = (int)(zn[j] / 4);
    z4 += zn[j] / 4;
  }
  a.nb_zero = (int)std::min<int64_t>((z4 + 1023) / 1024, 256);
}

// Host: the pad/gather job over P = B*H*W pixels (sets P, quad, nb_pad).
inline void prep_set_pad(PrepArgs& a, int64_t P) {
  if (a.C > 16 || a.Cp > 16 || (a.Cp % 8 != 0 && a.Cp != 4) || a.C > a.Cp)
    throw std::runtime_error("prep_step: input channels must pad to 4, 8 or 16");
  if (P >= (1ll << 31)) throw std::runtime_error("prep_step: too many pixels");
  if (P > 0 && (a.H <= 0 || a.W <= 0 || P % ((int64_t)a.H * a.W) != 0)) throw std::runtime_error("prep_step: P != B*H*W");
  a.P = (int)P;
  a.quad = (a.C == 3 && (a.Cp == 8 || a.Cp == 4) && P > 0 && a.W % 4 == 0) ? 1 : 0;
  a.nb_pad = a.quad ? (int)(P / ((int64_t)a.H * a.W)) : (int)std::min<int64_t>((P + 255) / 256, 1024);
}

// Host: the device-gather fields (batch b of step ctr[0] = sample
// order[(ctr[0]*B + b) mod n_order], normalised (v/255 - mean)/std).
inline void prep_set_gather(PrepArgs& a, uintptr_t img, uintptr_t order, uintptr_t lab_all, uintptr_t lab_out,
                            uintptr_t ctr, int n_order, int B, int C, const std::vector<float>& mean,
                            const std::vector<float>& stdv) {
  if (C > 3 || mean.size() < (size_t)C || stdv.size() < (size_t)C) throw std::runtime_error("prep_step_gather: C <= 3");
  if (n_order <= 0 || B <= 0) throw std::runtime_error("prep_step_gather: empty order / batch");
  if (!img || !order || !lab_all || !lab_out || !ctr) throw std::runtime_error("prep_step_gather: null pointer");
  a.img = (const uint8_t*)img; a.order = (const int*)order; a.lab_all = (const int64_t*)lab_all;
  a.lab_out = (int64_t*)lab_out; a.ctr = (const unsigned long long*)ctr; a.n_order = n_order; a.B = B;
  for (int c = 0; c < 3; ++c) {
    a.mean[c] = c < C ? mean[c] : 0.f;
    a.inv_std[c] = c < C ? 1.0f / stdv[c] : 1.f;
  }
}

}  // namespace dl
