// Classifier head: Linear(F, C) -> LogSoftMax -> ClassNLLCriterion (mean),
// forward AND backward fused (gfx950).
//
// Reference: grad.nn.Linear(512*2*2, 10) + grad.nn.LogSoftMax +
// grad.nn.ClassNLLCriterion (examples/cifar10.lua:132-143,159-163),
// util.logSoftMax + logMultinomialLoss (examples/mnist.lua:79,86); SURVEY §2.8
// K17/K18.  The head is tiny (B x 10 x 2048), so it is two kernels instead of
// six library calls:
//   head_fwd_bwd : one workgroup per sample: logits = W h + b, log-softmax, loss,
//                  dlogits = (softmax - onehot)/B, dh = W^T dlogits (bf16, feeds
//                  the last conv block's backward); or logits only (predict)
//   head_wgrad   : dW[c][j] = sum_b dlogits[b][c] h[b][j], db, mean loss
//                  (fixed summation order: deterministic)
#include "dl_common.h"
#include <vector>
#include "dl_ops.h"
#include "head_wgrad_dev.h"
#include "bn_fin_dev.h"
#include "wtrans_dev.h"

namespace dl {

// DL_HEAD_STAMPS builds only (diagnostics): s_memtime of thread 0 of every
// head_fwd_bwd block at its phase boundaries -> [block][8]
__device__ unsigned long long* g_head_stamps = nullptr;
#ifdef DL_HEAD_STAMPS
__device__ __forceinline__ unsigned long long hstamp() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
#define HEAD_STAMP(k) do { if (threadIdx.x == 0 && g_head_stamps) g_head_stamps[blockIdx.x * 8 + (k)] = hstamp(); } while (0)
#else
#define HEAD_STAMP(k) do { } while (0)
#endif

// POOL: the head's input h is not read but computed here from the last conv
// block's pre-BN output y [B][yH][yW][yC] (bf16) and its BN coefficients
// (coef [4][yC]: scale at 2*yC, shift at 3*yC) -- the work of
// bn_relu_pool_fwd for that block, with the identical operation order and
// bf16 rounding -- and written to h_out for head_wgrad (one launch and one
// pass over h fewer per step).  Needs F == 2048 (one 8-feature chunk per thread).
struct HeadPool {
  const bf16_t* y;
  const float* coef;
  bf16_t* h_out;
  int yH, yW, yC;
  BnFin fin;  // fin.sums != nullptr: derive the coefficients from the accumulated statistics (mode 1)
  // RED: the last conv block's BatchNorm backward reduce, fused: each block
  // adds its sample's sum(dz) / sum(dz * xhat) per channel into row
  // (blockIdx & (fin.R - 1)) of red_rows [R][dgamma (C); dbeta (C)] (zeroed by
  // the step's prep kernel) -- the work of bn_relu_pool_bwd_reduce for that
  // block, done while dP, the window values and the coefficients are in registers
  float* red_rows;
};

template <int NC, bool POOL = false, bool RED = false>
__global__ void __launch_bounds__(256) head_fwd_bwd_kernel(const bf16_t* __restrict__ h, const float* __restrict__ w,
                                                           const float* __restrict__ bias,
                                                           const int64_t* __restrict__ labels, int F, int B,
                                                           float* __restrict__ logits_out, float* __restrict__ dlogits,
                                                           float* __restrict__ loss_b, bf16_t* __restrict__ dh,
                                                           const HeadPool hp = HeadPool{},
                                                           const WTransArgs wt = WTransArgs{}) {
  if ((int)blockIdx.x >= B) {  // blocks past the batch: the step's dgrad weight transposes (wtrans_dev.h)
    wtrans_block(wt, (int)blockIdx.x - B);
    return;
  }
  HEAD_STAMP(0);
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  __shared__ float lgp[NC][257];  // per-thread logit partials, transposed (+1: conflict-free rows)
  __shared__ float redc[NC];
  __shared__ float dl[NC];
  // the label and the bias, loaded now: read by thread 0 after the logits
  // barrier they were one more dependent memory round trip on its serial path
  const int ylab = labels ? (int)labels[b] : -1;
  float bv[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) bv[c] = bias[c];
  const bf16_t* hb = h + (int64_t)b * F;
  float acc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) acc[c] = 0.f;
  // F == 2048 (the reference net): one 8-feature chunk per thread; its 8 x NC
  // weights stay in registers for the dh pass (W is read once per sample)
  const bool one = F == 256 * 8;
  float4 wc[NC][2];
  uint4 v[4];                           // RED: the window values, kept for the backward reduce
  float rsc[8], rsh[8], rmu[8], ris[8];  // RED: BN coefficients of the thread's 8 channels
  if (one) {
    const int j0 = tid * 8;
    // the classifier weights first: independent of everything below, so their
    // L2 round trip overlaps the window loads and the BN coefficient rows
    // (issued after bn_fin_block's barrier they were a third round trip)
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      wc[c][0] = *reinterpret_cast<const float4*>(w + (int64_t)c * F + j0);
      wc[c][1] = *reinterpret_cast<const float4*>(w + (int64_t)c * F + j0 + 4);
    }
    uint4 hv;
    if constexpr (POOL) {
      // feature j0 = (oh * Wo + ow) * yC + c0 of the pooled NHWC map
      const int Wo = hp.yW >> 1;
      const int pix = j0 / hp.yC, c0 = j0 - pix * hp.yC;
      const int oh = pix / Wo, ow = pix - oh * Wo;
      const bf16_t* base = hp.y + (((int64_t)b * hp.yH + 2 * oh) * hp.yW + 2 * ow) * hp.yC + c0;
      v[0] = *reinterpret_cast<const uint4*>(base);
      v[1] = *reinterpret_cast<const uint4*>(base + hp.yC);
      v[2] = *reinterpret_cast<const uint4*>(base + (int64_t)hp.yW * hp.yC);
      v[3] = *reinterpret_cast<const uint4*>(base + (int64_t)hp.yW * hp.yC + hp.yC);
      float sc[8], sh[8];
      if (hp.fin.sums != nullptr) {  // uniform over the block (bn_fin_block ends with a barrier)
        __shared__ float ssc[kFinMaxC], ssh[kFinMaxC];
        __shared__ float smu[RED ? kFinMaxC : 1], sis[RED ? kFinMaxC : 1];
        bn_fin_block(hp.fin, hp.yC, ssc, ssh, RED ? smu : nullptr, RED ? sis : nullptr);
        HEAD_STAMP(1);
#pragma unroll
        for (int k = 0; k < 8; ++k) { sc[k] = ssc[c0 + k]; sh[k] = ssh[c0 + k]; }
        if constexpr (RED) {
#pragma unroll
          for (int k = 0; k < 8; ++k) { rmu[k] = smu[c0 + k]; ris[k] = sis[c0 + k]; }
        }
      } else {
        const float4 sc0 = *reinterpret_cast<const float4*>(hp.coef + 2 * hp.yC + c0);
        const float4 sc1 = *reinterpret_cast<const float4*>(hp.coef + 2 * hp.yC + c0 + 4);
        const float4 sh0 = *reinterpret_cast<const float4*>(hp.coef + 3 * hp.yC + c0);
        const float4 sh1 = *reinterpret_cast<const float4*>(hp.coef + 3 * hp.yC + c0 + 4);
        sc[0] = sc0.x; sc[1] = sc0.y; sc[2] = sc0.z; sc[3] = sc0.w; sc[4] = sc1.x; sc[5] = sc1.y; sc[6] = sc1.z;
        sc[7] = sc1.w;
        sh[0] = sh0.x; sh[1] = sh0.y; sh[2] = sh0.z; sh[3] = sh0.w; sh[4] = sh1.x; sh[5] = sh1.y; sh[6] = sh1.z;
        sh[7] = sh1.w;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) { rsc[k] = sc[k]; rsh[k] = sh[k]; }
      float mx[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float f[8] = {lo_bf16(v[q].x), hi_bf16(v[q].x), lo_bf16(v[q].y), hi_bf16(v[q].y),
                            lo_bf16(v[q].z), hi_bf16(v[q].z), lo_bf16(v[q].w), hi_bf16(v[q].w)};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float z = fmaf(sc[k], f[k], sh[k]);
          mx[k] = q == 0 ? z : fmaxf(mx[k], z);
        }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) mx[k] = fmaxf(mx[k], 0.f);
      hv = make_uint4(pack_bf16x2(mx[0], mx[1]), pack_bf16x2(mx[2], mx[3]), pack_bf16x2(mx[4], mx[5]),
                      pack_bf16x2(mx[6], mx[7]));
      *reinterpret_cast<uint4*>(hp.h_out + (int64_t)b * F + j0) = hv;
    } else {
      hv = *reinterpret_cast<const uint4*>(hb + j0);
    }
    const float hf[8] = {lo_bf16(hv.x), hi_bf16(hv.x), lo_bf16(hv.y), hi_bf16(hv.y),
                         lo_bf16(hv.z), hi_bf16(hv.z), lo_bf16(hv.w), hi_bf16(hv.w)};
#pragma unroll
    for (int c = 0; c < NC; ++c)
      acc[c] = hf[0] * wc[c][0].x + hf[1] * wc[c][0].y + hf[2] * wc[c][0].z + hf[3] * wc[c][0].w +
               hf[4] * wc[c][1].x + hf[5] * wc[c][1].y + hf[6] * wc[c][1].z + hf[7] * wc[c][1].w;
  }
  for (int j0 = tid * 8; !one && j0 < F; j0 += 256 * 8) {
    const uint4 hv = *reinterpret_cast<const uint4*>(hb + j0);
    float hf[8] = {lo_bf16(hv.x), hi_bf16(hv.x), lo_bf16(hv.y), hi_bf16(hv.y),
                   lo_bf16(hv.z), hi_bf16(hv.z), lo_bf16(hv.w), hi_bf16(hv.w)};
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const float4 w0 = *reinterpret_cast<const float4*>(w + (int64_t)c * F + j0);
      const float4 w1 = *reinterpret_cast<const float4*>(w + (int64_t)c * F + j0 + 4);
      acc[c] += hf[0] * w0.x + hf[1] * w0.y + hf[2] * w0.z + hf[3] * w0.w + hf[4] * w1.x + hf[5] * w1.y +
                hf[6] * w1.z + hf[7] * w1.w;
    }
  }
  // logits: sum of the 256 threads' partials per class through LDS (16 threads
  // per class, 16 values each, then a 16-lane butterfly) instead of NC
  // 64-lane shuffle reductions (6 dependent ds_bpermute rounds each)
#pragma unroll
  for (int c = 0; c < NC; ++c) lgp[c][tid] = acc[c];
  HEAD_STAMP(2);
  __syncthreads();
  if (tid < NC * 16) {
    const int c = tid >> 4, j = tid & 15;
    float sp = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) sp += lgp[c][q * 16 + j];
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) sp += __shfl_xor(sp, o, 16);
    if (j == 0) redc[c] = sp;
  }
  __syncthreads();
  HEAD_STAMP(3);
  if (tid == 0) {
    float lg[NC], mx = -INFINITY;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      lg[c] = redc[c] + bv[c];
      mx = fmaxf(mx, lg[c]);
    }
    float se = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) se += __expf(lg[c] - mx);
    const float lse = mx + __logf(se);
    if (logits_out) {
#pragma unroll
      for (int c = 0; c < NC; ++c) logits_out[(int64_t)b * NC + c] = lg[c] - lse;  // log-probabilities
    }
    if (labels) {
      const int y = ylab;
      float lb = 0.f;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const float p = __expf(lg[c] - lse);
        const float d = (p - (c == y ? 1.f : 0.f)) / (float)B;
        dl[c] = d;
        dlogits[(int64_t)b * NC + c] = d;
        if (c == y) lb = lse - lg[c];
      }
      loss_b[b] = lb;
    }
  }
  if (!labels) return;
  __syncthreads();
  HEAD_STAMP(4);
  float d[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) d[c] = dl[c];
  if (one) {
    const int j0 = tid * 8;
    float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      o[0] += d[c] * wc[c][0].x; o[1] += d[c] * wc[c][0].y; o[2] += d[c] * wc[c][0].z; o[3] += d[c] * wc[c][0].w;
      o[4] += d[c] * wc[c][1].x; o[5] += d[c] * wc[c][1].y; o[6] += d[c] * wc[c][1].z; o[7] += d[c] * wc[c][1].w;
    }
    const uint4 dpk =
        make_uint4(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]), pack_bf16x2(o[4], o[5]), pack_bf16x2(o[6], o[7]));
    *reinterpret_cast<uint4*>(dh + (int64_t)b * F + j0) = dpk;
    HEAD_STAMP(5);
    if constexpr (POOL && RED) {
      // the backward reduce of this sample: dz routed to the pool argmax (ReLU
      // mask), sum(dz) and sum(dz * xhat) per channel, from the bf16 dP that the
      // apply kernel will read -- bwd_reduce_body's arithmetic, item for item
      float g[8], s1[8], s2[8];
      g[0] = lo_bf16(dpk.x); g[1] = hi_bf16(dpk.x); g[2] = lo_bf16(dpk.y); g[3] = hi_bf16(dpk.y);
      g[4] = lo_bf16(dpk.z); g[5] = hi_bf16(dpk.z); g[6] = lo_bf16(dpk.w); g[7] = hi_bf16(dpk.w);
      float yv[4][8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        yv[q][0] = lo_bf16(v[q].x); yv[q][1] = hi_bf16(v[q].x); yv[q][2] = lo_bf16(v[q].y); yv[q][3] = hi_bf16(v[q].y);
        yv[q][4] = lo_bf16(v[q].z); yv[q][5] = hi_bf16(v[q].z); yv[q][6] = lo_bf16(v[q].w); yv[q][7] = hi_bf16(v[q].w);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float best = -INFINITY;
        int arg = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const float r = fmaxf(fmaf(rsc[k], yv[w][k], rsh[k]), 0.f);
          if (r > best) { best = r; arg = w; }
        }
        s1[k] = 0.f;
        s2[k] = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const float dz = (w == arg && best > 0.f) ? g[k] : 0.f;
          s1[k] += dz;
          s2[k] += dz * (yv[w][k] - rmu[k]) * ris[k];
        }
      }
      // the 4 waves hold the 4 pooled pixels of the same 64 channel chunks
      __shared__ float rr[4][64][17];
#pragma unroll
      for (int k = 0; k < 8; ++k) { rr[wid][lane][k] = s1[k]; rr[wid][lane][8 + k] = s2[k]; }
      __syncthreads();
      HEAD_STAMP(6);
      // row = [dgamma (= sum dz*xhat) ; dbeta (= sum dz)]: thread t adds outputs
      // t, t + 256, ... so a wave's 64 atomics hit 64 consecutive floats (2 cache
      // lines; the chunk-major lane order spread them over 16)
      float* row = hp.red_rows + (int64_t)(blockIdx.x & (hp.fin.R - 1)) * 2 * hp.yC;
      for (int o = tid; o < 2 * hp.yC; o += 256) {
        const int which = o < hp.yC ? 1 : 0;  // rr: [0..8) sum dz, [8..16) sum dz*xhat
        const int c = o - (o < hp.yC ? 0 : hp.yC), ch = c >> 3, k = which * 8 + (c & 7);
        unsafeAtomicAdd(row + o, rr[0][ch][k] + rr[1][ch][k] + rr[2][ch][k] + rr[3][ch][k]);
      }
      HEAD_STAMP(7);
    }
    return;
  }
  for (int j0 = tid * 8; j0 < F; j0 += 256 * 8) {
    float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const float4 w0 = *reinterpret_cast<const float4*>(w + (int64_t)c * F + j0);
      const float4 w1 = *reinterpret_cast<const float4*>(w + (int64_t)c * F + j0 + 4);
      o[0] += d[c] * w0.x; o[1] += d[c] * w0.y; o[2] += d[c] * w0.z; o[3] += d[c] * w0.w;
      o[4] += d[c] * w1.x; o[5] += d[c] * w1.y; o[6] += d[c] * w1.z; o[7] += d[c] * w1.w;
    }
    *reinterpret_cast<uint4*>(dh + (int64_t)b * F + j0) =
        make_uint4(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]), pack_bf16x2(o[4], o[5]), pack_bf16x2(o[6], o[7]));
  }
}

// dW[c][j] (fp32, written into the flat grad), db[c], loss = mean(loss_b):
// head_wgrad_body (head_wgrad_dev.h).
template <int NC>
__global__ void __launch_bounds__(256) head_wgrad_kernel(const bf16_t* __restrict__ h,
                                                         const float* __restrict__ dlogits,
                                                         const float* __restrict__ loss_b, int F, int B,
                                                         float* __restrict__ dw, float* __restrict__ db,
                                                         float* __restrict__ loss, float* __restrict__ slot,
                                                         unsigned long long* __restrict__ step_ctr) {
  head_wgrad_body<NC>(h, dlogits, loss_b, F, B, dw, db, loss, slot, step_ctr, (int)blockIdx.x);
}

void head_fwd_bwd(uintptr_t h, uintptr_t w, uintptr_t bias, uintptr_t labels, int F, int B, int NC,
                  uintptr_t logits_out, uintptr_t dlogits, uintptr_t loss_b, uintptr_t dh, uintptr_t stream) {
  if (NC != 10) throw std::runtime_error("head_fwd_bwd: built for 10 classes");
  if (F % 8 != 0) throw std::runtime_error("head_fwd_bwd: F % 8 != 0");
  head_fwd_bwd_kernel<10><<<B, 256, 0, as_stream(stream)>>>((const bf16_t*)h, (const float*)w, (const float*)bias,
                                                            (const int64_t*)labels, F, B, (float*)logits_out,
                                                            (float*)dlogits, (float*)loss_b, (bf16_t*)dh);
  DL_HIP_CHECK(hipGetLastError());
}

// fin_sums != 0 (atomic modes, reduce_rows() rows): the last block's BN coefficients are derived from
// the accumulated statistics (block 0 also publishes coef + running stats)
void head_fwd_bwd_pool_wt(uintptr_t y, uintptr_t coef, int yH, int yW, int yC, uintptr_t h_out, uintptr_t w,
                          uintptr_t bias, uintptr_t labels, int B, int NC, uintptr_t logits_out, uintptr_t dlogits,
                          uintptr_t loss_b, uintptr_t dh, uintptr_t fin_sums, int64_t fin_m, uintptr_t gamma,
                          uintptr_t beta, uintptr_t conv_bias, uintptr_t rmean, uintptr_t rvar, float eps,
                          float momentum, uintptr_t red_rows, uintptr_t stream, std::vector<uintptr_t> tw,
                          std::vector<uintptr_t> twt, std::vector<int> tcout, std::vector<int> tcin, int taps) {
  if (NC != 10) throw std::runtime_error("head_fwd_bwd_pool: built for 10 classes");
  // optional: the dgrad weight flip-transposes ride this launch (blocks B..)
  WTransArgs wt{};
  if (tw.size() > 4 || twt.size() != tw.size() || tcout.size() != tw.size() || tcin.size() != tw.size())
    throw std::runtime_error("head_fwd_bwd_pool: up to 4 consistent transposes");
  wt.nt = (int)tw.size();
  wt.taps = taps;
  for (int j = 0; j < wt.nt; ++j) {
    if (tcin[j] % 64 != 0 || tcout[j] % 64 != 0 || taps <= 0)
      throw std::runtime_error("head_fwd_bwd_pool: transposes need channel counts that are multiples of 64");
    wt.tw[j] = (const bf16_t*)tw[j];
    wt.twt[j] = (bf16_t*)twt[j];
    wt.tcout[j] = tcout[j];
    wt.tcin[j] = tcin[j];
    wt.nb[j] = (tcin[j] / 64) * (tcout[j] / 64) * taps;
  }
  const int grid = B + wtrans_blocks(wt);
  const int F = (yH / 2) * (yW / 2) * yC;
  if (F != 2048 || yC % 8 != 0 || yH % 2 != 0 || yW % 2 != 0)
    throw std::runtime_error("head_fwd_bwd_pool: needs a 2048-feature pooled map, C % 8 == 0");
  if (fin_sums != 0 && (reduce_rows() < 1 || reduce_rows() > kMaxRows || yC > kFinMaxC))
    throw std::runtime_error("head_fwd_bwd_pool: accumulated statistics need an atomic reduction mode");
  if (red_rows != 0 && (fin_sums == 0 || labels == 0 || yC != 512))
    throw std::runtime_error("head_fwd_bwd_pool: the fused BN backward reduce needs the atomic statistics, labels, C 512");
  const HeadPool hp{(const bf16_t*)y, (const float*)coef, (bf16_t*)h_out, yH, yW, yC,
                    make_bn_fin(fin_sums, fin_m, gamma, beta, conv_bias, rmean, rvar, eps, momentum, coef, reduce_rows()),
                    (float*)red_rows};
  if (red_rows)
    head_fwd_bwd_kernel<10, true, true><<<grid, 256, 0, as_stream(stream)>>>(
        nullptr, (const float*)w, (const float*)bias, (const int64_t*)labels, F, B, (float*)logits_out,
        (float*)dlogits, (float*)loss_b, (bf16_t*)dh, hp, wt);
  else
    head_fwd_bwd_kernel<10, true><<<grid, 256, 0, as_stream(stream)>>>(
        nullptr, (const float*)w, (const float*)bias, (const int64_t*)labels, F, B, (float*)logits_out,
        (float*)dlogits, (float*)loss_b, (bf16_t*)dh, hp, wt);
  DL_HIP_CHECK(hipGetLastError());
}

void head_fwd_bwd_pool(uintptr_t y, uintptr_t coef, int yH, int yW, int yC, uintptr_t h_out, uintptr_t w,
                       uintptr_t bias, uintptr_t labels, int B, int NC, uintptr_t logits_out, uintptr_t dlogits,
                       uintptr_t loss_b, uintptr_t dh, uintptr_t fin_sums, int64_t fin_m, uintptr_t gamma,
                       uintptr_t beta, uintptr_t conv_bias, uintptr_t rmean, uintptr_t rvar, float eps, float momentum,
                       uintptr_t red_rows, uintptr_t stream) {
  head_fwd_bwd_pool_wt(y, coef, yH, yW, yC, h_out, w, bias, labels, B, NC, logits_out, dlogits, loss_b, dh, fin_sums,
                       fin_m, gamma, beta, conv_bias, rmean, rvar, eps, momentum, red_rows, stream, {}, {}, {}, {}, 0);
}

void head_wgrad(uintptr_t h, uintptr_t dlogits, uintptr_t loss_b, int F, int B, int NC, uintptr_t dw, uintptr_t db,
                uintptr_t loss, uintptr_t slot, uintptr_t step_ctr, uintptr_t stream) {
  if (NC != 10) throw std::runtime_error("head_wgrad: built for 10 classes");
  head_wgrad_kernel<10><<<(F + 31) / 32 + 1, 256, 0, as_stream(stream)>>>((const bf16_t*)h, (const float*)dlogits,
                                                                        (const float*)loss_b, F, B, (float*)dw,
                                                                        (float*)db, (float*)loss, (float*)slot,
                                                                        (unsigned long long*)step_ctr);
  DL_HIP_CHECK(hipGetLastError());
}

void set_head_stamps(uintptr_t buf) {
  unsigned long long* p = (unsigned long long*)buf;
  DL_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_head_stamps), &p, sizeof(p)));
}

}  // namespace dl
