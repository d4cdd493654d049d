// Device body of the classifier head's weight gradient (head.hip), shared by
// head_wgrad_kernel and the fused launch with the last conv block's BN
// backward reduce (bn_pool.hip: bn_bwd_reduce_head).  `bid` = the block's
// index within the head-wgrad part of the grid, (F + 31) / 32 + 1 blocks of
// 256 threads.
#pragma once
#include "dl_common.h"

namespace dl {

// dW[c][j] (fp32, written into the flat grad), db[c], loss = mean(loss_b).
// Block = 32 columns x 8 row groups; fixed-order reductions (deterministic).
template <int NC>
__device__ __forceinline__ void head_wgrad_body(const bf16_t* __restrict__ h, const float* __restrict__ dlogits,
                                                const float* __restrict__ loss_b, int F, int B,
                                                float* __restrict__ dw, float* __restrict__ db,
                                                float* __restrict__ loss, float* __restrict__ slot,
                                                unsigned long long* __restrict__ step_ctr, int bid) {
  __shared__ float red[8][NC + 1][33];
  const int tid = threadIdx.x, col = tid & 31, grp = tid >> 5;
  const int nblk_cols = (F + 31) / 32;
  if (bid < nblk_cols) {
    const int j = bid * 32 + col;
    float acc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = 0.f;
    if (j < F) {
      // rows in batches of 4 with every load issued before the FMAs (the
      // serial load->use chain was latency-bound)
      int b = grp;
      // 16 rows per trip (B = 128: the whole column in one memory round trip)
      for (; b + 8 * 15 < B; b += 128) {
        float hv[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) hv[u] = bf16_to_f32(h[(int64_t)(b + 8 * u) * F + j]);
#pragma unroll
        for (int u = 0; u < 16; ++u)
#pragma unroll
          for (int c = 0; c < NC; ++c) acc[c] += dlogits[(int64_t)(b + 8 * u) * NC + c] * hv[u];
      }
      for (; b + 24 < B; b += 32) {
        float hv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) hv[u] = bf16_to_f32(h[(int64_t)(b + 8 * u) * F + j]);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int c = 0; c < NC; ++c) acc[c] += dlogits[(int64_t)(b + 8 * u) * NC + c] * hv[u];
      }
      for (; b < B; b += 8) {
        const float hv = bf16_to_f32(h[(int64_t)b * F + j]);
#pragma unroll
        for (int c = 0; c < NC; ++c) acc[c] += dlogits[(int64_t)b * NC + c] * hv;
      }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) red[grp][c][col] = acc[c];
    __syncthreads();
    for (int o = tid; o < NC * 32; o += 256) {
      const int c = o / 32, cc = o % 32;
      float s = 0.f;
#pragma unroll
      for (int g = 0; g < 8; ++g) s += red[g][c][cc];
      const int jj = bid * 32 + cc;
      if (jj < F) dw[(int64_t)c * F + jj] = s;
    }
  } else {
    // bias gradient and mean loss: rows b split over 8 groups x 32 lanes
    float acc[NC + 1];
#pragma unroll
    for (int c = 0; c <= NC; ++c) acc[c] = 0.f;
    for (int b = tid; b < B; b += 256) {
#pragma unroll
      for (int c = 0; c < NC; ++c) acc[c] += dlogits[(int64_t)b * NC + c];
      acc[NC] += loss_b[b];
    }
#pragma unroll
    for (int c = 0; c <= NC; ++c) red[grp][c][col] = acc[c];
    __syncthreads();
    if (tid <= NC) {
      float s = 0.f;
      for (int g = 0; g < 8; ++g)
        for (int cc = 0; cc < 32; ++cc) s += red[g][tid][cc];
      if (tid < NC) {
        if (db) db[tid] = s;
      } else {
        if (loss) *loss = s / (float)B;
        // participation count of this node's gradient (flat-buffer header):
        // replaces a per-step fill of the whole gradient buffer, every other
        // gradient element is overwritten by its producing kernel
        if (slot) *slot = 1.0f;
        // device-side data path: the step's gather kernel (prep_step_gather)
        // read the step counter; advance it here, one kernel boundary later
        // (a plain read-modify-write by one lane, no arrival ticket)
        if (step_ctr) *step_ctr += 1ull;
      }
    }
  }
}

}  // namespace dl
