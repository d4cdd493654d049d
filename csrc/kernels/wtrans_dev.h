// dgrad weight flip-transposes as a block job: W [co][tap][ci] (bf16 shadow)
// -> WT [ci][taps-1-tap][co], one 64 (co) x 64 (ci) tile of one tap per
// 256-thread block through LDS, 16-byte loads and stores: in, 8 lanes sweep one
// 128-B weight row; out, the 64 lanes of a wave own 64 consecutive ci and each
// gathers 8 consecutive co (row stride 72 elements: the column reads are
// conflict-free).  Used by the step's prep launch and -- so the transposes run
// on the CUs the 128-block head kernel leaves idle -- by the head launch.
#pragma once
#include "dl_common.h"

namespace dl {

struct WTransArgs {
  const bf16_t* tw[4];
  bf16_t* twt[4];
  int tcout[4], tcin[4], nb[4];
  int nt, taps;
};

// host: block counts of the Cin % 64 == 0 && Cout % 64 == 0 tiles
inline int wtrans_blocks(const WTransArgs& a) {
  int n = 0;
  for (int j = 0; j < a.nt; ++j) n += a.nb[j];
  return n;
}

__device__ __forceinline__ void wtrans_tile(const bf16_t* __restrict__ src, bf16_t* __restrict__ dst, int Cin,
                                            int Cout, int taps, int blk, bf16_t (*tt)[72]) {
  const int nci = Cin / 64, nco = Cout / 64;
  const int tap = blk / (nci * nco);
  const int r = blk % (nci * nco);
  const int ci0 = (r % nci) * 64, co0 = (r / nci) * 64;
#pragma unroll
  for (int q = threadIdx.x; q < 512; q += 256) {
    const int row = q >> 3, ch = q & 7;
    *reinterpret_cast<uint4*>(&tt[row][ch * 8]) =
        *reinterpret_cast<const uint4*>(src + ((int64_t)(co0 + row) * taps + tap) * Cin + ci0 + ch * 8);
  }
  __syncthreads();
  const int ftap = taps - 1 - tap;
#pragma unroll
  for (int q = threadIdx.x; q < 512; q += 256) {
    const int ci = q & 63, ch = q >> 6;
    uint32_t w4[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      w4[e] = (uint32_t)tt[ch * 8 + 2 * e][ci] | ((uint32_t)tt[ch * 8 + 2 * e + 1][ci] << 16);
    *reinterpret_cast<uint4*>(dst + ((int64_t)(ci0 + ci) * taps + ftap) * Cout + co0 + ch * 8) =
        make_uint4(w4[0], w4[1], w4[2], w4[3]);
  }
}

// block `blk` of the job list (blocks of job j follow those of job j-1)
__device__ __forceinline__ void wtrans_block(const WTransArgs& a, int blk) {
  __shared__ __attribute__((aligned(16))) bf16_t tt[64][72];
  for (int j = 0; j < a.nt; ++j) {
    if (blk >= a.nb[j]) { blk -= a.nb[j]; continue; }
    wtrans_tile(a.tw[j], a.twt[j], a.tcin[j], a.tcout[j], a.taps, blk, tt);
    return;
  }
}

}  // namespace dl
