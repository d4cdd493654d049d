// Implicit-GEMM convolution on CDNA4 matrix cores (gfx950, bf16 in, fp32 acc).
//
// Replaces the reference's cunn SpatialConvolutionMM (im2col + cuBLAS GEMM;
// examples/cifar10.lua:108-126, examples/mnist.lua:57-62).
// Layouts are chosen for MFMA, not copied from Torch:
//   activations NHWC (channels-last), weights KRSC = [Cout][KS][KS][Cin].
// Then, for a stride-1 "same" convolution with M = B*H*W, N = Cout,
// K = KS*KS*Cin and k = (kh*KS + kw)*Cin + c:
//   forward  y[m][n]  = sum_k im2col(x)[m][k] * W[n][k]          (A gathered, B K-major)
//   dgrad    dx       = forward(dy, W') with W'[ci][kh][kw][co] = W[co][KS-1-kh][KS-1-kw][ci]
//   wgrad    dW[n][k] = sum_m dy[m][n] * im2col(x)[m][k]          (reduction over m)
// Cin is a power of two >= 8 (the 3-channel input layer is zero-padded to 8),
// so every 16-byte chunk of K (8 channels) lies inside one (kh, kw) tap and is
// one aligned vector load; padding taps and K tails load zeros.
//
// Kernels use v_mfma_f32_16x16x32_bf16 (lane l: A[l&15][8(l>>4)+j],
// B[8(l>>4)+j][l&15], C/D col = l&15, row = 4(l>>4)+j), 256-thread workgroups
// (2x2 waves of 64 lanes), register-staged double-buffered LDS tiles with XOR
// swizzles so that the fragment reads are bank-conflict free:
//   * forward / dgrad: both operands K-contiguous -> ds_read_b128 row reads;
//   * wgrad: both operands have the reduction index (m) as the *row* index of
//     an NHWC tensor -> tiles are staged [m][col] and read with the gfx950
//     hardware transpose ds_read_b64_tr_b16 (no shuffles).
// The forward epilogue also produces the per-channel sum / sum-of-squares
// partials of the bf16 output for train-mode BatchNorm (fused, deterministic:
// one partial row per M tile, reduced by bn_finalize).
#include "dl_common.h"
#include "dl_ops.h"

namespace dl {

struct ConvGeom {
  int B, H, W;
  int Cin, Cout;
  int KS, pad;
  int logW, logHW, logC8;  // log2(W), log2(H*W), log2(Cin/8)
  int M, K, Kch;           // M = B*H*W, K = KS*KS*Cin, Kch = K/8
};

static int ilog2_exact(int v, const char* what) {
  int l = 0;
  while ((1 << l) < v) ++l;
  if ((1 << l) != v) throw std::runtime_error(std::string(what) + " must be a power of two");
  return l;
}

static ConvGeom make_geom(int B, int H, int W, int Cin, int Cout, int KS) {
  ConvGeom g;
  g.B = B; g.H = H; g.W = W; g.Cin = Cin; g.Cout = Cout; g.KS = KS; g.pad = KS / 2;
  if (KS % 2 != 1) throw std::runtime_error("conv: odd kernel size required");
  if (Cin < 8) throw std::runtime_error("conv: Cin must be >= 8 (pad the input channels)");
  g.logW = ilog2_exact(W, "W");
  g.logHW = ilog2_exact(H * W, "H*W");
  g.logC8 = ilog2_exact(Cin / 8, "Cin/8");
  g.M = B * H * W;
  g.K = KS * KS * Cin;
  g.Kch = g.K / 8;
  return g;
}

// --------------------------------------------------------------------------
// LDS swizzles (16-byte chunk granularity)
// --------------------------------------------------------------------------
// Row reads (ds_read_b128, 16 lanes = 16 consecutive rows at one chunk): rows
// of CPR chunks; rows r and r + 16/CPR share a 256-B bank row, so XOR the
// chunk with (r / (16/CPR)) mod CPR.
template <int CPR>
__device__ __forceinline__ int swz_row(int row, int ch) {
  constexpr int RPB = 16 / CPR;  // rows per 256-B bank row
  return row * CPR + (ch ^ ((row / RPB) & (CPR - 1)));
}

// Transposed reads (ds_read_b64_tr_b16): a 32-lane half reads rows
// {r0..r0+3, r0+8..r0+11} (or +4) x two adjacent chunks; the XOR spreads those
// 8 rows over distinct 32-byte slot pairs of the 256-byte bank row.
template <int CPR>
__device__ __forceinline__ int swz_tr(int row, int ch) {
  if constexpr (CPR == 16) {
    const int f = 2 * ((row & 3) | (((row >> 3) & 1) << 2));
    return row * 16 + (ch ^ f);
  } else {
    static_assert(CPR == 8, "swz_tr: rows of 8 or 16 chunks");
    const int f = 2 * (((row >> 1) & 1) | (((row >> 3) & 1) << 1));
    return row * 8 + (ch ^ f);
  }
}

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

typedef short s16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ s16x4 ds_read_tr16(const void* lds_byte_ptr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(lds_byte_ptr));
}

// XCD-aware tile order: consecutive tiles (sharing weight panels) on one XCD.
__device__ __forceinline__ int xcd_swizzle(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// --------------------------------------------------------------------------
// forward / dgrad implicit GEMM
// --------------------------------------------------------------------------
template <int BM, int BN, int BK, bool STATS>
__global__ void __launch_bounds__(256) conv_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                       bf16_t* __restrict__ y, float* __restrict__ stats,
                                                       const ConvGeom g) {
  constexpr int NT = 256, WM = 2, WN = 2;
  constexpr int CPR = BK / 8;
  constexpr int A_PT = BM * CPR / NT, B_PT = BN * CPR / NT;
  static_assert(BM * CPR % NT == 0 && BN * CPR % NT == 0, "tile/thread mismatch");
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  constexpr int A_CH = BM * CPR, B_CH = BN * CPR;
  __shared__ __attribute__((aligned(16))) uint4 smem[2 * (A_CH + B_CH)];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int ntn = (g.Cout + BN - 1) / BN;
  const int ntm = (g.M + BM - 1) / BM;
  const int tile = xcd_swizzle(blockIdx.x, ntm * ntn);
  // n fastest: the ntn tiles sharing one activation panel run back to back
  const int tm = tile / ntn, tn = tile % ntn;
  const int m0 = tm * BM, n0 = tn * BN;
  const int HW = 1 << g.logHW, Wd = g.W, C8 = 1 << g.logC8;

  // per-thread A rows (fixed over the K loop)
  int a_row[A_PT], a_ch[A_PT], a_oh[A_PT], a_ow[A_PT];
  int64_t a_base[A_PT];
  bool a_ok[A_PT];
#pragma unroll
  for (int i = 0; i < A_PT; ++i) {
    const int q = tid + i * NT;
    a_row[i] = q / CPR;
    a_ch[i] = q % CPR;
    const int m = m0 + a_row[i];
    a_ok[i] = m < g.M;
    const int mm = a_ok[i] ? m : 0;
    const int b = mm >> g.logHW, rem = mm & (HW - 1);
    a_oh[i] = rem >> g.logW;
    a_ow[i] = rem & (Wd - 1);
    a_base[i] = (int64_t)b * HW * g.Cin;
  }
  int b_row[B_PT], b_ch[B_PT];
#pragma unroll
  for (int i = 0; i < B_PT; ++i) {
    const int q = tid + i * NT;
    b_row[i] = q / CPR;
    b_ch[i] = q % CPR;
  }

  uint4 ra[A_PT], rb[B_PT];
  const uint4 zero4 = make_uint4(0, 0, 0, 0);
  auto load_tiles = [&](int kt) {
#pragma unroll
    for (int i = 0; i < A_PT; ++i) {
      const int kc = kt * CPR + a_ch[i];
      const int kpos = kc >> g.logC8;
      const int c0 = (kc & (C8 - 1)) << 3;
      const int kh = kpos / g.KS, kw = kpos - kh * g.KS;
      const int ih = a_oh[i] + kh - g.pad, iw = a_ow[i] + kw - g.pad;
      const bool ok = a_ok[i] && kc < g.Kch && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)Wd;
      ra[i] = ok ? *reinterpret_cast<const uint4*>(x + a_base[i] + (((int64_t)ih << g.logW) + iw) * g.Cin + c0)
                 : zero4;
    }
#pragma unroll
    for (int i = 0; i < B_PT; ++i) {
      const int kc = kt * CPR + b_ch[i];
      const int n = n0 + b_row[i];
      const bool ok = n < g.Cout && kc < g.Kch;
      rb[i] = ok ? *reinterpret_cast<const uint4*>(w + (int64_t)n * g.K + (int64_t)kc * 8) : zero4;
    }
  };
  auto store_tiles = [&](int buf) {
    uint4* As = smem + buf * (A_CH + B_CH);
    uint4* Bs = As + A_CH;
#pragma unroll
    for (int i = 0; i < A_PT; ++i) As[swz_row<CPR>(a_row[i], a_ch[i])] = ra[i];
#pragma unroll
    for (int i = 0; i < B_PT; ++i) Bs[swz_row<CPR>(b_row[i], b_ch[i])] = rb[i];
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (g.Kch + CPR - 1) / CPR;
  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) load_tiles(kt + 1);
    const uint4* As = smem + cur * (A_CH + B_CH);
    const uint4* Bs = As + A_CH;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 af[FM], bfr[FN];
      const int ch = kk * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        uint4 v = As[swz_row<CPR>(wm * TM + i * 16 + (lane & 15), ch)];
        af[i] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        uint4 v = Bs[swz_row<CPR>(wn * TN + j * 16 + (lane & 15), ch)];
        bfr[j] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
    if (kt + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // ---- epilogue: bf16 store (+ BN statistics of the stored values)
  const int col_l = lane & 15, rq = lane >> 4;
  float s1[FN], s2[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * TN + j * 16 + col_l;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * TM + i * 16 + rq * 4 + r;
        const bf16_t hv = f32_to_bf16(acc[i][j][r]);
        if (m < g.M && n < g.Cout) y[(int64_t)m * g.Cout + n] = hv;
        if constexpr (STATS) {
          const float v = bf16_to_f32(hv);  // statistics of exactly what is stored (0 for m >= M)
          s1[j] += v;
          s2[j] += v * v;
        }
      }
    }
  }
  if constexpr (STATS) {
    float* red = reinterpret_cast<float*>(smem);  // [WM][2][BN]
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      s1[j] += __shfl_xor(s1[j], 16, 64);
      s1[j] += __shfl_xor(s1[j], 32, 64);
      s2[j] += __shfl_xor(s2[j], 16, 64);
      s2[j] += __shfl_xor(s2[j], 32, 64);
      if (rq == 0) {
        red[(wm * 2 + 0) * BN + wn * TN + j * 16 + col_l] = s1[j];
        red[(wm * 2 + 1) * BN + wn * TN + j * 16 + col_l] = s2[j];
      }
    }
    __syncthreads();
    for (int c = tid; c < BN; c += NT) {
      const int n = n0 + c;
      if (n < g.Cout) {
        float a = 0.f, b = 0.f;
#pragma unroll
        for (int q = 0; q < WM; ++q) { a += red[(q * 2) * BN + c]; b += red[(q * 2 + 1) * BN + c]; }
        stats[(int64_t)tm * 2 * g.Cout + n] = a;
        stats[(int64_t)tm * 2 * g.Cout + g.Cout + n] = b;
      }
    }
  }
}

// --------------------------------------------------------------------------
// wgrad implicit GEMM: out[split][co][k] = sum_{m in split} dy[m][co] * im2col(x)[m][k]
// --------------------------------------------------------------------------
template <int BM, int BN, int BK>
__global__ void __launch_bounds__(256) conv_wgrad_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                         float* __restrict__ out, const ConvGeom g, int m_per_split,
                                                         int ldo) {
  constexpr int NT = 256, WM = 2, WN = 2;
  constexpr int ACPR = BM / 8, BCPR = BN / 8;  // chunks per LDS row (row = one m)
  constexpr int A_CH = BK * ACPR, B_CH = BK * BCPR;
  constexpr int A_PT = A_CH / NT, B_PT = B_CH / NT;
  static_assert(A_CH % NT == 0 && B_CH % NT == 0, "tile/thread mismatch");
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  __shared__ __attribute__((aligned(16))) uint4 smem[2 * (A_CH + B_CH)];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int ntm = (g.Cout + BM - 1) / BM, ntn = (g.Kch * 8 + BN - 1) / BN;
  const int tile = xcd_swizzle(blockIdx.x, ntm * ntn);
  const int tm = tile % ntm, tn = tile / ntm;
  const int co0 = tm * BM, k0 = tn * BN;
  const int split = blockIdx.y;
  const int mbeg = split * m_per_split;
  const int mend = min(g.M, mbeg + m_per_split);
  const int HW = 1 << g.logHW, Wd = g.W, C8 = 1 << g.logC8;

  // A (dy) chunks: row r (m), chunk c (8 channels of co)
  int a_r[A_PT], a_c[A_PT];
#pragma unroll
  for (int i = 0; i < A_PT; ++i) {
    const int q = tid + i * NT;
    a_r[i] = q / ACPR;
    a_c[i] = q % ACPR;
  }
  // B (im2col) chunks: row r (m), chunk c -> fixed tap (dh, dw, c0)
  int b_r[B_PT], b_c[B_PT], b_dh[B_PT], b_dw[B_PT], b_c0[B_PT];
  bool b_kok[B_PT];
#pragma unroll
  for (int i = 0; i < B_PT; ++i) {
    const int q = tid + i * NT;
    b_r[i] = q / BCPR;
    b_c[i] = q % BCPR;
    const int kc = k0 / 8 + b_c[i];
    b_kok[i] = kc < g.Kch;
    const int kpos = kc >> g.logC8;
    b_c0[i] = (kc & (C8 - 1)) << 3;
    const int kh = kpos / g.KS;
    b_dh[i] = kh - g.pad;
    b_dw[i] = kpos - kh * g.KS - g.pad;
  }

  uint4 ra[A_PT], rb[B_PT];
  const uint4 zero4 = make_uint4(0, 0, 0, 0);
  auto load_tiles = [&](int kt) {
    const int mb = mbeg + kt * BK;
#pragma unroll
    for (int i = 0; i < A_PT; ++i) {
      const int m = mb + a_r[i];
      const int co = co0 + a_c[i] * 8;
      const bool ok = m < mend && co < g.Cout;
      ra[i] = ok ? *reinterpret_cast<const uint4*>(dy + (int64_t)m * g.Cout + co) : zero4;
    }
#pragma unroll
    for (int i = 0; i < B_PT; ++i) {
      const int m = mb + b_r[i];
      const int b = m >> g.logHW, rem = m & (HW - 1);
      const int ih = (rem >> g.logW) + b_dh[i], iw = (rem & (Wd - 1)) + b_dw[i];
      const bool ok = m < mend && b_kok[i] && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)Wd;
      rb[i] = ok ? *reinterpret_cast<const uint4*>(x + ((int64_t)b * HW + ((int64_t)ih << g.logW) + iw) * g.Cin +
                                                   b_c0[i])
                 : zero4;
    }
  };
  auto store_tiles = [&](int buf) {
    uint4* As = smem + buf * (A_CH + B_CH);
    uint4* Bs = As + A_CH;
#pragma unroll
    for (int i = 0; i < A_PT; ++i) As[swz_tr<ACPR>(a_r[i], a_c[i])] = ra[i];
#pragma unroll
    for (int i = 0; i < B_PT; ++i) Bs[swz_tr<BCPR>(b_r[i], b_c[i])] = rb[i];
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed-read lane roles: group gq = lane>>4 (k rows 8gq..8gq+7),
  // within the group lane 4q+p -> row q, columns 4p..4p+3
  const int gq = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  const int nk = (mend - mbeg + BK - 1) / BK;
  if (nk > 0) {
    load_tiles(0);
    store_tiles(0);
  }
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) load_tiles(kt + 1);
    const char* As = reinterpret_cast<const char*>(smem + cur * (A_CH + B_CH));
    const char* Bs = As + A_CH * 16;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int col = wm * TM + i * 16 + 4 * p4;  // first of 4 columns (co)
        const int ch = col >> 3, sub = (col & 7) * 2;
        const int r0 = kk * 32 + gq * 8 + q4;
        s16x4 lo = ds_read_tr16(As + swz_tr<ACPR>(r0, ch) * 16 + sub);
        s16x4 hi = ds_read_tr16(As + swz_tr<ACPR>(r0 + 4, ch) * 16 + sub);
        af[i] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = wn * TN + j * 16 + 4 * p4;
        const int ch = col >> 3, sub = (col & 7) * 2;
        const int r0 = kk * 32 + gq * 8 + q4;
        s16x4 lo = ds_read_tr16(Bs + swz_tr<BCPR>(r0, ch) * 16 + sub);
        s16x4 hi = ds_read_tr16(Bs + swz_tr<BCPR>(r0 + 4, ch) * 16 + sub);
        bfr[j] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
    if (kt + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  float* o = out + (int64_t)split * g.Cout * ldo;
  const int col_l = lane & 15, rq = lane >> 4;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int k = k0 + wn * TN + j * 16 + col_l;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wm * TM + i * 16 + rq * 4 + r;
        if (co < g.Cout && k < ldo) o[(int64_t)co * ldo + k] = acc[i][j][r];
      }
    }
}

// Sum `splits` fp32 slabs [splits][Cout][Kp] (Kp = taps*Cp) into dst
// [Cout][taps][C] (C <= Cp: drops zero-padded input channels).
__global__ void __launch_bounds__(256) slab_reduce_kernel(const float* __restrict__ slabs, float* __restrict__ dst,
                                                          int splits, int Cout, int taps, int Cp, int C) {
  const int64_t total = (int64_t)Cout * taps * C;
  const int64_t slab = (int64_t)Cout * taps * Cp;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const int64_t rest = i / C;  // co*taps + tap
    const int64_t src = rest * Cp + c;
    float s = 0.f;
    for (int sp = 0; sp < splits; ++sp) s += slabs[sp * slab + src];
    dst[i] = s;
  }
}

// --------------------------------------------------------------------------
// weight / input re-layouts (bf16)
// --------------------------------------------------------------------------
// W [Cout][KS][KS][Cin] -> Wt [Cin][KS][KS][Cout] with the taps flipped (dgrad B operand)
__global__ void __launch_bounds__(256) weight_flip_transpose_kernel(const bf16_t* __restrict__ w,
                                                                    bf16_t* __restrict__ wt, int Cout, int Cin,
                                                                    int KS) {
  __shared__ bf16_t t[32][33];
  const int taps = KS * KS;
  const int tap = blockIdx.z;
  const int ci0 = blockIdx.x * 32, co0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int r = ty; r < 32; r += 8) {
    const int co = co0 + r, ci = ci0 + tx;
    t[r][tx] = (co < Cout && ci < Cin) ? w[((int64_t)co * taps + tap) * Cin + ci] : (bf16_t)0;
  }
  __syncthreads();
  const int ftap = taps - 1 - tap;  // (KS-1-kh, KS-1-kw)
  for (int r = ty; r < 32; r += 8) {
    const int ci = ci0 + r, co = co0 + tx;
    if (ci < Cin && co < Cout) wt[((int64_t)ci * taps + ftap) * Cout + co] = t[tx][r];
  }
}

// fp32 [Cout][taps][C] -> bf16 [Cout][taps][Cp] (zero channels C..Cp-1)
__global__ void __launch_bounds__(256) pack_weight_kernel(const float* __restrict__ w, bf16_t* __restrict__ wp,
                                                          int Cout, int taps, int C, int Cp) {
  const int64_t total = (int64_t)Cout * taps * Cp;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cp);
    const int64_t rest = i / Cp;
    wp[i] = c < C ? f32_to_bf16(w[rest * C + c]) : (bf16_t)0;
  }
}

// bf16 [P][C] -> bf16 [P][Cp] (zero channels C..Cp-1); one thread per pixel
__global__ void __launch_bounds__(256) pad_channels_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ xp,
                                                           int64_t P, int C, int Cp) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < P; p += (int64_t)gridDim.x * blockDim.x) {
    for (int c = 0; c < Cp; ++c) xp[p * Cp + c] = c < C ? x[p * C + c] : (bf16_t)0;
  }
}

// --------------------------------------------------------------------------
// host launchers
// --------------------------------------------------------------------------
template <int BM, int BN, int BK, bool STATS>
static void launch_fwd(const ConvGeom& g, uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t stats, hipStream_t s) {
  const int ntm = (g.M + BM - 1) / BM, ntn = (g.Cout + BN - 1) / BN;
  conv_fwd_kernel<BM, BN, BK, STATS><<<ntm * ntn, 256, 0, s>>>((const bf16_t*)x, (const bf16_t*)w, (bf16_t*)y,
                                                                (float*)stats, g);
}

int conv_fwd_mtile(int B, int H, int W, int Cin, int Cout, int KS, int tile) {
  (void)B; (void)H; (void)W; (void)Cin; (void)Cout; (void)KS;
  return tile == 1 ? 64 : 128;
}

// tile: 0 = 128x128, 1 = 64x64, 2 = 128x64   (BK = 64; BK = 32 when K is small)
void conv_fwd(uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t stats, int B, int H, int W, int Cin, int Cout, int KS,
              int tile, uintptr_t stream) {
  ConvGeom g = make_geom(B, H, W, Cin, Cout, KS);
  hipStream_t s = as_stream(stream);
  const bool st = stats != 0;
  const bool smallK = g.K <= 256;
#define DL_FWD(BM_, BN_, BK_)                                        \
  do {                                                               \
    if (st) launch_fwd<BM_, BN_, BK_, true>(g, x, w, y, stats, s);   \
    else launch_fwd<BM_, BN_, BK_, false>(g, x, w, y, stats, s);     \
  } while (0)
  if (tile == 0) {
    if (smallK) DL_FWD(128, 128, 32); else DL_FWD(128, 128, 64);
  } else if (tile == 1) {
    if (smallK) DL_FWD(64, 64, 32); else DL_FWD(64, 64, 64);
  } else if (tile == 2) {
    if (smallK) DL_FWD(128, 64, 32); else DL_FWD(128, 64, 64);
  } else {
    throw std::runtime_error("conv_fwd: bad tile id");
  }
#undef DL_FWD
  DL_HIP_CHECK(hipGetLastError());
}

// out: fp32 [splits][Cout][ldo], ldo >= K (K = KS*KS*Cin)
void conv_wgrad(uintptr_t dy, uintptr_t x, uintptr_t out, int B, int H, int W, int Cin, int Cout, int KS, int splits,
                int ldo, int tile, uintptr_t stream) {
  ConvGeom g = make_geom(B, H, W, Cin, Cout, KS);
  if (ldo < g.K) throw std::runtime_error("conv_wgrad: ldo < K");
  if (splits < 1) splits = 1;
  int mps = (g.M + splits - 1) / splits;
  hipStream_t s = as_stream(stream);
  if (tile == 0) {
    constexpr int BM = 128, BN = 64, BK = 32;
    const int nt = ((g.Cout + BM - 1) / BM) * ((g.K + BN - 1) / BN);
    conv_wgrad_kernel<BM, BN, BK><<<dim3(nt, splits), 256, 0, s>>>((const bf16_t*)dy, (const bf16_t*)x, (float*)out,
                                                                   g, mps, ldo);
  } else {
    constexpr int BM = 64, BN = 64, BK = 32;
    const int nt = ((g.Cout + BM - 1) / BM) * ((g.K + BN - 1) / BN);
    conv_wgrad_kernel<BM, BN, BK><<<dim3(nt, splits), 256, 0, s>>>((const bf16_t*)dy, (const bf16_t*)x, (float*)out,
                                                                   g, mps, ldo);
  }
  DL_HIP_CHECK(hipGetLastError());
}

void slab_reduce(uintptr_t slabs, uintptr_t dst, int splits, int Cout, int taps, int Cp, int C, uintptr_t stream) {
  const int64_t total = (int64_t)Cout * taps * C;
  slab_reduce_kernel<<<stream_grid(total), 256, 0, as_stream(stream)>>>((const float*)slabs, (float*)dst, splits,
                                                                        Cout, taps, Cp, C);
  DL_HIP_CHECK(hipGetLastError());
}

void weight_flip_transpose(uintptr_t w, uintptr_t wt, int Cout, int Cin, int KS, uintptr_t stream) {
  dim3 grid((Cin + 31) / 32, (Cout + 31) / 32, KS * KS);
  weight_flip_transpose_kernel<<<grid, 256, 0, as_stream(stream)>>>((const bf16_t*)w, (bf16_t*)wt, Cout, Cin, KS);
  DL_HIP_CHECK(hipGetLastError());
}

void pack_weight(uintptr_t w, uintptr_t wp, int Cout, int taps, int C, int Cp, uintptr_t stream) {
  const int64_t total = (int64_t)Cout * taps * Cp;
  pack_weight_kernel<<<stream_grid(total), 256, 0, as_stream(stream)>>>((const float*)w, (bf16_t*)wp, Cout, taps, C,
                                                                        Cp);
  DL_HIP_CHECK(hipGetLastError());
}

void pad_channels(uintptr_t x, uintptr_t xp, int64_t P, int C, int Cp, uintptr_t stream) {
  pad_channels_kernel<<<stream_grid(P), 256, 0, as_stream(stream)>>>((const bf16_t*)x, (bf16_t*)xp, P, C, Cp);
  DL_HIP_CHECK(hipGetLastError());
}

}  // namespace dl
