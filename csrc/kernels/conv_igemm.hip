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
#include "slab_reduce_dev.h"
#include "bn_fin_dev.h"
#include "prep_dev.h"
#include "sgd_dev.h"
#include "wtrans_dev.h"

#include <algorithm>
#include <type_traits>
#include <vector>

namespace dl {

// Reduction mode of the train-mode BatchNorm statistics (set_reduce_atomic):
// 0 = one deterministic partial row per M tile (reduced by bn_finalize),
// R >= 1 (a power of two) = every workgroup atomically adds its per-channel
// totals into row (tile & (R-1)) of R zero-initialised [2][C] rows (the
// consumer -- bn_relu_pool_fwd_fin / the head -- sums the R rows and derives
// the BN coefficients itself: no finalize launch).  R = 1 is the single-row
// mode; R > 1 stripes the same-address atomics (measured: 1024 workgroups
// adding into one row serialise in the memory-side atomic unit, layer-1
// forward 31 vs 11 us).  Read once per workgroup epilogue (wave-uniform).
__device__ int g_red_atomic = 0;

__device__ __forceinline__ void put_stats(float* __restrict__ stats, int64_t row, int C, int n, float sa, float sb) {
  if (const int R = g_red_atomic) {
    float* s = stats + (int64_t)(row & (R - 1)) * 2 * C;
    unsafeAtomicAdd(s + n, sa);
    unsafeAtomicAdd(s + C + n, sb);
  } else {
    stats[row * 2 * C + n] = sa;
    stats[row * 2 * C + C + n] = sb;
  }
}

// BatchNorm backward reduce fused into a dgrad epilogue (BNRED): the dgrad's
// output is dP, the gradient of the pooled output of the previous block; for
// every stored element the epilogue also loads that block's pre-BN values y
// under the 2x2 pool window, routes dP to the window's argmax of relu(BN(y))
// and accumulates sum(dz) and sum(dz * xhat) per channel (bn_pool.hip
// bwd_reduce_body's arithmetic) -- the stand-alone reduce launch, and its
// re-read of dP, are gone.  rows: mode 0 = one partial row per M tile
// [T][sum dz (C); sum dz*xhat (C)], atomic modes = R striped rows
// [R][dgamma = sum dz*xhat (C); dbeta = sum dz (C)] (the layouts of the reduce).
// (BNR 2 / 3, the same reduce for the ResNet-50 channels-last BatchNorms in
// the 1x1 dgrad epilogues, measured slower than the reduce pass -- the
// epilogue's re-read of the BN input costs more than it saves,
// profiles/r5_resnet_bn_dgrad_ab.txt -- and was removed in round 6.)
struct BnRedArgs {
  const bf16_t* y;     // [B][2Ho][2Wo][C] pre-BN output of the previous block
  const float* coef;   // [4][C] mean, invstd, scale, shift
  float* rows;
};

// (A BatchNorm -> ReLU applied to the A operand on load of the ResNet-50
// b2 -> c3 1x1 GEMM measured slower than the apply pass it removed, 25.43 vs
// 24.64 ms/step, profiles/r4_resnet_bn_on_load_ab.txt; removed in round 6.)

struct ConvGeom {
  int B, H, W;
  int Hp, Wp;  // spatially zero-padded input dims (H + 2 pad, W + 2 pad)
  int Cin, Cout;
  int KS, pad;
  int logW, logHW, logC8;  // log2(W), log2(H*W) (valid when pow2), log2(Cin/8)
  int M, K, Kch;           // M = B*H*W, K = KS*KS*Cin, Kch = K/8
  int pow2;                // H and W powers of two (the region / c8 kernels and the shift addressing)
  int posm;                // streaming kernel: position-major M tiles with padding taps skipped (fwd_posm)
  float inv_HW, inv_W;     // reciprocals for the non-pow2 pixel decomposition (fdivmod)
  // Generalised geometry (make_geom_ex; the streaming forward and the wgrad
  // kernels only, non-pow2 addressing): tap (kh, kw) of output pixel (oh, ow)
  // reads padded input pixel (S*oh + kh, S*ow + kw) of the [B][Hp][Wp][Cin]
  // buffer; kernels may be KH x KW (K = KH*KW*Cin, taps row-major).
  int S, KH, KW;
  int kwstep;  // wgrad B chunks: tap column kw * kwstep (2: the pair-packed first layer, make_geom_pair)
  int dsep, dHp, dWp, dpad;  // wgrad: dy has its own buffer geometry [B][dHp][dWp][Cout], interior at dpad
  // epilogue output-row map (om != 0): output pixel (b, oh, ow) is stored at
  // row b*omHW + (omS*oh + omH0)*omW + omS*ow + omW0 (the phases of a strided
  // convolution's input gradient, written interleaved into the full tensor)
  int om, omS, omH0, omW0, omW, omHW;
};

// q = n / d, r = n - q*d for 0 <= n < 2^24 via a float reciprocal and one
// correction step (the ResNet-50 spatial sizes 56/28/14/7 are not powers of two)
__device__ __forceinline__ int fdivmod(int n, int d, float inv_d, int& r) {
  int q = (int)((float)n * inv_d);
  r = n - q * d;
  if (r < 0) { --q; r += d; }
  else if (r >= d) { ++q; r -= d; }
  return q;
}

// padded pixel index (b*Hp + S*oh)*Wp + S*ow of tap (0, 0) of output pixel m
// (any H, W; pow2 addressing only ever runs with S == 1)
__device__ __forceinline__ int out_pix(const ConvGeom& g, int m) {
  if (g.pow2) {
    const int b = m >> g.logHW, rem = m & ((1 << g.logHW) - 1);
    return (b * g.Hp + (rem >> g.logW)) * g.Wp + (rem & (g.W - 1));
  }
  int rem, ow;
  const int b = fdivmod(m, g.H * g.W, g.inv_HW, rem);
  const int oh = fdivmod(rem, g.W, g.inv_W, ow);
  return (b * g.Hp + g.S * oh) * g.Wp + g.S * ow;
}

// wgrad with a separate dy geometry (g.dsep): interior pixel of output m in dy
__device__ __forceinline__ int dy_pix(const ConvGeom& g, int m) {
  int rem, ow;
  const int b = fdivmod(m, g.H * g.W, g.inv_HW, rem);
  const int oh = fdivmod(rem, g.W, g.inv_W, ow);
  return (b * g.dHp + oh + g.dpad) * g.dWp + ow + g.dpad;
}

// epilogue row of output pixel m under the output map (g.om)
__device__ __forceinline__ int om_row(const ConvGeom& g, int m) {
  int rem, ow;
  const int b = fdivmod(m, g.H * g.W, g.inv_HW, rem);
  const int oh = fdivmod(rem, g.W, g.inv_W, ow);
  return b * g.omHW + (g.omS * oh + g.omH0) * g.omW + g.omS * ow + g.omW0;
}

// K steps (64 channels of one tap) of a position-major tile at output pixel
// pos: the taps whose input pixel is inside the image, times Cin / 64
__host__ __device__ __forceinline__ int posm_nk(const ConvGeom& g, int pos) {
  const int oh = pos / g.W, ow = pos - oh * g.W;
  const int th = min(g.KS, g.H + g.pad - oh) - max(0, g.pad - oh);
  const int tw = min(g.KS, g.W + g.pad - ow) - max(0, g.pad - ow);
  return th * tw * (g.Cin / 64);
}

static int ilog2_exact(int v, const char* what) {
  int l = 0;
  while ((1 << l) < v) ++l;
  if ((1 << l) != v) throw std::runtime_error(std::string(what) + " must be a power of two");
  return l;
}

static bool is_pow2(int v) { return v > 0 && (v & (v - 1)) == 0; }

static ConvGeom make_geom(int B, int H, int W, int Cin, int Cout, int KS) {
  ConvGeom g{};  // value-initialised: a field added later must not read stack garbage
  g.B = B; g.H = H; g.W = W; g.Cin = Cin; g.Cout = Cout; g.KS = KS; g.pad = KS / 2;
  g.Hp = H + 2 * g.pad; g.Wp = W + 2 * g.pad;
  if (KS % 2 != 1) throw std::runtime_error("conv: odd kernel size required");
  if (Cin < 8) throw std::runtime_error("conv: Cin must be >= 8 (pad the input channels)");
  g.pow2 = is_pow2(W) && is_pow2(H) ? 1 : 0;
  g.posm = 0;
  g.S = 1; g.KH = KS; g.KW = KS; g.kwstep = 1;
  g.dsep = 0; g.dHp = g.Hp; g.dWp = g.Wp; g.dpad = g.pad;
  g.om = 0; g.omS = 1; g.omH0 = 0; g.omW0 = 0; g.omW = W; g.omHW = H * W;
  g.logW = g.pow2 ? ilog2_exact(W, "W") : 0;
  g.logHW = g.pow2 ? ilog2_exact(H * W, "H*W") : 0;
  g.inv_HW = 1.0f / (float)(H * W);
  g.inv_W = 1.0f / (float)W;
  g.logC8 = ilog2_exact(Cin / 8, "Cin/8");
  if (!g.pow2 && (int64_t)B * H * W >= (1 << 24))
    throw std::runtime_error("conv: non-power-of-two H/W needs B*H*W < 2^24 (float pixel decomposition)");
  g.M = B * H * W;
  g.K = KS * KS * Cin;
  g.Kch = g.K / 8;
  if ((int64_t)B * g.Hp * g.Wp * std::max(Cin, Cout) >= (1ll << 31) || (int64_t)Cout * g.K >= (1ll << 31))
    throw std::runtime_error("conv: operand too large for 32-bit offsets");
  return g;
}

// The pair-packed first layer (4-channel padded input, <= 4 real channels):
// one 16-byte K chunk = channels 0-3 of two horizontally adjacent taps
// (dl_common.h pack1_index, cp = -KS), K = KS * ceil(KS/2) * 8.  For the
// wgrad kernel's B operand the chunk is 2 adjacent pixels of the [.][Wp][4]
// buffer: KW = ceil(KS/2) chunk columns at tap column 2 * kw.
static ConvGeom make_geom_pair(int B, int H, int W, int Cout, int KS) {
  ConvGeom g = make_geom(B, H, W, 8, Cout, KS);
  const int cpr = (KS + 1) / 2;
  g.Cin = 4; g.logC8 = 0;
  g.KW = cpr; g.kwstep = 2;
  g.Kch = KS * cpr; g.K = g.Kch * 8;
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
// CPR = 32 (512-B rows, the 256-wide wgrad tile): chunks ch and ch + 16 share
// banks, so the CPR = 16 XOR on the low four chunk bits spreads the rows the same.
template <int CPR>
__device__ __forceinline__ int swz_tr(int row, int ch) {
  if constexpr (CPR == 16 || CPR == 32) {
    const int f = 2 * ((row & 3) | (((row >> 3) & 1) << 2));
    return row * CPR + (ch ^ f);
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
// LDS-DMA staging (global_load_lds_dwordx4): one wave instruction writes
// 64 lanes x 16 B = 1 KiB contiguously at a wave-uniform LDS base.  The LDS
// image stays lane-linear; the swizzle is applied to the per-lane SOURCE chunk
// (the XORs above are involutions), and zero padding (halo taps, K tails,
// M/N tails) is read from a 16-byte zero line in global memory.
// --------------------------------------------------------------------------
__device__ uint4 g_zero16[4];
static unsigned long long* g_conv_dbg = nullptr;  // debug: per-workgroup s_memtime stamps

__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

__device__ __forceinline__ void glds16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// Buffer-descriptor LDS-DMA (buffer_load_dwordx4 ... offen lds): per-lane 32-bit
// byte offset in a VGPR + wave-uniform byte offset in an SGPR (soffset), so a
// load whose per-lane part is loop-invariant costs no VALU at all; offsets at
// or past `bytes` read zeros (hardware range check), which replaces the zero
// line for K/M tails.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr unsigned kOOB = 0x40000000u;  // a voffset past every operand: loads zeros
// streaming fwd/dgrad kernel main loop (set_conv_fwd_pf; A/B): 1 = register
// prefetch of the next step's fragments + unconditional DMA pipeline (4 stages)
__constant__ int g_fwd_pf = 1;

__device__ __forceinline__ rsrc_t make_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ void blds16(rsrc_t r, unsigned voff, unsigned soff, void* lds_wave_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_wave_base, 16, (int)voff,
                                           (int)soff, 0, 0);
}

// The same LDS-DMA as inline asm, for loops that read the staged tiles with
// ds_read_b64_tr_b16: hipcc (ROCm 7.2) puts an `s_waitcnt vmcnt(0)` in front of
// every __builtin_amdgcn_ds_read_tr16_b64 while a builtin LDS-DMA may be in
// flight (it cannot tell which LDS bytes the transposed read touches), which
// drains the whole DMA ring at every K step -- the wgrad kernel waited for the
// stages it had just issued.  Issued from asm, the DMA is invisible to that
// analysis; the kernel's own counted `s_waitcnt vmcnt(N)` before each barrier
// orders it (and the compiler still tracks lgkmcnt for the tr16 results).
// M0 carries the LDS base (nothing else in those kernels uses M0).
typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4 make_rsrc4(const void* p, unsigned bytes) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(p);
  return i32x4{(int)(unsigned)a, (int)(unsigned)(a >> 32), (int)bytes, 0x00020000};
}

__device__ __forceinline__ void blds16_asm(const i32x4& r, unsigned voff, unsigned soff, void* lds_wave_base) {
  // wave-uniform operands in SGPRs (readfirstlane: the compiler may not prove them uniform)
  const unsigned m0 = __builtin_amdgcn_readfirstlane(
      (unsigned)reinterpret_cast<unsigned long long>((__attribute__((address_space(3))) char*)lds_wave_base));
  const unsigned so = __builtin_amdgcn_readfirstlane(soff);
  const i32x4 rs{__builtin_amdgcn_readfirstlane(r[0]), __builtin_amdgcn_readfirstlane(r[1]),
                 __builtin_amdgcn_readfirstlane(r[2]), __builtin_amdgcn_readfirstlane(r[3])};
  asm volatile("s_mov_b32 m0, %3\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(rs), "s"(so),
               "s"(m0)
               : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until at most `n` stages (of LPS LDS-DMA loads each) are still in flight
template <int LPS>
__device__ __forceinline__ void wait_stages(int n) {
  switch (n) {
    case 0: wait_vmcnt<0>(); break;
    case 1: wait_vmcnt<LPS>(); break;
    case 2: wait_vmcnt<2 * LPS>(); break;
    case 3: wait_vmcnt<3 * LPS>(); break;
    case 4: wait_vmcnt<(4 * LPS < 63 ? 4 * LPS : 63)>(); break;
    case 5: wait_vmcnt<(5 * LPS < 63 ? 5 * LPS : 63)>(); break;
    default: wait_vmcnt<(6 * LPS < 63 ? 6 * LPS : 63)>(); break;
  }
}

__device__ __forceinline__ void block_sync_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// Forward / dgrad epilogue shared by the implicit-GEMM kernels: SLAB = fp32
// split-K partials; else bf16 y (+ STATS: per-M-tile channel sum / sum of
// squares of exactly the stored bf16 values, one deterministic partial row
// per M tile, reduced through `smem`, which the caller no longer uses).
// ADD (!SLAB): y = bf16(acc + addend) with addend a bf16 [M][Cout] tensor passed
// through the (otherwise unused) slab pointer -- the dgrad of a 1x1 conv whose
// input also feeds a residual branch adds that branch's gradient in place of a
// separate elementwise pass (ops/conv.py).
template <int BM, int BN, bool STATS, bool SLAB, int WM, int WN, bool ADD = false>
__device__ __forceinline__ void conv_fwd_epilogue(const f32x4 (&acc)[BM / WM / 16][BN / WN / 16], const ConvGeom& g,
                                                  bf16_t* __restrict__ y, float* __restrict__ stats,
                                                  float* __restrict__ slab, int split, int tm, int m0, int n0,
                                                  char* smem, int pm_b0 = 0, int pm_pos = 0) {
  // position-major tiles (g.posm): logical row ml -> stored row (pm_b0 + ml - m0) * HW + pm_pos
  auto phys = [&](int ml) {
    return g.posm ? (pm_b0 + ml - m0) * (g.H * g.W) + pm_pos : (g.om ? om_row(g, ml) : ml);
  };
  constexpr int NT = 64 * WM * WN, TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  const int col_l = lane & 15, rq = lane >> 4;
  if constexpr (SLAB) {
    float* o = slab + (int64_t)split * g.M * g.Cout;
#pragma unroll
    for (int a = 0; a < FM; ++a)
#pragma unroll
      for (int b = 0; b < FN; ++b) {
        const int n = n0 + wn * TN + b * 16 + col_l;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * TM + a * 16 + rq * 4 + r;
          if (m < g.M && n < g.Cout) o[(int64_t)phys(m) * g.Cout + n] = acc[a][b][r];
        }
      }
  } else {
    float s1[FN], s2[FN];
#pragma unroll
    for (int b = 0; b < FN; ++b) { s1[b] = 0.f; s2[b] = 0.f; }
#pragma unroll
    for (int a = 0; a < FM; ++a) {
#pragma unroll
      for (int b = 0; b < FN; ++b) {
        const int n = n0 + wn * TN + b * 16 + col_l;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * TM + a * 16 + rq * 4 + r;
          float v0 = acc[a][b][r];
          const int64_t mo = (int64_t)phys(m) * g.Cout + n;
          if constexpr (ADD) {  // (ADD: stats carries the addend's optional mask bits, see conv_fwd_add)
            const uint8_t* mb = reinterpret_cast<const uint8_t*>(stats);
            if (m < g.M && n < g.Cout &&
                (mb == nullptr || ((mb[(int64_t)phys(m) * (g.Cout >> 3) + (n >> 3)] >> (n & 7)) & 1u)))
              v0 += bf16_to_f32(reinterpret_cast<const bf16_t*>(slab)[mo]);
          }
          const bf16_t hv = f32_to_bf16(v0);
          if (m < g.M && n < g.Cout) y[mo] = hv;
          if constexpr (STATS) {
            const float v = m < g.M ? bf16_to_f32(hv) : 0.f;  // statistics of exactly what is stored
            s1[b] += v;
            s2[b] += v * v;
          }
        }
      }
    }
    if constexpr (STATS) {
      __syncthreads();  // every wave done with the LDS ring (no DMA in flight: the K loop drained it)
      float* red = reinterpret_cast<float*>(smem);  // [WM][2][BN]
#pragma unroll
      for (int b = 0; b < FN; ++b) {
        s1[b] += __shfl_xor(s1[b], 16, 64);
        s1[b] += __shfl_xor(s1[b], 32, 64);
        s2[b] += __shfl_xor(s2[b], 16, 64);
        s2[b] += __shfl_xor(s2[b], 32, 64);
        if (rq == 0) {
          red[(wm * 2 + 0) * BN + wn * TN + b * 16 + col_l] = s1[b];
          red[(wm * 2 + 1) * BN + wn * TN + b * 16 + col_l] = s2[b];
        }
      }
      __syncthreads();
      for (int c = tid; c < BN; c += NT) {
        const int n = n0 + c;
        if (n < g.Cout) {
          float sa = 0.f, sb = 0.f;
#pragma unroll
          for (int q = 0; q < WM; ++q) { sa += red[(q * 2) * BN + c]; sb += red[(q * 2 + 1) * BN + c]; }
          put_stats(stats, tm, g.Cout, n, sa, sb);
        }
      }
    }
  }
}

// Inclusive sum over the 16 lanes of each DPP row: lane 15 of the row ends
// with the row total (row_shr 1, 2, 4, 8 with zero fill; fixed order).
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x111, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x112, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x114, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x118, 0xf, 0xf, true));
  return v;
}

// Transposed epilogue (region kernel, and the streaming kernel whenever its
// wave tile has an even number of N fragments).  The MFMAs compute C^T
// (weights as the A operand), so lane l holds, per 16-pixel M fragment a and
// N-fragment pair p, the 8 CONSECUTIVE channels n0 + wn*TN + 32p + 8*(l>>4) +
// 0..7 of pixel m0 + wm*TM + 16a + (l&15) (fragments 2p / 2p+1 hold channel
// quads 0..3 / 4..7, see the B row map b_frag_row): one 16-byte bf16 store (or
// two 16-byte fp32 slab stores) per (a, p) instead of 8 scattered 2-byte
// stores.  Measured on the ResNet-50 1x1 shapes (scripts/bench_gemm1x1.py):
// the write-heavy GEMMs (Cout = 4 Cin) ran at ~2.6 TB/s with the scattered
// stores vs ~5 TB/s for the read-heavy ones.  BN statistics: DPP row sums
// over the 16 pixels of a lane group, then a fixed-order sum over the WM wave
// rows through LDS (deterministic).  ADD: + a bf16 [M][Cout] addend (16-byte
// loads), passed through the slab pointer.
template <int BM, int BN, bool STATS, bool SLAB, int WM, int WN, int FM, int FN, bool ADD = false, int BNR = 0>
__device__ __forceinline__ void conv_fwd_epilogue_t(const f32x4 (&acc)[FM][FN], const ConvGeom& g,
                                                    bf16_t* __restrict__ y, float* __restrict__ stats,
                                                    float* __restrict__ slab, int split, int tm, int m0, int n0,
                                                    char* smem, int pm_b0 = 0, int pm_pos = 0,
                                                    const BnRedArgs br = BnRedArgs{}) {
  constexpr int NT = 64 * WM * WN, TM = BM / WM, TN = BN / WN, NP = FN / 2;
  static_assert(!(ADD && (SLAB || STATS)), "ADD: plain bf16 output only");
  constexpr bool BNRED = BNR != 0;
  static_assert(BNR == 0 || BNR == 1, "BNR 1: the pooled BN backward reduce");
  static_assert(!(BNRED && (SLAB || STATS || ADD)), "BNRED: plain bf16 output");
  static_assert(FN % 2 == 0, "N fragments pair up");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  const int nl = wn * TN + 8 * (lane >> 4);  // + 32p: local channel of the lane's 8-run
  float s1[NP][8], s2[NP][8];
#pragma unroll
  for (int q = 0; q < NP; ++q)
#pragma unroll
    for (int k = 0; k < 8; ++k) { s1[q][k] = 0.f; s2[q][k] = 0.f; }
  // vmcnt(0) before any output store: the k loop's trailing LDS-DMA (zero-fill
  // past nk, inline asm the compiler does not track) has landed, so the LDS-only
  // barriers of the statistics below need not wait for this tile's stores
  if constexpr ((STATS || BNRED) && !SLAB) __builtin_amdgcn_s_waitcnt(0x0F70);
  // BNRED: the lane's channels are fixed per q -- their BN coefficients once
  float rmu[BNRED ? NP : 1][8], ris[BNRED ? NP : 1][8], rsc[BNRED ? NP : 1][8], rsh[BNRED ? NP : 1][8];
  if constexpr (BNR == 1) {
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const int n = n0 + nl + 32 * q;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        rmu[q][k] = br.coef[n + k];
        ris[q][k] = br.coef[g.Cout + n + k];
        rsc[q][k] = br.coef[2 * g.Cout + n + k];
        rsh[q][k] = br.coef[3 * g.Cout + n + k];
      }
    }
  }
  // the stored row of fragment a (position-major tiles hold image pm_b0 + r at
  // output pixel pm_pos)
  auto row_of = [&](int a, bool& ok) {
    const int ml = m0 + wm * TM + a * 16 + (lane & 15);
    ok = ml < g.M;
    return g.posm ? (pm_b0 + ml - m0) * (g.H * g.W) + pm_pos : (g.om && ok ? om_row(g, ml) : ml);
  };
  // ADD (plain): every fragment's addend (and mask byte) loaded before the
  // first store -- y may alias it as far as the compiler knows, so a load left
  // in the loop below waits behind each store, one memory latency per
  // fragment: ResNet-50 c1 dgrads with the residual addend 827 vs 956 / 538 vs
  // 575 us per step (profiles/r5_resnet_bn_dgrad_ab.txt).  Not for BNR 1
  // (the CIFAR region dgrad's pool windows: 24.3 vs 23.7-24.0 us)
  constexpr bool PA = ADD && BNR == 0;
  uint4 pad_[PA ? FM : 1][PA ? NP : 1];
  unsigned padm_[PA ? FM : 1][PA ? NP : 1];
  if constexpr (PA) {
#pragma unroll
    for (int a = 0; a < FM; ++a) {
      bool ok;
      const int m = row_of(a, ok);
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        const int n = n0 + nl + 32 * q;
        const int64_t o = (int64_t)(ok ? m : 0) * g.Cout + n, ob = (int64_t)(ok ? m : 0) * (g.Cout >> 3) + (n >> 3);
        {
          // (ADD: stats carries the addend's optional mask bits, conv_fwd_add: the
          // residual gradient = dy of the BN + residual + ReLU, masked here)
          const uint8_t* mb = reinterpret_cast<const uint8_t*>(stats);
          pad_[a][q] = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(slab) + o);
          padm_[a][q] = mb != nullptr ? mb[ob] : 0xffu;
        }
      }
    }
  }
#pragma unroll
  for (int a = 0; a < FM; ++a) {
    bool ok;
    const int m = row_of(a, ok);
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const int n = n0 + nl + 32 * q;
      float v[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[j] = acc[a][2 * q][j]; v[4 + j] = acc[a][2 * q + 1][j]; }
      if constexpr (ADD) {
        if (ok) {
          const uint8_t* mb = reinterpret_cast<const uint8_t*>(stats);
          const uint4 ad = PA ? pad_[a][q]
                                    : *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(slab) +
                                                                      (int64_t)m * g.Cout + n);
          const unsigned bits = PA ? padm_[a][q] : (mb != nullptr ? mb[(int64_t)m * (g.Cout >> 3) + (n >> 3)] : 0xffu);
          const float a8[8] = {lo_bf16(ad.x), hi_bf16(ad.x), lo_bf16(ad.y), hi_bf16(ad.y),
                               lo_bf16(ad.z), hi_bf16(ad.z), lo_bf16(ad.w), hi_bf16(ad.w)};
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] += (bits >> k) & 1u ? a8[k] : 0.f;
        }
      }
      if constexpr (SLAB) {
        float* o = slab + ((int64_t)split * g.M + m) * g.Cout + n;
        if (ok) {
          *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
          *reinterpret_cast<float4*>(o + 4) = make_float4(v[4], v[5], v[6], v[7]);
        }
      } else {
        const uint4 pk = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                                    pack_bf16x2(v[6], v[7]));
        if (ok) *reinterpret_cast<uint4*>(y + (int64_t)m * g.Cout + n) = pk;
        if constexpr (BNR == 1) {
          if (ok) {
            // pooled pixel m = (b, oh, ow) of the [B][H][W] dgrad output; its window in y
            int rem, ow;
            const int b = fdivmod(m, g.H * g.W, g.inv_HW, rem);
            const int oh = fdivmod(rem, g.W, g.inv_W, ow);
            const int W2 = 2 * g.W;
            const bf16_t* base = br.y + ((int64_t)(b * 2 * g.H + 2 * oh) * W2 + 2 * ow) * g.Cout + n;
            const uint4 w0 = *reinterpret_cast<const uint4*>(base);
            const uint4 w1 = *reinterpret_cast<const uint4*>(base + g.Cout);
            const uint4 w2 = *reinterpret_cast<const uint4*>(base + (int64_t)W2 * g.Cout);
            const uint4 w3 = *reinterpret_cast<const uint4*>(base + (int64_t)W2 * g.Cout + g.Cout);
            const uint4 wv[4] = {w0, w1, w2, w3};
            const float gd[8] = {lo_bf16(pk.x), hi_bf16(pk.x), lo_bf16(pk.y), hi_bf16(pk.y),
                                 lo_bf16(pk.z), hi_bf16(pk.z), lo_bf16(pk.w), hi_bf16(pk.w)};
            float yv[4][8];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
              yv[w][0] = lo_bf16(wv[w].x); yv[w][1] = hi_bf16(wv[w].x); yv[w][2] = lo_bf16(wv[w].y);
              yv[w][3] = hi_bf16(wv[w].y); yv[w][4] = lo_bf16(wv[w].z); yv[w][5] = hi_bf16(wv[w].z);
              yv[w][6] = lo_bf16(wv[w].w); yv[w][7] = hi_bf16(wv[w].w);
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              float best = -INFINITY;
              int arg = 0;
#pragma unroll
              for (int w = 0; w < 4; ++w) {
                const float r = fmaxf(fmaf(rsc[q][k], yv[w][k], rsh[q][k]), 0.f);
                if (r > best) { best = r; arg = w; }
              }
#pragma unroll
              for (int w = 0; w < 4; ++w) {
                const float dz = (w == arg && best > 0.f) ? gd[k] : 0.f;
                s1[q][k] += dz;
                s2[q][k] += dz * (yv[w][k] - rmu[q][k]) * ris[q][k];
              }
            }
          }
        }
        if constexpr (STATS) {
          const float h[8] = {lo_bf16(pk.x), hi_bf16(pk.x), lo_bf16(pk.y), hi_bf16(pk.y),
                              lo_bf16(pk.z), hi_bf16(pk.z), lo_bf16(pk.w), hi_bf16(pk.w)};
#pragma unroll
          for (int k = 0; k < 8; ++k) {  // statistics of exactly what is stored
            const float hv = ok ? h[k] : 0.f;
            s1[q][k] += hv;
            s2[q][k] += hv * hv;
          }
        }
      }
    }
  }
  if constexpr ((STATS || BNRED) && !SLAB) {
#pragma unroll
    for (int q = 0; q < NP; ++q)
#pragma unroll
      for (int k = 0; k < 8; ++k) { s1[q][k] = row16_sum(s1[q][k]); s2[q][k] = row16_sum(s2[q][k]); }
    // LDS-only barriers: __syncthreads() would also wait for this wave's output
    // stores (vmcnt(0)) before the tile's statistics, exposing their latency per
    // tile.  No LDS-DMA is in flight (waited above); the ring's reads are lgkm.
    block_sync_lds();  // lgkmcnt(0) (a compiler memory fence) + barrier: every wave done with the ring
    float* red = reinterpret_cast<float*>(smem);  // [WM][2][BN]
    if ((lane & 15) == 15) {
#pragma unroll
      for (int q = 0; q < NP; ++q)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          red[(wm * 2 + 0) * BN + nl + 32 * q + k] = s1[q][k];
          red[(wm * 2 + 1) * BN + nl + 32 * q + k] = s2[q][k];
        }
    }
    block_sync_lds();
    for (int c = tid; c < BN; c += NT) {
      float sa = 0.f, sb = 0.f;
#pragma unroll
      for (int q = 0; q < WM; ++q) { sa += red[(q * 2) * BN + c]; sb += red[(q * 2 + 1) * BN + c]; }
      if constexpr (BNR == 1) {
        // sa = sum dz, sb = sum dz*xhat; atomic rows hold [dgamma; dbeta] (the reduce's layouts)
        if (g_red_atomic) put_stats(br.rows, tm, g.Cout, n0 + c, sb, sa);
        else put_stats(br.rows, tm, g.Cout, n0 + c, sa, sb);
      } else {
        put_stats(stats, tm, g.Cout, n0 + c, sa, sb);
      }
    }
  }
}

// B-tile chunk swizzle of the region kernel: conflict-free ds_read_b128 for
// its permuted fragment rows 8(i>>2) + 4b + (i&3) (and for identity rows)
__device__ __forceinline__ int swz_b(int row) { return ((row >> 1) ^ (row >> 3)) & 7; }

// B fragment row of lane group i (0..15) for N fragment b of a transposed
// (C^T) wave tile: fragment pair p = b/2 covers 32 channels, and lane group
// i>>2 reads channels 8(i>>2) + 4(b&1) + (i&3), so the accumulator lane of
// output row 4(l>>4)+r holds channel 32p + 8(l>>4) + 4(b&1) + r.
__device__ __forceinline__ int b_frag_row(int b, int i) { return 32 * (b >> 1) + 8 * (i >> 2) + 4 * (b & 1) + (i & 3); }

// In-launch split-K combine (FIX, conv_fwd_fix).  Every K slice of a tile
// publishes its fp32 partial tile write-through (sc1 16-byte buffer stores),
// drains its stores (every wave: s_waitcnt vmcnt(0)), and after a workgroup
// barrier one lane adds to the tile's arrival counter (relaxed, agent scope).
// The slice whose add returns splits - 1 is the reducer: it reads EVERY slice
// (its own included) with sc1 loads -- which bypass the CU's L1, so no acquire
// fence is needed -- and sums them in slice order, bitwise the sums of
// splitk_combine / combine_bwd_reduce; it then runs the plain bf16 epilogue
// (BN statistics, or the BN backward reduce of the block below).  The other
// slices exit.  Correct for any placement of a tile's slices over CUs and
// XCDs (cdna_hip_programming.md §5 "in-launch split-K reduction", §6
// Guideline 16: sc1 payload + drained stores + counter, sc1 loads): the
// separate combine launch and its ~1.5-2 us kernel boundary are gone.  The
// reducer resets the counter for the next launch (the counters start zeroed:
// a __device__ array).
__device__ int g_fix_cnt[1 << 16];
constexpr int kFixCnt = 1 << 16;

template <int BM, int BN, int WM, int WN, int FM, int FN>
__device__ __forceinline__ bool splitk_fixup(f32x4 (&acc)[FM][FN], const ConvGeom& g, float* __restrict__ slab,
                                             int split, int splits, int m0, int n0, int pm_b0, int pm_pos, int* cnt,
                                             char* smem) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  constexpr int TM = BM / WM, TN = BN / WN, NP = FN / 2;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  const int nl = wn * TN + 8 * (lane >> 4);
  const rsrc_t sr = make_rsrc(slab, (unsigned)((int64_t)splits * g.M * g.Cout * 4));
  unsigned off[FM][NP];  // byte offset of the lane's 8 channels in slice 0 (or kOOB: M tail)
#pragma unroll
  for (int a = 0; a < FM; ++a) {
    const int ml = m0 + wm * TM + a * 16 + (lane & 15);
    const int row = g.posm ? (pm_b0 + ml - m0) * (g.H * g.W) + pm_pos : ml;
#pragma unroll
    for (int q = 0; q < NP; ++q)
      off[a][q] = ml < g.M ? (unsigned)(((int64_t)row * g.Cout + n0 + nl + 32 * q) * 4) : kOOB;
  }
  const unsigned sstride = (unsigned)((int64_t)g.M * g.Cout * 4);
#pragma unroll
  for (int a = 0; a < FM; ++a)
#pragma unroll
    for (int q = 0; q < NP; ++q)
      if (off[a][q] != kOOB) {
        const unsigned o = off[a][q] + (unsigned)split * sstride;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[a][2 * q]), sr, (int)o, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[a][2 * q + 1]), sr, (int)(o + 16), 0, 16);
      }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its slice is out of the CU
  __syncthreads();
  int* flag = reinterpret_cast<int*>(smem);  // the k loop is done with the ring (barrier above)
  if (tid == 0) {
    const int t = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == splits - 1 ? 1 : 0;
    if (last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag[0] = last;
  }
  __syncthreads();
  const int last = flag[0];
  __syncthreads();  // flag read by every wave before the epilogue reuses the LDS
  if (!last) return false;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction) keep the loads below the counter
  if (splits <= 4) {
    // the other slices only (the reducer's own is in registers): up to 3 loads
    // per fragment half, all in flight; unconditional (a slice index past the
    // others re-reads the last one and is not used)
    u32x4 ld[3][FM][NP][2];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int o_s = min(u < split ? u : u + 1, splits - 1);  // u-th slice other than `split`
      const unsigned so = (unsigned)o_s * sstride;
#pragma unroll
      for (int a = 0; a < FM; ++a)
#pragma unroll
        for (int q = 0; q < NP; ++q) {
          const unsigned o = off[a][q] == kOOB ? kOOB : off[a][q] + so;
          ld[u][a][q][0] = __builtin_amdgcn_raw_buffer_load_b128(sr, (int)o, 0, 16);
          ld[u][a][q][1] = __builtin_amdgcn_raw_buffer_load_b128(sr, (int)(o + 16), 0, 16);
        }
    }
#pragma unroll
    for (int a = 0; a < FM; ++a)
#pragma unroll
      for (int q = 0; q < NP; ++q)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4 own = acc[a][2 * q + h];
          f32x4 d = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < 4; ++s) {  // slice order; selects on values, never on loads
            const f32x4 lo = __builtin_bit_cast(f32x4, ld[s < 3 ? s : 2][a][q][h]);
            const f32x4 hi = __builtin_bit_cast(f32x4, ld[s > 0 ? s - 1 : 0][a][q][h]);
            const f32x4 x = s < split ? lo : (s == split ? own : hi);
            if (s == 0) d = x;  // (0 + x would turn -0 into +0)
            else if (s < splits) d = f32x4{d[0] + x[0], d[1] + x[1], d[2] + x[2], d[3] + x[3]};
          }
          acc[a][2 * q + h] = d;
        }
    return true;
  }
  // more slices: every slice (its own re-read), 4 at a time with all their loads in flight
#pragma unroll
  for (int a = 0; a < FM; ++a)
#pragma unroll
    for (int b = 0; b < FN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int s0 = 0; s0 < splits; s0 += 4) {
    u32x4 ld[4][FM][NP][2];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const unsigned so = (unsigned)min(s0 + u, splits - 1) * sstride;
#pragma unroll
      for (int a = 0; a < FM; ++a)
#pragma unroll
        for (int q = 0; q < NP; ++q) {
          const unsigned o = off[a][q] == kOOB ? kOOB : off[a][q] + so;
          ld[u][a][q][0] = __builtin_amdgcn_raw_buffer_load_b128(sr, (int)o, 0, 16);
          ld[u][a][q][1] = __builtin_amdgcn_raw_buffer_load_b128(sr, (int)(o + 16), 0, 16);
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool use = s0 + u < splits;
#pragma unroll
      for (int a = 0; a < FM; ++a)
#pragma unroll
        for (int q = 0; q < NP; ++q)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const f32x4 v = __builtin_bit_cast(f32x4, ld[u][a][q][h]);
            f32x4& d = acc[a][2 * q + h];
            if (s0 + u == 0) d = v;
            else if (use) d = f32x4{d[0] + v[0], d[1] + v[1], d[2] + v[2], d[3] + v[3]};
          }
    }
  }
  return true;
}

// --------------------------------------------------------------------------
// forward / dgrad implicit GEMM, split-K capable
//   C[m][n] = sum_{k in split} im2col(x)[m][k] * w[n][k]
//   splits == 1: bf16 y (+ BN partial sums per M tile)   splits > 1: fp32 slab[split][M][N]
// 256 threads = 4 waves (2 x 2), wave tile (BM/2) x (BN/2), BK = 64,
// 3-stage LDS ring filled by LDS-DMA, one barrier per K step.
// --------------------------------------------------------------------------
// FIX: split-K with the in-launch combine (splitk_fixup): `slab` holds the
// slices, the reducer of each tile runs the plain (STATS / BNR) epilogue;
// fixcnt = the launch's per-tile arrival counters.
template <int BM, int BN, bool STATS, bool SLAB, bool TAPU, int STAGES, int WM = 2, int WN = 2, bool ADD = false,
          bool TRP = true, int BNR = 0, bool FIX = false>
__global__ void __launch_bounds__(64 * WM * WN) conv_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                       bf16_t* __restrict__ y, float* __restrict__ stats,
                                                       float* __restrict__ slab, const ConvGeom g, int splits,
                                                       int kt_per_split, unsigned long long* dbg,
                                                       const BnRedArgs br = BnRedArgs{},
                                                       const SgdJob side = SgdJob{},
                                                       int* __restrict__ fixcnt = nullptr) {
  // side job (set_conv_side_sgd): the last side.nblk workgroups run part of
  // the step's SGD update on the CUs the convolution's one-workgroup-per-CU
  // grid leaves free (its gradients are final by the time this conv runs)
  const int conv_grid = (int)gridDim.x - side.nblk;
  if ((int)blockIdx.x >= conv_grid) {
    sgd_side_block(side, (int)blockIdx.x - conv_grid);
    return;
  }
  // x is the SPATIALLY ZERO-PADDED input [B][Hp][Wp][Cin]: every tap of every
  // output pixel is in bounds, so an activation load is (per-lane pixel base)
  // + (wave-uniform tap offset) with no bounds test.  Cout % BN == 0
  // (host-checked); rows of an M tail load a valid pixel and are masked out
  // of the stores and BN statistics.
  const unsigned long long t_start = dbg ? stamp() : 0ull;
  constexpr int BK = 64, CPR = 8, NW = WM * WN, PD = STAGES - 1;
  static_assert(STAGES >= 2 && STAGES <= 4, "2..4 stages");
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int A_INS = A_BYTES / 1024 / NW, B_INS = B_BYTES / 1024 / NW;  // glds per wave per stage
  constexpr int LPS = A_INS + B_INS;
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  // transposed accumulators (16-byte epilogue stores) unless FN is odd (TRP = false: the old layout)
  constexpr bool TR = TRP && FN % 2 == 0;
  static_assert(A_INS >= 1 && B_INS >= 1, "tile too small");
  static_assert(A_INS * NW * 1024 == A_BYTES && B_INS * NW * 1024 == B_BYTES, "DMA split");
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE_BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int ntm = (g.M + BM - 1) / BM;
  // Panel-major order: the workgroups of one XCD (consecutive ids after the
  // swizzle) share one (n-tile, K-split) weight panel and sweep the M tiles,
  // so the panel is fetched into that XCD's L2 once instead of every XCD
  // streaming the whole weight tensor from the Infinity Cache.
  // (M-tile-major measured 0.8 % slower, r2_fwd_order_ab.txt; per-pixel
  // balanced position-major split-K no faster, r2_posm_balance_ab.txt: both
  // removed in round 6)
  const int npanel = (g.Cout / BN) * splits;
  const int id = xcd_swizzle(blockIdx.x, ntm * npanel);
  const int tm = id % ntm;
  const int panel = id / ntm;
  const int split = panel % splits;
  const int tn = panel / splits;
  const int m0 = tm * BM, n0 = tn * BN;
  const int C8 = 1 << g.logC8;
  // Position-major tiles (g.posm, host-enabled for TAPU layers whose output is
  // smaller than twice the kernel, B % BM == 0): M tile tm holds images b0..b0+BM-1
  // at ONE output pixel, so every row of the tile has the same valid taps and
  // the taps that only read the zero border are skipped (4x4 output, 5x5
  // kernel: 9-16 of 25 taps per pixel).  K steps are split evenly per tile.
  int pm_b0 = 0, pm_pos = 0, kh0 = 0, kh1 = g.KS, kw0 = 0, kw1 = g.KS;
  int nkt_total = (g.Kch + CPR - 1) / CPR, ktps = kt_per_split;
  if (TAPU && g.posm) {
    const int nbt = g.B / BM;
    pm_pos = tm / nbt;
    pm_b0 = (tm - pm_pos * nbt) * BM;
    const int oh = pm_pos / g.W, ow = pm_pos - oh * g.W;
    kh0 = max(0, g.pad - oh);
    kh1 = min(g.KS, g.H + g.pad - oh);
    kw0 = max(0, g.pad - ow);
    kw1 = min(g.KS, g.W + g.pad - ow);
    nkt_total = (kh1 - kh0) * (kw1 - kw0) * (g.Cin / BK);
    ktps = (nkt_total + splits - 1) / splits;
  }
  const int kt_beg = split * ktps;
  const int kt_end = min(nkt_total, kt_beg + ktps);
  const int nk = max(0, kt_end - kt_beg);

  // per-lane source roles (fixed over the K loop); 32-bit element offsets.
  // A: instruction j of this wave covers rows 8*(wid*A_INS + j) .. +7;
  //    a_base = padded pixel of tap (0,0) of output pixel m (+ chunk for TAPU)
  int a_base[A_INS], a_ch[A_INS];
#pragma unroll
  for (int j = 0; j < A_INS; ++j) {
    const int row = 8 * (wid * A_INS + j) + (lane >> 3);
    a_ch[j] = (lane & 7) ^ ((row >> 1) & 7);
    const int m = (TAPU && g.posm) ? (pm_b0 + row) * (g.H * g.W) + pm_pos
                                   : min(m0 + row, g.M - 1);  // M tail: any valid pixel (masked in the epilogue)
    a_base[j] = out_pix(g, m) * g.Cin + (TAPU ? a_ch[j] * 8 : 0);
  }
  int b_off[B_INS], b_k[B_INS];
#pragma unroll
  for (int j = 0; j < B_INS; ++j) {
    const int row = 8 * (wid * B_INS + j) + (lane >> 3);
    const int ch = (lane & 7) ^ swz_b(row);
    b_k[j] = ch * 8;
    b_off[j] = (n0 + row) * g.K + ch * 8;
  }
  const rsrc_t xr = make_rsrc(x, (unsigned)((int64_t)g.B * g.Hp * g.Wp * g.Cin * 2));
  const rsrc_t wr = make_rsrc(w, (unsigned)((int64_t)g.Cout * g.K * 2));

  // Wave-uniform tap state of the next K step to load (TAPU: one step = 64
  // channels of one tap): off = (kh*Wp + kw)*Cin + c0 (activation), wk =
  // (kh*KS + kw)*Cin + c0 (weight column), advanced incrementally (no
  // divisions in the loop).
  struct Tap { int off, c0, kw, kh, wk; };
  Tap tnext{0, 0, 0, 0, 0};
  if constexpr (TAPU) {
    int kh, kw;
    if (g.posm) {
      const int chunks = g.Cin / BK, t = kt_beg / chunks, nkw = kw1 - kw0;
      tnext.c0 = (kt_beg - t * chunks) * BK;
      kh = kh0 + t / nkw;
      kw = kw0 + (t - (t / nkw) * nkw);
    } else {
      const int k0 = kt_beg * BK;
      const int kpos = k0 >> (g.logC8 + 3);
      kh = kpos / g.KW;
      kw = kpos - kh * g.KW;
      tnext.c0 = k0 & (g.Cin - 1);
    }
    tnext.kw = kw;
    tnext.kh = kh;
    tnext.off = (kh * g.Wp + kw) * g.Cin + tnext.c0;
    tnext.wk = (kh * g.KW + kw) * g.Cin + tnext.c0;
  }
  auto tap_advance = [&](Tap& t) {
    if constexpr (TAPU) {
      t.off += BK;
      t.wk += BK;
      t.c0 += BK;
      if (t.c0 == g.Cin) {
        t.c0 = 0;
        if (g.posm) {  // next valid tap of the tile's window
          if (++t.kw == kw1) { t.kw = kw0; ++t.kh; }
          t.off = (t.kh * g.Wp + t.kw) * g.Cin;
          t.wk = (t.kh * g.KS + t.kw) * g.Cin;
        } else if (++t.kw == g.KW) {
          t.kw = 0;
          t.off += (g.Wp - g.KW) * g.Cin;
        }
      }
    }
  };
  // One LDS-DMA load (q < A_INS: activation row block, else weight row block)
  // of K step kt into ring slot `slot`.
  auto issue_one = [&](int q, int kt, int slot, const Tap& t) {
    char* sA = smem + slot * STAGE_BYTES;
    char* sB = sA + A_BYTES;
    if (q < A_INS) {
      const int j = q;
      if constexpr (TAPU) {
        blds16(xr, 2u * (unsigned)a_base[j], 2u * (unsigned)t.off, sA + (wid * A_INS + j) * 1024);
      } else {
        // first layer (Cin < 64): a 64-wide K step spans several taps, per lane
        const int kc = kt * CPR + a_ch[j];
        const int kpos = kc >> g.logC8;
        const int c0 = (kc & (C8 - 1)) << 3;
        const int kh = kpos / g.KW, kw = kpos - kh * g.KW;
        const unsigned off = kc < g.Kch ? 2u * (unsigned)(a_base[j] + (kh * g.Wp + kw) * g.Cin + c0) : kOOB;
        blds16(xr, off, 0u, sA + (wid * A_INS + j) * 1024);
      }
    } else {
      const int j = q - A_INS;
      const int kadd = TAPU ? t.wk : kt * BK;
      unsigned voff = 2u * (unsigned)b_off[j];
      if constexpr (!TAPU) voff = (kadd + b_k[j]) < g.K ? voff : kOOB;  // K tail (first layer only)
      blds16(wr, voff, 2u * (unsigned)kadd, sB + (wid * B_INS + j) * 1024);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const unsigned long long t_setup = dbg ? stamp() : 0ull;
  // Fragment-prefetch pipeline (g_fwd_pf, STAGES >= 3): every step issues one
  // stage unconditionally (zero-fill past nk keeps the vmcnt count constant),
  // right after the barrier and before the fragment reads (asm DMA: the reads
  // cannot be hoisted above it, and hipcc's LDS-DMA alias waits stay out);
  // the fragments of step i+1 are read while the MFMAs of step i run.  The
  // plain loop below read each step's fragments and waited for them before
  // its first MFMA: the LDS latency was exposed at every step.
  // (4 stages: two in flight beyond the one being read; at 3 the step waited
  // for the stage issued one step earlier: 0.352 vs 0.341 ms/step, at 4 0.336)
  bool done = false;
  if constexpr (STAGES >= 4) {
    if (g_fwd_pf) {
      done = true;
      const i32x4 xr4 = make_rsrc4(x, (unsigned)((int64_t)g.B * g.Hp * g.Wp * g.Cin * 2));
      const i32x4 wr4 = make_rsrc4(w, (unsigned)((int64_t)g.Cout * g.K * 2));
      auto issue_stage = [&](int kt, int slot, bool valid) {
        char* sA = smem + slot * STAGE_BYTES;
        char* sB = sA + A_BYTES;
#pragma unroll
        for (int j = 0; j < A_INS; ++j) {
          if constexpr (TAPU) {
            blds16_asm(xr4, valid ? 2u * (unsigned)a_base[j] : kOOB, valid ? 2u * (unsigned)tnext.off : 0u,
                       sA + (wid * A_INS + j) * 1024);
          } else {
            const int kc = kt * CPR + a_ch[j];
            const int kpos = kc >> g.logC8;
            const int c0 = (kc & (C8 - 1)) << 3;
            const int kh = kpos / g.KW, kw = kpos - kh * g.KW;
            const unsigned off =
                (valid && kc < g.Kch) ? 2u * (unsigned)(a_base[j] + (kh * g.Wp + kw) * g.Cin + c0) : kOOB;
            blds16_asm(xr4, off, 0u, sA + (wid * A_INS + j) * 1024);
          }
        }
#pragma unroll
        for (int j = 0; j < B_INS; ++j) {
          const int kadd = TAPU ? tnext.wk : kt * BK;
          unsigned voff = 2u * (unsigned)b_off[j];
          if constexpr (!TAPU) voff = (kadd + b_k[j]) < g.K ? voff : kOOB;
          blds16_asm(wr4, valid ? voff : kOOB, valid ? 2u * (unsigned)kadd : 0u, sB + (wid * B_INS + j) * 1024);
        }
        if (valid) tap_advance(tnext);
      };
      auto read_frags = [&](int slot, bf16x8 (&af)[BK / 32][FM], bf16x8 (&bfr)[BK / 32][FN]) {
        const uint4* As = reinterpret_cast<const uint4*>(smem + slot * STAGE_BYTES);
        const uint4* Bs = reinterpret_cast<const uint4*>(smem + slot * STAGE_BYTES + A_BYTES);
#pragma unroll
        for (int kk = 0; kk < BK / 32; ++kk) {
          const int ch = kk * 4 + (lane >> 4);
#pragma unroll
          for (int a = 0; a < FM; ++a)
            af[kk][a] = __builtin_bit_cast(bf16x8, As[swz_row<CPR>(wm * TM + a * 16 + (lane & 15), ch)]);
#pragma unroll
          for (int b = 0; b < FN; ++b) {
            const int row = wn * TN + (TR ? b_frag_row(b, lane & 15) : b * 16 + (lane & 15));
            bfr[kk][b] = __builtin_bit_cast(bf16x8, Bs[row * CPR + (ch ^ swz_b(row))]);
          }
        }
      };
#pragma unroll
      for (int p = 0; p < PD; ++p) issue_stage(kt_beg + p, p, p < nk);
      constexpr int NRD = (BK / 32) * (FM + FN);  // ds_read_b128 per step
      constexpr int NMF = (BK / 32) * FM * FN;
      bf16x8 fa0[BK / 32][FM], fb0[BK / 32][FN], fa1[BK / 32][FM], fb1[BK / 32][FN];
      wait_vmcnt<(PD - 1) * LPS>();  // stage 0 landed
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      read_frags(0, fa0, fb0);
      int kt_next = kt_beg + PD, slot_n = PD % STAGES, slot_r = 1 % STAGES;
      auto step = [&](int i, bf16x8 (&fca)[BK / 32][FM], bf16x8 (&fcb)[BK / 32][FN], bf16x8 (&fna)[BK / 32][FM],
                      bf16x8 (&fnb)[BK / 32][FN]) {
        wait_vmcnt<(PD - 2) * LPS>();        // stage i+1 landed
        __builtin_amdgcn_s_waitcnt(0xC07F);  // step i's fragments in registers
        __builtin_amdgcn_s_barrier();        // every wave done reading slot i-1
        __builtin_amdgcn_sched_barrier(0);
        issue_stage(kt_next, slot_n, i + PD < nk);
        ++kt_next;
        slot_n = slot_n + 1 == STAGES ? 0 : slot_n + 1;
        __builtin_amdgcn_sched_barrier(0);
        read_frags(slot_r, fna, fnb);  // (past nk: zeros, never used)
        slot_r = slot_r + 1 == STAGES ? 0 : slot_r + 1;
#pragma unroll
        for (int kk = 0; kk < BK / 32; ++kk)
#pragma unroll
          for (int a = 0; a < FM; ++a)
#pragma unroll
            for (int b = 0; b < FN; ++b)
              acc[a][b] = TR ? mfma16(fcb[kk][b], fca[kk][a], acc[a][b]) : mfma16(fca[kk][a], fcb[kk][b], acc[a][b]);
        constexpr int P1 = NRD < NMF ? NRD : NMF;  // (MFMA, read) pairs
#pragma unroll
        for (int q = 0; q < P1; ++q) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        if constexpr (NRD > P1) __builtin_amdgcn_sched_group_barrier(0x100, NRD - P1, 0);
        if constexpr (NMF > P1) __builtin_amdgcn_sched_group_barrier(0x008, NMF - P1, 0);
        __builtin_amdgcn_sched_barrier(0);
      };
      int i = 0;
      for (; i + 1 < nk; i += 2) {
        step(i, fa0, fb0, fa1, fb1);
        step(i + 1, fa1, fb1, fa0, fb0);
      }
      if (i < nk) step(i, fa0, fb0, fa1, fb1);
      wait_vmcnt<0>();  // the trailing zero-fill DMAs still target the ring (the epilogue reuses it)
    }
  }
  if (!done) {
#pragma unroll
    for (int p = 0; p < PD; ++p)
      if (p < nk) {
#pragma unroll
        for (int q = 0; q < LPS; ++q) issue_one(q, kt_beg + p, p, tnext);
        tap_advance(tnext);
      }
    // MFMAs per K step and the spacing of the next stage's DMA issues between them
    constexpr int NMF = (BK / 32) * FM * FN;
    constexpr int IL = NMF / LPS > 0 ? NMF / LPS : 1;
    int slot_c = 0, slot_n = PD % STAGES;
    auto kstep = [&](int i) {
      block_sync_lds();  // stage i landed for every wave; slot (i+PD)%STAGES no longer read
      const bool pf = i + PD < nk;
      const int kt_n = kt_beg + i + PD;
      const uint4* As = reinterpret_cast<const uint4*>(smem + slot_c * STAGE_BYTES);
      const uint4* Bs = reinterpret_cast<const uint4*>(smem + slot_c * STAGE_BYTES + A_BYTES);
      bf16x8 af[BK / 32][FM], bfr[BK / 32][FN];
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        const int ch = kk * 4 + (lane >> 4);
#pragma unroll
        for (int a = 0; a < FM; ++a)
          af[kk][a] = __builtin_bit_cast(bf16x8, As[swz_row<CPR>(wm * TM + a * 16 + (lane & 15), ch)]);
#pragma unroll
        for (int b = 0; b < FN; ++b) {
          const int row = wn * TN + (TR ? b_frag_row(b, lane & 15) : b * 16 + (lane & 15));
          bfr[kk][b] = __builtin_bit_cast(bf16x8, Bs[row * CPR + (ch ^ swz_b(row))]);
        }
      }
      // the next stage's LDS-DMA issues ride between the MFMAs (their issue cost
      // overlaps matrix-core execution instead of serialising in front of it)
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk)
#pragma unroll
        for (int a = 0; a < FM; ++a)
#pragma unroll
          for (int b = 0; b < FN; ++b) {
            acc[a][b] = TR ? mfma16(bfr[kk][b], af[kk][a], acc[a][b]) : mfma16(af[kk][a], bfr[kk][b], acc[a][b]);
            const int idx = (kk * FM + a) * FN + b;
            if (idx % IL == IL - 1 && idx / IL < LPS) {
              if (pf) issue_one(idx / IL, kt_n, slot_n, tnext);
              __builtin_amdgcn_sched_barrier(0);
            }
          }
      if (pf) tap_advance(tnext);
      slot_c = slot_c + 1 == STAGES ? 0 : slot_c + 1;
      slot_n = slot_n + 1 == STAGES ? 0 : slot_n + 1;
    };
    // steady state (constant wait: stage i landed, PD-1 younger stages in flight), then the drain
    int i = 0;
    for (; i < nk - (PD - 1); ++i) {
      wait_vmcnt<(PD - 1) * LPS>();
      kstep(i);
    }
    for (; i < nk; ++i) {
      wait_stages<LPS>(nk - 1 - i);
      kstep(i);
    }

  }

  const unsigned long long t_loop = dbg ? stamp() : 0ull;
  auto dbg_out = [&]() {
    if (dbg && threadIdx.x == 0) {
      unsigned long long* d = dbg + (size_t)blockIdx.x * 4;
      d[0] = t_start; d[1] = t_setup; d[2] = t_loop; d[3] = stamp();
    }
  };
  static_assert(BNR == 0 || TR, "the fused BN reduce needs the transposed epilogue");
  if constexpr (FIX) {
    static_assert(TR && !SLAB && !ADD, "FIX: transposed plain epilogue after the in-launch combine");
    if (!splitk_fixup<BM, BN, WM, WN, FM, FN>(acc, g, slab, split, splits, m0, n0, pm_b0, pm_pos, fixcnt + tn * ntm + tm,
                                              smem)) {
      dbg_out();
      return;
    }
  }
  if constexpr (TR)
    conv_fwd_epilogue_t<BM, BN, STATS, SLAB, WM, WN, FM, FN, ADD, BNR>(acc, g, y, stats, slab, split, tm, m0, n0, smem,
                                                                       pm_b0, pm_pos, br);
  else
    conv_fwd_epilogue<BM, BN, STATS, SLAB, WM, WN, ADD>(acc, g, y, stats, slab, split, tm, m0, n0, smem, pm_b0,
                                                        pm_pos);
  dbg_out();
}

// --------------------------------------------------------------------------
// forward / dgrad implicit GEMM with the activation REGION resident in LDS
// (tap reuse).  The generic kernel above streams the A operand tap by tap:
// each of the KS*KS k-steps of a 64-channel chunk re-reads an almost
// identical shifted window of the input through the L2 -> LDS path, which is
// what bounds it (~25 B/clk/CU of LDS-DMA fill).  Here a workgroup's M tile
// (BM = 128 output pixels = whole output rows of one image, or whole images)
// loads the padded input pixels it touches ONCE per 64-channel chunk, and
// every tap reads its A fragments from that region at a wave-uniform offset;
// only the weight tile (B) is streamed per k-step (3-stage LDS-DMA ring).
// Fill bytes per FLOP drop ~1.8-2.6x.
//
// Region image: pixel-major, S = 10 16-byte slots per pixel (8 data + 2 pad),
// row stride RS = RW*S + RP slots, image stride IS = RH*RS (host-chosen, see
// region_geom): with these paddings the ds_read_b128 fragment reads of 16
// output pixels are bank-conflict free for W = 4, 8, 16, 32 at every tap,
// and a tap is a plain address offset (no per-tap swizzle arithmetic).
// Pad slots are loaded from an out-of-range offset (zeros, no traffic).
// --------------------------------------------------------------------------
struct RegionGeom {
  int S, RS, IS;    // slots per pixel / region row / region image
  int RW, RH;       // region row width (= Wp) and rows per region image
  int nimg;         // images per region (rows mode: 1)
  int rows_mode;    // 1: M tile = BM/W output rows of one image; 0: BM/HW whole images
  int nslot;        // slots per region (multiple of 64)
  int cpw;          // 64-channel chunks per workgroup (1 or 2)
  float inv_S, inv_RS, inv_IS;  // exact slot -> (img,row,col,chunk) decomposition (slots < 2^16)
};


template <int BN, bool STATS, bool SLAB, int STAGES, int WM, int WN, bool BNRED = false>
__global__ void __launch_bounds__(64 * WM * WN) conv_fwd_region_kernel(const bf16_t* __restrict__ x,
                                                              const bf16_t* __restrict__ w, bf16_t* __restrict__ y,
                                                              float* __restrict__ stats, float* __restrict__ slab,
                                                              const ConvGeom g, const RegionGeom rg, int splits,
                                                              unsigned long long* dbg, int ablate,
                                                              const BnRedArgs br) {
  const unsigned long long t_start = dbg ? stamp() : 0ull;
  constexpr int BM = 128, BK = 64, CPR = 8, NW = WM * WN, PD = STAGES - 1;
  constexpr int B_BYTES = BN * BK * 2, B_INS = B_BYTES / 1024 / NW, LPS = B_INS;
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  static_assert(B_INS >= 1 && B_INS * NW * 1024 == B_BYTES, "B DMA split");
  static_assert(FN % 2 == 0, "the 16-byte epilogue pairs N fragments");
  static_assert(STAGES >= 3, "fragment prefetch needs >= 3 ring slots");
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int region_bytes = rg.nslot * 16;
  char* sR = smem;                          // cpw region images
  char* sB = smem + rg.cpw * region_bytes;  // B ring

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int ntm = (g.M + BM - 1) / BM;
  const int npanel = (g.Cout / BN) * splits;
  const int id = xcd_swizzle(blockIdx.x, ntm * npanel);
  const int tm = id % ntm;
  const int panel = id / ntm;
  const int split = panel % splits, tn = panel / splits;
  const int m0 = tm * BM, n0 = tn * BN;
  const int HW = 1 << g.logHW, Wd = g.W;
  const int HpWp = g.Hp * g.Wp;
  const int taps = g.KS * g.KS;
  const int nk = rg.cpw * taps;
  const int img0 = m0 >> g.logHW, oh0 = (m0 & (HW - 1)) >> g.logW;  // oh0 = 0 in images mode
  const int start_pix = img0 * HpWp + oh0 * g.Wp;
  const rsrc_t xr = make_rsrc(x, (unsigned)((int64_t)g.B * HpWp * g.Cin * 2));
  const rsrc_t wr = make_rsrc(w, (unsigned)((int64_t)g.Cout * g.K * 2));
  const int cbase = split * rg.cpw;  // first 64-channel chunk of this workgroup

  // ---- region loads (once per chunk): lane-linear slots -> source pixel/chunk
  {
    const int nq = rg.nslot >> 6;
    // slot -> (region row R, pixel in row, chunk): the region's image rows
    // are consecutive padded rows (rows mode: RH rows of one image; images
    // mode: RH = Hp, whole images), so the source pixel is start + R*Wp + col
    const int nrows = rg.nimg * rg.RH;
    for (int q = wid; q < nq; q += NW) {
      const int sl = q * 64 + lane;
      const int R = (int)(((float)sl + 0.5f) * rg.inv_RS);
      const int r2 = sl - R * rg.RS;
      const int col = (r2 * 6554) >> 16;  // r2 / 10 (exact for r2 < 16384; S == 10)
      const int ch = r2 - col * 10;
      const bool ok = R < nrows && col < rg.RW && ch < 8;
      const int pix = start_pix + R * g.Wp + col;
      const unsigned voff = ok ? 2u * (unsigned)(pix * g.Cin + ch * 8) : kOOB;
      for (int c = 0; c < rg.cpw; ++c)
        blds16(xr, voff, 2u * (unsigned)((cbase + c) * 64), sR + c * region_bytes + q * 1024);
    }
  }
  // ---- B (weight) stream: k-step ks = (chunk c, tap t): k offset t*Cin + (cbase+c)*64
  int b_v[B_INS];
#pragma unroll
  for (int j = 0; j < B_INS; ++j) {
    const int row = 8 * (wid * B_INS + j) + (lane >> 3);
    const int ch = (lane & 7) ^ swz_b(row);
    b_v[j] = 2 * ((n0 + row) * g.K + ch * 8);
  }
  int ld_c = 0, ld_t = 0, ld_slot = 0;  // next k-step to load (wave-uniform)
  // Every step issues its DMA unconditionally (k-steps past the end load
  // zeros from an out-of-range offset into a slot nobody reads again), so the
  // number of loads in flight is the same at every wait and the loop body is
  // one basic block the scheduler can interleave.
  auto issue_b = [&](int q, bool live) {
    const unsigned soff = 2u * (unsigned)(ld_t * g.Cin + (cbase + ld_c) * 64);
    blds16(wr, live ? (unsigned)b_v[q] : kOOB, soff, sB + ld_slot * B_BYTES + (wid * B_INS + q) * 1024);
  };
  int ld_k = 0;
  auto advance_ld = [&]() {  // branch-free (keeps the step one basic block)
    ++ld_k;
    ++ld_t;
    const int wrap = ld_t == taps;
    ld_t -= wrap * taps;
    ld_c = min(ld_c + wrap, rg.cpw - 1);
    ++ld_slot;
    ld_slot -= (ld_slot == STAGES) * STAGES;
  };

  // ---- per-lane A fragment bases (slot of the tap-(0,0) pixel + lane's chunk)
  int a_base[FM];
#pragma unroll
  for (int a = 0; a < FM; ++a) {
    const int m = min(m0 + wm * TM + a * 16 + (lane & 15), g.M - 1);
    const int im = (m >> g.logHW) - img0;
    const int oh = ((m & (HW - 1)) >> g.logW) - oh0;
    const int ow = m & (Wd - 1);
    a_base[a] = (im * rg.IS + oh * rg.RS + ow * rg.S + (lane >> 4)) * 16;
  }
  // B fragment rows: N fragment b, MFMA row i -> channel
  // 32*(b>>1) + 8*(i>>2) + 4*(b&1) + (i&3) of the wave's TN channels (so a
  // lane's fragments 2p, 2p+1 cover 8 consecutive channels of the
  // transposed accumulator)
  int b_row[FN];
#pragma unroll
  for (int b = 0; b < FN; ++b) {
    const int i = lane & 15;
    b_row[b] = wn * TN + 32 * (b >> 1) + 8 * (i >> 2) + 4 * (b & 1) + (i & 3);
  }

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: region + PD B stages in flight
#pragma unroll
  for (int p = 0; p < PD; ++p) {
#pragma unroll
    for (int q = 0; q < LPS; ++q) issue_b(q, ld_k < nk);
    advance_ld();
  }
  const unsigned long long t_issued = dbg ? stamp() : 0ull;

  // fragment reads of k-step (rc, rkh, rkw) from ring slot rslot
  int rc = 0, rkh = 0, rkw = 0, rslot = 0;
  auto read_frags = [&](bf16x8 (&fa)[BK / 32][FM], bf16x8 (&fb)[BK / 32][FN]) {
    const char* As = sR + rc * region_bytes + (rkh * rg.RS + rkw * rg.S) * 16;  // wave-uniform tap offset
    const uint4* Bs = reinterpret_cast<const uint4*>(sB + rslot * B_BYTES);
    {  // advance the read state, branch-free
      ++rkw;
      const int ww = rkw == g.KS;
      rkw -= ww * g.KS;
      rkh += ww;
      const int wh = rkh == g.KS;
      rkh -= wh * g.KS;
      rc = min(rc + wh, rg.cpw - 1);
      ++rslot;
      rslot -= (rslot == STAGES) * STAGES;
    }
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int ch = kk * 4 + (lane >> 4);
#pragma unroll
      for (int b = 0; b < FN; ++b) fb[kk][b] = __builtin_bit_cast(bf16x8, Bs[b_row[b] * CPR + (ch ^ swz_b(b_row[b]))]);
#pragma unroll
      for (int a = 0; a < FM; ++a) fa[kk][a] = *reinterpret_cast<const bf16x8*>(As + a_base[a] + kk * 64);
    }
  };
  // Step i: [wait stage i+1, barrier] -> prefetch fragments of step i+1 ->
  // MFMAs of step i (C^T += W * X^T) with the DMA of stage i+PD (into the
  // slot read two steps ago), reads and MFMAs interleaved 1:1 so that a
  // read stalled on a full LDS queue never holds back more than one MFMA.
  constexpr int NRD = (BK / 32) * (FM + FN);  // fragment reads per step
  constexpr int NMF = (BK / 32) * FM * FN;    // MFMAs per step
  bf16x8 fa0[BK / 32][FM], fb0[BK / 32][FN], fa1[BK / 32][FM], fb1[BK / 32][FN];
  wait_vmcnt<(PD - 1) * LPS>();  // region + stage 0 landed
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t_first = dbg ? stamp() : 0ull;
  read_frags(fa0, fb0);
  auto step = [&](bf16x8 (&fca)[BK / 32][FM], bf16x8 (&fcb)[BK / 32][FN], bf16x8 (&fna)[BK / 32][FM],
                  bf16x8 (&fnb)[BK / 32][FN]) {
    wait_vmcnt<(PD - 2) * LPS>();  // stage i+1 landed (stages i+2 .. i+PD-1 may fly)
    // The fragments of step i must be in registers: the builtin wait is seen
    // by the compiler's waitcnt pass (an inline-asm one is not, and it would
    // then wait lgkmcnt(0) at the first MFMA, i.e. also for the prefetch).
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();        // stage i+1 visible to all waves; slot of step i-1 fully read
    __builtin_amdgcn_sched_barrier(0);
    const bool live = ld_k < nk;
    read_frags(fna, fnb);
#pragma unroll
    for (int q = 0; q < LPS; ++q) issue_b(q, live);
    advance_ld();
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk)
#pragma unroll
      for (int a = 0; a < FM; ++a)
#pragma unroll
        for (int b = 0; b < FN; ++b) acc[a][b] = mfma16(fcb[kk][b], fca[kk][a], acc[a][b]);
    // issue order: (MFMA, read) pairs, leftover reads, (MFMA, DMA) pairs, the rest
    constexpr int P1 = NRD < NMF ? NRD : NMF;
    constexpr int P2 = LPS < NMF - P1 ? LPS : NMF - P1;
#pragma unroll
    for (int q = 0; q < P1; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    if constexpr (NRD > P1) __builtin_amdgcn_sched_group_barrier(0x100, NRD - P1, 0);
#pragma unroll
    for (int q = 0; q < LPS; ++q) {
      if (q < P2) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    }
    if constexpr (NMF - P1 - P2 > 0) __builtin_amdgcn_sched_group_barrier(0x008, NMF - P1 - P2, 0);
  };
  int i = 0;
  for (; i + 1 < nk; i += 2) {
    step(fa0, fb0, fa1, fb1);
    step(fa1, fb1, fa0, fb0);
  }
  if (i < nk) step(fa0, fb0, fa1, fb1);
  const unsigned long long t_loop = dbg ? stamp() : 0ull;
  conv_fwd_epilogue_t<128, BN, STATS, SLAB, WM, WN, FM, FN, false, BNRED ? 1 : 0>(acc, g, y, stats, slab, split, tm,
                                                                                 m0, n0, smem, 0, 0, br);
  if (dbg && threadIdx.x == 0) {
    unsigned long long* d = dbg + (size_t)blockIdx.x * 5;
    d[0] = t_start; d[1] = t_issued; d[2] = t_first; d[3] = t_loop; d[4] = stamp();
  }
}

// s_waitcnt immediate (gfx9 encoding) for vmcnt(n), expcnt / lgkmcnt unconstrained
constexpr int vmcnt_imm(int n) { return (n & 15) | ((n >> 4) << 14) | 0x70 | 0xF00; }

// --------------------------------------------------------------------------
// First layer (Cin = 8 after the 3 -> 8 channel pad; K = KS*KS*8 = 200): the
// whole problem of a workgroup fits in LDS at once -- its 128 output pixels'
// padded input rows (16 B per pixel) and the 64 x K weight panel -- so it is
// one DMA burst, one barrier and ceil(K/32) MFMA steps; a 32-deep k-step
// covers 4 taps (lane group q = l>>4 reads tap 4s+q at its own pixel offset).
// The streaming kernel spent most of its time on per-lane tap arithmetic and
// on re-reading each input pixel through the L2 for 25 taps.
// Output: transposed accumulator -> conv_fwd_epilogue_t (16-byte stores, BN
// statistics per M tile).
// --------------------------------------------------------------------------
template <bool STATS, bool PAIR = false>
__global__ void __launch_bounds__(512) conv_fwd_c8_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                          bf16_t* __restrict__ y, float* __restrict__ stats,
                                                          const ConvGeom g, int region_rows, int mt,
                                                          unsigned long long* dbg) {
  // mt consecutive 128-pixel M tiles per workgroup (whole output rows of one
  // image): the weight panel (BN x taps x 16 B = 25.6 KiB for the reference's
  // layer 1) is DMA'd once per workgroup instead of once per tile, the region
  // covers the mt tiles' rows + the kernel halo, and the tiles are computed
  // one after the other from LDS (epilogue scratch after the region).
  constexpr int BM = 128, BN = 64, WM = 4, WN = 2, NW = 8, TM = 32, TN = 32, FM = 2, FN = 2;
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const unsigned long long t_start = dbg ? stamp() : 0;  // (set_conv_debug: phase stamps)
  // PAIR: the input has <= 4 real channels and the weights are pair-packed
  // (pack1_index, cp = -KS): one 16-byte K chunk = channels 0-3 of two
  // horizontally adjacent taps, read as the first 8 bytes of two adjacent
  // region pixels -- K = KS * ceil(KS/2) * 8 (120 for 5x5) instead of
  // KS * KS * 8 (200), 4 k-steps instead of 7 and a 15.4 instead of a 25.6 KiB
  // weight panel.  (The odd last tap's partner is a zero weight; the pixel it
  // reads is the next padded row's zero border, or a zero slot.)
  const int cpr = (g.KS + 1) >> 1;
  const int taps = PAIR ? g.KS * cpr : g.KS * g.KS;  // K chunks (16 B) per output channel
  const int nsteps = (taps + 3) / 4;                 // 32-deep k-steps (4 chunks each)
  const int rpix = region_rows * g.Wp;               // region pixels (PAIR: 8 B each, else 16 B)
  const int rslots = PAIR ? (rpix + 1) / 2 : rpix;   // 16-byte region slots
  const int rslots_p = (rslots + 2 + 63) / 64 * 64;  // + >= 2 zero slots, whole DMA pieces
  // weight panel: BN rows x taps 16-B chunks.  (Its B-fragment reads put rows
  // r and r+16 on the same banks; spreading them with 4 empty chunks per 16
  // rows measured no change -- the k loop is not LDS-bound, 12.96 vs 13.24 us,
  // profiles/r6_c8_stamps.txt.)
  const int wslots = BN * taps;
  const int wslots_p = (wslots + 63) / 64 * 64;
  char* sR = smem;
  char* sW = smem + rslots_p * 16;
  char* sX = sW + wslots_p * 16;  // epilogue scratch ([WM][2][BN] floats)

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int ntm = (g.M + BM - 1) / BM, ngr = ntm / mt;  // host: mt | ntm, mt * BM | H * W
  const int id = xcd_swizzle(blockIdx.x, ngr * (g.Cout / BN));
  const int tg = id % ngr, tn = id / ngr;
  const int mg0 = tg * mt * BM, n0 = tn * BN;
  const int HW = 1 << g.logHW;
  const int img0 = mg0 >> g.logHW, oh0 = (mg0 & (HW - 1)) >> g.logW;
  const int start_pix = (img0 * g.Hp + oh0) * g.Wp;
  const rsrc_t xr = make_rsrc(x, (unsigned)((int64_t)g.B * g.Hp * g.Wp * (PAIR ? 8 : 16)));
  const rsrc_t wr = make_rsrc(w, (unsigned)((int64_t)g.Cout * taps * 16));
  // one DMA burst: region pixels (contiguous padded rows) then the weight panel
  for (int q = wid; q < rslots_p / 64; q += NW) {
    const int sl = q * 64 + lane;
    blds16(xr, sl < rslots ? (PAIR ? 8u * (unsigned)start_pix + 16u * (unsigned)sl : 16u * (unsigned)(start_pix + sl))
                           : kOOB, 0u, sR + q * 1024);
  }
  for (int q = wid; q < wslots_p / 64; q += NW) {
    const int sl = q * 64 + lane;
    blds16(wr, sl < wslots ? 16u * (unsigned)(n0 * taps + sl) : kOOB, 0u, sW + q * 1024);
  }
  const int i = lane & 15, qg = lane >> 4;
  int b_row[FN];
#pragma unroll
  for (int b = 0; b < FN; ++b) b_row[b] = wn * TN + 8 * (i >> 2) + 4 * b + (i & 3);
  wait_vmcnt<0>();
  block_sync_lds();
  const unsigned long long t_dma = dbg ? stamp() : 0;
  unsigned long long t_mfma = 0;
  const int zero_slot = rslots;  // loaded from an out-of-range offset: zeros
  for (int t_ = 0; t_ < mt; ++t_) {
  const int tm = tg * mt + t_, m0 = tm * BM;
  int a_pix[FM];
#pragma unroll
  for (int a = 0; a < FM; ++a) {
    const int m = min(m0 + wm * TM + a * 16 + i, g.M - 1) - mg0;  // group-local output pixel
    a_pix[a] = (m >> g.logW) * g.Wp + (m & (g.W - 1));
  }
  f32x4 acc[FM][FN];
#pragma unroll
  for (int a = 0; a < FM; ++a)
#pragma unroll
    for (int b = 0; b < FN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int st = 0; st < nsteps; ++st) {
    const int t = 4 * st + qg;  // this lane group's tap (PAIR: tap pair)
    const int kh = PAIR ? t / cpr : t / g.KS, kw = PAIR ? 2 * (t - kh * cpr) : t - kh * g.KS;
    const int toff = kh * g.Wp + kw;
    bf16x8 fa[FM], fb[FN];
#pragma unroll
    for (int a = 0; a < FM; ++a) {
      if constexpr (PAIR) {  // 8-byte pixels: the chunk is pixels q, q+1 (two 8-byte-aligned reads)
        const int q = a_pix[a] + (t < taps ? toff : 0);
        const uint2 lo = *reinterpret_cast<const uint2*>(sR + q * 8);
        const uint2 hi = *reinterpret_cast<const uint2*>(sR + q * 8 + 8);
        const bool ok = t < taps;  // past the last chunk: zeros (the weights there are clamped, not zero)
        fa[a] = __builtin_bit_cast(bf16x8, make_uint4(ok ? lo.x : 0u, ok ? lo.y : 0u, ok ? hi.x : 0u, ok ? hi.y : 0u));
      } else {
        fa[a] = *reinterpret_cast<const bf16x8*>(sR + (t < taps ? a_pix[a] + toff : zero_slot) * 16);
      }
    }
#pragma unroll
    for (int b = 0; b < FN; ++b)
      fb[b] = *reinterpret_cast<const bf16x8*>(sW + (b_row[b] * taps + min(t, taps - 1)) * 16);
#pragma unroll
    for (int a = 0; a < FM; ++a)
#pragma unroll
      for (int b = 0; b < FN; ++b) acc[a][b] = mfma16(fb[b], fa[a], acc[a][b]);
  }
  if (dbg) t_mfma = stamp();
  conv_fwd_epilogue_t<128, BN, STATS, false, WM, WN, FM, FN>(acc, g, y, stats, nullptr, 0, tm, m0, n0, sX);
  }
  if (dbg && threadIdx.x == 0) {
    unsigned long long* d = dbg + (size_t)blockIdx.x * 4;
    d[0] = t_start; d[1] = t_dma; d[2] = t_mfma; d[3] = stamp();
  }
}

// split-K combine: y = bf16(sum_s slab[s]) (+ BN partial sums, one row per block)
template <bool STATS>
__global__ void __launch_bounds__(256) splitk_combine_kernel(const float* __restrict__ slab, bf16_t* __restrict__ y,
                                                             float* __restrict__ stats, int splits, int M, int N,
                                                             int rows_per_block, const ConvGeom g) {
  const int N8 = N >> 3;
  const int tpr = N8;                 // threads per row (one 8-column chunk each)
  const int rpi = 256 / tpr;          // rows per iteration
  const int c8 = threadIdx.x % tpr, rsub = threadIdx.x / tpr;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  float s1[8], s2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { s1[k] = 0.f; s2[k] = 0.f; }
  if (rsub < rpi) {
    for (int m = r0 + rsub; m < r1; m += rpi) {
      const int splits_m = splits;
      float v[8];
      const float* p = slab + (int64_t)m * N + c8 * 8;
      {
        const float4 a = *reinterpret_cast<const float4*>(p);
        const float4 b = *reinterpret_cast<const float4*>(p + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
      }
      // splits in batches of 4 with every load of a batch issued before the
      // first add (a load->add chain per split was latency-bound); the adds
      // keep the split order
      auto add8 = [&](const float4& a, const float4& b) {
        v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
      };
      int s = 1;
      for (; s + 3 < splits_m; s += 4) {
        float4 a[4], b[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float* q = p + (int64_t)(s + u) * M * N;
          a[u] = *reinterpret_cast<const float4*>(q);
          b[u] = *reinterpret_cast<const float4*>(q + 4);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) add8(a[u], b[u]);
      }
      for (; s < splits_m; ++s) {
        const float* q = p + (int64_t)s * M * N;
        add8(*reinterpret_cast<const float4*>(q), *reinterpret_cast<const float4*>(q + 4));
      }
      uint4 o;
      o.x = pack_bf16x2(v[0], v[1]); o.y = pack_bf16x2(v[2], v[3]);
      o.z = pack_bf16x2(v[4], v[5]); o.w = pack_bf16x2(v[6], v[7]);
      *reinterpret_cast<uint4*>(y + (int64_t)m * N + c8 * 8) = o;
      if constexpr (STATS) {
        const float h[8] = {lo_bf16(o.x), hi_bf16(o.x), lo_bf16(o.y), hi_bf16(o.y),
                            lo_bf16(o.z), hi_bf16(o.z), lo_bf16(o.w), hi_bf16(o.w)};
#pragma unroll
        for (int k = 0; k < 8; ++k) { s1[k] += h[k]; s2[k] += h[k] * h[k]; }
      }
    }
  }
  if constexpr (STATS) {
    __shared__ float red[256][17];
#pragma unroll
    for (int k = 0; k < 8; ++k) { red[threadIdx.x][k] = s1[k]; red[threadIdx.x][8 + k] = s2[k]; }
    __syncthreads();
    for (int c = threadIdx.x; c < N; c += 256) {
      const int ch = c >> 3, k = c & 7;
      float a = 0.f, b = 0.f;
      for (int t = ch; t < rpi * tpr; t += tpr) { a += red[t][k]; b += red[t][8 + k]; }
      put_stats(stats, blockIdx.x, N, c, a, b);
    }
  }
}

// --------------------------------------------------------------------------
// wgrad implicit GEMM: out[split][co][k] = sum_{m in split} dy[m][co] * im2col(x)[m][k]
// Tiles are staged [m][col] (rows = the reduction index) by LDS-DMA and read
// as MFMA operands with ds_read_b64_tr_b16.  BK = 64 rows of m per stage.
// --------------------------------------------------------------------------
// DL_WGRAD_STAMPS builds only (diagnostics): per-workgroup s_memtime phase
// sums of waves 0 and NW-1 -> [wg][2][6] = start, loop begin, sum of the
// steps' wait+barrier, sum of the steps' issue work, loop end, end
__device__ unsigned long long* g_wgrad_stamps = nullptr;

// (Removed in round 6 after losing their A/B: atomic split-K accumulation,
// r2_mode1_timeline.txt; 256x128 tiles, r3_wgrad_tile256_ab.txt; position-major
// steps, r5_wgrad_posm_ab.txt; the read-before-DMA loop order and the
// read-then-compute loop, r3_wgrad_order_ab.txt.)
template <int BM, int BN, int STAGES, int WM = 2, int WN = 2, int BK_ = 64>
__global__ void __launch_bounds__(64 * WM * WN) conv_wgrad_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                         float* __restrict__ out, const ConvGeom g, int m_per_split,
                                                         int ldo, const SgdJob side = SgdJob{}) {
  // side job (set_conv_side_sgd, as conv_fwd_kernel): the last side.nblk
  // workgroups run part of the step's SGD update beside the weight gradient
  const int wg_grid = (int)gridDim.x - side.nblk;
  if ((int)blockIdx.x >= wg_grid) {
    sgd_side_block(side, (int)blockIdx.x - wg_grid);
    return;
  }
  // dy and x are both spatially zero-padded [B][Hp][Wp][C] (dy: interior at
  // (pad, pad)).  A 64-row M step starts at a multiple of 64 output pixels;
  // with W | 64 and (H*W | 64 or 64 | H*W) the padded position of row r of the
  // step is U(step) + L(r): a wave-uniform part plus a per-lane constant, so
  // a load is one add, no bounds test (m_per_split % 64 == 0, Cout % BM == 0);
  // only a partial last step (M % 64 != 0) tests rows (wave-uniform branch).
  // BK_ = 32 (the 256x128 tile): 32-row steps, which start at multiples of 32
  // -- the host then needs W | 32 for the pow2 decomposition (H*W and 32 are
  // powers of two, so one divides the other)
  constexpr int BK = BK_, NW = WM * WN, PD = STAGES - 1;
  static_assert(BK == 32 || BK == 64, "32- or 64-row steps");
  static_assert(STAGES >= 2 && STAGES <= 8, "2..8 stages");
  constexpr int ACPR = BM / 8, BCPR = BN / 8;  // chunks per LDS row (row = one m)
  constexpr int A_BYTES = BK * BM * 2, B_BYTES = BK * BN * 2, STAGE_BYTES = A_BYTES + B_BYTES;
  constexpr int A_INS = A_BYTES / 1024 / NW, B_INS = B_BYTES / 1024 / NW;
  constexpr int LPS = A_INS + B_INS;
  constexpr int A_RPI = 64 / ACPR, B_RPI = 64 / BCPR;  // rows per glds instruction
  static_assert(A_INS * NW * 1024 == A_BYTES && B_INS * NW * 1024 == B_BYTES, "DMA split");
  constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  static_assert(A_INS >= 1 && B_INS >= 1, "tile too small");
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE_BYTES];

#ifdef DL_WGRAD_STAMPS
  unsigned long long st_start = stamp(), st_loop = 0, st_wait = 0, st_work = 0, st_prev = 0, st_lend = 0;
#endif
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int ntm = g.Cout / BM, ntn = (g.Kch * 8 + BN - 1) / BN;
  // split-major XCD-aware order: the workgroups of one K split (same dy rows,
  // same x pixels, different taps / channel tiles) get consecutive ids after
  // the swizzle, i.e. one XCD, so the split's rows are fetched into that XCD's
  // L2 once instead of once per XCD (wgrad1 15.3 -> 11.0 us, r2_wgrad_xcd_ab.txt)
  const int id = xcd_swizzle(blockIdx.x, wg_grid);
  const int split = id / (ntm * ntn);
  const int tile = id - split * (ntm * ntn);
  const int tm = tile % ntm, tn = tile / ntm;
  const int co0 = tm * BM, k0 = tn * BN;
  const int mbeg = split * m_per_split;
  const int mend = min(g.M, mbeg + m_per_split);
  const int HW = 1 << g.logHW, Wd = g.W, C8 = 1 << g.logC8;
  const int HpWp = g.Hp * g.Wp;
  // padded pixel offset of row r inside a 64-aligned step (pow2 H, W: the step's
  // pixel decomposes as wave-uniform step base + per-lane row part; otherwise
  // every lane decomposes its own pixel each step, out_pix)
  auto lane_pix = [&](int r) {
    return g.pow2 ? (r >> g.logHW) * HpWp + ((r & (HW - 1)) >> g.logW) * g.Wp + (r & (Wd - 1)) : 0;
  };

  // A (dy) lanes: row = A_RPI*(wid*A_INS + j) + lane/ACPR, chunk fixed
  int a_off[A_INS], a_row[A_INS];
#pragma unroll
  for (int j = 0; j < A_INS; ++j) {
    const int row = A_RPI * (wid * A_INS + j) + lane / ACPR;
    a_row[j] = row;
    const int ch = swz_tr<ACPR>(row, lane % ACPR) - row * ACPR;  // logical chunk (involution)
    a_off[j] = (lane_pix(row) + (g.dsep ? 0 : g.pad * g.Wp + g.pad)) * g.Cout + co0 + ch * 8;
  }
  // B (im2col of x) lanes: chunk -> fixed tap (kh, kw, c0)
  int b_off[B_INS], b_row[B_INS];
  bool b_kok[B_INS];
#pragma unroll
  for (int j = 0; j < B_INS; ++j) {
    const int row = B_RPI * (wid * B_INS + j) + lane / BCPR;
    b_row[j] = row;
    const int ch = swz_tr<BCPR>(row, lane % BCPR) - row * BCPR;
    const int kc = k0 / 8 + ch;
    b_kok[j] = kc < g.Kch;
    const int kpos = kc >> g.logC8;
    const int kh = kpos / g.KW, kw = (kpos - kh * g.KW) * g.kwstep;
    b_off[j] = (lane_pix(row) + kh * g.Wp + kw) * g.Cin + ((kc & (C8 - 1)) << 3);
  }
  const i32x4 dyr = make_rsrc4(dy, (unsigned)((int64_t)g.B * g.dHp * g.dWp * g.Cout * 2));
  const i32x4 xr = make_rsrc4(x, (unsigned)((int64_t)g.B * g.Hp * g.Wp * g.Cin * 2));
  unsigned a_v[A_INS], b_v[B_INS];  // per-lane byte offsets (K-tail lanes: out of range -> zeros)
#pragma unroll
  for (int j = 0; j < A_INS; ++j) a_v[j] = 2u * (unsigned)a_off[j];
#pragma unroll
  for (int j = 0; j < B_INS; ++j) b_v[j] = b_kok[j] ? 2u * (unsigned)b_off[j] : kOOB;

  // One stage's LDS-DMA (branch-free: rows past the end -- a partial last
  // step, or a k-step past nk issued by the unconditional pipeline -- read
  // zeros from an out-of-range offset).
  auto issue = [&](int kt, int slot) {
    char* sA = smem + slot * STAGE_BYTES;
    char* sB = sA + A_BYTES;
    const int ms = mbeg + kt * BK;  // 64-aligned first row of the step
    const int left = mend - ms;     // rows left (uniform)
    if (g.pow2) {
      const int u = (ms >> g.logHW) * HpWp + ((ms & (HW - 1)) >> g.logW) * g.Wp;  // wave-uniform
      const unsigned ua = 2u * (unsigned)(u * g.Cout), ub = 2u * (unsigned)(u * g.Cin);
#pragma unroll
      for (int j = 0; j < A_INS; ++j)
        blds16_asm(dyr, a_row[j] < left ? a_v[j] : kOOB, ua, sA + (wid * A_INS + j) * 1024);
#pragma unroll
      for (int j = 0; j < B_INS; ++j)
        blds16_asm(xr, b_row[j] < left ? b_v[j] : kOOB, ub, sB + (wid * B_INS + j) * 1024);
    } else {
#pragma unroll
      for (int j = 0; j < A_INS; ++j) {
        const bool ok = a_row[j] < left;
        const int mr = ok ? ms + a_row[j] : 0;
        const int px = g.dsep ? dy_pix(g, mr) : out_pix(g, mr);
        blds16_asm(dyr, ok ? a_v[j] + 2u * (unsigned)(px * g.Cout) : kOOB, 0u, sA + (wid * A_INS + j) * 1024);
      }
#pragma unroll
      for (int j = 0; j < B_INS; ++j) {
        const bool ok = b_row[j] < left;
        const int px = out_pix(g, ok ? ms + b_row[j] : 0);
        blds16_asm(xr, ok && b_v[j] != kOOB ? b_v[j] + 2u * (unsigned)(px * g.Cin) : kOOB, 0u,
                   sB + (wid * B_INS + j) * 1024);
      }
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int gq = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  const int nk = max(0, (mend - mbeg + BK - 1) / BK);
  // (as conv_fwd_region_kernel) every step issues one stage unconditionally,
  // fragments of step i+1 are read (transposed LDS reads) while the MFMAs of
  // step i run, interleaved 1:1 -- needs >= 4 stages to keep DMA lookahead
  static_assert(STAGES >= 3, "fragment prefetch needs >= 3 ring slots");
#pragma unroll
  for (int p = 0; p < PD; ++p) issue(p, p);
  int rslot = 0, dslot = PD % STAGES;
  auto read_frags = [&](bf16x8 (&af)[BK / 32][FM], bf16x8 (&bf)[BK / 32][FN]) {
    const char* As = smem + rslot * STAGE_BYTES;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int r0 = kk * 32 + gq * 8 + q4;
#pragma unroll
      for (int a = 0; a < FM; ++a) {
        const int col = wm * TM + a * 16 + 4 * p4;
        const int ch = col >> 3, sub = (col & 7) * 2;
        s16x4 lo = ds_read_tr16(As + swz_tr<ACPR>(r0, ch) * 16 + sub);
        s16x4 hi = ds_read_tr16(As + swz_tr<ACPR>(r0 + 4, ch) * 16 + sub);
        af[kk][a] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int b = 0; b < FN; ++b) {
        const int col = wn * TN + b * 16 + 4 * p4;
        const int ch = col >> 3, sub = (col & 7) * 2;
        s16x4 lo = ds_read_tr16(Bs + swz_tr<BCPR>(r0, ch) * 16 + sub);
        s16x4 hi = ds_read_tr16(Bs + swz_tr<BCPR>(r0 + 4, ch) * 16 + sub);
        bf[kk][b] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
    }
    ++rslot;
    rslot -= (rslot == STAGES) * STAGES;
  };
  constexpr int NRD = (BK / 32) * (FM + FN) * 2;  // ds_read_b64_tr_b16 per step
  constexpr int NMF = (BK / 32) * FM * FN;
  bf16x8 fa0[BK / 32][FM], fb0[BK / 32][FN], fa1[BK / 32][FM], fb1[BK / 32][FN];
  {
  wait_vmcnt<(PD - 1) * LPS>();  // stage 0 landed
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  read_frags(fa0, fb0);
  int kt_next = PD;
  // The step's LDS-DMA is issued right after the barrier, BEFORE the
  // fragment reads.  The asm DMA carries a memory
  // clobber, so reads issued before it cannot move past it: in the old order
  // (reads, DMA, MFMAs) the 24 reads were bunched ahead of all MFMAs and the
  // compiler hoisted the next step's lgkmcnt(0) + barrier to after the 4th
  // MFMA -- the reads' latency was covered by 4 MFMAs and the other 12 ran
  // with no reads beside them.  DMA first, the reads and MFMAs share one
  // scheduling region and interleave (MFMA, 2 reads) as the group barriers
  // ask, and a closing sched_barrier keeps the next barrier after them.
  auto step = [&](bf16x8 (&fca)[BK / 32][FM], bf16x8 (&fcb)[BK / 32][FN], bf16x8 (&fna)[BK / 32][FM],
                  bf16x8 (&fnb)[BK / 32][FN]) {
#ifdef DL_WGRAD_STAMPS
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long sa = stamp();
    __builtin_amdgcn_sched_barrier(0);
#endif
    wait_vmcnt<(PD - 2) * LPS>();        // stage i+1 landed
    __builtin_amdgcn_s_waitcnt(0xC07F);  // step i's fragments in registers (compiler-visible wait)
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#ifdef DL_WGRAD_STAMPS
    {
      const unsigned long long sb = stamp();
      __builtin_amdgcn_sched_barrier(0);
      st_wait += sb - sa;
      if (st_prev) st_work += sa - st_prev;
      st_prev = sb;
    }
#endif
    issue(kt_next, dslot);  // into the slot read two steps ago
    ++kt_next;
    ++dslot;
    dslot -= (dslot == STAGES) * STAGES;
    __builtin_amdgcn_sched_barrier(0);
    read_frags(fna, fnb);
    // C^T (k x co): lane holds 4 consecutive k of one co -> 16-byte stores
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk)
#pragma unroll
      for (int a = 0; a < FM; ++a)
#pragma unroll
        for (int b = 0; b < FN; ++b) acc[a][b] = mfma16(fcb[kk][b], fca[kk][a], acc[a][b]);
    constexpr int P1 = NRD / 2 < NMF ? NRD / 2 : NMF;  // (MFMA, 2 reads) pairs
#pragma unroll
    for (int q = 0; q < P1; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
    if constexpr (NRD > 2 * P1) __builtin_amdgcn_sched_group_barrier(0x100, NRD - 2 * P1, 0);
    if constexpr (NMF > P1) __builtin_amdgcn_sched_group_barrier(0x008, NMF - P1, 0);
    __builtin_amdgcn_sched_barrier(0);
  };
  int i = 0;
#ifdef DL_WGRAD_STAMPS
  st_loop = stamp();
#endif
  for (; i + 1 < nk; i += 2) {
    step(fa0, fb0, fa1, fb1);
    step(fa1, fb1, fa0, fb0);
  }
  if (i < nk) step(fa0, fb0, fa1, fb1);
  }

#ifdef DL_WGRAD_STAMPS
  st_lend = stamp();
  struct StampOut {
    unsigned long long* p;
    unsigned long long v[5];
    int w;
    __device__ ~StampOut() {
      if (p && (threadIdx.x & 63) == 0 && (w == 0 || w == (int)(blockDim.x >> 6) - 1)) {
        unsigned long long* d = p + ((size_t)(blockIdx.x + blockIdx.y * gridDim.x) * 2 + (w ? 1 : 0)) * 6;
        d[0] = v[0]; d[1] = v[1]; d[2] = v[2]; d[3] = v[3]; d[4] = v[4]; d[5] = stamp();
      }
    }
  } stamp_out{g_wgrad_stamps, {st_start, st_loop, st_wait, st_work, st_lend}, wid};
#endif
  const int col_l = lane & 15, rq = lane >> 4;
  float* o = out + (int64_t)split * g.Cout * ldo;
  if constexpr (BN >= 128) {  // (64-wide tiles: measured no gain)
    // Slab rows through LDS: straight from the accumulators a store
    // instruction writes 16 rows x 64 B; staged, every instruction writes whole
    // BN*4-byte rows (64 lanes x 16 B).  The C^T tile goes into the (drained)
    // DMA ring as [co][k] fp32 with a 16-byte row pad (row stride 2^n + 16 B:
    // the 16 co rows of a store group fall on distinct banks).
    constexpr int LROW = BN + 4;
    static_assert(BM * LROW * 4 <= STAGES * STAGE_BYTES, "staged slab tile fits the ring");
    wait_vmcnt<0>();  // the unconditional pipeline's trailing (zero-fill) DMAs still target the ring
    block_sync_lds();
    float* st = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int a = 0; a < FM; ++a)
#pragma unroll
      for (int b = 0; b < FN; ++b)
        *reinterpret_cast<float4*>(st + (wm * TM + a * 16 + col_l) * LROW + wn * TN + b * 16 + rq * 4) =
            make_float4(acc[a][b][0], acc[a][b][1], acc[a][b][2], acc[a][b][3]);
    block_sync_lds();
    constexpr int C4 = BN / 4, NTH = 64 * NW;  // 16-byte chunks per row, threads
    static_assert(BM * C4 % NTH == 0, "whole store passes");
#pragma unroll
    for (int i = 0; i < BM * C4 / NTH; ++i) {
      const int idx = tid + i * NTH, r = idx / C4, c4 = idx - r * C4;
      const int co = co0 + r, k = k0 + 4 * c4;
      if (co < g.Cout && k < ldo)
        *reinterpret_cast<float4*>(o + (int64_t)co * ldo + k) =
            *reinterpret_cast<const float4*>(st + r * LROW + 4 * c4);
    }
    return;
  }
#pragma unroll
  for (int a = 0; a < FM; ++a)
#pragma unroll
    for (int b = 0; b < FN; ++b) {
      const int k = k0 + wn * TN + b * 16 + rq * 4;
      const int co = co0 + wm * TM + a * 16 + col_l;
      if (co < g.Cout && k < ldo)  // ldo % 4 == 0 and k % 4 == 0: the 4-run is in bounds
        *reinterpret_cast<float4*>(o + (int64_t)co * ldo + k) =
            make_float4(acc[a][b][0], acc[a][b][1], acc[a][b][2], acc[a][b][3]);
    }
}

// Sum `splits` fp32 slabs [splits][Cout][Kp] (Kp = taps*Cp) into dst
// [Cout][taps][C] (body and options: slab_reduce_dev.h).
template <int TPO, bool ACC = false, bool OIHW = false>
__global__ void __launch_bounds__(256) slab_reduce_kernel(const float* __restrict__ slabs, float* __restrict__ dst,
                                                          int splits, int Cout, int taps, int Cp, int C) {
  slab_reduce_body<TPO, ACC, OIHW>(slabs, dst, splits, Cout, taps, Cp, C, (int)blockIdx.x, (int)gridDim.x);
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
// Many [rows][cols] bf16 matrices transposed in ONE launch (the ResNet-50 1x1
// weights for their dgrads, once per step: 33 weight_flip_transpose launches
// of ~5 us each before).  Entries sorted by tile0; 64x64 tiles.
struct TrEntry {
  int64_t src, dst;
  int rows, cols, tile0, tiles_c;
};

__global__ void __launch_bounds__(256) transpose_many_kernel(const TrEntry* __restrict__ tab, int n) {
  __shared__ bf16_t t[64][65];
  const int b = blockIdx.x;
  int e = 0;
  for (int i = 1; i < n; ++i)
    if (tab[i].tile0 <= b) e = i;
  const TrEntry en = tab[e];
  const bf16_t* __restrict__ src = reinterpret_cast<const bf16_t*>(en.src);
  bf16_t* __restrict__ dst = reinterpret_cast<bf16_t*>(en.dst);
  const int local = b - en.tile0;
  const int r0 = (local / en.tiles_c) * 64, c0 = (local % en.tiles_c) * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4)
    t[r][tx] = (r0 + r < en.rows && c0 + tx < en.cols) ? src[(int64_t)(r0 + r) * en.cols + c0 + tx] : (bf16_t)0;
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int c = c0 + r, rr = r0 + tx;
    if (c < en.cols && rr < en.rows) dst[(int64_t)c * en.rows + rr] = t[tx][r];
  }
}

// Many conv weights [Cout][Cin][KK] -> channels-last [Cout][KK][Cin] in ONE
// launch (the ResNet-50 MIOpen convolutions read channels-last weights: torch
// converted each one on every call, 34 copy kernels per step).
// blockIdx.y = entry, grid-stride over that entry's elements in dst order.
struct ClEntry {
  int64_t src, dst;
  int cout, cin, kk, pad;
};

__global__ void __launch_bounds__(256) weights_to_cl_kernel(const ClEntry* __restrict__ tab) {
  const ClEntry en = tab[blockIdx.y];
  const bf16_t* __restrict__ src = reinterpret_cast<const bf16_t*>(en.src);
  bf16_t* __restrict__ dst = reinterpret_cast<bf16_t*>(en.dst);
  const int64_t total = (int64_t)en.cout * en.kk * en.cin;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < total; j += (int64_t)gridDim.x * blockDim.x) {
    const int ci = (int)(j % en.cin);
    const int64_t r = j / en.cin;  // co * kk + t
    const int t = (int)(r % en.kk);
    const int64_t co = r / en.kk;
    dst[j] = src[(co * en.cin + ci) * en.kk + t];
  }
}

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
// Per-step operand preparation in ONE launch (was 5): zero-pad the input
// image channels, pack the first layer's fp32 weights to padded bf16, and
// flip+transpose the bf16 weights of every later layer for its dgrad.
// Job = blockIdx range; each transpose block moves one 32x32 (co, ci) tile of
// one tap through LDS.
// --------------------------------------------------------------------------
// (PrepArgs and the pad / zero jobs: prep_dev.h, shared with the SGD launch
// that prepares the next step of an unrolled graph.)
__global__ void __launch_bounds__(256) prep_step_kernel(const PrepArgs a) {
  __shared__ bf16_t t[32][33];
  int blk = blockIdx.x;
  if (blk < a.nb_pad) {
    prep_pad_block(a, blk);
    return;
  }
  blk -= a.nb_pad;
  if (blk < a.nb_pack) {
    if (a.w1_cp < 0) {  // pair-packed (pack1_index): scatter the real elements, pads stay zero
      const int total = a.w1_cout * a.taps * a.w1_c;
      for (int e = blk * 256 + threadIdx.x; e < total; e += a.nb_pack * 256)
        a.w1p[pack1_index(e, a.w1_c, a.w1_cp)] = f32_to_bf16(a.w1[e]);
      return;
    }
    const int total = a.w1_cout * a.taps * a.w1_cp;
    for (int i = blk * 256 + threadIdx.x; i < total; i += a.nb_pack * 256) {
      const int c = i % a.w1_cp;
      a.w1p[i] = c < a.w1_c ? f32_to_bf16(a.w1[(i / a.w1_cp) * a.w1_c + c]) : (bf16_t)0;
    }
    return;
  }
  blk -= a.nb_pack;
  if (blk < a.nb_zero) {
    prep_zero_block(a, blk);
    return;
  }
  blk -= a.nb_zero;
  for (int j = 0; j < a.nt; ++j) {
    if (blk >= a.nb_t[j]) { blk -= a.nb_t[j]; continue; }
    const int Cin = a.tcin[j], Cout = a.tcout[j], taps = a.taps;
    if (Cin % 64 == 0 && Cout % 64 == 0) {
      // (wtrans_dev.h.  Tiles of 4 consecutive taps per block with every load
      // issued first measured slower: 0.3314-0.3332 vs 0.3296-0.3307 ms/step,
      // 4x fewer blocks and 4x the static LDS of the whole prep launch,
      // profiles/r3_prep_taps_ab.txt.)
      __shared__ __attribute__((aligned(16))) bf16_t tt[64][72];
      wtrans_tile(a.tw[j], a.twt[j], Cin, Cout, taps, blk, tt);
      return;
    }
    const int nci = (Cin + 31) / 32, nco = (Cout + 31) / 32;
    const int tap = blk / (nci * nco);
    const int r = blk % (nci * nco);
    const int ci0 = (r % nci) * 32, co0 = (r / nci) * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int q = ty; q < 32; q += 8) {
      const int co = co0 + q, ci = ci0 + tx;
      t[q][tx] = (co < Cout && ci < Cin) ? a.tw[j][((int64_t)co * taps + tap) * Cin + ci] : (bf16_t)0;
    }
    __syncthreads();
    const int ftap = taps - 1 - tap;
    for (int q = ty; q < 32; q += 8) {
      const int ci = ci0 + q, co = co0 + tx;
      if (ci < Cin && co < Cout) a.twt[j][((int64_t)ci * taps + ftap) * Cout + co] = t[tx][q];
    }
    return;
  }
}

static void launch_prep(PrepArgs& a, int64_t P, uintptr_t w1, uintptr_t w1p, int w1_cout, int taps, int w1_c,
                        int w1_cp, const std::vector<uintptr_t>& tw, const std::vector<uintptr_t>& twt,
                        const std::vector<int>& tcout, const std::vector<int>& tcin,
                        const std::vector<uintptr_t>& zp, const std::vector<int64_t>& zn, uintptr_t stream) {
  prep_set_zero(a, zp, zn);
  prep_set_pad(a, P);
  a.w1 = (const float*)w1; a.w1p = (bf16_t*)w1p; a.w1_cout = w1_cout; a.taps = taps; a.w1_c = w1_c; a.w1_cp = w1_cp;
  a.nt = (int)tw.size();
  if (a.nt > 4 || twt.size() != tw.size() || tcout.size() != tw.size() || tcin.size() != tw.size())
    throw std::runtime_error("prep_step: up to 4 consistent transposes");
  if (w1_cp < 0 && (w1_c > 4 || taps != w1_cp * w1_cp)) throw std::runtime_error("prep_step: pair pack needs C <= 4, a square kernel");
  a.nb_pack = (int)std::min<int64_t>(((int64_t)w1_cout * taps * (w1_cp > 0 ? w1_cp : w1_c) + 255) / 256, 256);
  int total = a.nb_pad + a.nb_pack + a.nb_zero;
  for (int j = 0; j < a.nt; ++j) {
    a.tw[j] = (const bf16_t*)tw[j]; a.twt[j] = (bf16_t*)twt[j];
    a.tcout[j] = tcout[j]; a.tcin[j] = tcin[j];
    a.nb_t[j] = (tcin[j] % 64 == 0 && tcout[j] % 64 == 0) ? (tcin[j] / 64) * (tcout[j] / 64) * taps
                                                          : ((tcin[j] + 31) / 32) * ((tcout[j] + 31) / 32) * taps;
    total += a.nb_t[j];
  }
  if (total == 0) return;
  prep_step_kernel<<<total, 256, 0, as_stream(stream)>>>(a);
  DL_HIP_CHECK(hipGetLastError());
}

void prep_step(uintptr_t x, uintptr_t xp, int64_t P, int C, int Cp, int H, int W, int sp, uintptr_t w1, uintptr_t w1p,
               int w1_cout, int taps, int w1_c, int w1_cp, std::vector<uintptr_t> tw, std::vector<uintptr_t> twt,
               std::vector<int> tcout, std::vector<int> tcin, std::vector<uintptr_t> zp, std::vector<int64_t> zn,
               uintptr_t stream) {
  PrepArgs a{};
  a.x = (const bf16_t*)x; a.xp = (bf16_t*)xp; a.C = C; a.Cp = Cp;
  a.H = H; a.W = W; a.sp = sp;
  launch_prep(a, P, w1, w1p, w1_cout, taps, w1_c, w1_cp, tw, twt, tcout, tcin, zp, zn, stream);
}

// Same launch with the step's input gathered on the device: batch b of step
// s (= ctr[0]) is sample order[(s*B + b) mod n_order] of the uint8 NHWC
// dataset `img`, normalised ((v/255 - mean)/std), channel- and spatially
// padded into xp; its label goes to lab_out[b].  head_wgrad advances ctr[0]
// later in the step, so a captured graph replays consecutive batches.
void prep_step_gather(uintptr_t img, uintptr_t order, uintptr_t lab_all, uintptr_t lab_out, uintptr_t ctr,
                      int n_order, int B, int C, std::vector<float> mean, std::vector<float> stdv, uintptr_t xp,
                      int Cp, int H, int W, int sp, uintptr_t w1, uintptr_t w1p, int w1_cout, int taps, int w1_c,
                      int w1_cp, std::vector<uintptr_t> tw, std::vector<uintptr_t> twt, std::vector<int> tcout,
                      std::vector<int> tcin, std::vector<uintptr_t> zp, std::vector<int64_t> zn, uintptr_t stream) {
  PrepArgs a{};
  a.xp = (bf16_t*)xp; a.C = C; a.Cp = Cp; a.H = H; a.W = W; a.sp = sp;
  prep_set_gather(a, img, order, lab_all, lab_out, ctr, n_order, B, C, mean, stdv);
  launch_prep(a, (int64_t)B * H * W, w1, w1p, w1_cout, taps, w1_c, w1_cp, tw, twt, tcout, tcin, zp, zn, stream);
}

// --------------------------------------------------------------------------
// host launchers
// --------------------------------------------------------------------------
static int fwd_bm(int tile) { return tile == 1 ? 64 : 128; }
static int fwd_bn(int tile) { return tile == 0 ? 128 : 64; }

static int combine_rows_per_block(int M, int N) {
  const int rpi = 256 / (N / 8);
  int rpb = (M + 383) / 384;            // ~384 blocks
  rpb = ((rpb + rpi - 1) / rpi) * rpi;  // whole iterations
  return rpb < rpi ? rpi : rpb;
}


// number of BN partial-sum rows conv_fwd writes for this configuration
int conv_fwd_stat_rows(int B, int H, int W, int Cin, int Cout, int KS, int tile, int splits) {
  tile &= 15;
  ConvGeom g = make_geom(B, H, W, Cin, Cout, KS);
  if (splits <= 1) return (g.M + fwd_bm(tile) - 1) / fwd_bm(tile);
  const int rpb = combine_rows_per_block(g.M, Cout);
  return (g.M + rpb - 1) / rpb;
}

static SgdJob g_side_sgd{};         // set_conv_side_sgd: side SGD job of the next conv_fwd / conv_wgrad launch
static uintptr_t g_fwd_addend = 0;  // conv_fwd_add: bf16 [M][Cout] added in the epilogue
static uintptr_t g_fwd_addend_mask = 0;  // conv_fwd_add: optional uint8 [M][Cout/8] mask bits of the addend
static int g_fwd_keep_slabs = 0;    // FwdCfg bit 20: leave the split-K slabs (the caller combines them)
static int g_c8_pair = 0;           // FwdCfg bit 24: pair-packed first-layer weights (conv_fwd_c8_kernel PAIR)
static int g_red_atomic_host = 0;   // host mirror of g_red_atomic
static BnRedArgs g_bnred{};         // conv_fwd_bnred: fused BN backward reduce (region dgrad only)
// conv_fwd_fix: the current conv_fwd call combines its split-K slices in-launch
// (FIX); bnred.rows != nullptr: its epilogue is the BN backward reduce of the
// block below (BNR 1) instead of the BN statistics
struct FixState {
  bool on = false;
  BnRedArgs bnred{};
};
static FixState g_fix{};
static int g_fix_next = 0;  // next free arrival counter (round robin over g_fix_cnt)

// Position-major tiles with padding taps skipped (conv_fwd_kernel, g.posm):
// for TAPU layers whose output is smaller than twice the kernel (most output
// pixels then have padding-only taps), the batch a multiple of BM and no
// addend.  (8x8 outputs added in round 6: CIFAR layer-3 dgrad 27.2 -> 25.7 us,
// 28 % of its taps read only the border; the per-tile work is then uneven, and
// 4 splits to even it out lost, profiles/r6_posm8_ab.txt.)
// set_conv_posm(0) = the pixel-major tiles (A/B).
static int g_posm = 1;
void set_conv_posm(int on) { g_posm = on ? 1 : 0; }

template <int BM, int BN, bool TAPU, int ST, int WM, int WN>
static void launch_fwd_w(ConvGeom& g, uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t stats,
                         uintptr_t slab, int splits, hipStream_t s) {
  g.posm = (g_posm && TAPU && !g_fwd_addend && g.B % BM == 0 && (g.H < 2 * g.KS || g.W < 2 * g.KS) && g.S == 1 && !g.om &&
            g.KH == g.KS && g.KW == g.KS && g.Hp == g.H + 2 * g.pad && g.Wp == g.W + 2 * g.pad) ? 1 : 0;
  const int ntm = (g.M + BM - 1) / BM, ntn = (g.Cout + BN - 1) / BN;
  const int nkt = (g.Kch + 7) / 8;
  const int ktps = (nkt + splits - 1) / splits;
  SgdJob side = g_side_sgd;  // one-shot: consumed by this launch
  g_side_sgd.nblk = 0;
  constexpr int kNT = 64 * WM * WN;
  if (side.nblk < 0)  // auto: one float4 per thread (2048 x 512 measured best of 256..2048 workgroups)
    side.nblk = (int)std::max<int64_t>(1, (side.hi4 - side.lo4 + kNT - 1) / kNT);
  const int grid = ntm * ntn * splits + side.nblk;
  constexpr int NT = 64 * WM * WN;
  constexpr bool kTR = (BN / WN / 16) % 2 == 0;
  if (g_fix.on) {
    if constexpr (kTR && TAPU && BM == 128 && BN == 64 && WM == 4 && WN == 2) {
      if (splits < 2 || g.om || g_fwd_addend)
        throw std::runtime_error("conv_fwd_fix: split-K without output maps / addends");
      const int ntiles = ntm * ntn;
      if (ntiles > kFixCnt) throw std::runtime_error("conv_fwd_fix: too many tiles");
      static int* cnt0 = nullptr;
      if (!cnt0) DL_HIP_CHECK(hipGetSymbolAddress((void**)&cnt0, HIP_SYMBOL(g_fix_cnt)));
      if (g_fix_next + ntiles > kFixCnt) g_fix_next = 0;
      int* cnt = cnt0 + g_fix_next;  // distinct counters per call site (graph replays reuse them in order)
      g_fix_next += ntiles;
      if (g_fix.bnred.rows != nullptr) {
        if (stats) throw std::runtime_error("conv_fwd_fix: BN reduce epilogue has no statistics");
        conv_fwd_kernel<BM, BN, false, false, TAPU, ST, WM, WN, false, true, 1, true><<<grid, NT, 0, s>>>(
            (const bf16_t*)x, (const bf16_t*)w, (bf16_t*)y, nullptr, (float*)slab, g, splits, ktps, g_conv_dbg,
            g_fix.bnred, side, cnt);
      } else if (stats) {
        conv_fwd_kernel<BM, BN, true, false, TAPU, ST, WM, WN, false, true, 0, true><<<grid, NT, 0, s>>>(
            (const bf16_t*)x, (const bf16_t*)w, (bf16_t*)y, (float*)stats, (float*)slab, g, splits, ktps, g_conv_dbg,
            BnRedArgs{}, side, cnt);
      } else {
        conv_fwd_kernel<BM, BN, false, false, TAPU, ST, WM, WN, false, true, 0, true><<<grid, NT, 0, s>>>(
            (const bf16_t*)x, (const bf16_t*)w, (bf16_t*)y, nullptr, (float*)slab, g, splits, ktps, g_conv_dbg,
            BnRedArgs{}, side, cnt);
      }
      return;
    } else {
      throw std::runtime_error("conv_fwd_fix: only the 128x64 streaming tile (8 waves) combines in-launch");
    }
  }
  if (g_fwd_addend && (splits > 1 || stats)) throw std::runtime_error("conv_fwd_add: no split-K / statistics");
  if (g_fwd_addend)
    conv_fwd_kernel<BM, BN, false, false, TAPU, ST, WM, WN, true><<<grid, NT, 0, s>>>(
        (const bf16_t*)x, (const bf16_t*)w, (bf16_t*)y, (float*)g_fwd_addend_mask, (float*)g_fwd_addend, g, 1, ktps,
        g_conv_dbg, BnRedArgs{}, side);
  else if (splits > 1)
    conv_fwd_kernel<BM, BN, false, true, TAPU, ST, WM, WN><<<grid, NT, 0, s>>>(
        (const bf16_t*)x, (const bf16_t*)w, nullptr, nullptr, (float*)slab, g, splits, ktps, g_conv_dbg, BnRedArgs{}, side);
  else if (stats)
    conv_fwd_kernel<BM, BN, true, false, TAPU, ST, WM, WN><<<grid, NT, 0, s>>>(
        (const bf16_t*)x, (const bf16_t*)w, (bf16_t*)y, (float*)stats, nullptr, g, 1, ktps, g_conv_dbg, BnRedArgs{}, side);
  else
    conv_fwd_kernel<BM, BN, false, false, TAPU, ST, WM, WN><<<grid, NT, 0, s>>>(
        (const bf16_t*)x, (const bf16_t*)w, (bf16_t*)y, nullptr, nullptr, g, 1, ktps, g_conv_dbg, BnRedArgs{}, side);
}

static int g_fwd_waves = 8;
static int g_fwd_stages = 3;  // set_conv_stages (the dgrads of an overlapped step run 2 stages)

// Per-call streaming-kernel configuration packed into the tile id:
// bits 0-3 tile, bits 4-7 LDS ring stages (0 = the global default), bits 8-11
// waves per workgroup (0 = default).  The ResNet-50 1x1 GEMMs pick 2 stages
// (96 -> 64 KiB of LDS: two workgroups per CU, which is what the short-K
// GEMMs need -- scripts/bench_gemm1x1.py SWEEP=1, ops/conv.py _plan_1x1),
// while the CIFAR layers keep the tuned global default.
// bit 20: keep the split-K slabs -- no combine launch; the consumer sums them
// (bn_pool.hip combine_bwd_reduce: a dgrad's combine fused with the BN
// backward reduce of the block below).
struct FwdCfg {
  int saved_st, saved_wv;
  explicit FwdCfg(int& tile) : saved_st(g_fwd_stages), saved_wv(g_fwd_waves) {
    const int st = (tile >> 4) & 15, wv = (tile >> 8) & 15;
    g_fwd_keep_slabs = (tile >> 20) & 1;
    g_c8_pair = (tile >> 24) & 1;
    tile &= 15;
    if (st && (st < 2 || st > 4)) throw std::runtime_error("conv_fwd: packed stages must be 2..4");
    if (wv && wv != 4 && wv != 8) throw std::runtime_error("conv_fwd: packed waves must be 4 or 8");
    if (st) g_fwd_stages = st;
    if (wv) g_fwd_waves = wv;
  }
  ~FwdCfg() {
    g_fwd_stages = saved_st; g_fwd_waves = saved_wv; g_fwd_keep_slabs = 0; g_c8_pair = 0;
  }
};

template <int BM, int BN, bool TAPU, int ST>
static void launch_fwd_t(ConvGeom& g, uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t stats,
                         uintptr_t slab, int splits, hipStream_t s) {
  if (g_fwd_waves == 8) {
    if constexpr (BN >= 128) launch_fwd_w<BM, BN, TAPU, ST, 2, 4>(g, x, w, y, stats, slab, splits, s);
    else if constexpr (BM >= 128) launch_fwd_w<BM, BN, TAPU, ST, 4, 2>(g, x, w, y, stats, slab, splits, s);
    else launch_fwd_w<BM, BN, TAPU, ST, 2, 4>(g, x, w, y, stats, slab, splits, s);
  } else {
    launch_fwd_w<BM, BN, TAPU, ST, 2, 2>(g, x, w, y, stats, slab, splits, s);
  }
}

void set_conv_waves(int waves) {
  if (waves != 4 && waves != 8) throw std::runtime_error("waves must be 4 or 8");
  g_fwd_waves = waves;
}

void set_conv_fwd_pf(int on) {
  const int v = on ? 1 : 0;
  DL_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_fwd_pf), &v, sizeof(int)));
}
void set_conv_debug(uintptr_t buf) { g_conv_dbg = (unsigned long long*)buf; }
void set_conv_wgrad_stamps(uintptr_t buf) {
  unsigned long long* p = (unsigned long long*)buf;
  DL_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_wgrad_stamps), &p, sizeof(p)));
}

void set_conv_stages(int fwd, int wgrad) {
  if (fwd < 2 || fwd > 4 || wgrad != 0)
    throw std::runtime_error("stages: fwd 2..4, wgrad 0 (the per-tile default; other rings removed in round 6)");
  g_fwd_stages = fwd;
}

template <int BM, int BN>
static void launch_fwd(ConvGeom& g, uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t stats,
                       uintptr_t slab, int splits, hipStream_t s) {
  const int st = (BM * 64 * 2 + BN * 64 * 2) * 4 > 160 * 1024 ? std::min(g_fwd_stages, 3) : g_fwd_stages;
  if (g.Cin >= 64) {
    if (st == 2) launch_fwd_t<BM, BN, true, 2>(g, x, w, y, stats, slab, splits, s);
    else if (st == 3) launch_fwd_t<BM, BN, true, 3>(g, x, w, y, stats, slab, splits, s);
    else launch_fwd_t<BM, BN, true, 4>(g, x, w, y, stats, slab, splits, s);
  } else {
    launch_fwd_t<BM, BN, false, 3>(g, x, w, y, stats, slab, splits, s);
  }
}

// ---- tap-reuse (LDS-resident region) forward path --------------------------
// set_conv_region(0) forces the streaming kernel (A/B); 1 = region kernel
// for row tiles (H*W % 128 == 0), 2 = also for whole-image tiles.  Measured
// (MI355X, batch 128, rocprofv3): rows mode wins (conv2 fwd 19.3 -> 17.7 us,
// dgrad 22.8 -> 20.5 us); images mode loses (conv3/conv4 21-25 vs 19.7 us:
// the 4x4/8x8 outputs need 8x8/12x12 padded inputs, the region fill does not
// amortise over 25 k-steps), so it is off by default.
static int g_region = 1, g_region_images = 0;
void set_conv_region(int on) {
  g_region = on ? 1 : 0;
  g_region_images = on >= 2 ? 1 : 0;
}

// LDS budget of one region-kernel workgroup: the CU's 160 KiB minus room for
// one co-resident RCCL collective workgroup (rcclGenericKernel: 19,744 B of
// LDS, 256 threads, <= 280 VGPRs -- read from librccl's gfx950 code object),
// so the bucket all-reduce that overlaps the backward at N > 1 never evicts
// a conv workgroup from a CU (a 1-workgroup-per-CU grid would otherwise need
// a second round for the CUs RCCL holds).  The dgrad instance (BN = 64, the
// one that runs beside the all-reduce) also stays at <= 112 VGPRs, so two
// of its waves fit a SIMD next to a 288-VGPR RCCL wave; the BN = 128
// instance (127 VGPRs) only runs in the forward, before any collective.
// Measured with one CU held by a workgroup of RCCL's footprint
// (bench_conv.py --occupy 1): the dgrad instance (~126 KiB) +1 us, while the
// streaming kernel's 3-stage ring (96 KiB, 90 VGPRs) loses 14 us -- the executor
// switches the overlapped dgrads to its 2-stage ring (models/cifar_hip.py).
constexpr int kRegionLdsCap = 160 * 1024 - 20 * 1024;

// Region geometry for a BM = 128 tile, or false if the shape does not fit the
// region kernel (then the streaming kernel runs).
static bool region_geom(const ConvGeom& g, int BN, int splits, RegionGeom& rg) {
  constexpr int BM = 128, STAGES = 3;
  if (!g.pow2 || !g_region || g.Cin % 64 != 0 || g.W > BM || BM % g.W != 0) return false;
  const int HW = g.H * g.W;
  const int chunks = g.Cin / 64;
  if (chunks % splits != 0) return false;
  rg.cpw = chunks / splits;
  if (rg.cpw > 2) return false;
  rg.S = 10;  // the kernel's region loader divides by 10 with a multiply
  rg.RW = g.Wp;
  if (HW % BM == 0) {  // M tile = BM / W whole output rows of one image
    rg.rows_mode = 1;
    rg.nimg = 1;
    rg.RH = BM / g.W + g.KS - 1;
    rg.RS = rg.RW * rg.S;
  } else if (BM % HW == 0 && g_region_images) {  // M tile = BM / HW whole images
    rg.rows_mode = 0;
    rg.nimg = BM / HW;
    rg.RH = g.Hp;
    rg.RS = rg.RW * rg.S + 8;  // + 8 slots per region row: conflict-free fragment reads across rows
  } else {
    return false;
  }
  rg.IS = rg.RH * rg.RS;
  rg.nslot = (rg.nimg * rg.IS + 63) / 64 * 64;
  if (rg.RS >= 16384) return false;
  if (rg.nslot >= (1 << 16)) return false;
  rg.inv_S = 1.0f / rg.S;
  rg.inv_RS = 1.0f / rg.RS;
  rg.inv_IS = 1.0f / rg.IS;
  const int lds = rg.cpw * rg.nslot * 16 + STAGES * BN * 64 * 2;  // at least a 3-stage B ring
  return lds <= kRegionLdsCap;
}

static int g_region_waves = 8;  // 8: 2 waves per SIMD; 4: one wave per SIMD with 2x wider wave tiles
void set_conv_region_waves(int w) {
  if (w != 4 && w != 8) throw std::runtime_error("region waves must be 4 or 8");
  g_region_waves = w;
}
static int g_region_ablate = 0;  // debug: bit 0 = no in-loop weight DMA, bit 1 = no MFMAs
void set_conv_region_ablate(int a) { g_region_ablate = a; }
static int g_region_stages = 0;  // 0 = as many B stages as the LDS holds (max 8)
void set_conv_region_stages(int st) { g_region_stages = st; }

template <int BN, int WM, int WN, int ST>
static void launch_fwd_region_st(const ConvGeom& g, const RegionGeom& rg, uintptr_t x, uintptr_t w, uintptr_t y,
                                 uintptr_t stats, uintptr_t slab, int splits, hipStream_t s) {
  const int ntm = (g.M + 127) / 128;
  const int grid = ntm * (g.Cout / BN) * splits;
  const size_t lds = (size_t)rg.cpw * rg.nslot * 16 + ST * BN * 64 * 2;
  auto go = [&](auto kern, bf16_t* yy, float* st, float* sl) {
    static bool attr = false;  // per instantiation: allow > 64 KiB of dynamic LDS
    if (!attr) {
      DL_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
      attr = true;
    }
    kern<<<grid, 64 * WM * WN, lds, s>>>((const bf16_t*)x, (const bf16_t*)w, yy, st, sl, g, rg, splits, g_conv_dbg,
                                         g_region_ablate, g_bnred);
  };
  if (g_bnred.rows != nullptr) {
    if (splits > 1 || stats) throw std::runtime_error("conv_fwd_bnred: plain unsplit dgrad only");
    go(conv_fwd_region_kernel<BN, false, false, ST, WM, WN, true>, (bf16_t*)y, nullptr, nullptr);
  } else if (splits > 1)
    go(conv_fwd_region_kernel<BN, false, true, ST, WM, WN>, nullptr, nullptr, (float*)slab);
  else if (stats)
    go(conv_fwd_region_kernel<BN, true, false, ST, WM, WN>, (bf16_t*)y, (float*)stats, nullptr);
  else
    go(conv_fwd_region_kernel<BN, false, false, ST, WM, WN>, (bf16_t*)y, nullptr, nullptr);
}

// The LDS-DMA issue -> landed latency is ~1.1 us while a k-step computes in
// ~0.2 us: the B ring must keep ~5 k-steps in flight, so it takes every
// stage the LDS has left after the region.
template <int BN, int WM, int WN>
static void launch_fwd_region(const ConvGeom& g, const RegionGeom& rg, uintptr_t x, uintptr_t w, uintptr_t y,
                              uintptr_t stats, uintptr_t slab, int splits, hipStream_t s) {
  const int free_b = kRegionLdsCap - rg.cpw * rg.nslot * 16;
  int st = std::min(8, free_b / (BN * 64 * 2));
  if (g_region_stages > 0) st = std::min(st, g_region_stages);
  if (st >= 8) launch_fwd_region_st<BN, WM, WN, 8>(g, rg, x, w, y, stats, slab, splits, s);
  else if (st >= 6) launch_fwd_region_st<BN, WM, WN, 6>(g, rg, x, w, y, stats, slab, splits, s);
  else if (st >= 5) launch_fwd_region_st<BN, WM, WN, 5>(g, rg, x, w, y, stats, slab, splits, s);
  else if (st >= 4) launch_fwd_region_st<BN, WM, WN, 4>(g, rg, x, w, y, stats, slab, splits, s);
  else launch_fwd_region_st<BN, WM, WN, 3>(g, rg, x, w, y, stats, slab, splits, s);
}

// a region kernel takes the shape (the streaming kernel otherwise).  (The
// direct-B region kernel -- weights streamed into registers, no LDS ring --
// measured slower, layer-2 k-loop 24.3 k vs 23.6 k cycles, layer-3 49.9 k vs
// 34.0 k, README round 5 / scripts/stamp_region.py; removed in round 6.)
static bool any_region_geom(const ConvGeom& g, int tile, int splits, RegionGeom& rg) {
  return (tile == 2 && region_geom(g, 64, splits, rg)) || (tile == 0 && region_geom(g, 128, splits, rg));
}

// tile: 0 = 128x128, 1 = 64x64, 2 = 128x64 (BM x BN, BK = 64).  splits > 1:
// split-K into `slab` (fp32 [splits][M][Cout]) + combine (bf16 y, BN partials).
// Returns the number of BN partial rows written to `stats` (if non-null).
// M tiles per workgroup of the first-layer (Cin = 8) kernel (upper bound; set_conv_c8_mt).
// Measured at batch 128 (profiles/r2_c8_mt_ab.txt): 1 tile (1024 workgroups, 4 per CU)
// 12.0 us, 4 tiles (256 workgroups, one weight-panel DMA each) 14.8 us: the kernel is
// bound by its epilogue stores overlapping across workgroups, not by the weight DMA.
static int g_c8_mt = 1;
void set_conv_c8_mt(int mt) {
  if (mt != 1 && mt != 2 && mt != 4 && mt != 8) throw std::runtime_error("c8 tiles per workgroup: 1, 2, 4 or 8");
  g_c8_mt = mt;
}

// fwd/dgrad workgroup order after the XCD swizzle (A/B knob): 0 = panel-major
// (an XCD's workgroups share a weight panel and sweep M tiles), 1 = M-major
// (they share M tiles and sweep the panels)

int conv_fwd(uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t stats, uintptr_t slab, int B, int H, int W, int Cin,
             int Cout, int KS, int tile, int splits, uintptr_t stream) {
  const FwdCfg cfg(tile);
  if (g_c8_pair && Cin != 4) throw std::runtime_error("conv_fwd: pair-packed weights need the 4-channel input");
  ConvGeom g = g_c8_pair ? make_geom_pair(B, H, W, Cout, KS) : make_geom(B, H, W, Cin, Cout, KS);
  hipStream_t s = as_stream(stream);
  if (splits < 1) splits = 1;
  if (splits > 1 && !slab) throw std::runtime_error("conv_fwd: split-K needs a slab");
  if (Cout % 8 != 0) throw std::runtime_error("conv_fwd: Cout % 8 != 0");
  if (tile < 0 || tile > 2) throw std::runtime_error("conv_fwd: bad tile id");
  if (Cout % fwd_bn(tile) != 0) throw std::runtime_error("conv_fwd: Cout must be a multiple of the N tile");
  RegionGeom rg{};
  // c8 kernel: mt M tiles per workgroup (largest of g_c8_mt, ..., 2, 1 that keeps
  // >= 256 workgroups and divides the tiles of one image)
  int c8_mt = 1;
  const int c8_ntm = (H * W) % 128 == 0 ? g.M / 128 : 0;
  for (int mt = g_c8_mt; mt > 1; mt /= 2) {
    if (c8_ntm > 0 && (H * W) % (mt * 128) == 0 && c8_ntm % mt == 0 && (c8_ntm / mt) * std::max(1, Cout / 64) >= 256) {
      c8_mt = mt;
      break;
    }
  }
  const int c8_rows = c8_mt * 128 / std::max(1, W) + KS - 1;
  const int c8_chunks = g_c8_pair ? KS * ((KS + 1) / 2) : KS * KS;  // weight chunks per output channel
  const int c8_rslots = g_c8_pair ? (c8_rows * g.Wp + 1) / 2 : c8_rows * g.Wp;  // 16-B region slots (pair: 2 pixels)
  const size_t c8_lds =
      (size_t)((c8_rslots + 2 + 63) / 64 * 64 + (64 * c8_chunks + 63) / 64 * 64) * 16 + 4 * 2 * 64 * 4;
  // the NHWC BN reduce epilogue and the in-launch split-K combine are on the streaming kernel
  const bool streaming_only = g_fix.on;
  if (!streaming_only && tile == 2 && splits == 1 && g_region && g.pow2 && (Cin == 8 || g_c8_pair) && W <= 128 && 128 % W == 0 && (H * W) % 128 == 0 &&
      Cout % 64 == 0 && c8_lds <= 160 * 1024) {
    const int grid = (g.M / 128 / c8_mt) * (Cout / 64);
    auto go = [&](auto kern) {
      static bool attr = false;
      if (!attr) {
        DL_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr = true;
      }
      kern<<<grid, 512, c8_lds, s>>>((const bf16_t*)x, (const bf16_t*)w, (bf16_t*)y, (float*)stats, g, c8_rows,
                                     c8_mt, g_conv_dbg);
    };
    if (g_c8_pair) {
      if (stats) go(conv_fwd_c8_kernel<true, true>);
      else go(conv_fwd_c8_kernel<false, true>);
    } else if (stats) {
      go(conv_fwd_c8_kernel<true>);
    } else {
      go(conv_fwd_c8_kernel<false>);
    }
  } else if (g_c8_pair) {
    throw std::runtime_error("conv_fwd: pair-packed weights need the first-layer kernel (Cin 8, tile 2, no split)");
  } else if (!streaming_only && tile == 0 && region_geom(g, 128, splits, rg)) {
    if (g_region_waves == 4) launch_fwd_region<128, 2, 2>(g, rg, x, w, y, stats, slab, splits, s);
    else launch_fwd_region<128, 2, 4>(g, rg, x, w, y, stats, slab, splits, s);
  } else if (!streaming_only && tile == 2 && region_geom(g, 64, splits, rg)) {
    if (g_region_waves == 4) launch_fwd_region<64, 2, 2>(g, rg, x, w, y, stats, slab, splits, s);
    else launch_fwd_region<64, 4, 2>(g, rg, x, w, y, stats, slab, splits, s);
  }
  else if (tile == 0) launch_fwd<128, 128>(g, x, w, y, stats, slab, splits, s);
  else if (tile == 1) launch_fwd<64, 64>(g, x, w, y, stats, slab, splits, s);
  else if (tile == 2) launch_fwd<128, 64>(g, x, w, y, stats, slab, splits, s);
  else throw std::runtime_error("conv_fwd: bad tile id");
  DL_HIP_CHECK(hipGetLastError());
  if (g_side_sgd.nblk != 0) {  // armed, but this call ran on the region / c8 kernel
    g_side_sgd.nblk = 0;
    throw std::runtime_error("set_conv_side_sgd: the next conv_fwd call must run on the streaming kernel");
  }
  if (splits == 1 || g_fix.on) return (g.M + fwd_bm(tile) - 1) / fwd_bm(tile);
  if (g_fwd_keep_slabs) {
    if (stats) throw std::runtime_error("conv_fwd keep-slabs: no statistics");
    return 0;
  }
  if (256 % (Cout / 8) != 0) throw std::runtime_error("conv_fwd split-K combine: Cout/8 must divide 256");
  const int rpb = combine_rows_per_block(g.M, Cout);
  const int nb = (g.M + rpb - 1) / rpb;
  if (stats)
    splitk_combine_kernel<true><<<nb, 256, 0, s>>>((const float*)slab, (bf16_t*)y, (float*)stats, splits, g.M, Cout,
                                                   rpb, g);
  else
    splitk_combine_kernel<false><<<nb, 256, 0, s>>>((const float*)slab, (bf16_t*)y, nullptr, splits, g.M, Cout, rpb,
                                                    g);
  DL_HIP_CHECK(hipGetLastError());
  return nb;
}

// The next streaming conv_fwd launch also runs the fused SGD update of the
// elements [lo, hi) of the flat buffer p (gradient g, or the split-K slabs of
// the given ranges; bf16 shadow p16 required) as nblk extra workgroups
// (0: one float4 per thread).  One-shot; the caller's final update skips [lo, hi).
void set_conv_side_sgd(uintptr_t p, uintptr_t g, uintptr_t mom, uintptr_t p16, uintptr_t slot, float lr,
                       float momentum, float wd, int64_t lo, int64_t hi, std::vector<int64_t> offs,
                       std::vector<int64_t> lens, std::vector<uintptr_t> slabs, std::vector<int> splits, int nblk) {
  if (!p16) throw std::runtime_error("set_conv_side_sgd: needs the bf16 shadow");
  SgdJob j = make_sgd_job(p, g, mom, p16, slot, lr, momentum, wd, lo, hi, offs, lens, slabs, splits, {}, 0);
  j.nblk = nblk > 0 ? nblk : -1;  // -1: sized by the launch (one float4 per thread)
  g_side_sgd = j;
}

// The next streaming conv_fwd launch sums the split-K weight-gradient slabs of
// the given in-place ranges into the gradient buffer g (a reduce-only side job,
// sgd_dev.h: bitwise slab_reduce's sums) as nblk extra workgroups (0: one
// float4 per thread): a multi-node step's weight gradient, materialised for
// its all-reduce on the CUs the dgrad leaves free instead of in a launch of
// its own.  One-shot.
void set_conv_side_reduce(uintptr_t g, int64_t lo, int64_t hi, std::vector<int64_t> offs, std::vector<int64_t> lens,
                          std::vector<uintptr_t> slabs, std::vector<int> splits, int nblk) {
  if (offs.empty()) throw std::runtime_error("set_conv_side_reduce: no slab range");
  SgdJob j = make_reduce_job(g, lo, hi, offs, lens, slabs, splits, {}, 0);
  j.nblk = nblk > 0 ? nblk : -1;
  g_side_sgd = j;
}

// Whether conv_fwd runs this unsplit shape on the region (tap-reuse) kernel --
// the kernel that carries the fused BN backward reduce epilogue.
int conv_region_ok(int B, int H, int W, int Cin, int Cout, int KS, int tile, int splits) {
  ConvGeom g = make_geom(B, H, W, Cin, Cout, KS);
  RegionGeom rg{};
  const int t = tile & 15;
  if (splits < 1) splits = 1;
  return any_region_geom(g, t, splits, rg) ? 1 : 0;
}

// conv_fwd (a dgrad) with the previous block's BatchNorm backward reduce in its
// epilogue (BnRedArgs): only the region kernel path; returns the number of
// rows written (M tiles, mode 0) or throws if the shape takes another kernel.
int conv_fwd_bnred(uintptr_t x, uintptr_t w, uintptr_t y, int B, int H, int W, int Cin, int Cout, int KS, int tile,
                   uintptr_t y_prev, uintptr_t coef, uintptr_t rows, uintptr_t stream) {
  ConvGeom g = make_geom(B, H, W, Cin, Cout, KS);
  RegionGeom rg{};
  const int t = tile & 15;
  if (!any_region_geom(g, t, 1, rg))
    throw std::runtime_error("conv_fwd_bnred: the shape does not take the region kernel");
  if (!rows || !coef || !y_prev) throw std::runtime_error("conv_fwd_bnred: null operand");
  g_bnred = BnRedArgs{(const bf16_t*)y_prev, (const float*)coef, (float*)rows};
  int T;
  try {
    T = conv_fwd(x, w, y, 0, 0, B, H, W, Cin, Cout, KS, tile, 1, stream);
  } catch (...) {
    g_bnred = BnRedArgs{};
    throw;
  }
  g_bnred = BnRedArgs{};
  return T;
}

// conv_fwd of a split-K plan whose slices are combined inside the launch
// (FIX, splitk_fixup) instead of by splitk_combine / combine_bwd_reduce: the
// reducer of each tile writes bf16 y and either the BN statistics (stats) or,
// y_prev != 0 (a dgrad), the BatchNorm backward reduce of the block below
// into rows (conv_fwd_bnred's epilogue, BNR 1).  128x64 streaming tiles only
// (conv_fix_ok).  Returns the rows written (M tiles).
int conv_fwd_fix(uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t stats, uintptr_t slab, int B, int H, int W, int Cin,
                 int Cout, int KS, int tile, int splits, uintptr_t y_prev, uintptr_t coef, uintptr_t rows,
                 uintptr_t stream) {
  if (splits < 2 || !slab) throw std::runtime_error("conv_fwd_fix: a split-K plan with a slab");
  if ((y_prev != 0) != (rows != 0) || (y_prev && !coef)) throw std::runtime_error("conv_fwd_fix: BN reduce operands");
  g_fix.on = true;
  g_fix.bnred = y_prev ? BnRedArgs{(const bf16_t*)y_prev, (const float*)coef, (float*)rows} : BnRedArgs{};
  int T;
  try {
    T = conv_fwd(x, w, y, stats, slab, B, H, W, Cin, Cout, KS, tile, splits, stream);
  } catch (...) {
    g_fix = FixState{};
    throw;
  }
  g_fix = FixState{};
  return T;
}

// Whether conv_fwd_fix serves this plan (the 128x64 streaming tile, 8 waves,
// the transposed epilogue; no balanced position-major split).
int conv_fix_ok(int B, int H, int W, int Cin, int Cout, int KS, int tile, int splits) {
  (void)B; (void)H; (void)W;
  const int t = tile & 15, wv = (tile >> 8) & 15;
  return (t == 2 && splits >= 2 && Cin >= 64 && Cout % 64 == 0 && KS >= 1 && (wv == 0 ? g_fwd_waves : wv) == 8 &&
          true)
             ? 1
             : 0;
}

// y = conv(x, w) + addend (bf16, same layout as y), streaming kernel only
// (KS = 1 or the region kernels disabled for the shape), no split-K / stats.
void conv_fwd_add(uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t addend, int B, int H, int W, int Cin, int Cout,
                  int KS, int tile, uintptr_t stream, uintptr_t addend_mask) {
  const FwdCfg cfg(tile);
  ConvGeom g = make_geom(B, H, W, Cin, Cout, KS);
  hipStream_t s = as_stream(stream);
  if (!addend) throw std::runtime_error("conv_fwd_add: null addend");
  if (Cout % fwd_bn(tile) != 0) throw std::runtime_error("conv_fwd_add: Cout must be a multiple of the N tile");
  if (KS != 1 && g_region) throw std::runtime_error("conv_fwd_add: only the streaming kernel (KS = 1)");
  g_fwd_addend = addend;
  g_fwd_addend_mask = addend_mask;
  try {
    if (tile == 0) launch_fwd<128, 128>(g, x, w, y, 0, 0, 1, s);
    else if (tile == 1) launch_fwd<64, 64>(g, x, w, y, 0, 0, 1, s);
    else if (tile == 2) launch_fwd<128, 64>(g, x, w, y, 0, 0, 1, s);
    else throw std::runtime_error("conv_fwd_add: bad tile id");
  } catch (...) {
    g_fwd_addend = g_fwd_addend_mask = 0;
    throw;
  }
  g_fwd_addend = g_fwd_addend_mask = 0;
  DL_HIP_CHECK(hipGetLastError());
}

// ---- generalised geometry (strided / KH x KW / phase-mapped convolutions) ----
// The ResNet-50 convolutions that are not stride-1 odd-square: the stride-2
// 1x1 downsample and 3x3 convs, the stem (a stride-2 7x7 over 3 channels,
// rewritten as a 4x4 stride-1 conv over its 2x2 space-to-depth image: 12 -> 16
// channels), and the stride-2 convs' input gradients (one phase conv per
// output parity, stored interleaved through the epilogue's output map).
// Streaming forward kernel and wgrad kernel only, float-reciprocal pixel
// addressing (never the pow2 / region / c8 paths).
static ConvGeom make_geom_ex(int B, int Ho, int Wo, int Hp, int Wp, int Cin, int Cout, int KH, int KW, int S) {
  if (KH < 1 || KW < 1 || S < 1) throw std::runtime_error("conv_ex: bad kernel / stride");
  if (Hp < S * (Ho - 1) + KH || Wp < S * (Wo - 1) + KW) throw std::runtime_error("conv_ex: input buffer too small");
  ConvGeom g = make_geom(B, Ho, Wo, Cin, Cout, 1);
  g.KS = std::max(KH, KW);
  g.pad = 0;
  g.Hp = Hp; g.Wp = Wp;
  g.S = S; g.KH = KH; g.KW = KW;
  g.dHp = Ho; g.dWp = Wo; g.dpad = 0;
  g.pow2 = 0;
  g.K = KH * KW * Cin;
  g.Kch = g.K / 8;
  if ((int64_t)B * Ho * Wo >= (1 << 24)) throw std::runtime_error("conv_ex: B*Ho*Wo must be < 2^24");
  if ((int64_t)B * Hp * Wp * std::max(Cin, Cout) >= (1ll << 31) || (int64_t)Cout * g.K >= (1ll << 31))
    throw std::runtime_error("conv_ex: operand too large for 32-bit offsets");
  return g;
}

// y[om(m)] = conv(x, w)[m] (+ addend[om(m)] when addend != 0: an in-place
// accumulate when addend == y) with the generalised geometry; om_S == 0: no
// output map.  Returns the number of BN statistics rows (stats != 0, no split).
int conv_fwd_ex(uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t stats, uintptr_t slab, int B, int Ho, int Wo, int Hp,
                int Wp, int Cin, int Cout, int KH, int KW, int S, int om_S, int om_H0, int om_W0, int om_W, int om_HW,
                uintptr_t addend, int tile, int splits, uintptr_t stream) {
  const FwdCfg cfg(tile);
  ConvGeom g = make_geom_ex(B, Ho, Wo, Hp, Wp, Cin, Cout, KH, KW, S);
  if (om_S > 0) {
    g.om = 1; g.omS = om_S; g.omH0 = om_H0; g.omW0 = om_W0; g.omW = om_W; g.omHW = om_HW;
    if ((int64_t)B * om_HW * std::max(Cin, Cout) >= (1ll << 31)) throw std::runtime_error("conv_fwd_ex: output too large");
  }
  hipStream_t s = as_stream(stream);
  if (splits < 1) splits = 1;
  if (splits > 1 && (!slab || addend || g.om)) throw std::runtime_error("conv_fwd_ex: split-K needs a slab, no addend / map");
  if (stats && (addend || splits > 1)) throw std::runtime_error("conv_fwd_ex: statistics need a plain, unsplit output");
  if (Cin % 8 != 0 || (Cin < 64 && Cin % 8 != 0)) throw std::runtime_error("conv_fwd_ex: Cin % 8 != 0");
  if (Cin >= 64 && Cin % 64 != 0) throw std::runtime_error("conv_fwd_ex: Cin >= 64 must be a multiple of 64");
  if (tile < 0 || tile > 2) throw std::runtime_error("conv_fwd_ex: bad tile id");
  if (Cout % fwd_bn(tile) != 0) throw std::runtime_error("conv_fwd_ex: Cout must be a multiple of the N tile");
  g_fwd_addend = addend;
  try {
    if (tile == 0) launch_fwd<128, 128>(g, x, w, y, stats, slab, splits, s);
    else if (tile == 1) launch_fwd<64, 64>(g, x, w, y, stats, slab, splits, s);
    else launch_fwd<128, 64>(g, x, w, y, stats, slab, splits, s);
  } catch (...) {
    g_fwd_addend = 0;
    throw;
  }
  g_fwd_addend = 0;
  DL_HIP_CHECK(hipGetLastError());
  if (splits == 1) return (g.M + fwd_bm(tile) - 1) / fwd_bm(tile);
  if (g_fwd_keep_slabs) return 0;
  if (256 % (Cout / 8) != 0) throw std::runtime_error("conv_fwd_ex split-K combine: Cout/8 must divide 256");
  const int rpb = combine_rows_per_block(g.M, Cout);
  const int nb = (g.M + rpb - 1) / rpb;
  splitk_combine_kernel<false><<<nb, 256, 0, s>>>((const float*)slab, (bf16_t*)y, nullptr, splits, g.M, Cout, rpb, g);
  DL_HIP_CHECK(hipGetLastError());
  return nb;
}

// out: fp32 [splits][Cout][ldo] weight-gradient slabs of a generalised-geometry
// conv: x as in conv_fwd_ex, dy [B][dHp][dWp][Cout] with the output interior at dpad.
void conv_wgrad_ex(uintptr_t dy, uintptr_t x, uintptr_t out, int B, int Ho, int Wo, int Hp, int Wp, int dHp, int dWp,
                   int dpad, int Cin, int Cout, int KH, int KW, int S, int splits, int ldo, int tile,
                   uintptr_t stream);

// out: fp32 [splits][Cout][ldo], ldo >= K (K = KS*KS*Cin); tile 1 = 64x64, 2 = 128x128 (co x k)
static void conv_wgrad_g(const ConvGeom& g, uintptr_t dy, uintptr_t x, uintptr_t out, int splits, int ldo, int tile,
                         uintptr_t stream);

void conv_wgrad(uintptr_t dy, uintptr_t x, uintptr_t out, int B, int H, int W, int Cin, int Cout, int KS, int splits,
                int ldo, int tile, int atomic_creal, uintptr_t stream) {
  if (atomic_creal != 0) throw std::runtime_error("conv_wgrad: atomic split-K was removed in round 6 (pass 0)");
  if ((tile >> 24) & 1) {  // pair-packed first layer (make_geom_pair): x is [B][Hp][Wp][4]
    if (Cin != 4) throw std::runtime_error("conv_wgrad: the pair-packed layout needs a 4-channel input");
    conv_wgrad_g(make_geom_pair(B, H, W, Cout, KS), dy, x, out, splits, ldo, tile & 15, stream);
    return;
  }
  conv_wgrad_g(make_geom(B, H, W, Cin, Cout, KS), dy, x, out, splits, ldo, tile, stream);
}

void conv_wgrad_ex(uintptr_t dy, uintptr_t x, uintptr_t out, int B, int Ho, int Wo, int Hp, int Wp, int dHp, int dWp,
                   int dpad, int Cin, int Cout, int KH, int KW, int S, int splits, int ldo, int tile,
                   uintptr_t stream) {
  ConvGeom g = make_geom_ex(B, Ho, Wo, Hp, Wp, Cin, Cout, KH, KW, S);
  g.dsep = 1; g.dHp = dHp; g.dWp = dWp; g.dpad = dpad;
  if (dHp < Ho + dpad || dWp < Wo + dpad) throw std::runtime_error("conv_wgrad_ex: dy buffer too small");
  if ((int64_t)B * dHp * dWp * Cout >= (1ll << 31)) throw std::runtime_error("conv_wgrad_ex: dy too large");
  conv_wgrad_g(g, dy, x, out, splits, ldo, tile, stream);
}

static void conv_wgrad_g(const ConvGeom& g, uintptr_t dy, uintptr_t x, uintptr_t out, int splits, int ldo, int tile,
                         uintptr_t stream) {
  const int Cout = g.Cout, W = g.W;
  if (tile != 1 && tile != 2) throw std::runtime_error("conv_wgrad: tile 1 (64x64) or 2 (128x128)");
  if (ldo < g.K) throw std::runtime_error("conv_wgrad: ldo < K");
  if (ldo % 4 != 0) throw std::runtime_error("conv_wgrad: ldo % 4 != 0 (16-byte slab stores)");
  if (Cout % 8 != 0) throw std::runtime_error("conv_wgrad: Cout % 8 != 0");
  const int bm = tile == 1 ? 64 : 128;
  if (Cout % bm != 0) throw std::runtime_error("conv_wgrad: Cout must be a multiple of the Cout tile");
  if (g.pow2 && W > 64) throw std::runtime_error("conv_wgrad: needs W <= 64");
  if (splits < 1) splits = 1;
  int mps = (g.M + splits - 1) / splits;
  mps = (mps + 63) / 64 * 64;  // 64-row aligned M steps (padded-layout addressing)
  hipStream_t s = as_stream(stream);
  // 4-stage LDS-DMA rings with fragment prefetch: 64x64 tiles (2 WGs per CU:
  // wgrad1 22.1 -> 16.8 us vs 3 stages), 128x128 tiles (1 WG per CU, 128 KiB
  // LDS, 141 VGPRs: wgrad2/3/4 31.7/29.7/28.4 us as 128x64 -> 24.7/23.0/21.8 us;
  // the waves wait on the LDS-DMA ring, so the deeper ring wins over occupancy)
  SgdJob side = g_side_sgd;  // one-shot: consumed by this launch
  g_side_sgd.nblk = 0;
  auto go = [&](auto kern, int BM_, int BN_, int NT_) {
    const int nt = ((g.Cout + BM_ - 1) / BM_) * ((g.K + BN_ - 1) / BN_);
    if (side.nblk < 0) side.nblk = (int)std::max<int64_t>(1, (side.hi4 - side.lo4 + NT_ - 1) / NT_);
    kern<<<nt * splits + side.nblk, NT_, 0, s>>>((const bf16_t*)dy, (const bf16_t*)x, (float*)out, g, mps, ldo, side);
  };
  if (tile == 2) go(conv_wgrad_kernel<128, 128, 4, 2, 4>, 128, 128, 512);
  else go(conv_wgrad_kernel<64, 64, 4, 2, 4>, 64, 64, 512);
  DL_HIP_CHECK(hipGetLastError());
}

void set_reduce_atomic_conv(int rows) {
  if (rows < 0 || rows > 64 || (rows & (rows - 1)) != 0)
    throw std::runtime_error("set_reduce_atomic: rows must be 0 or a power of two <= 64");
  const int v = rows;
  DL_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_red_atomic), &v, sizeof(int)));
  g_red_atomic_host = rows;
}

template <bool ACC, bool OIHW = false>
static void slab_reduce_t(uintptr_t slabs, uintptr_t dst, int splits, int Cout, int taps, int Cp, int C,
                          uintptr_t stream) {
  auto s = as_stream(stream);
  const int g = slab_reduce_grid(splits, Cout, taps, C);
  const int tpo = slab_reduce_tpo(splits);
  if (tpo == 32)
    slab_reduce_kernel<32, ACC, OIHW><<<g, 256, 0, s>>>((const float*)slabs, (float*)dst, splits, Cout, taps, Cp, C);
  else if (tpo == 8)
    slab_reduce_kernel<8, ACC, OIHW><<<g, 256, 0, s>>>((const float*)slabs, (float*)dst, splits, Cout, taps, Cp, C);
  else
    slab_reduce_kernel<1, ACC, OIHW><<<g, 256, 0, s>>>((const float*)slabs, (float*)dst, splits, Cout, taps, Cp, C);
  DL_HIP_CHECK(hipGetLastError());
}

void slab_reduce(uintptr_t slabs, uintptr_t dst, int splits, int Cout, int taps, int Cp, int C, uintptr_t stream) {
  slab_reduce_t<false>(slabs, dst, splits, Cout, taps, Cp, C, stream);
}

// dst += sum of the slabs (the ResNet-50 1x1 weight gradients: plain slab
// stores + this reduce beat the atomic split-K 1.3-2.3x, profiles/r2_gemm1x1_wgrad_slab.jsonl)
void slab_reduce_add(uintptr_t slabs, uintptr_t dst, int splits, int Cout, int taps, int Cp, int C, uintptr_t stream) {
  slab_reduce_t<true>(slabs, dst, splits, Cout, taps, Cp, C, stream);
}

// dst [Cout][C][taps] (OIHW, the flat gradient of a KxK conv weight) += sum of the slabs
void slab_reduce_add_oihw(uintptr_t slabs, uintptr_t dst, int splits, int Cout, int taps, int Cp, int C,
                          uintptr_t stream) {
  slab_reduce_t<true, true>(slabs, dst, splits, Cout, taps, Cp, C, stream);
}

void weight_flip_transpose(uintptr_t w, uintptr_t wt, int Cout, int Cin, int KS, uintptr_t stream) {
  dim3 grid((Cin + 31) / 32, (Cout + 31) / 32, KS * KS);
  weight_flip_transpose_kernel<<<grid, 256, 0, as_stream(stream)>>>((const bf16_t*)w, (bf16_t*)wt, Cout, Cin, KS);
  DL_HIP_CHECK(hipGetLastError());
}

// table_dev: n TrEntry on the device (32 bytes each; built once by the caller,
// ops/conv.py WeightTransposes, and reused by every step / graph replay).
void transpose_many(uintptr_t table_dev, int n, int total_tiles, uintptr_t stream) {
  if (n <= 0) return;
  if (total_tiles <= 0) throw std::runtime_error("transpose_many: no tiles");
  transpose_many_kernel<<<total_tiles, 256, 0, as_stream(stream)>>>((const TrEntry*)table_dev, n);
  DL_HIP_CHECK(hipGetLastError());
}

int transpose_entry_bytes() { return (int)sizeof(TrEntry); }

void weights_to_cl(uintptr_t table_dev, int n, uintptr_t stream) {
  if (n <= 0) return;
  weights_to_cl_kernel<<<dim3(256, n), 256, 0, as_stream(stream)>>>((const ClEntry*)table_dev);
  DL_HIP_CHECK(hipGetLastError());
}

int cl_entry_bytes() { return (int)sizeof(ClEntry); }

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
