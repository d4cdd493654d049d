// Host-side launcher declarations for every HIP kernel in csrc/kernels.
// All take raw device pointers (uintptr_t) and a HIP stream handle so that the
// Python layer can enqueue them on torch streams (and inside hipGraph capture).
#pragma once
#include <stdint.h>

#include <vector>

namespace dl {

// flat_ops.hip -------------------------------------------------------------
void sgd_update(uintptr_t p, uintptr_t g, uintptr_t mom, uintptr_t p16, uintptr_t slot, float lr, float momentum,
                float wd, int64_t n, uintptr_t stream);
void scale_by_count(uintptr_t x, uintptr_t slot, int64_t n, uintptr_t stream);
void elastic_step(uintptr_t p, uintptr_t c, uintptr_t pending, uintptr_t out, uintptr_t p16, float alpha, int64_t n,
                  uintptr_t stream);
void add_inplace(uintptr_t y, uintptr_t x, int64_t n, uintptr_t stream);
void fill_f32(uintptr_t x, float v, int64_t n, int64_t slot_index, float slot_value, uintptr_t stream);
void elastic_step_wire16(uintptr_t p, uintptr_t c, uintptr_t out, uintptr_t out16, uintptr_t p16, float alpha,
                         int64_t n, uintptr_t stream);
void stamp_time(uintptr_t slot, uintptr_t stream);
int wall_clock_khz();
void cast_f32_bf16(uintptr_t x, uintptr_t y, int64_t n, uintptr_t stream);
void cast_bf16_f32(uintptr_t x, uintptr_t y, int64_t n, uintptr_t stream);
// the next streaming conv_fwd launch also runs the SGD of flat elements [lo, hi)
// as nblk extra workgroups (conv_igemm.hip; flat_ops' update then skips them)
void set_conv_side_sgd(uintptr_t p, uintptr_t g, uintptr_t mom, uintptr_t p16, uintptr_t slot, float lr,
                       float momentum, float wd, int64_t lo, int64_t hi, std::vector<int64_t> offs,
                       std::vector<int64_t> lens, std::vector<uintptr_t> slabs, std::vector<int> splits, int nblk);
// ... or sums split-K weight-gradient slabs into the gradient buffer g instead
// (reduce-only side job: a multi-node step's gradients before the all-reduce)
void set_conv_side_reduce(uintptr_t g, int64_t lo, int64_t hi, std::vector<int64_t> offs, std::vector<int64_t> lens,
                          std::vector<uintptr_t> slabs, std::vector<int> splits, int nblk);
void sgd_update_g16(uintptr_t p, uintptr_t g16, uintptr_t mom, uintptr_t p16, uintptr_t slot, float lr,
                    float momentum, float wd, int64_t n, uintptr_t stream);
// sgd_update whose gradient in up to 4 ranges [offs, offs+lens) is the sum of the
// split-K slabs [splits][lens] at slabs[j], and in one optional channel-padded
// "tail" range (offset, numel, splits, Cout, taps, Cp, C) the sum of tail_slab
// (bitwise slab_reduce's sums); elements [skip_lo, skip_hi) are left alone (a
// conv launch's side job updated them: set_conv_side_sgd)
void sgd_update_slabs(uintptr_t p, uintptr_t g, uintptr_t mom, uintptr_t p16, uintptr_t slot, float lr,
                      float momentum, float wd, int64_t n, std::vector<int64_t> offs, std::vector<int64_t> lens,
                      std::vector<uintptr_t> slabs, std::vector<int> splits, std::vector<int64_t> tail,
                      uintptr_t tail_slab, int64_t skip_lo, int64_t skip_hi, uintptr_t stream);
// one-shot: the next sgd_update_slabs launch also prepares the next step of an
// unrolled graph -- gathers its batch into xp, zeroes its accumulators (prep_dev.h)
// and writes the first layer's updated weights into the packed bf16 operand w1p
// (from the slab tail, or from the main loop's elements [pack_off, +pack_len))
void arm_sgd_next_prep(uintptr_t img, uintptr_t order, uintptr_t lab_all, uintptr_t lab_out, uintptr_t ctr,
                       int n_order, int B, int C, std::vector<float> mean, std::vector<float> stdv, uintptr_t xp,
                       int Cp, int H, int W, int sp, std::vector<uintptr_t> zp, std::vector<int64_t> zn,
                       uintptr_t w1p, int w1_cp, int64_t pack_off, int64_t pack_len);
bool sgd_next_prep_armed();
// reduce-only launch: split-K slabs of up to 4 ranges + 1 padded tail summed into g
void slab_reduce_multi(uintptr_t g, int64_t n, std::vector<int64_t> offs, std::vector<int64_t> lens,
                       std::vector<uintptr_t> slabs, std::vector<int> splits, std::vector<int64_t> tail,
                       uintptr_t tail_slab, uintptr_t stream);
void set_sgd_trim(bool on);  // update grid sized to the elements before a skipped suffix (default on)
void disarm_sgd_next_prep();

// metrics.hip ---------------------------------------------------------------
// channels-last training BatchNorm (+ReLU, +residual) for the ResNet-50 path
void bn_nhwc_fwd_pad(uintptr_t x, uintptr_t res, uintptr_t y, uintptr_t acc, uintptr_t w, uintptr_t b,
                     uintptr_t save, uintptr_t run_mean, uintptr_t run_var, int64_t M, int C, double eps,
                     double momentum, int relu, int have_stats, int H, int W, int opad, uintptr_t stream,
                     uintptr_t mbits = 0, uintptr_t rbn_acc = 0, uintptr_t rbn_w = 0, uintptr_t rbn_b = 0,
                     uintptr_t rbn_save = 0, uintptr_t rbn_rm = 0, uintptr_t rbn_rv = 0, double rbn_eps = 1e-5,
                     double rbn_momentum = 0.1);
void bn_nhwc_bwd_pad(uintptr_t dy, uintptr_t y, uintptr_t x, uintptr_t save, uintptr_t w, uintptr_t b,
                     uintptr_t acc, uintptr_t dx, uintptr_t dres, uintptr_t dw, uintptr_t db, int64_t M, int C,
                     int relu, int H, int W, int opad, uintptr_t stream, int have_sums = 0, uintptr_t mbits = 0,
                     uintptr_t rbn_x = 0, uintptr_t rbn_save = 0, uintptr_t rbn_w = 0, uintptr_t rbn_acc = 0,
                     uintptr_t rbn_dw = 0, uintptr_t rbn_db = 0);
void zero_border_nhwc(uintptr_t buf, int N, int H, int W, int C, int pad, uintptr_t stream);
void bn_nhwc_fwd(uintptr_t x, uintptr_t res, uintptr_t y, uintptr_t acc, uintptr_t w, uintptr_t b, uintptr_t save,
                 uintptr_t run_mean, uintptr_t run_var, int64_t M, int C, double eps, double momentum, int relu, int have_stats,
                 uintptr_t stream);
void set_bn_reduce_blocks(int n);
void set_bn_tuning(int apply_rows, int reduce_threads);
void set_bn_minw(int fwd, int bwd);
// acc[0:2C] += the column sums of T partial rows [T][2][C] (acc zeroed by the caller)
void bn_rows_reduce(uintptr_t rows, int T, int C, uintptr_t acc, uintptr_t stream);
void bn_nhwc_bwd(uintptr_t dy, uintptr_t y, uintptr_t x, uintptr_t save, uintptr_t w, uintptr_t b, uintptr_t acc,
                 uintptr_t dx,
                 uintptr_t dres, uintptr_t dw, uintptr_t db, int64_t M, int C, int relu, uintptr_t stream);
void confusion_update(uintptr_t pred, int pred_is_bf16, uintptr_t target, uintptr_t mat, int B, int C,
                      uintptr_t stream);
void gather_normalize(uintptr_t images, uintptr_t idx, uintptr_t out, int B, int HW, int Cs, int Cd, float m0,
                      float m1, float m2, float s0, float s1, float s2, uintptr_t stream);

// conv_igemm.hip --------------------------------------------------------------
// NHWC activations, KRSC weights, stride 1, same padding, Cin power of two >= 8.
int conv_fwd(uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t stats, uintptr_t slab, int B, int H, int W, int Cin,
             int Cout, int KS, int tile, int splits, uintptr_t stream);
int conv_fwd_stat_rows(int B, int H, int W, int Cin, int Cout, int KS, int tile, int splits);
void set_conv_region(int on);
void set_bn_bwd_items(int n);
void set_conv_region_ablate(int a);
void set_conv_region_waves(int w);
void set_conv_region_stages(int st);
void set_conv_stages(int fwd, int wgrad);
void set_conv_waves(int waves);
void set_conv_debug(uintptr_t buf);
void set_conv_fwd_pf(int on);
void set_head_stamps(uintptr_t buf);
void set_bn_stamps(uintptr_t buf);
void set_conv_wgrad_stamps(uintptr_t buf);
// the next conv_fwd (region kernel, forward with statistics) pools its input on load
// from the previous block's pre-BN output (BN coefficients from its accumulated sums)
int conv_region_ok(int B, int H, int W, int Cin, int Cout, int KS, int tile, int splits = 1);
int conv_fwd_fix(uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t stats, uintptr_t slab, int B, int H, int W, int Cin,
                 int Cout, int KS, int tile, int splits, uintptr_t y_prev, uintptr_t coef, uintptr_t rows,
                 uintptr_t stream);
int conv_fix_ok(int B, int H, int W, int Cin, int Cout, int KS, int tile, int splits);
int conv_fwd_bnred(uintptr_t x, uintptr_t w, uintptr_t y, int B, int H, int W, int Cin, int Cout, int KS, int tile,
                   uintptr_t y_prev, uintptr_t coef, uintptr_t rows, uintptr_t stream);
int conv_fwd_ex(uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t stats, uintptr_t slab, int B, int Ho, int Wo, int Hp,
                int Wp, int Cin, int Cout, int KH, int KW, int S, int om_S, int om_H0, int om_W0, int om_W, int om_HW,
                uintptr_t addend, int tile, int splits, uintptr_t stream);
void conv_wgrad_ex(uintptr_t dy, uintptr_t x, uintptr_t out, int B, int Ho, int Wo, int Hp, int Wp, int dHp, int dWp,
                   int dpad, int Cin, int Cout, int KH, int KW, int S, int splits, int ldo, int tile,
                   uintptr_t stream);
// first-layer weight gradient from an LDS-resident input region (Cin 8, Cout 64):
// fp32 slabs [B * H / R][64][ldo]; returns the split count
// position-major wgrad plan at `steps` K steps per workgroup: {max splits a
// column tile needs, workgroups with work} ({0, 0}: B does not take it)
void conv_wgrad(uintptr_t dy, uintptr_t x, uintptr_t out, int B, int H, int W, int Cin, int Cout, int KS, int splits,
                int ldo, int tile, int atomic_creal, uintptr_t stream);
void set_reduce_atomic_conv(int rows);
void conv_fwd_add(uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t addend, int B, int H, int W, int Cin, int Cout,
                  int KS, int tile, uintptr_t stream, uintptr_t addend_mask = 0);
void set_conv_posm(int on);
void set_conv_c8_mt(int mt);
void slab_reduce(uintptr_t slabs, uintptr_t dst, int splits, int Cout, int taps, int Cp, int C, uintptr_t stream);
void slab_reduce_add(uintptr_t slabs, uintptr_t dst, int splits, int Cout, int taps, int Cp, int C, uintptr_t stream);
void slab_reduce_add_oihw(uintptr_t slabs, uintptr_t dst, int splits, int Cout, int taps, int Cp, int C,
                          uintptr_t stream);
void transpose_many(uintptr_t table_dev, int n, int total_tiles, uintptr_t stream);
int transpose_entry_bytes();
void weights_to_cl(uintptr_t table_dev, int n, uintptr_t stream);
int cl_entry_bytes();
void weight_flip_transpose(uintptr_t w, uintptr_t wt, int Cout, int Cin, int KS, uintptr_t stream);
void pack_weight(uintptr_t w, uintptr_t wp, int Cout, int taps, int C, int Cp, uintptr_t stream);
void pad_channels(uintptr_t x, uintptr_t xp, int64_t P, int C, int Cp, uintptr_t stream);
void prep_step(uintptr_t x, uintptr_t xp, int64_t P, int C, int Cp, int H, int W, int sp, uintptr_t w1, uintptr_t w1p,
               int w1_cout, int taps, int w1_c, int w1_cp, std::vector<uintptr_t> tw, std::vector<uintptr_t> twt,
               std::vector<int> tcout, std::vector<int> tcin, std::vector<uintptr_t> zp, std::vector<int64_t> zn,
               uintptr_t stream);
void prep_step_gather(uintptr_t img, uintptr_t order, uintptr_t lab_all, uintptr_t lab_out, uintptr_t ctr,
                      int n_order, int B, int C, std::vector<float> mean, std::vector<float> stdv, uintptr_t xp,
                      int Cp, int H, int W, int sp, uintptr_t w1, uintptr_t w1p, int w1_cout, int taps, int w1_c,
                      int w1_cp, std::vector<uintptr_t> tw, std::vector<uintptr_t> twt, std::vector<int> tcout,
                      std::vector<int> tcin, std::vector<uintptr_t> zp, std::vector<int64_t> zn, uintptr_t stream);

// bn_pool.hip -----------------------------------------------------------------
void bn_finalize(uintptr_t partial, int T, int C, int64_t M, uintptr_t gamma, uintptr_t beta, uintptr_t bias,
                 uintptr_t rmean, uintptr_t rvar, float eps, float momentum, int mode, uintptr_t coef,
                 uintptr_t stream);
void bn_relu_pool_fwd(uintptr_t y, uintptr_t coef, uintptr_t out, int B, int H, int W, int C, int opad,
                      uintptr_t stream);
int bn_bwd_blocks(int B, int H, int W, int C);
int combine_bwd_reduce(uintptr_t slab, int splits, uintptr_t dP, uintptr_t y, uintptr_t coef, uintptr_t partial, int B,
                       int H, int W, int C, uintptr_t stream);
int combine_bwd_reduce_blocks(int B, int H, int W, int C);
void bn_relu_pool_bwd_reduce(uintptr_t y, uintptr_t dP, uintptr_t coef, uintptr_t partial, int B, int H, int W, int C,
                             int blocks, uintptr_t stream);
void bn_bwd_finalize(uintptr_t partial, int T, int C, int64_t M, uintptr_t gamma, uintptr_t coef, uintptr_t dgamma,
                     uintptr_t dbeta, uintptr_t acoef, uintptr_t stream);
void bn_relu_pool_bwd_apply(uintptr_t y, uintptr_t dP, uintptr_t coef, uintptr_t acoef, uintptr_t dy, int B, int H,
                            int W, int C, int opad, uintptr_t stream);
void bn_relu_pool_bwd_apply_sums(uintptr_t y, uintptr_t dP, uintptr_t coef, uintptr_t dgb, uintptr_t gamma, int64_t M,
                                 uintptr_t dy, int B, int H, int W, int C, int opad, uintptr_t dgamma_out,
                                 uintptr_t dbeta_out, uintptr_t stream);
void bn_relu_pool_fwd_fin(uintptr_t y, uintptr_t sums, int64_t M, uintptr_t gamma, uintptr_t beta, uintptr_t bias,
                          uintptr_t rmean, uintptr_t rvar, float eps, float momentum, uintptr_t coef, uintptr_t out,
                          int B, int H, int W, int C, int opad, uintptr_t stream);
void set_reduce_atomic_bn(int rows);
int reduce_rows();
void set_bn_fin_grid(int cap);

// head.hip --------------------------------------------------------------------
void head_fwd_bwd(uintptr_t h, uintptr_t w, uintptr_t bias, uintptr_t labels, int F, int B, int NC,
                  uintptr_t logits_out, uintptr_t dlogits, uintptr_t loss_b, uintptr_t dh, uintptr_t stream);
void bn_bwd_reduce_slab(uintptr_t y, uintptr_t dP, uintptr_t coef, uintptr_t partial, int B, int H, int W, int C,
                        int blocks, uintptr_t slabs, uintptr_t dst, int splits, int Cout, int taps, int Cp, int Creal,
                        uintptr_t stream);
void bn_bwd_reduce_head(uintptr_t y, uintptr_t dP, uintptr_t coef, uintptr_t partial, int B, int H, int W, int C,
                        int blocks, uintptr_t h, uintptr_t dlogits, uintptr_t loss_b, int F, int NC, uintptr_t dw,
                        uintptr_t db, uintptr_t loss, uintptr_t slot, uintptr_t step_ctr, uintptr_t stream);
void head_fwd_bwd_pool(uintptr_t y, uintptr_t coef, int yH, int yW, int yC, uintptr_t h_out, uintptr_t w,
                       uintptr_t bias, uintptr_t labels, int B, int NC, uintptr_t logits_out, uintptr_t dlogits,
                       uintptr_t loss_b, uintptr_t dh, uintptr_t fin_sums, int64_t fin_m, uintptr_t gamma,
                       uintptr_t beta, uintptr_t conv_bias, uintptr_t rmean, uintptr_t rvar, float eps, float momentum,
                       uintptr_t red_rows, uintptr_t stream);
void head_fwd_bwd_pool_wt(uintptr_t y, uintptr_t coef, int yH, int yW, int yC, uintptr_t h_out, uintptr_t w,
                          uintptr_t bias, uintptr_t labels, int B, int NC, uintptr_t logits_out, uintptr_t dlogits,
                          uintptr_t loss_b, uintptr_t dh, uintptr_t fin_sums, int64_t fin_m, uintptr_t gamma,
                          uintptr_t beta, uintptr_t conv_bias, uintptr_t rmean, uintptr_t rvar, float eps,
                          float momentum, uintptr_t red_rows, uintptr_t stream, std::vector<uintptr_t> tw,
                          std::vector<uintptr_t> twt, std::vector<int> tcout, std::vector<int> tcin, int taps);
void bn_bwd_apply_head(uintptr_t y, uintptr_t dP, uintptr_t coef, uintptr_t dgb, uintptr_t gamma, int64_t M,
                       uintptr_t dy, int B, int H, int W, int C, int opad, uintptr_t dgamma_out, uintptr_t dbeta_out,
                       uintptr_t h, uintptr_t dlogits, uintptr_t loss_b, int F, int NC, uintptr_t dw, uintptr_t db,
                       uintptr_t loss, uintptr_t slot, uintptr_t step_ctr, uintptr_t stream);
void head_wgrad(uintptr_t h, uintptr_t dlogits, uintptr_t loss_b, int F, int B, int NC, uintptr_t dw, uintptr_t db,
                uintptr_t loss, uintptr_t slot, uintptr_t step_ctr, uintptr_t stream);

// pool_nhwc.hip ----------------------------------------------------------------
// stem max-pool backward fused with its input BN + ReLU's backward (pool_nhwc.hip)
void maxpool_bn_bwd(uintptr_t dy, uintptr_t idx, uintptr_t x, uintptr_t save, uintptr_t w, uintptr_t b,
                    uintptr_t acc, uintptr_t dx, uintptr_t dw, uintptr_t db, int N, int H, int W, int C,
                    uintptr_t stream);
void maxpool_nhwc_fwd(uintptr_t x, uintptr_t y, uintptr_t idx, int N, int H, int W, int C, int K, int S, int P,
                      uintptr_t stream, uintptr_t bn_acc = 0, uintptr_t bn_w = 0, uintptr_t bn_b = 0,
                      uintptr_t bn_save = 0, uintptr_t bn_rm = 0, uintptr_t bn_rv = 0, double bn_eps = 1e-5,
                      double bn_momentum = 0.1);
void maxpool_nhwc_bwd(uintptr_t dy, uintptr_t idx, uintptr_t dx, int N, int H, int W, int C, int K, int S, int P,
                      uintptr_t stream);

// mnist.hip -------------------------------------------------------------------
void mnist_step(uintptr_t x, int x_bf16, uintptr_t labels, uintptr_t w1, uintptr_t b1, uintptr_t w2, uintptr_t b2,
                uintptr_t wf, uintptr_t bf, uintptr_t gw1, uintptr_t gb1, uintptr_t gw2, uintptr_t gb2, uintptr_t gwf,
                uintptr_t gbf, uintptr_t logp, uintptr_t loss_b, uintptr_t scratch, int B, uintptr_t stream);
int64_t mnist_scratch_bytes(int B);

// resnet_glue.hip ---------------------------------------------------------------
void s2d_stem_input(uintptr_t x, uintptr_t S, int N, int H, int W, int Hs, int Ws, int pad, uintptr_t stream);
void stem_weight_pack(uintptr_t w7, uintptr_t w4, int Cout, uintptr_t stream);
void stem_wgrad_unpack(uintptr_t slab, uintptr_t dw7, int splits, int Cout, uintptr_t stream);
void phase_weights(uintptr_t wt, uintptr_t out, int Cin, int Cout, uintptr_t stream);
void head_pool(uintptr_t h, uintptr_t f, int B, int HW, int C, uintptr_t loss, uintptr_t stream);
void head_softmax_nll(uintptr_t slab, int splits, int B, int NC, int NCp, uintptr_t bias, uintptr_t labels,
                      uintptr_t logp, uintptr_t loss_b, uintptr_t dl, float dscale, uintptr_t db, uintptr_t loss,
                      uintptr_t stream);
void head_weight_prep(uintptr_t w, uintptr_t wb, uintptr_t wbt, int NC, int NCp, int C, uintptr_t stream);
void head_broadcast(uintptr_t df, uintptr_t dh, int B, int HW, int C, uintptr_t stream);
void head_wgrad_reduce(uintptr_t slab, uintptr_t dw, int splits, int NC, int NCp, int C, float scale,
                       uintptr_t stream);

}  // namespace dl
