/* ifd training ops — the C ABI of the fp32 training step (BASELINE configs[4]).
 *
 * Replaces, for the 9-channel UNet of code/unet.py / code/nn.py, what the reference's
 * `train_epoch` (code/train_inpainting.py:15-79) gets from torch autograd + optim:
 *   loss = diffusion.training_losses(model, x_start, t, model_kwargs)['loss']
 *                                        (code/gaussian_diffusion.py:540-614)
 *   loss.backward()                      (code/train_inpainting.py:61)
 *   clip_grad_norm_(params, 1.0)         (:64)
 *   AdamW(lr, wd, betas=(0.9, 0.999)).step()   (:66, :394-399)
 * The host side (ifd/train.py) orchestrates these ops over the reference's module graph; every
 * tensor argument is a DEVICE pointer, activations are NHWC fp32 [N][H][W][C], weights are in the
 * reference's torch layouts ([Cout][Cin][kh][kw], Linear [out][in]). All launches are async on
 * `stream`; reductions run in a fixed order (bit-reproducible). Status 0 = ok, else see
 * ifd_last_error(). Accumulating outputs (dw, db, dgamma, dbeta, dss) are added into (+=).
 */
#ifndef IFD_TRAIN_H
#define IFD_TRAIN_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* conv weight W[cout][cin][taps] -> the fp32 conv kernel's packing; transpose=1 packs the dgrad kernel
 * (out channels = cin, in channels = cout, taps flipped). cin_pad / cout_pad / bn are the PACKED conv's
 * (bn = 64 if its out count % 64 == 0 else 32; cin_pad a multiple of 8). */
int ifd_tr_pack_conv(const float* w, int cout, int cin, int taps, int bn, int cin_pad, int cout_pad, int transpose,
                     float* wpack, void* stream);
/* out[N,H,H,cout] = conv(concat(x0[c0], x1[c1])) + bias (+ res): nn.Conv2d 3x3 pad 1 (taps 9) or 1x1
 * (code/nn.py:12-20,184,252,254); cout % 4 == 0 (pad: weights packed with zero rows);
 * split-K slabs in `part` (size: ifd_tr_conv_part_floats). */
int64_t ifd_tr_conv_part_floats(int N, int H, int cin_pad, int cout, int cout_pad, int bn, int taps);
int ifd_tr_conv(const float* x0, int c0, const float* x1, int c1, int N, int H, const float* wpack, const float* bias,
                int cin_pad, int cout, int cout_pad, int bn, int taps, const float* res, float* out, float* part,
                int64_t part_floats, void* stream);
/* 3xf16 training convs (the sampler's split kernel, conv_x3.hip, on a materialised input: no prologue).
 * ifd_tr_pack_conv_x3: W[cout][cin][9] (transpose=1: the dgrad conv, taps flipped) -> the split packing
 * [cout_pad/64][cin_pad16/16][9][part][h][64][8] f16 (wx3: cout_pad * cin_pad16 * 9 floats); taps = 1: the
 * 1x1 chunk packing [cout_pad/64][cin/32][2][part][h][64][8] (cout_pad * cin floats); sets bit 2 of
 * *guard when a weight is outside the split's range (|w| >= 32).
 * ifd_tr_conv_x3: the same contract as ifd_tr_conv for 3x3 convs with cout % 64 == 0, cin % 16 == 0 and
 * maps of >= 16x16 (8x8: N % 4 == 0); returns 3 (nothing launched) for any other shape, so the caller runs
 * ifd_tr_conv. Operands with |a| >= 65504 set bit 1 of *guard (the step must then be re-run in fp32). */
int ifd_tr_pack_conv_x3(const float* w, int cout, int cin, int taps, int cin_pad16, int cout_pad, int transpose,
                        void* wx3, unsigned* guard, void* stream);
/* Every ifd_tr_pack_conv_x3 of a step in one launch: desc = a device array of ndesc records (ifd_tr_pack_desc_bytes
 * bytes each: const float* w; void* dst; int cout, cin, pad (cin_pad16 or the 1x1 operand's channel pad),
 * cout_pad, transpose, taps; int64 first block), in block order, each record's blocks = ceil(packed f16 pairs /
 * 8192) (256 threads x 32 elements); nblocks = the total. */
int64_t ifd_tr_pack_desc_bytes(void);
int ifd_tr_pack_x3_batch(const void* desc, int ndesc, int64_t nblocks, unsigned* guard, void* stream);
int64_t ifd_tr_conv_x3_part_floats(int N, int H, int cin_pad, int cout);
int ifd_tr_conv_x3(const float* x0, int c0, const float* x1, int c1, int N, int H, const void* wx3, const float* bias,
                   int cin_pad, int cout, const float* res, float* out, float* part, int64_t part_floats,
                   unsigned* guard, void* stream);
/* ifd_tr_conv_x3 for 3x3 (taps 9) or 1x1 (taps 1: cin % 32 == 0, weights packed by ifd_tr_pack_conv_x3 with
 * taps 1, part size from ifd_tr_conv_x3_part_floats). nprod: 3 (the fp32-class split) or 1 (the reduced-
 * precision f16 training mode: the hi x hi product only, same packing). */
int ifd_tr_conv_x3_taps(const float* x0, int c0, const float* x1, int c1, int N, int H, const void* wx3,
                        const float* bias, int cin_pad, int cout, const float* res, float* out, float* part,
                        int64_t part_floats, unsigned* guard, int taps, int nprod, void* stream);
/* ifd_tr_conv_x3_taps that also writes the output's GroupNorm granule statistics when the launch geometry
 * has them (cout % 128 == 0; single-image 256-pixel tiles or a split-K reduction): gstat[n][cout/4][E] =
 * (mean, M2) of *gstat_cnt values each; *gstat_E = E, or 0 when none were written (then use ifd_tr_gn_fwd).
 * gstat needs ifd_tr_gstat_floats(N, H, cout) floats. Replaces the statistics pass of the GroupNorm that
 * follows a conv (code/unet.py ResBlock in_layers / out_layers). */
int64_t ifd_tr_gstat_floats(int N, int H, int cout);
int ifd_tr_conv_x3_gstat(const float* x0, int c0, const float* x1, int c1, int N, int H, const void* wx3,
                         const float* bias, int cin_pad, int cout, const float* res, float* out, float* part,
                         int64_t part_floats, unsigned* guard, int taps, float* gstat, int64_t gstat_floats,
                         int* gstat_E, float* gstat_cnt, int nprod, void* stream);
/* GroupNorm-apply prologue variants: the conv reads the RAW GroupNorm input x = concat(x0, x1) and
 * computes silu(actA[n][c] x + actB[n][c]) per staged value (zero padding after the activation), as the
 * sampler's convs do; actA / actB from ifd_tr_gn_coef. The normalised activation of a ResBlock's
 * in_layers / out_layers (code/nn.py:189-212) and the output head (code/unet.py:197-200) is then never
 * written. ifd_tr_conv_x3_gn: 3x3 only, else as ifd_tr_conv_x3_gstat (returns 3 when not eligible);
 * ifd_tr_conv_gn: the fp32 kernel, as ifd_tr_conv. */
int ifd_tr_conv_x3_gn(const float* x0, int c0, const float* x1, int c1, int N, int H, const void* wx3,
                      const float* bias, int cin_pad, int cout, const float* actA, const float* actB, const float* res,
                      float* out, float* part, int64_t part_floats, unsigned* guard, float* gstat,
                      int64_t gstat_floats, int* gstat_E, float* gstat_cnt, int nprod, void* stream);
int ifd_tr_conv_gn(const float* x0, int c0, const float* x1, int c1, int N, int H, const float* wpack,
                   const float* bias, int cin_pad, int cout, int cout_pad, int bn, int taps, const float* actA,
                   const float* actB, const float* res, float* out, float* part, int64_t part_floats, void* stream);
/* The output head's forward (code/unet.py:197-200: GroupNorm + SiLU + conv 3x3 -> 6) on the sampler's split
 * head kernel (conv_head.hip): out[N,H,H,8] = conv(silu(actA x + actB)) + bias8 with channels 6, 7 zero
 * (bias8 padded with zeros); w = the raw [cout][cin][3][3] weight (cout <= 8), re-packed on the device
 * into wpack (ifd_tr_head_x3_pack_floats(cin) floats; |w| >= 32 sets bit 2 of *guard). cin % 32 == 0,
 * cin <= 128, H % 16 == 0; returns 3 (nothing launched) otherwise. */
int64_t ifd_tr_head_x3_pack_floats(int cin);
int ifd_tr_conv_head_x3(const float* x, int cin, int N, int H, const float* w, int cout, float* wpack,
                        const float* bias8, const float* actA, const float* actB, float* out, unsigned* guard,
                        void* stream);
/* x[i] *= s (the loss scale of the 3xf16 backward and its removal from the gradients). */
int ifd_tr_scale(float* x, int64_t n, float s, void* stream);
/* dw[cout][c0+c1][taps] += sum_pixels dy (x) shifted concat(x0, x1); db[cout] += column sums of dy. */
int64_t ifd_tr_wgrad_part_floats(int cout, int cin, int taps, int64_t P, int* splits);
int ifd_tr_conv_wgrad(const float* dy, int cout, const float* x0, int c0, const float* x1, int c1, int N, int H,
                      int taps, float* dw, float* db, float* part, int64_t part_floats, float* colpart,
                      int64_t colpart_floats, void* stream);
/* ifd_tr_conv_wgrad with the 3xf16 split kernel for 3x3 / 1x1 convs on maps >= 8x8, X = concat(x0, x1) with
 * c0 % 64 == 0 when c1 > 0 (both
 * operands split on the fly, three f16 products per MAC, fp32 accumulation; |operand| >= 65504 sets bit 1
 * of *guard); other shapes run ifd_tr_conv_wgrad. Same workspaces. nprod 1: the hi x hi product only (the
 * reduced-precision f16 training mode). */
int ifd_tr_conv_wgrad_x3(const float* dy, int cout, const float* x0, int c0, const float* x1, int c1, int N, int H,
                         int taps, float* dw, float* db, float* part, int64_t part_floats, float* colpart,
                         int64_t colpart_floats, unsigned* guard, int nprod, void* stream);
/* ifd_tr_conv_wgrad_x3 (3x3) of the weight whose forward ran ifd_tr_conv_x3_gn: X = silu(actA x + actB),
 * recomputed at staging from the raw x = concat(x0[c0], x1[c1]) (c1 > 0: c0 % 64 == 0). Returns 3 (nothing launched) for shapes the split kernel does not
 * take: the caller then materialises X (ifd_tr_act_apply) and calls ifd_tr_conv_wgrad[_x3]. */
int ifd_tr_conv_wgrad_x3_gn(const float* dy, int cout, const float* x0, int c0, const float* x1, int c1, int N, int H,
                            const float* actA, const float* actB, float* dw, float* db, float* part,
                            int64_t part_floats, float* colpart, int64_t colpart_floats, unsigned* guard, int nprod,
                            void* stream);
/* GroupNorm statistics and apply coefficients without the apply pass: stats[n][32][2] = (mean, rstd) as
 * ifd_tr_gn_fwd's, A[n][c] = rstd gamma (1 + scale), B[n][c] = (beta - mean rstd gamma)(1 + scale) + shift
 * (ss as ifd_tr_gn_fwd's, or NULL). From granules (gstat0 != NULL: ifd_tr_gn_fwd_gstat's contract, x unused)
 * or one statistics pass over x (work: N * ifd_tr_gn_slices(HW, N, C) * 64 doubles). */
int ifd_tr_gn_coef(const float* x, int N, int HW, int C, const float* gamma, const float* beta, const float* ss,
                   int ss_stride, const float* gstat0, int C0, const float* gstat1, int E, float cnt, float* stats,
                   float* A, float* B, double* work, int64_t work_doubles, void* stream);
/* out = act(A[n][c] x + B[n][c]) (silu != 0: SiLU, else the affine only), the convs' prologue arithmetic:
 * materialises a GroupNorm-applied activation when a consumer cannot apply it on load. */
int ifd_tr_act_apply(const float* x, int N, int HW, int C, const float* A, const float* B, int silu, float* out,
                     void* stream);
/* The resampling ResBlocks' input side in one pass (code/nn.py:189-195 with nn.py:151-152): out =
 * resample(silu(A[n][c] x + B[n][c])) and out_raw = resample(x), mode 1 nearest-up x2, mode 2 AvgPool2d(2)
 * (the sampler's act_pool arithmetic), at the output resolution. */
int ifd_tr_act_resample(const float* x, int N, int Hin, int C, const float* A, const float* B, int mode, float* out,
                        float* out_raw, void* stream);
/* Pixel slices per image of the GroupNorm passes (ifd_tr_gn_fwd / _coef / _bwd work sizes use it): 256-pixel
 * slices, smaller on small maps so that the grid keeps >= 1024 blocks. */
int64_t ifd_tr_gn_slices(int HW, int N, int C);
/* GroupNorm(32, C) (+ scale/shift: ss[n][0:C] = scale, ss[n][C:2C] = shift, row stride ss_stride) (+ SiLU).
 * stats[n][32][2] = (mean, rstd) saved for the backward; work: N * ifd_tr_gn_slices(HW, N, C) * 64 doubles. */
int ifd_tr_gn_fwd(const float* x, int N, int HW, int C, const float* gamma, const float* beta, const float* ss,
                  int ss_stride, int act_silu, float* out, float* stats, double* work, int64_t work_doubles,
                  void* stream);
/* ifd_tr_gn_fwd with the statistics merged from ifd_tr_conv_x3_gstat's granules of x (C % 128 == 0): no
 * statistics pass over x. x = concat(a[C0], b[C - C0]) (the output blocks' skip concat) takes a's granules
 * in gstat0 and b's in gstat1 (equal E and cnt); a single source passes C0 = C, gstat1 = NULL. */
int ifd_tr_gn_fwd_gstat(const float* x, int N, int HW, int C, const float* gamma, const float* beta, const float* ss,
                        int ss_stride, int act_silu, const float* gstat0, int C0, const float* gstat1, int E,
                        float cnt, float* out, float* stats, void* stream);
/* its backward: dx (= or +=), dgamma/dbeta +=, dss (d scale, d shift) +=.
 * work: N * ifd_tr_gn_slices(HW, N, C) * C * 3 + N*C*3 + N*64 floats. */
int ifd_tr_gn_bwd(const float* dout, const float* x, int N, int HW, int C, const float* gamma, const float* beta,
                  const float* ss, int ss_stride, int act_silu, const float* stats, float* dx, int accumulate,
                  float* dgamma, float* dbeta, float* dss, float* work, int64_t work_floats, void* stream);
/* ifd_tr_gn_bwd of a concat input x = concat(x0[C0], x1[C - C0]) read by channel range (the output blocks'
 * cat(h, skip), code/unet.py:170); dx is the concat's gradient as one [N][HW][C] tensor. add (optional, else
 * NULL): dx also gets add[p * add_stride + c] (a channel range of a wider tensor: the skip part of an output
 * block's concat gradient, which joins the encoder chain's gradient here instead of by a separate pass).
 * dx1 (optional, else NULL; C0 < C, accumulate 0): the gradient split per concat source - dx [N][HW][C0] gets
 * channels [0, C0), dx1 [N][HW][C - C0] channels [C0, C) (no channel copy out of a C-wide gradient). */
int ifd_tr_gn_bwd_cat(const float* dout, const float* x0, int C0, const float* x1, int N, int HW, int C,
                      const float* gamma, const float* beta, const float* ss, int ss_stride, int act_silu,
                      const float* stats, float* dx, int accumulate, float* dgamma, float* dbeta, float* dss,
                      float* work, int64_t work_floats, const float* add, int add_stride, float* dx1,
                      void* stream);
/* ifd_tr_gn_bwd (no scale/shift, one source) for a resampling ResBlock's in_layers GroupNorm (code/nn.py:
 * 189-195): dout at the block's output resolution (mode 1: nearest-up x2, 2H; mode 2: AvgPool2d(2), H/2) is read
 * through the resample adjoint, and radd (optional, same resolution: the skip path's gradient) joins dx through
 * it too — no materialised adjoint. x: [N][H][H][C]; dx (=, at H) also gets add as ifd_tr_gn_bwd_cat. */
int ifd_tr_gn_bwd_resampled(const float* dout, const float* x, int N, int H, int C, const float* gamma,
                            const float* beta, int act_silu, const float* stats, int mode, const float* radd, float* dx,
                            float* dgamma, float* dbeta, const float* add, int add_stride, float* work,
                            int64_t work_floats, void* stream);
/* The dgrad conv that feeds a GroupNorm backward, with that backward's pass 1 fused into its epilogue
 * (code/train_inpainting.py:15-79 backward of nn.py:46-48,151-152,203-207): out = conv^T(dy) on the split
 * kernel (ifd_tr_conv_x3_taps, 3x3, no residual), and for GroupNorm input x = concat(gx0[gc0], gx1) (cout
 * channels), stats / gamma / beta / ss as ifd_tr_gn_bwd: gpart[N][*gpart_nsl][cout][3] = per 64-pixel block
 * sum dz, sum dz nrm, sum dz (1 + s) xhat. *gpart_nsl = 0 when the geometry cannot fuse (split-K, 8x8 tiles):
 * the conv still ran, and the caller runs ifd_tr_gn_bwd_cat. gpart: ifd_tr_gnb_part_floats floats. */
int64_t ifd_tr_gnb_part_floats(int N, int H, int cout);
int ifd_tr_conv_x3_gnb(const float* dy, int cdy, int N, int H, const void* wx3, const float* bias, int cin_pad,
                       int cout, float* out, float* part, int64_t part_floats, unsigned* guard, const float* gx0, int gc0,
                       const float* gx1, const float* stats, const float* gamma, const float* beta, const float* ss,
                       int ss_stride, int act_silu, float* gpart, int64_t gpart_floats, int* gpart_nsl, int nprod,
                       void* stream);
/* The same, and when act_out is non-null (and the geometry fuses, *gpart_nsl > 0) the epilogue also writes the
 * GroupNorm's forward output act = silu(z) (z without act_silu), z = GN(x) (1 + s) + shift, to act_out
 * [N][H][W][cout] - the input of the conv whose weight gradient comes next (round 6), from the values the pass-1
 * sums compute anyway, so that weight gradient need not re-apply the GroupNorm + SiLU on load
 * (ifd_tr_conv_wgrad_x3 on act_out instead of ifd_tr_conv_wgrad_x3_gn on x). */
int ifd_tr_conv_x3_gnb_act(const float* dy, int cdy, int N, int H, const void* wx3, const float* bias, int cin_pad,
                           int cout, float* out, float* part, int64_t part_floats, unsigned* guard, const float* gx0,
                           int gc0, const float* gx1, const float* stats, const float* gamma, const float* beta,
                           const float* ss, int ss_stride, int act_silu, float* gpart, int64_t gpart_floats,
                           int* gpart_nsl, float* act_out, int nprod, void* stream);
/* ifd_tr_gn_bwd_cat with pass 1 done (gpart from ifd_tr_conv_x3_gnb): reduce, group, parameter and dx passes
 * (add, dx1 as there). work: N*C*3 + N*64 floats. */
int ifd_tr_gn_bwd_from_part(const float* dout, const float* x0, int C0, const float* x1, int N, int HW, int C,
                            const float* gamma, const float* beta, const float* ss, int ss_stride, int act_silu,
                            const float* stats, const float* part, int part_nsl, float* dx, int accumulate,
                            float* dgamma, float* dbeta, float* dss, float* work, int64_t work_floats, const float* add,
                            int add_stride, float* dx1, void* stream);
/* 1x1 conv out[px][co] = bias[co] + sum_k W[co][k] cat(x0[c0], x1[c1])[px][k] (code/nn.py:184 skip_connection,
 * and its dgrad with transpose = 1: W^T, cout <-> cin) on the dedicated split 1x1 kernel (the sampler's
 * skip_x3.hip), the weights W[cout][cin] packed on the device into wpack (ifd_tr_conv1x1_pack_floats floats).
 * Returns 3 when the shape is not eligible (c0, c1 multiples of 16, c0 + c1 a multiple of 64, N*H*H a multiple of
 * 32): the caller uses ifd_tr_conv_x3_taps. nprod 3 (3xf16) or 1 (f16). */
int64_t ifd_tr_conv1x1_pack_floats(int cout, int cin, int transpose);
int ifd_tr_conv1x1_x3(const float* x0, int c0, const float* x1, int c1, int N, int H, const float* w, int cout, int cin,
                      int transpose, const float* bias, float* out, void* wpack, int64_t wpack_floats, unsigned* guard,
                      int nprod, void* stream);
/* nearest-up x2 (mode 1) / AvgPool2d(2) (mode 2) (code/nn.py:92-133) and the adjoint (dx at Hin). */
int ifd_tr_resample(const float* x, int N, int Hin, int C, int mode, float* out, void* stream);
int ifd_tr_resample_bwd(const float* dy, int N, int Hin, int C, int mode, float* dx, int accumulate, void* stream);
int ifd_tr_add(const float* a, const float* b, float* out, int64_t n, void* stream);
/* dst[p][doff+c] (=|+=) src[p][soff+c], c < nc: the skip concat (code/unet.py:170) and its gradient split */
int ifd_tr_copy_channels(const float* src, int cs, int soff, float* dst, int cd, int doff, int nc, int64_t npix,
                         int accumulate, void* stream);
/* QKVAttention (code/nn.py:222-235) on qkv [N][T][3C] -> out [N][T][C], and its backward (dqkv written). */
int ifd_tr_attention(const float* qkv, int N, int T, int C, float scale, float* out, void* stream);
int64_t ifd_tr_attention_bwd_scratch_floats(int N, int T, int C);
int ifd_tr_attention_bwd(const float* qkv, const float* dout, int N, int T, int C, float scale, float* dqkv,
                         float* scratch, int64_t scratch_floats, void* stream);
/* y[M][N] = post(pre(x) W^T + b), W [N][K] (nn.Linear), pre/post SiLU optional; backward: dx (= or +=,
 * times pre'(x)), dw +=, db +=. */
int ifd_tr_linear(const float* x, int M, int K, const float* w, const float* b, int N, int pre_silu, int post_silu,
                  float* y, void* stream);
int ifd_tr_linear_bwd(const float* dy, const float* x, int M, int K, const float* w, int N, int pre_silu, float* dx,
                      int dx_accumulate, float* dw, float* db, void* stream);
int ifd_tr_silu_bwd(const float* z, const float* dy, float* dz, int64_t n, void* stream);
/* timestep_embedding (code/nn.py:51-61) from an fp32 frequency table freqs[dim/2]. */
int ifd_tr_temb(const int64_t* t, const float* freqs, int N, int dim, float* out, void* stream);
/* the 9-channel input [x, masked_image, mask x3] (code/unet.py:199) as NHWC with 16 channels (7 zero). */
int ifd_tr_pack_input(const float* x, const float* masked_image, const float* mask, int N, int HW, float* out16,
                      void* stream);
/* x_t = q_sample(x0, t, noise); inject: keep * q_sample(x0, t[0], cached) + (1 - keep) * x_t, keep = 1 - mask
 * (code/gaussian_diffusion.py:566-582). sqrt_ac / sqrt_1m_ac: the fp32-rounded float64 tables. NCHW. */
int ifd_tr_q_sample_inject(const float* x0, const float* noise, const float* cached, const float* mask,
                           const int64_t* t, const float* sqrt_ac, const float* sqrt_1m_ac, int N, int HW, int inject,
                           float* xt, void* stream);
/* masked eps-MSE (code/gaussian_diffusion.py:595-610) on channels 0-2 of the model output (NHWC, channel
 * stride cs >= 6): loss[0] and d loss / d out (same layout, other channels 0). work: 6N floats. */
int ifd_tr_masked_mse(const float* out6_nhwc, int cs, const float* noise, const float* mask, int N, int HW,
                      float* loss, float* dout6_nhwc, float* work, void* stream);
/* clip_grad_norm_(max_norm) then AdamW over one flat parameter buffer; norm_coef[0] = grad norm,
 * [1] = clip coefficient (device; no host sync). work: 1024 doubles. step >= 1. */
/* The optimizer's scalars arrive as doubles (Python floats): 1 - lr*wd, 1 - b1, 1 - b2, lr / (1 - b1^k) and
 * sqrt(1 - b2^k) are formed in double and rounded to fp32 once, as torch's AdamW forms them. */
int ifd_tr_clip_adamw(float* p, float* g, float* m, float* v, int64_t n, float max_norm, double lr, double b1, double b2,
                      double eps, double wd, int step, double* work, float* norm_coef, void* stream);

#ifdef __cplusplus
}
#endif
#endif
