// Fused implicit-GEMM convolution on fp32 MFMA (v_mfma_f32_32x32x2_f32), NHWC activations.
//
// One launch computes, for a 128-pixel x BN-channel output tile:
//   out = conv3x3( act( xform( concat(in0, in1) ) ) ) [+ conv1x1(concat(s0, s1))] + bias [+ residual]
// where
//   act(v)   = silu(A[n,c] * v + B[n,c])   (GroupNorm-apply [+ scale/shift] + SiLU, fused prologue)
//            | A[n,c] * v + B[n,c]         (GroupNorm-apply only: attention qkv)
//            | v                           (no prologue)
//   xform    = identity | nearest-up x2 | avg-pool 2x2   (ResBlock h_upd, code/nn.py:190-195)
//   residual = identity | up x2 | down 2x2 of a raw tensor (ResBlock x_upd + identity skip, nn.py:212)
// and zero padding is applied AFTER act, as torch pads the activated tensor (code/nn.py:153,176).
// The 1x1 segment is the ResBlock skip_connection (code/nn.py:184) accumulated into the same
// MFMA accumulators, so `skip(x) + h` costs no extra pass over HBM.
#pragma once
#include "common.h"

namespace ifd {

enum ConvAct : int { ACT_NONE = 0, ACT_AFFINE = 1, ACT_AFFINE_SILU = 2 };
enum ConvXform : int { XF_NONE = 0, XF_UP = 1, XF_DOWN = 2 };
enum ConvEpi : int { EPI_NHWC = 0, EPI_NCHW = 1, EPI_DDIM = 2, EPI_DDPM = 3 };

// Per-step sampler coefficients, float64-derived on the host and rounded to fp32 once
// (exactly what torch does when a float64 0-dim tensor multiplies an fp32 tensor).
struct StepCoeffs {
  // DDIM (code/test_inp_ddim_50.py:523-574)
  float c_sqrt_1m_at;  // sqrt(1 - a_t)
  float c_sqrt_at;     // sqrt(a_t)              (divisor)
  float c_sqrt_ap;     // sqrt(a_prev)
  float c_dir;         // sqrt(1 - a_prev - sigma^2)
  float c_sigma;       // sigma
  // DDPM (code/gaussian_diffusion.py:213-298 + test_inp_ddim_50.py:442-466)
  float c_min_log, c_max_log, c_recip, c_recipm1, c_coef1, c_coef2, c_nonzero;
  // injection (both): img*mask + (c_inj_a*gt + c_inj_b*known)*(1-mask)
  float c_inj_a, c_inj_b;
  int use_noise;  // DDIM: noise tensor present (tau > 0 and eta > 0)
  int inject;     // tau > 0
  int clip;       // clip_denoised
  int pad;
};

struct ConvParams {
  // primary input (concat of two NHWC sources along C)
  const float* in0; int c0;
  const float* in1; int c1;
  int N, Hin, Win;   // input spatial size (before xform)
  int H, W;          // conv / output spatial size
  int act;           // ConvAct
  const float* actA; const float* actB;  // [N, c0 + c1]
  // weights
  const float* wpack;  // [Cout_pad/BN][Cin_pad/8][TAPS][2][BN][4]
  const float* bias;   // [Cout] (main + skip bias folded in)
  int cin_pad, cout, cout_pad;
  // 1x1 segment (ResBlock skip_connection), raw inputs at output resolution
  const float* s0; int sc0;
  const float* s1; int sc1;
  const float* wskip;  // [Cout_pad/BN][Cs_pad/8][1][2][BN][4]
  int cs_pad;
  // residual (raw tensor with `cout` channels)
  const float* res; int res_xform; int res_H, res_W;
  // output
  float* out;
  int epi;
  // tile geometry (host-computed)
  int bm;  // pixel-tile size (128 or 256), chosen by conv_geometry
  int TW, TH, IMGS, tiles_x, tiles_y, npix_tiles;
  int lg_tw, lg_tpi;  // log2(TW), log2(TH*TW): tile dims are powers of two
  // split-K (low-resolution layers): blockIdx.z = split; split z accumulates main-segment chunks
  // [z*n/S, (z+1)*n/S) (+ the 1x1 segment when z == S-1) and writes raw sums to
  // part[z][N][H][W][cout]; splitk_reduce adds the S slabs in order, then bias and residual.
  int ksplit;
  float* part;
  // sampler epilogue (EPI_DDIM / EPI_DDPM): all NCHW [N,3,H,W] except mask [N,1,H,W]
  float* img; const float* gt; const float* mask; const float* noise; const float* known;
  StepCoeffs sc;
  // IFD_TRACE builds only: per-block timestamps (see conv.hip / conv_stream.hip)
  unsigned long long* trace;
  // optional GroupNorm granule statistics of the output (norm.hip): gstat[n][cout/4][e] =
  // (mean, M2); e = the tile's index within its image (x4 + consumer wave in conv_stream2).
  // Written only for single-image tiles without split-K (the host checks).
  float* gstat;
  int gstat_E;
  // handle options (read once at ifd_create, ifd_set_option): development overrides and the
  // batch-invariant geometry (split-K and tile kind chosen per image, not per batch, so an image's
  // result does not depend on how many other images share the launch)
  int opt_bm128;  // fp32 kernel: 128-pixel tiles only (the training 1x1 convs)
  int opt_invariant;
  // the split kernel's four-image 8 x 8 tiles at any batch (a partial last tile, conv_x3.hip unit_of): set by
  // the sampler (unet.h fill_opts) and the training ops (train_ops.hip conv_x3_params). Round 6 fixed the
  // fault this was gated on: the ACT_NONE coefficient loads read from the moved tile origin, below the tensor.
  int opt_img8_partial;
  // 3xf16 range guard (conv_x3.hip): set to 1 when an operand's magnitude reaches the f16 range
  // (|a| >= 65504 would split into inf). The host re-runs the eval in fp32 when it is set.
  unsigned* guard;
  // split kernel products per MAC: 3 (IFD_PREC_3XF16, fp32-class) or 1 (IFD_PREC_F16, f16 operands)
  int x3_nprod;
};

// Training (conv_x3's GNB instantiation, single-image tiles, no split-K, no residual): the conv's output is the
// upstream gradient da of a GroupNorm(32) (+ scale/shift) (+ SiLU) whose input x = concat(x0[c0], x1) has `cout`
// channels at the output's pixels; the epilogue also writes that GroupNorm backward's pass-1 partial sums
// (train_ops.hip gn_bwd_partial_kernel's A1 = sum dz, A2 = sum dz nrm, A3 = sum dz (1 + s) xhat) per
// (image, 64-pixel wave block e, channel): part[((n * nsl + e) * cout + c) * 3 + k]. A separate kernel
// argument, so the sampler's instantiations keep their ConvParams-only signature (and register allocation).
struct GnbParams {
  const float* x0; const float* x1; int c0;
  const float* stats;  // [N][32][2] (mean, rstd)
  const float* gamma; const float* beta;
  const float* ss; int ss_stride;  // optional scale [n][c], shift [n][cout + c]
  int silu;
  float* part; int nsl;
  float* act;  // optional: the GroupNorm's forward output silu(z) (or z), [N][H][W][cout] (the next weight gradient's input)
};
int launch_conv_x3_gnb(const ConvParams& p, const GnbParams& g, hipStream_t stream);

// Launch with the tile configuration chosen from (cout, taps, xform). Returns hipError_t.
int launch_conv(const ConvParams& p, int taps, int xform, int bn, hipStream_t stream);
int conv_pick_bn(int cout, int taps, int H, int W, int N);
// Tile geometry + split-K choice shared by the launcher and the workspace planner.
void conv_geometry(ConvParams& p, int H, int W, int N, int bn, int nchunks, bool x3 = false);
int launch_splitk_reduce(const ConvParams& p, hipStream_t stream);
// splitk_reduce + the GroupNorm granule statistics of the output into p.gstat (E entries per image
// of cnt values each); p.gstat must hold N * E * cout/4 * 2 floats with E = max(H*W / 64, 1).
int launch_splitk_gstat(const ConvParams& p, int* E, float* cnt, hipStream_t stream);
// Persistent streaming kernel for the wide layers (conv_stream.hip).
bool conv_stream_eligible(const ConvParams& p, int taps, int xform, int bn);
int launch_conv_stream(const ConvParams& p, int xform, int mode, hipStream_t stream);
// 3xf16 split-precision streaming kernel (conv_x3.hip); wpack = the x3 packing (pack_conv_x3).
bool conv_x3_eligible(const ConvParams& p, int taps, int xform, int bn);
int launch_conv_x3(const ConvParams& p, int xform, hipStream_t stream);

// A ResBlock's 1x1 skip_connection on split f16 MFMAs as its own launch (skip_x3.hip):
// out = bias + W * cat(s0, s1) per pixel, NHWC fp32 in and out; conv2 then adds it as its residual.
struct Skip1x1Params {
  const float* s0; int sc0;
  const float* s1; int sc1;
  int npix;           // N * H * W (a multiple of 32)
  int cout;
  const void* wpack;  // pack_skip1x1_x3 (unet.hip): [cout/ntc][K/16][part][h][ntc][8] f16
  const float* bias;  // [cout] (the skip bias only)
  float* out;         // [npix][cout]
  unsigned* guard;    // range guard word (ConvParams::guard)
  int ntc;            // output channels per block, skip_x3_ntc(K, cout)
  int nprod;          // 3 (3xf16) or 1 (f16)
};
int skip_x3_ntc(int K, int cout);  // 128, 64 or 32 (the tile's split weights fit 128 KiB of LDS); 0 if none
bool skip_x3_eligible(const Skip1x1Params& p);
int launch_skip_x3(const Skip1x1Params& p, hipStream_t stream);

// fp32 output-head conv (conv_head.hip): 3x3, cout 6 or 3, NCHW / sampler-step epilogues.
bool conv_head_eligible(const ConvParams& p, int taps, int xform);
size_t conv_head_pack_floats(int cin);
void conv_head_pack(const float* w, int cout, int cin, float* dst);
int launch_conv_head(const ConvParams& p, const float* wh, hipStream_t stream);
// the same head on f16 MFMAs with split operands (3xf16 mode): weights packed by conv_head_x3_pack
bool conv_head_x3_eligible(const ConvParams& p, int taps, int xform);
size_t conv_head_x3_pack_floats(int cin);
bool conv_head_x3_pack(const float* w, int cout, int cin, float* dst);
int launch_conv_head_x3(const ConvParams& p, const float* wx, hipStream_t stream);
// the training forward's head on the same kernel (NHWC, 8 channels) and its device-side weight packing
bool conv_head_x3_nhwc_eligible(const ConvParams& p);
int launch_pack_head_x3(const float* w, int cout, int cin, float* dst, unsigned* guard, hipStream_t stream);

// Shared elementwise step math, also used by the standalone step kernels (sampler.hip).
__device__ __forceinline__ float ddim_step_value(const StepCoeffs& s, float img, float eps, float noise,
                                                float gt, float mask, float known) {
#pragma clang fp contract(off)
  float x0 = (img - s.c_sqrt_1m_at * eps) / s.c_sqrt_at;
  if (s.clip) x0 = fminf(fmaxf(x0, -1.0f), 1.0f);
  float dir = s.c_dir * eps;
  float v = s.c_sqrt_ap * x0 + dir;
  if (s.use_noise) v = v + s.c_sigma * noise;
  if (s.inject) {
    float keep = 1.0f - mask;
    v = v * mask + (s.c_inj_a * gt + s.c_inj_b * known) * keep;
  }
  return v;
}

__device__ __forceinline__ float ddpm_step_value(const StepCoeffs& s, float x, float eps, float var_v, float noise,
                                                float gt, float mask, float known) {
#pragma clang fp contract(off)
  float frac = (var_v + 1.0f) / 2.0f;
  float logvar = frac * s.c_max_log + (1.0f - frac) * s.c_min_log;
  float x0 = s.c_recip * x - s.c_recipm1 * eps;
  if (s.clip) x0 = fminf(fmaxf(x0, -1.0f), 1.0f);
  float mean = s.c_coef1 * x0 + s.c_coef2 * x;
  float v = mean + (s.c_nonzero * expf(0.5f * logvar)) * noise;
  if (s.inject) {
    float keep = 1.0f - mask;
    v = v * mask + (s.c_inj_a * gt + s.c_inj_b * known) * keep;
  }
  return v;
}

}  // namespace ifd
