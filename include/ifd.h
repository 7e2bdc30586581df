/* ifd — MI355X-native masked-inpainting diffusion sampler: the drop-in C ABI.
 *
 * Plain C, plain pointers and sizes; no torch types. All tensor arguments are DEVICE pointers
 * to contiguous fp32 (int64 for timesteps) memory on the handle's device; every launch is
 * asynchronous on `stream` (a hipStream_t passed as void*, e.g. torch's current stream).
 * Status: 0 = ok, non-zero = error; the message is in ifd_last_error() (thread-local).
 *
 * Reference interfaces each entry point replaces (paths relative to the reference repo):
 *   ifd_create / ifd_param_* / ifd_load_weights / ifd_finalize
 *       create_model_and_diffusion (code/train_inpainting.py:199-262): UNetModel(...) +
 *       DiffusionInpaintingModel(base, 9) (code/unet.py:176-195) + load_state_dict(strict=False)
 *       (code/train_inpainting.py:241; code/test_inp_ddim_50.py:349). Names are the reference's
 *       state_dict keys, with or without the "base_model." prefix.
 *   ifd_unet_forward
 *       DiffusionInpaintingModel.forward(x, t, masked_image, mask) (code/unet.py:197-200)
 *       -> UNetModel.forward (code/unet.py:154-173); NCHW in, NCHW [B,6,H,W] out.
 *   ifd_ddim_step
 *       one iteration of InpaintingSampler.inpainting_ddim_sample_loop
 *       (code/test_inp_ddim_50.py:501-574): model_fn (:373-385) + UNet + the DDIM update and the
 *       known-region re-injection, fused into the last conv's epilogue; updates img in place.
 *   ifd_ddpm_step
 *       one iteration of inpainting_p_sample_loop (code/test_inp_ddim_50.py:424-466) with
 *       p_mean_variance (code/gaussian_diffusion.py:213-298), fused likewise.
 *   ifd_ddim_update / ifd_ddpm_update
 *       the same update math applied to an already computed model output [B,6,H,W].
 *   ifd_blend
 *       final blend result*mask + gt*(1-mask) (code/test_inp_ddim_50.py:692-696).
 */
#ifndef IFD_H
#define IFD_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ifd_config {
  int image_size;          /* 256 */
  int in_channels;         /* 9 (x, masked_image, mask x3) */
  int model_channels;      /* 128 */
  int out_channels;        /* 6 (eps + learned-range variance) */
  int num_res_blocks;      /* 1 */
  int num_levels;          /* len(channel_mult) = 6 */
  int channel_mult[8];     /* 1,1,2,2,4,4 */
  int num_attention;       /* number of entries in attention_ds */
  int attention_ds[8];     /* downsample factors with attention: 16 */
  int num_head_channels;   /* 64 */
} ifd_config;

/* Sampler coefficients: float64 on the host, rounded to fp32 once (torch semantics). */
typedef struct ifd_step_coeffs {
  float c_sqrt_1m_at, c_sqrt_at, c_sqrt_ap, c_dir, c_sigma;                        /* DDIM */
  float c_min_log, c_max_log, c_recip, c_recipm1, c_coef1, c_coef2, c_nonzero;   /* DDPM */
  float c_inj_a, c_inj_b;                                                          /* injection */
  int use_noise, inject, clip, pad;
} ifd_step_coeffs;

typedef struct ifd_handle ifd_handle;

int ifd_create(const ifd_config* cfg, ifd_handle** out);
void ifd_destroy(ifd_handle* h);
const char* ifd_last_error(void);
/* Clears the thread-local message (ifd._lib.check does after reporting one, so a message is never reported
 * for a later status). Every non-zero status sets its own message naming the entry point that returned it. */
void ifd_clear_error(void);

/* Parameter inventory of the model (state_dict order, names without "base_model."). No GPU use. */
int ifd_num_params(ifd_handle* h, int* n);
int ifd_param_info(ifd_handle* h, int i, const char** name, int64_t* shape4, int* ndim);

/* Copy one parameter (host or device pointer, fp32 contiguous). The handle keeps its own copy. */
int ifd_load_weights(ifd_handle* h, const char* name, const float* data, const int64_t* shape, int ndim);
/* Pack every loaded parameter into the device layouts. Missing parameters are an error. */
int ifd_finalize(ifd_handle* h);
/* Conv arithmetic of the handle (default IFD_PREC_FP32):
 *   IFD_PREC_FP32   every conv on v_mfma_f32_32x32x2_f32: an exact fp32 fma chain.
 *   IFD_PREC_3XF16  layers with a split kernel (every 3x3 conv, the 1x1 convs, the output head) run
 *                   each fp32 operand as two f16 parts (hi + 2^-11 lo) and three f16 MFMAs into one
 *                   fp32 accumulator: fp32-level error, 5.3x the fp32 MFMA rate; the
 *                   other layers stay fp32. Takes effect on the next call.
 * The reference has no such switch: its model runs in the caller's dtype (fp32 on this path). */
#define IFD_PREC_FP32 0
#define IFD_PREC_3XF16 1
/* IFD_PREC_F16: the reduced-precision variant (the reference's `.half()` experiment,
 * code/test_quant.py:390-409, reported separately): the split kernels with the hi parts only — f16
 * operands, one f16 MFMA per MAC, fp32 accumulation; GroupNorm, attention, the head and the sampler
 * update stay fp32. Not fp32-class: errors ~1e-3 relative per eval. */
#define IFD_PREC_F16 2
int ifd_set_precision(ifd_handle* h, int prec);
/* 3xf16 range guard. The split needs every conv operand below the f16 range (|a| < 65504; the
 * weights are checked at finalize). The 3xf16 kernels set a device word when an operand reaches it
 * (activations in the producers, the raw 1x1-skip residual stream in the consumers). reset: async
 * on `stream`; read: synchronises `stream`, *tripped = 1 if any launch since the reset saw an
 * out-of-range operand — that eval's output is not fp32-accurate and must be recomputed in
 * IFD_PREC_FP32 (ifd.model / ifd.sampler do this automatically). */
int ifd_guard_reset(ifd_handle* h, void* stream);
int ifd_guard_read(ifd_handle* h, int* tripped, void* stream);
/* The guard word, without a synchronisation: enqueues on `stream` a copy of the word into *host_dst
 * (4 bytes; page-locked host memory, or the copy is not asynchronous) and returns. The value is valid
 * once the work enqueued on `stream` before this call has finished (an event recorded after it).
 * ifd.model's default "lazy" guard uses it so that a caller-driven loop of forwards (the reference
 * scripts' model() per step) never waits on the GPU; see DiffusionInpaintingModel(guard=...). */
int ifd_guard_copy_async(ifd_handle* h, unsigned* host_dst, void* stream);
int ifd_get_precision(ifd_handle* h, int* prec);
/* Handle options. No reference counterpart: execution choices of this library that never change
 * the arithmetic of a single image except where noted. Initial values are read from the
 * environment once, in ifd_create (IFD_BATCH_INVARIANT, IFD_CONV_STREAM, IFD_GN_FUSED, IFD_X3_OFF,
 * IFD_SKIP_SEP); nothing is read per launch. Keys:
 *   "batch_invariant" 0/1  tile kind and split-K chosen per image, so an image's output is
 *                          bit-identical whatever batch it shares a launch with (multi-GPU parity
 *                          mode: N ranks x B/N images == one rank x B images). Slower on small layers.
 *   "conv_stream"     0..2 wide fp32 layers: one tile per workgroup / persistent 1 or 2 per CU
 *   "gn_fused"        0/1  GroupNorm statistics fused into the producing conv (1) or a separate pass
 *   "skip_sep"        >= 0 split modes: a ResBlock's 1x1 skip as its own launch at resolutions >= this
 *   "x3_off"               bisecting mask of the split kernels (bit 32 keeps the output head on the
 *                          fp32 VALU kernel in the 3xf16 mode) */
int ifd_set_option(ifd_handle* h, const char* key, int value);
int ifd_get_option(ifd_handle* h, const char* key, int* value);
/* Bytes of device workspace the handle holds (weights + activations). */
int ifd_memory(ifd_handle* h, int64_t* weight_bytes, int64_t* workspace_bytes);
/* Bytes of activation workspace a forward at batch B would allocate (the arena plan: resident
 * skip tensors, rotating block buffers, split-K slabs of the convs the plan runs, statistics).
 * Host arithmetic only, no GPU use; the handle's current arena is not changed. */
int ifd_workspace_plan(ifd_handle* h, int64_t B, int64_t* workspace_bytes);

int ifd_unet_forward(ifd_handle* h, const float* x, const float* masked_image, const float* mask,
                     const int64_t* t, int64_t B, int H, int W, float* out6, void* stream);

/* img [B,3,H,W] in/out; gt [B,3,H,W]; mask [B,1,H,W] (1 = hole); noise / known [B,3,H,W]
 * (noise may be NULL when c->use_noise == 0 for DDIM; known may be NULL when c->inject == 0). */
int ifd_ddim_step(ifd_handle* h, const int64_t* t, int64_t B, int H, int W, float* img, const float* gt,
                  const float* mask, const float* noise, const float* known, const ifd_step_coeffs* c,
                  void* stream);
int ifd_ddpm_step(ifd_handle* h, const int64_t* t, int64_t B, int H, int W, float* img, const float* gt,
                  const float* mask, const float* noise, const float* known, const ifd_step_coeffs* c,
                  void* stream);

int ifd_ddim_update(const float* out6, int64_t B, int H, int W, float* img, const float* gt, const float* mask,
                    const float* noise, const float* known, const ifd_step_coeffs* c, void* stream);
int ifd_ddpm_update(const float* out6, int64_t B, int H, int W, float* img, const float* gt, const float* mask,
                    const float* noise, const float* known, const ifd_step_coeffs* c, void* stream);
int ifd_blend(const float* result, const float* gt, const float* mask, int64_t B, int C, int H, int W, float* out,
              void* stream);
/* Output conversion toU8 (code/test_inp_ddim_50.py:33-41): sample NCHW fp32 -> out NHWC u8
 * [B,H,W,C], ((x + 1) * 127.5).clamp(0, 255) with a truncating cast. B == 0 is a no-op. */
int ifd_to_u8(const float* sample, int64_t B, int C, int H, int W, uint8_t* out_nhwc, void* stream);
/* Mask convention of OrderedMaskDataset (code/data/dataset.py:278-286): gray u8 (already resized)
 * -> mask fp32, 1 where gray/255 < 0.5 (black = hole), else 0. n elements, n == 0 is a no-op. */
int ifd_mask_from_gray(const uint8_t* gray, int64_t n, float* mask, void* stream);

/* Library loops (GaussianDiffusion.p_sample_loop / ddim_sample_loop, code/gaussian_diffusion.py:357-538):
 *   ifd_lib_inject: apply_inpainting_injection (:114-157): out = keep * (ca * gt + cb * noise) + (1 - keep) * x,
 *     keep [B,1,H,W] broadcast over C; ca, cb the fp32 q_sample coefficients of the step (cached-noise
 *     path: sqrt_alphas_cumprod / sqrt_one_minus; fresh-noise path: fp32 sqrt of the extracted ac).
 *   ifd_lib_update: ddim != 0: ddim_sample (:447-485), else p_sample (:357-388), from the model output
 *     out6 [B,6,H,W] (eps, learned-range v) and the step noise: sample (and pred_xstart, may be NULL). */
typedef struct ifd_lib_coeffs {
  float c_recip, c_recipm1;   /* sqrt_recip_alphas_cumprod[t], sqrt_recipm1_alphas_cumprod[t] */
  float c_ab, c_abp, c_eta;   /* DDIM: alphas_cumprod[t], alphas_cumprod_prev[t], eta */
  float c_nonzero;            /* (t != 0) */
  float c_min_log, c_max_log, c_coef1, c_coef2;  /* DDPM: posterior_log_variance_clipped, log(betas), coefs */
  int clip, pad;
} ifd_lib_coeffs;
int ifd_lib_inject(const float* x, const float* gt, const float* keep, const float* noise, float ca, float cb,
                   int64_t B, int C, int H, int W, float* out, void* stream);
int ifd_lib_update(int ddim, const float* x, const float* out6, const float* noise, int64_t B, int H, int W,
                   const ifd_lib_coeffs* c, float* sample, float* pred_xstart, void* stream);

/* Input-side data formats (OrderedMaskDataset / InpaintingDataset transforms, code/data/dataset.py:
 * 231-240, 273-286) on the device. No GPU use by ifd_resize_coeffs / ifd_resize_u8_workspace.
 *   ifd_resize_u8: Pillow BILINEAR resample (torchvision Resize((Hout, Wout)) of a PIL image), bit-exact,
 *     NHWC uint8 [N,Hin,Win,C] -> [N,Hout,Wout,C]; `work` >= ifd_resize_u8_workspace(...) bytes.
 *   ifd_resize_coeffs: the fixed-point coefficients (bounds[out][2] = first, count; coeffs[out][ksize]).
 *   ifd_image_to_float: ToTensor + Normalize(0.5, 0.5): NHWC u8 -> NCHW fp32 in [-1, 1].
 *   ifd_make_inpaint_batch: ordered mask cycling + mask rule + masked image for a batch: mask[n] =
 *     (bank[idx[n] % M] / 255 < 0.5), masked_image = images * (1 - mask); bank u8 [M][H][W];
 *     images / masked_image [N,3,H,W], mask [N,1,H,W] fp32 (either output may be NULL). */
int ifd_resize_coeffs(int in_size, int out_size, int* bounds, int* coeffs, int* ksize);
int64_t ifd_resize_u8_workspace(int64_t N, int C, int Hin, int Win, int Hout, int Wout);
int ifd_resize_u8(const uint8_t* src, int64_t N, int C, int Hin, int Win, int Hout, int Wout, uint8_t* dst,
                  uint8_t* work, int64_t work_bytes, void* stream);
int ifd_image_to_float(const uint8_t* src_nhwc, int64_t N, int C, int H, int W, float* dst_nchw, void* stream);
int ifd_make_inpaint_batch(const float* images, int64_t N, int H, int W, const uint8_t* mask_bank, int M,
                           const int64_t* idx, float* mask, float* masked_image, void* stream);

/* Per-launch profiler: when enabled, every kernel the handle launches is bracketed by hipEvents on
 * its stream; after the caller synchronises, ifd_profile_report writes a JSON summary per kernel
 * name {"count", "ms", "flops" (algorithmic 2*MAC), "bytes" (algorithmic)} and clears it. */
int ifd_profile_enable(ifd_handle* h, int on);  /* 0 off, 1 by kernel, 2 by kernel + layer shape */
/* Record only the launches whose kernel name starts with `prefix` ("" or NULL: all), so a timed
 * region carries event packets only around the kernel it measures. */
int ifd_profile_filter(ifd_handle* h, const char* prefix);
int ifd_profile_report(ifd_handle* h, char* buf, int64_t buflen);
const char* ifd_version(void);

#ifdef __cplusplus
}
#endif
#endif
