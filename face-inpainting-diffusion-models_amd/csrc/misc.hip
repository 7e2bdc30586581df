// Small kernels around the conv core: input assembly, timestep embedding + MLP, the batched
// ResBlock emb projections, QKV attention, and the standalone sampler step / blend kernels.
#include "conv.h"
#include "conv_dev.h"
#include "kernels.h"

namespace ifd {

// ---------------------------------------------------------------------------------------------
// Input assembly (code/unet.py:197-200 + code/test_inp_ddim_50.py:373-385):
//   [x(3), masked_image(3), mask, mask, mask] NCHW fp32  ->  NHWC with 16 channels (9 used, 7 zero)
// mode 0: (x, masked_image, mask) given directly (model.forward)
// mode 1: (img, gt, masks) from the sampler: masked = gt*keep + 0*(1-keep), mask_in = 1 - keep,
//         keep = 1 - masks, bit-for-bit the fp32 ops of model_fn.
__global__ void pack_input_kernel(const float* __restrict__ x, const float* __restrict__ a,
                                  const float* __restrict__ m, int mode, int N, int HW, float* __restrict__ out) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= N * HW) return;
  const int n = idx / HW, px = idx - n * HW;
  const float* xn = x + (size_t)n * 3 * HW + px;
  const float* an = a + (size_t)n * 3 * HW + px;
  float mk = m[(size_t)n * HW + px];
  f32x4 o0, o1, o2, o3;
  o0[0] = xn[0]; o0[1] = xn[HW]; o0[2] = xn[2 * HW];
  float m0, m1, m2;
  if (mode == 0) {
    m0 = an[0]; m1 = an[HW]; m2 = an[2 * HW];
  } else {
#pragma clang fp contract(off)
    const float keep = 1.0f - mk;
    const float zk = 0.0f * (1.0f - keep);
    m0 = an[0] * keep + zk; m1 = an[HW] * keep + zk; m2 = an[2 * HW] * keep + zk;
    mk = 1.0f - keep;
  }
  o0[3] = m0; o1[0] = m1; o1[1] = m2; o1[2] = mk; o1[3] = mk;
  o2[0] = mk; o2[1] = 0.f; o2[2] = 0.f; o2[3] = 0.f;
  o3[0] = 0.f; o3[1] = 0.f; o3[2] = 0.f; o3[3] = 0.f;
  f32x4* dst = reinterpret_cast<f32x4*>(out + (size_t)idx * 16);
  dst[0] = o0; dst[1] = o1; dst[2] = o2; dst[3] = o3;
}

void launch_pack_input(const float* x, const float* a, const float* m, int mode, int N, int HW, float* out,
                       hipStream_t s) {
  const int tot = N * HW;
  hipLaunchKernelGGL(pack_input_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, x, a, m, mode, N, HW, out);
}

// ---------------------------------------------------------------------------------------------
// The embedding MLPs as skinny GEMMs: out[n][j] = post(sum_k pre(in)[n][k] * Wt[k][j] + b[j]) for
// the N <= 16 images of a pass, Wt pre-transposed to [K][J] so a wave's weight loads coalesce.
//   time_embed.0 (code/unet.py:44-48, nn.py:51-61): pre = timestep_embedding(t), post = SiLU
//   time_embed.2: pre = identity (the stored h1 is already SiLU'd), post = identity
//   all 30 ResBlock emb_layers (nn.py:167-170,199) in one launch: pre = SiLU, post = identity
// Block = 64 columns x 4 K-quarters (one wave each); the input rows sit in LDS as [k][16] so a
// k step is 1 coalesced weight load + 4 broadcast ds_read_b128 + 16 FMAs; the quarters are summed
// in a fixed order (deterministic). Bound: the weight stream (K x J x 4 B, read once per pass).
enum SkPre : int { SK_PRE_NONE = 0, SK_PRE_SILU = 1, SK_PRE_TEMB = 2 };
constexpr int SK_NB = 16;  // images per pass
constexpr int SK_JB = 64;  // columns per block
__global__ __launch_bounds__(256) void skinny_kernel(const float* __restrict__ in, const int64_t* __restrict__ t,
                                                     const float* __restrict__ freqs, int pre, int post_silu, int K,
                                                     int N, const float* __restrict__ wt,
                                                     const float* __restrict__ b, int J, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float sk[];  // [K][SK_NB] inputs, then [4][SK_NB][SK_JB]
  float* red = sk + (size_t)K * SK_NB;
  const int tid = threadIdx.x, jj = tid & (SK_JB - 1), kq = tid / SK_JB;
  const int j = blockIdx.x * SK_JB + jj;
  const int kc = K / 4, k0 = kq * kc;
  for (int nb = 0; nb < N; nb += SK_NB) {
    const int nn = min(SK_NB, N - nb);
    __syncthreads();
    for (int i = tid; i < K * SK_NB; i += 256) {
      const int kk = i / SK_NB, q = i % SK_NB;
      float v = 0.f;
      if (q < nn) {
        if (pre == SK_PRE_TEMB) {
          const int half = K / 2;
          const float arg = (float)t[nb + q] * freqs[kk < half ? kk : kk - half];
          v = kk < half ? cosf(arg) : sinf(arg);
        } else {
          v = in[(size_t)(nb + q) * K + kk];
          if (pre == SK_PRE_SILU) v = silu_f(v);
        }
      }
      sk[i] = v;
    }
    __syncthreads();
    float acc[SK_NB];
#pragma unroll
    for (int q = 0; q < SK_NB; ++q) acc[q] = 0.f;
    if (j < J) {
      // (16 weight loads in flight per wave: the loop is latency-bound at ~1 wave per SIMD; the
      // accumulation order per slot is unchanged)
#pragma unroll 16
      for (int kk = k0; kk < k0 + kc; ++kk) {
        const float w = wt[(size_t)kk * J + j];
        const f32x4* s4 = reinterpret_cast<const f32x4*>(sk + (size_t)kk * SK_NB);
#pragma unroll
        for (int g = 0; g < SK_NB / 4; ++g) {
          const f32x4 s = s4[g];
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[4 * g + c] = fmaf(w, s[c], acc[4 * g + c]);  // one rounding in every slot
        }
      }
    }
#pragma unroll
    for (int q = 0; q < SK_NB; ++q) red[(kq * SK_NB + q) * SK_JB + jj] = acc[q];
    __syncthreads();
    for (int i = tid; i < SK_NB * SK_JB; i += 256) {
      const int q = i / SK_JB, c = i % SK_JB, jo = blockIdx.x * SK_JB + c;
      if (q < nn && jo < J) {
        float v = ((red[(0 * SK_NB + q) * SK_JB + c] + red[(1 * SK_NB + q) * SK_JB + c]) +
                   red[(2 * SK_NB + q) * SK_JB + c]) + red[(3 * SK_NB + q) * SK_JB + c];
        v += b[jo];
        if (post_silu) v = silu_f(v);
        out[(size_t)(nb + q) * J + jo] = v;
      }
    }
  }
}

static void launch_skinny(const float* in, const int64_t* t, const float* freqs, int pre, int post_silu, int K, int N,
                          const float* wt, const float* b, int J, float* out, hipStream_t s) {
  const size_t lds = ((size_t)K * SK_NB + 4 * SK_NB * SK_JB) * sizeof(float);
  hipLaunchKernelGGL(skinny_kernel, dim3((J + SK_JB - 1) / SK_JB), dim3(256), lds, s, in, t, freqs, pre, post_silu, K,
                     N, wt, b, J, out);
}

// emb = time_embed(timestep_embedding(t, mc)); h1 (SiLU'd first layer) in `h1` [N][E]
void launch_temb(const int64_t* t, const float* freqs, int mc, const float* w0t, const float* b0, const float* w2t,
                 const float* b2, int E, int N, float* h1, float* emb, hipStream_t s) {
  launch_skinny(nullptr, t, freqs, SK_PRE_TEMB, 1, mc, N, w0t, b0, E, h1, s);
  launch_skinny(h1, nullptr, nullptr, SK_PRE_NONE, 0, E, N, w2t, b2, E, emb, s);
}

// All 30 ResBlock emb projections of one eval: Eall[n][j] = sum_k Wt[k][j] * silu(emb[n][k]) + b[j]
void launch_emb_proj(const float* emb, int E, int N, const float* wt, const float* b, int J, float* out,
                     hipStream_t s) {
  launch_skinny(emb, nullptr, nullptr, SK_PRE_SILU, 0, E, N, wt, b, J, out, s);
}

// ---------------------------------------------------------------------------------------------
// QKVAttention (code/nn.py:222-235), "chunk first" order: q = qkv[..., 0:C], k = [C:2C], v = [2C:3C],
// head h = channels [64h, 64h+64) of each. w = softmax((q*s)(k*s)^T) in fp32, a = w v.
// One block per (n, head, 32 queries); the whole score row (T <= 256) stays in LDS so the softmax
// is the exact max-subtract / exp / multiply-by-reciprocal of the reference (no online rescale).
constexpr int AT_QB = 32;
constexpr int AT_CH = 64;
constexpr int AT_KB = 64;

__global__ __launch_bounds__(256) void attention_kernel(const float* __restrict__ qkv, int T, int C, float scale,
                                                        float* __restrict__ out) {
  __shared__ float Qs[AT_QB][AT_CH + 1];
  __shared__ float KV[AT_KB][AT_CH + 1];
  __shared__ float S[AT_QB][256 + 1];
  const int tid = threadIdx.x;
  const int qb = blockIdx.x, head = blockIdx.y, n = blockIdx.z;
  const int t0 = qb * AT_QB;
  const size_t rowstride = 3 * (size_t)C;
  const float* base = qkv + (size_t)n * T * rowstride;
  for (int i = tid; i < AT_QB * AT_CH; i += 256) {
    const int r = i / AT_CH, c = i % AT_CH;
    const int tq = t0 + r;
    Qs[r][c] = tq < T ? base[(size_t)tq * rowstride + head * AT_CH + c] * scale : 0.f;
  }
  const int r = tid / 8, u = tid % 8;
  for (int kt = 0; kt < T; kt += AT_KB) {
    __syncthreads();
    for (int i = tid; i < AT_KB * AT_CH; i += 256) {
      const int s = i / AT_CH, c = i % AT_CH;
      const int ts = kt + s;
      KV[s][c] = ts < T ? base[(size_t)ts * rowstride + C + head * AT_CH + c] * scale : 0.f;
    }
    __syncthreads();
    for (int jj = 0; jj < AT_KB / 8; ++jj) {
      const int s = u + 8 * jj;
      if (kt + s < T) {
        float acc = 0.f;
        for (int c = 0; c < AT_CH; ++c) acc += Qs[r][c] * KV[s][c];
        S[r][kt + s] = acc;
      }
    }
  }
  __syncthreads();
  // softmax: 4 waves x 8 rows, lanes stride over the row
  {
    const int wave = tid / 64, lane = tid % 64;
    for (int rr = 0; rr < AT_QB / 4; ++rr) {
      const int row = wave * (AT_QB / 4) + rr;
      float mx = -INFINITY;
      for (int s = lane; s < T; s += 64) mx = fmaxf(mx, S[row][s]);
      for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
      float sum = 0.f;
      for (int s = lane; s < T; s += 64) {
        const float e = expf(S[row][s] - mx);
        S[row][s] = e;
        sum += e;
      }
      for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
      const float inv = 1.0f / sum;
      for (int s = lane; s < T; s += 64) S[row][s] = S[row][s] * inv;
    }
  }
  float acc[8];
  for (int q = 0; q < 8; ++q) acc[q] = 0.f;
  for (int kt = 0; kt < T; kt += AT_KB) {
    __syncthreads();
    for (int i = tid; i < AT_KB * AT_CH; i += 256) {
      const int s = i / AT_CH, c = i % AT_CH;
      const int ts = kt + s;
      KV[s][c] = ts < T ? base[(size_t)ts * rowstride + 2 * C + head * AT_CH + c] : 0.f;
    }
    __syncthreads();
    const int smax = min(AT_KB, T - kt);
    for (int s = 0; s < smax; ++s) {
      const float pw = S[r][kt + s];
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += pw * KV[s][u + 8 * q];
    }
  }
  const int tq = t0 + r;
  if (tq < T)
    for (int q = 0; q < 8; ++q) out[((size_t)n * T + tq) * C + head * AT_CH + u + 8 * q] = acc[q];
}

// The same attention on fp32 MFMA (v_mfma_f32_32x32x2_f32: an exact fp32 fma chain at the fp32
// vector rate, 1/16 of the f16 matrix rate - attention is 0.1 % of the FLOPs, so exactness wins),
// for T a multiple of 32 up to 256. Block = (n, head, 128 queries), 4 waves x 32 queries; the
// head's K (pre-scaled) and V for all T keys sit in LDS. Per wave:
//   S^T = K Q^T as KT = T/32 tiles of 32 keys x 32 queries: lane (query l32, half h) gets the
//     keys 8(r>>2) + 4h + (r&3) of each tile in its 16 accumulator registers; the channel order
//     of the 32 k-steps is permuted (half h supplies channel 32h + t) on both operands.
//   softmax over keys: in-register max / exp / sum plus one exchange with lane ^ 32 (the other
//     key half), then multiply by the reciprocal - the arithmetic of attention_kernel.
//   O = P V: P is used straight from the accumulators as the A operand (lane (query, h) supplies
//     key 8(r>>2) + 4h + (r&3) of k-step (tile, r)), V from LDS as B; lane l32 = channel on output.
constexpr int AM_KS = 68;  // K row stride (floats): ds_read_b128 of 32 rows conflict-free
constexpr int AM_VS = 72;  // V row stride: rows 4 keys apart (the two lane halves) 32 banks apart
template <int KT>
__global__ __launch_bounds__(256, 1) void attention_mfma_kernel(const float* __restrict__ qkv, int C, float scale,
                                                                float* __restrict__ out) {
  constexpr int T = 32 * KT;
  extern __shared__ __attribute__((aligned(16))) float am[];
  float* Ks = am;                 // [T][AM_KS]
  float* Vs = am + T * AM_KS;     // [T][AM_VS]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int head = blockIdx.y, n = blockIdx.z;
  const size_t rs = 3 * (size_t)C;
  const float* base = qkv + (size_t)n * T * rs + head * AT_CH;
  for (int i = tid; i < T * (AT_CH / 4); i += 256) {
    const int row = i / (AT_CH / 4), c4 = 4 * (i % (AT_CH / 4));
    f32x4 kv = gld4(base + (size_t)row * rs + C + c4);
#pragma unroll
    for (int j = 0; j < 4; ++j) kv[j] = kv[j] * scale;
    *(f32x4*)(Ks + row * AM_KS + c4) = kv;
    *(f32x4*)(Vs + row * AM_VS + c4) = gld4(base + (size_t)row * rs + 2 * C + c4);
  }
  __syncthreads();
  const int q0 = blockIdx.x * 128 + 32 * w;
  if (q0 >= T) return;
  float qv[32];  // Q[q0 + l32][32h .. 32h + 32) * scale
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const f32x4 v = gld4(base + (size_t)(q0 + l32) * rs + 32 * h + 4 * j);
#pragma unroll
    for (int c = 0; c < 4; ++c) qv[4 * j + c] = v[c] * scale;
  }
  f32x16 s[KT];
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
#pragma unroll
    for (int r = 0; r < 16; ++r) s[kt][r] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const f32x4 kf = *(const f32x4*)(Ks + (kt * 32 + l32) * AM_KS + 32 * h + 4 * j);
#pragma unroll
      for (int c = 0; c < 4; ++c) s[kt] = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[c], qv[4 * j + c], s[kt], 0, 0, 0);
    }
  }
  float mx = -INFINITY;
#pragma unroll
  for (int kt = 0; kt < KT; ++kt)
#pragma unroll
    for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[kt][r]);
  mx = fmaxf(mx, __shfl_xor(mx, 32));
  float sum = 0.f;
#pragma unroll
  for (int kt = 0; kt < KT; ++kt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float e = expf(s[kt][r] - mx);
      s[kt][r] = e;
      sum += e;
    }
  sum += __shfl_xor(sum, 32);
  const float inv = 1.0f / sum;
  f32x16 o0, o1;
#pragma unroll
  for (int r = 0; r < 16; ++r) o0[r] = o1[r] = 0.f;
#pragma unroll
  for (int kt = 0; kt < KT; ++kt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float pw = s[kt][r] * inv;
      const float* vr = Vs + (kt * 32 + 8 * (r >> 2) + 4 * h + (r & 3)) * AM_VS + l32;
      o0 = __builtin_amdgcn_mfma_f32_32x32x2f32(pw, vr[0], o0, 0, 0, 0);
      o1 = __builtin_amdgcn_mfma_f32_32x32x2f32(pw, vr[32], o1, 0, 0, 0);
    }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int q = q0 + 8 * (r >> 2) + 4 * h + (r & 3);
    float* o = out + ((size_t)n * T + q) * C + head * AT_CH + l32;
    o[0] = o0[r];
    o[32] = o1[r];
  }
}

template <int KT>
static void launch_attention_mfma(const float* qkv, int N, int C, float scale, float* out, hipStream_t s) {
  constexpr int T = 32 * KT;
  const size_t lds = (size_t)T * (AM_KS + AM_VS) * sizeof(float);
  static bool attr[kMaxDevices] = {};
  (void)set_lds_attr_once(attr, reinterpret_cast<const void*>(&attention_mfma_kernel<KT>), (int)lds);
  dim3 grid((T + 127) / 128, C / AT_CH, N);
  hipLaunchKernelGGL(attention_mfma_kernel<KT>, grid, dim3(256), lds, s, qkv, C, scale, out);
}

void launch_attention(const float* qkv, int N, int T, int C, float scale, float* out, hipStream_t s) {
  if (C % AT_CH == 0) {
    if (T == 256) return launch_attention_mfma<8>(qkv, N, C, scale, out, s);
    if (T == 128) return launch_attention_mfma<4>(qkv, N, C, scale, out, s);
    if (T == 64) return launch_attention_mfma<2>(qkv, N, C, scale, out, s);
    if (T == 32) return launch_attention_mfma<1>(qkv, N, C, scale, out, s);
  }
  dim3 grid((T + AT_QB - 1) / AT_QB, C / AT_CH, N);
  hipLaunchKernelGGL(attention_kernel, grid, dim3(256), 0, s, qkv, T, C, scale, out);
}

// ---------------------------------------------------------------------------------------------
// Standalone sampler updates on a model output [N,6,H,W] (same math as the fused conv epilogue).
__global__ void step_kernel(int mode, const StepCoeffs sc, const float* __restrict__ out6, float* __restrict__ img,
                            const float* __restrict__ gt, const float* __restrict__ mask,
                            const float* __restrict__ noise, const float* __restrict__ known, int N, int HW) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= N * 3 * HW) return;
  const int px = idx % HW, nc = idx / HW, c = nc % 3, n = nc / 3;
  const float eps = out6[((size_t)n * 6 + c) * HW + px];
  const size_t om = (size_t)n * HW + px;
  const float mk = sc.inject ? mask[om] : 0.f;
  const float g = sc.inject ? gt[idx] : 0.f;
  const float kn = sc.inject ? known[idx] : 0.f;
  float v;
  if (mode == EPI_DDIM) {
    v = ddim_step_value(sc, img[idx], eps, sc.use_noise ? noise[idx] : 0.f, g, mk, kn);
  } else {
    const float var_v = out6[((size_t)n * 6 + c + 3) * HW + px];
    v = ddpm_step_value(sc, img[idx], eps, var_v, noise[idx], g, mk, kn);
  }
  img[idx] = v;
}

void launch_step(int mode, const StepCoeffs& sc, const float* out6, float* img, const float* gt, const float* mask,
                 const float* noise, const float* known, int N, int HW, hipStream_t s) {
  const int tot = N * 3 * HW;
  hipLaunchKernelGGL(step_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, mode, sc, out6, img, gt, mask, noise,
                     known, N, HW);
}

// final blend (code/test_inp_ddim_50.py:692-696): out = result*mask + gt*(1 - mask)
__global__ void blend_kernel(const float* __restrict__ res, const float* __restrict__ gt,
                             const float* __restrict__ mask, float* __restrict__ out, int N, int C, int HW) {
#pragma clang fp contract(off)
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= N * C * HW) return;
  const int px = idx % HW, n = idx / (C * HW);
  const float m = mask[(size_t)n * HW + px];
  const float keep = 1.0f - m;
  out[idx] = res[idx] * m + gt[idx] * keep;
}

void launch_blend(const float* res, const float* gt, const float* mask, float* out, int N, int C, int HW,
                  hipStream_t s) {
  const int tot = N * C * HW;
  hipLaunchKernelGGL(blend_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, res, gt, mask, out, N, C, HW);
}

// toU8 (code/test_inp_ddim_50.py:33-41): NCHW fp32 in [-1,1] -> NHWC u8,
// ((x + 1) * 127.5).clamp(0, 255) then a truncating cast. One thread per pixel: channel reads are
// coalesced across the wave (stride HW), the C output bytes of a pixel are contiguous.
__global__ void to_u8_kernel(const float* __restrict__ x, unsigned char* __restrict__ out, int N, int C, int HW) {
#pragma clang fp contract(off)
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= N * HW) return;
  const int px = idx % HW, n = idx / HW;
  const float* src = x + (size_t)n * C * HW + px;
  unsigned char* dst = out + (size_t)idx * C;
  for (int c = 0; c < C; ++c) {
    float v = (src[(size_t)c * HW] + 1.0f) * 127.5f;
    v = fminf(fmaxf(v, 0.0f), 255.0f);
    dst[c] = (unsigned char)(int)v;
  }
}

void launch_to_u8(const float* x, unsigned char* out, int N, int C, int HW, hipStream_t s) {
  const int tot = N * HW;
  hipLaunchKernelGGL(to_u8_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, x, out, N, C, HW);
}

// OrderedMaskDataset mask convention (code/data/dataset.py:278-286): ToTensor's gray/255 in fp32,
// then (m < 0.5).float() -> 1 = hole (black), 0 = keep (white).
__global__ void mask_from_gray_kernel(const unsigned char* __restrict__ g, float* __restrict__ m, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  m[i] = ((float)g[i] / 255.0f < 0.5f) ? 1.0f : 0.0f;
}

void launch_mask_from_gray(const unsigned char* g, float* m, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(mask_from_gray_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g, m, n);
}

// act + 2x2 average pool, 4 channels per thread (16-byte loads/stores, coalesced along C).
__global__ __launch_bounds__(256) void act_pool_kernel(const float* __restrict__ x, int C, int N, int Hin, int act,
                                                       const float* __restrict__ A, const float* __restrict__ B,
                                                       float* __restrict__ out, float* __restrict__ out_raw) {
  const int Ho = Hin / 2, Q = C / 4;
  const size_t tot = (size_t)N * Ho * Ho * Q;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= tot) return;
  const int q = (int)(i % Q);
  const size_t pix = i / Q;
  const int xo = (int)(pix % Ho), yo = (int)((pix / Ho) % Ho), n = (int)(pix / ((size_t)Ho * Ho));
  const float* b = x + (((size_t)n * Hin + 2 * yo) * Hin + 2 * xo) * C + 4 * q;
  const f32x4 v00 = *(const f32x4*)b, v01 = *(const f32x4*)(b + C);
  const f32x4 v10 = *(const f32x4*)(b + (size_t)Hin * C), v11 = *(const f32x4*)(b + (size_t)Hin * C + C);
  f32x4 a = {1.f, 1.f, 1.f, 1.f}, c = {0.f, 0.f, 0.f, 0.f};
  if (act != ACT_NONE) {
    a = *(const f32x4*)(A + (size_t)n * C + 4 * q);
    c = *(const f32x4*)(B + (size_t)n * C + 4 * q);
  }
  f32x4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    auto f = [&](float v) {
      if (act == ACT_NONE) return v;
      const float t = a[j] * v + c[j];
      return act == ACT_AFFINE_SILU ? silu_fast(t) : t;
    };
    float s = f(v00[j]);
    s = s + f(v01[j]);
    s = s + f(v10[j]);
    s = s + f(v11[j]);
    r[j] = s * 0.25f;
  }
  *(f32x4*)(out + pix * C + 4 * q) = r;
  if (out_raw) {  // the down-ResBlock's residual pool(x) from the same four reads
    f32x4 rr;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float s = v00[j];
      s = s + v01[j];
      s = s + v10[j];
      s = s + v11[j];
      rr[j] = s * 0.25f;
    }
    *(f32x4*)(out_raw + pix * C + 4 * q) = rr;
  }
}

// act(A[n,c] x + B[n,c]) of an NHWC tensor, materialised for the split kernel's 1x1 chunks (the
// attention qkv conv's GroupNorm prologue): the arithmetic of the conv prologues.
__global__ __launch_bounds__(256) void act_apply_kernel(const float* __restrict__ x, int C, int HW, int act,
                                                        const float* __restrict__ A, const float* __restrict__ B,
                                                        size_t tot, float* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= tot) return;
  const int Q = C / 4;
  const int q = (int)(i % Q);
  const int n = (int)(i / ((size_t)Q * HW));
  const f32x4 v = *(const f32x4*)(x + 4 * i);
  const f32x4 a = *(const f32x4*)(A + (size_t)n * C + 4 * q), c = *(const f32x4*)(B + (size_t)n * C + 4 * q);
  f32x4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float t = a[j] * v[j] + c[j];
    r[j] = act == ACT_AFFINE_SILU ? silu_fast(t) : t;
  }
  *(f32x4*)(out + 4 * i) = r;
}

int launch_act_apply(const float* x, int C, int N, int HW, int act, const float* A, const float* B, float* out,
                     hipStream_t s) {
  const size_t tot = (size_t)N * HW * (C / 4);
  hipLaunchKernelGGL(act_apply_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, x, C, HW, act, A, B, tot,
                     out);
  return IFD_LAUNCH_STATUS();
}

int launch_act_pool(const float* x, int C, int N, int Hin, int act, const float* A, const float* B, float* out,
                    float* out_raw, hipStream_t s) {
  const size_t tot = (size_t)N * (Hin / 2) * (Hin / 2) * (C / 4);
  hipLaunchKernelGGL(act_pool_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, x, C, N, Hin, act, A, B,
                     out, out_raw);
  return IFD_LAUNCH_STATUS();
}

}  // namespace ifd
