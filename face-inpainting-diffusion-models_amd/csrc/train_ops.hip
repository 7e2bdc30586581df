// Training step ops (BASELINE configs[4]): the fp32 forward pieces the
// backward needs saved, and every backward kernel of the 9-channel UNet — conv dgrad (the forward
// fp32 MFMA conv on transposed-flipped weights) and wgrad (fp32 MFMA over pixels), GroupNorm +
// scale/shift + SiLU backward, nearest-up / avg-pool backward, QKV attention backward, the
// time-embedding linears, the masked eps-MSE loss and its gradient, grad-norm clipping and AdamW.
// Reference: code/train_inpainting.py:15-79 (train_epoch: loss.backward, clip_grad_norm_(1.0),
// AdamW.step), code/gaussian_diffusion.py:540-614 (training_losses), code/nn.py / code/unet.py
// (the modules differentiated). Activations are NHWC fp32; weights live in the reference's
// torch layouts inside one flat parameter buffer (ifd/train.py) and are packed per step.
// Every reduction runs in a fixed order (no atomics): a step is bit-reproducible.
#include <type_traits>
#include "../../include/ifd_train.h"

#include <cmath>
#include <cstring>

#include "conv.h"
#include "conv_dev.h"
#include "kernels.h"

namespace ifd {
namespace {

constexpr int TB = 256;

inline int grid1(int64_t n, int per = TB) { return (int)((n + per - 1) / per); }

// ---------------------------------------------------------------------------------------------
// Weight packing on the device (weights change every step). Layout of conv.hip:
// [Cout_pad/BN][Cin_pad/8][taps][q=2][BN][4], element W'[ct*BN + col][ch*8 + q*4 + j][tap].
// cout / cin are the weight tensor's dims W[cout][cin][taps]; cin_pad / cout_pad the packed conv's.
// transpose = 0: W' = W (forward). transpose = 1: dgrad, W'[ci][co][tap] = W[co][ci][taps-1-tap]
// (the transposed convolution of a stride-1, pad-1 3x3 conv is a 3x3 conv with the kernel flipped).
__global__ void pack_conv_kernel(const float* __restrict__ w, int cout, int cin, int taps, int bn, int cin_pad,
                                 int cout_pad, int transpose, float* __restrict__ dst) {
  const int64_t tot = (int64_t)cout_pad * cin_pad * taps;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= tot) return;
  // decode the destination index
  const int jj = (int)(i & 3);
  int64_t r = i >> 2;
  const int col = (int)(r % bn);
  r /= bn;
  const int q = (int)(r & 1);
  r >>= 1;
  const int tap = (int)(r % taps);
  r /= taps;
  const int nch = cin_pad / 8;
  const int chk = (int)(r % nch);
  const int ct = (int)(r / nch);
  const int o = ct * bn + col, c = chk * 8 + q * 4 + jj;  // packed (out, in) channel
  float v = 0.f;
  if (transpose == 0) {
    if (o < cout && c < cin) v = w[((size_t)o * cin + c) * taps + tap];
  } else {  // packed out channel o = the forward's input channel, packed in channel c = its output
    if (o < cin && c < cout) v = w[((size_t)c * cin + o) * taps + (taps - 1 - tap)];
  }
  dst[i] = v;
}

// ---------------------------------------------------------------------------------------------
// Weight gradient on fp32 MFMA (v_mfma_f32_32x32x2f32):
//   dW[co][ci][tap] = sum over pixels (n, y, x) of dY[n,y,x,co] * X[n, y + ky - 1, x + kx - 1, ci]
// with X = concat(x0, x1) along channels, zero padding. GEMM view: M = co, N = ci (one tap per
// block), K = pixels. Block = 4 waves, tile 64 co x 64 ci; wave w owns rows 32 (w & 1), cols
// 32 (w >> 1). Per chunk of 32 pixels the block stages dY^T [64][32] and X^T [64][32] (pixel
// contiguous) in LDS; an MFMA's k pair is pixels (j, 16 + j) so a lane reads its 16 pixels with
// four ds_read_b128. K is split over blockIdx.y: the partial sums go to slab z of `part`
// [S][cout][cin][taps] and wgrad_reduce adds the slabs in order (deterministic).
constexpr int WG_CH = 32;     // pixels per chunk
constexpr int WG_LD = 36;     // LDS row stride (floats): 16-B aligned rows
struct WgArgs {
  const float* dy; int cout;
  const float* x0; int c0;
  const float* x1; int c1;
  int N, H, W, taps;
  int64_t P;           // N * H * W
  int chunks_per_split;
  float* part;         // [S][cout][cin][taps]
  // wgrad_ws_kernel<.., GNA = true>: X = silu(actA[n][c] x + actB[n][c]) of the raw x0, zero padded after the
  // activation (the forward conv's GroupNorm + SiLU prologue, recomputed at staging instead of materialised)
  const float* actA; const float* actB;
};

__global__ __launch_bounds__(256) void wgrad_kernel(WgArgs a) {
  __shared__ __attribute__((aligned(16))) float dyt[64 * WG_LD];
  __shared__ __attribute__((aligned(16))) float xt[64 * WG_LD];
  const int cin = a.c0 + a.c1;
  const int nci = (cin + 63) / 64;
  int b = blockIdx.x;
  const int tap = b % a.taps;
  b /= a.taps;
  const int cit = b % nci, cot = b / nci;
  const int co0 = cot * 64, ci0 = cit * 64;
  const int ky = a.taps == 9 ? tap / 3 - 1 : 0, kx = a.taps == 9 ? tap % 3 - 1 : 0;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int wr = 32 * (wave & 1), wc = 32 * (wave >> 1);
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const int64_t nch = (a.P + WG_CH - 1) / WG_CH;
  const int64_t c_beg = (int64_t)blockIdx.y * a.chunks_per_split;
  const int64_t c_end = c_beg + a.chunks_per_split < nch ? c_beg + a.chunks_per_split : nch;
  const int HW = a.H * a.W;
  // staging assignment: thread -> (pixel pr = tid / 16 and pr + 16, channel quad 4 (tid % 16))
  const int pr = tid >> 4, cq = 4 * (tid & 15);
  for (int64_t ch = c_beg; ch < c_end; ++ch) {
    const int64_t p0 = ch * WG_CH;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int pl = pr + 16 * half;
      const int64_t pix = p0 + pl;
      f32x4 vy = {0.f, 0.f, 0.f, 0.f}, vx = {0.f, 0.f, 0.f, 0.f};
      if (pix < a.P) {
        const int co = co0 + cq;
        if (co < a.cout) {
          if (co + 3 < a.cout && (a.cout & 3) == 0) {
            vy = *reinterpret_cast<const f32x4*>(a.dy + pix * a.cout + co);
          } else {
            for (int j = 0; j < 4; ++j)
              if (co + j < a.cout) vy[j] = a.dy[pix * a.cout + co + j];
          }
        }
        const int n = (int)(pix / HW), rem = (int)(pix - (int64_t)n * HW);
        const int y = rem / a.W + ky, x = rem % a.W + kx;
        const int ci = ci0 + cq;
        if (y >= 0 && y < a.H && x >= 0 && x < a.W && ci < cin) {
          const int64_t sp = ((int64_t)n * a.H + y) * a.W + x;
          for (int j = 0; j < 4; ++j) {
            const int c = ci + j;
            if (c < a.c0) vx[j] = a.x0[sp * a.c0 + c];
            else if (c < cin) vx[j] = a.x1[sp * a.c1 + (c - a.c0)];
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dyt[(cq + j) * WG_LD + pl] = vy[j];
        xt[(cq + j) * WG_LD + pl] = vx[j];
      }
    }
    __syncthreads();
    f32x4 av[4], bv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      av[k] = *reinterpret_cast<const f32x4*>(&dyt[(wr + l32) * WG_LD + 16 * h + 4 * k]);
      bv[k] = *reinterpret_cast<const f32x4*>(&xt[(wc + l32) * WG_LD + 16 * h + 4 * k]);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[k][j], bv[k][j], acc, 0, 0, 0);
    __syncthreads();
  }
  // C[i][j], i = 8 (r >> 2) + 4 h + (r & 3) (co), j = l32 (ci)
  float* slab = a.part + (size_t)blockIdx.y * a.cout * cin * a.taps;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int co = co0 + wr + 8 * (r >> 2) + 4 * h + (r & 3);
    const int ci = ci0 + wc + l32;
    if (co < a.cout && ci < cin) slab[((size_t)co * cin + ci) * a.taps + tap] = acc[r];
  }
}

// Weight gradient, all taps of a 64 co x 64 ci tile per block (v_mfma_f32_32x32x2f32):
//   dW[co][ci][tap] = sum over output pixels p of dY[p][co] X[p + offset(tap)][ci]
// K = output pixels in chunks of 32: a 32-pixel row segment, or 32 / W whole rows when W < 32. Per
// chunk the block stages dY [32 px][64 co] and the X halo [(R + 2) rows][(Wc + 2) cols][64 ci] in LDS
// pixel-major and channel-contiguous (straight 16-B copies, no transpose), double-buffered: the
// next chunk's loads are in registers while this chunk's MFMAs run. Wave w owns the 32 x 32
// quadrant (co 32 (w & 1), ci 32 (w >> 1)) of every tap: TAPS x 16 accumulator registers. Per k pair
// (chunk pixels j and j + 16, one per lane half) one LDS read of dY serves all taps, and each tap
// reads X at its shift. The halo makes each X value serve 9 taps (the one-tap-per-block kernel,
// wgrad_kernel, re-read dY and X per tap at 61 TFLOP/s).
constexpr int W9_LDS = 32 * 64 + 3 * 34 * 64;  // floats per stage: dY + the largest halo (W >= 32)
template <int TAPS>
__global__ __launch_bounds__(256) void wgrad9_kernel(WgArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[2][W9_LDS];
  const int cin = a.c0 + a.c1;
  const int nci = (cin + 63) / 64;
  const int cit = blockIdx.x % nci, cot = blockIdx.x / nci;
  const int co0 = cot * 64, ci0 = cit * 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int wr = 32 * (wave & 1), wc = 32 * (wave >> 1);
  const int Wc = a.W < 32 ? a.W : 32, R = 32 / Wc;       // chunk: R rows of Wc pixels
  const int HWc = Wc + 2, HP = (R + 2) * HWc;            // halo row length, halo pixels
  const int segs = a.W / Wc, rows_per_img = a.H / R;      // chunks per image row block / per image
  const int64_t nch = (int64_t)a.N * rows_per_img * segs;
  const int64_t c_beg = (int64_t)blockIdx.y * a.chunks_per_split;
  const int64_t c_end = c_beg + a.chunks_per_split < nch ? c_beg + a.chunks_per_split : nch;
  f32x16 acc[TAPS];
#pragma unroll
  for (int t = 0; t < TAPS; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  if (c_beg >= c_end) return;  // (never for the host's split choice)

  // staging items: dY 512 quads (2 per thread), halo HP x 16 quads (<= 7 per thread); the items'
  // positions within the chunk are fixed per thread (no divisions in the chunk loop)
  constexpr int XI = 7;
  f32x4 dyv[2], xv[XI];
  const int lwc = __builtin_ctz(Wc);
  int dyo[2], xr[XI], xc[XI];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int px = (tid + 256 * k) >> 4;
    dyo[k] = (px >> lwc) * a.W + (px & (Wc - 1));  // pixel offset from the chunk origin
  }
#pragma unroll
  for (int k = 0; k < XI; ++k) {
    const int hp = (tid + 256 * k) >> 4;
    xr[k] = hp < HP ? hp / HWc - 1 : -1000000;  // halo row / column relative to the chunk origin
    xc[k] = hp % HWc - 1;
  }
  auto chunk_origin = [&](int64_t c, int& n, int& y0, int& x0) {
    const int64_t per_img = (int64_t)rows_per_img * segs;
    n = (int)(c / per_img);
    const int rem = (int)(c - (int64_t)n * per_img);
    y0 = (rem / segs) * R;
    x0 = (rem % segs) * Wc;
  };
  auto load = [&](int64_t c) {
    int n, y0, x0;
    chunk_origin(c, n, y0, x0);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = tid + 256 * k, co = co0 + 4 * (i & 15);
      const int64_t pix = ((int64_t)n * a.H + y0) * a.W + x0 + dyo[k];
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (co + 3 < a.cout) {
        v = *reinterpret_cast<const f32x4*>(a.dy + pix * a.cout + co);
      } else {
        for (int j = 0; j < 4; ++j)
          if (co + j < a.cout) v[j] = a.dy[pix * a.cout + co + j];
      }
      dyv[k] = v;
    }
#pragma unroll
    for (int k = 0; k < XI; ++k) {
      const int i = tid + 256 * k, ci = ci0 + 4 * (i & 15);
      const int y = y0 + xr[k], x = x0 + xc[k];
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (y >= 0 && y < a.H && x >= 0 && x < a.W && ci < cin) {
        const int64_t sp = ((int64_t)n * a.H + y) * a.W + x;
        v = ci < a.c0 ? *reinterpret_cast<const f32x4*>(a.x0 + sp * a.c0 + ci)
                      : *reinterpret_cast<const f32x4*>(a.x1 + sp * a.c1 + (ci - a.c0));
      }
      xv[k] = v;
    }
  };
  auto store = [&](float* L) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = tid + 256 * k;
      *reinterpret_cast<f32x4*>(L + (i >> 4) * 64 + 4 * (i & 15)) = dyv[k];
    }
    float* X = L + 32 * 64;
#pragma unroll
    for (int k = 0; k < XI; ++k) {
      const int i = tid + 256 * k;
      if ((i >> 4) < HP) *reinterpret_cast<f32x4*>(X + (i >> 4) * 64 + 4 * (i & 15)) = xv[k];
    }
  };
  load(c_beg);
  for (int64_t c = c_beg; c < c_end; ++c) {
    float* L = lds[c & 1];
    store(L);
    __syncthreads();  // (the other buffer's readers passed this barrier after their previous chunk)
    if (c + 1 < c_end) load(c + 1);
    const float* D = L;
    const float* X = L + 32 * 64;
    // software-pipelined one k pair ahead: the next pair's LDS reads (1 dY + TAPS X values) are
    // issued before this pair's MFMAs (left to itself, hipcc waited on each read before its MFMA)
    float av[2], bv[2][TAPS];
    auto fetch = [&](int j, int slot) {
      const int m = j + 16 * h;  // this lane half's pixel of the k pair
      av[slot] = D[m * 64 + wr + l32];
      const int hp0 = (m >> lwc) * HWc + (m & (Wc - 1));  // halo pixel of tap (ky, kx) = hp0 + ky HWc + kx
#pragma unroll
      for (int t = 0; t < TAPS; ++t) {
        const int ky = TAPS == 9 ? t / 3 : 1, kx = TAPS == 9 ? t % 3 : 1;
        bv[slot][t] = X[(hp0 + ky * HWc + kx) * 64 + wc + l32];
      }
    };
    // (the next pair's reads go out after this pair's first MFMAs: LDS reads in flight stay within
    // the 15 lgkmcnt can track, beyond which the wave stalls at issue)
    constexpr int TH = TAPS > 1 ? TAPS / 2 + 1 : 1;
    fetch(0, 0);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int cur = j & 1;
#pragma unroll
      for (int t = 0; t < TH; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[cur], bv[cur][t], acc[t], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (j + 1 < 16) fetch(j + 1, cur ^ 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = TH; t < TAPS; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[cur], bv[cur][t], acc[t], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // C[i][j], i = 8 (r >> 2) + 4 h + (r & 3) (co), j = l32 (ci); slab [z][cout][cin][taps]
  float* slab = a.part + (size_t)blockIdx.y * a.cout * cin * TAPS;
  const int ci = ci0 + wc + l32;
#pragma unroll
  for (int t = 0; t < TAPS; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = co0 + wr + 8 * (r >> 2) + 4 * h + (r & 3);
      if (co < a.cout && ci < cin) slab[((size_t)co * cin + ci) * TAPS + t] = acc[t][r];
    }
}

// 3xf16 weight gradient (training precision "3xf16"), all taps of a 64 co x 64 ci tile per block:
//   dW[co][ci][tap] = sum_p dY[p][co] X[p + offset(tap)][ci]
// with both operands split on the fly (hi = f16(v), lo = f16(v - hi), conv_x3.hip's split) and three
// f16 products per MAC (dY_hi X_hi + dY_hi X_lo + dY_lo X_hi) into fp32 accumulators
// (v_mfma_f32_32x32x16_f16, K = 16 output pixels). Per chunk of 64 output pixels (2 rows of 32, or
// 64 / W whole rows) the block stages, pixel-major as they sit in HBM (16-B loads, no transpose):
//   D [part][64 px][64 co]      X [part][halo px, row-major (R + 2) x (Wc + 2) <= 136][64 ci]   f16
// (one row per pixel at a 96-f16 pitch, WX_P below) and the MFMA operands, which want 8 consecutive
// pixels of one channel per lane, come from ds_read_b64_tr_b16 (4 pixel rows x 16 channels per
// 16-lane group, delivered column-major): a tap's shift only changes which halo rows a lane
// addresses. Double-buffered; the waves' quadrants and tap groups are described at WxCfg. dY carries
// the backward's loss scale; |v| >= 65504 sets the range guard.
// (A first version staged both operands transposed through dword loads and read the shifted X rows
// unaligned: it ran no faster than the fp32 wgrad9_kernel; the loads and the unaligned reads each
// cost more than the MFMAs.)
#ifndef WX_IL
#define WX_IL 1  // staging items interleaved with the MFMA pairs (0: one slice after each k-step)
#endif
#ifndef WX_ABL
#define WX_ABL 0  // development timing ablations (outputs garbage): 2 no global loads after the first chunk,
                  // 3 no staging (split + LDS writes) after the first chunk, 4 no MFMAs, 5 no fragment
                  // reads after each chunk's first
#endif
constexpr int WX_PX = 64;                 // output pixels per chunk
constexpr int WX_HMAX = 136;              // halo pixels: 4 x 34, 6 x 18, 10 x 10
// LDS rows (one pixel's 64 channels) at a pitch of 96 f16 = 192 B = 48 banks: any 4 consecutive rows
// start 48 r mod 64 = {0, 48, 32, 16} banks apart, so a transposed read's 4 rows x 64 B cover all 64 banks
// whatever its first row - a tap's shift is then a plain row offset (an immediate or one add), not a
// per-read swizzle (the XOR-swizzled 64-f16 rows of round 2 cost ~5 VALU per fragment read)
constexpr int WX_P = 96;
constexpr int WX_OOB = 0x7ffffff0;  // a buffer offset past mkrsrc's range: the load returns zeros
constexpr int WX_D = 2 * WX_PX * WX_P;    // f16 per stage: dY, both parts
constexpr int WX_X = 2 * WX_HMAX * WX_P;  // X halo, both parts
static_assert(2 * (WX_D + WX_X) * 2 <= 160 * 1024, "two stages fit the LDS");
typedef _Float16 wx_h8 __attribute__((ext_vector_type(8)));
typedef _Float16 wx_h4 __attribute__((ext_vector_type(4)));
typedef unsigned wx_u2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) wx_u2 wx_lds_u2;

#if WX_ABL == 4
#define WX_MFMA(a, b, c, x, y, z) ([&]() { asm volatile("" ::"v"(a), "v"(b)); return (c); }())
#else
#define WX_MFMA __builtin_amdgcn_mfma_f32_32x32x16_f16
#endif
// The split of two values (conv_x3.hip's split2): hi = f16 RNE of both by one v_cvt_pk_f16_f32, lo =
// f16(v - hi) by v_fma_mix{lo,hi}_f16 reading hi's halves as f16 (v - hi is exact in fp32, rounded once);
// the empty asm keeps v an fp32 register value (no folding of its producer into the conversion)
__device__ __forceinline__ void wx_split2(float v0, float v1, unsigned& h, unsigned& l) {
  asm volatile("" : "+v"(v0), "+v"(v1));
  typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
  typedef float f2_t __attribute__((ext_vector_type(2)));
  h = __builtin_bit_cast(unsigned, __builtin_convertvector(f2_t{v0, v1}, h2_t));
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%3 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %2, 1.0, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(l)
      : "v"(v0), "v"(v1), "v"(h));
}
// element offset of channel c of row r
__device__ __forceinline__ int wx_off(int r, int c) { return r * WX_P + c; }

typedef __fp16 wx_hv4 __attribute__((__vector_size__(4 * sizeof(__fp16))));
__device__ __forceinline__ wx_h4 wx_tr(const _Float16* L, int off) {
  return __builtin_bit_cast(wx_h4, __builtin_amdgcn_ds_read_tr16_b64_v4f16((__attribute__((address_space(3))) wx_hv4*)(L + off)));
}

// Threads per block of the 1x1 kernel: 4 waves, one 32 x 32 quadrant of the 64 co x 64 ci tile each.
template <int TAPS>
struct WxCfg {
  static_assert(TAPS == 1, "wgrad_x3_kernel is the 1x1 weight gradient (3x3: wgrad_ws_kernel)");
  static constexpr int NT = 256;
  static constexpr int DI = WX_PX * 16 / NT;                   // dY 16-B items per thread
  static constexpr int XI = (WX_HMAX * 16 + NT - 1) / NT;      // X items per thread
  static constexpr int NTMAX = 1;                              // accumulators per wave
};

// colpart (optional): the bias gradient's column sums of dY, fused: the ci-tile-0 blocks add their
// split's pixels per channel (fixed order: per thread over chunks, then the pixel lanes in lane
// order) into colpart[split][cout]; colsum_final_kernel adds the splits in order.
// NPROD = 3 (fp32-class: three split products) or 1 (the reduced-precision f16 training mode: the hi x hi
// product only; no lo planes are staged or read).
// The 1x1 weight gradients (skip connections, qkv, proj_out): X = the chunk's own pixels, no halo. The 3x3
// ones run wgrad_ws_kernel (below), whose consumer waves carry no staging (a 3x3 form of this kernel, every
// wave staging beside its MFMAs, measured 1.98 vs 1.79 ms, profiles/r04b/wgrad_exp; removed in round 5).
template <int NPROD>
__global__ __launch_bounds__(WxCfg<1>::NT, 1) void wgrad_x3_kernel(WgArgs a, unsigned* guard, float* colpart) {
  constexpr int TAPS = 1;
  using Cf = WxCfg<TAPS>;
  constexpr int NT = Cf::NT, WX_DI = Cf::DI, WX_XI = Cf::XI, NTMAX = Cf::NTMAX;
  constexpr int HALO = 0;
  __shared__ __attribute__((aligned(16))) _Float16 lds[2][WX_D + WX_X];
  f32x4* const csred = reinterpret_cast<f32x4*>(&lds[0][0]);  // after the chunk loop (its last barrier)
  const int cin = a.c0 + a.c1;  // (X = concat(x0[c0], x1[c1]): a 64-channel tile never straddles them)
  const int nci = (cin + 63) / 64;
  // (channel tile, pixel split z) of this block. Workgroups go to the 8 XCDs round-robin in launch order;
  // when the split count allows, the tiles of one z (the same dY rows and X halos) are put on one XCD so
  // the second co / ci tile re-reads them from that XCD's L2 instead of HBM
  int tile = blockIdx.x, zs = blockIdx.y;
  if ((gridDim.y & 7) == 0) {
    const int L = blockIdx.x + blockIdx.y * gridDim.x, j = L >> 3;
    tile = j % gridDim.x;
    zs = (j / gridDim.x) * 8 + (L & 7);
  }
  const int cit = tile % nci, cot = tile / nci;
  const int co0 = cot * 64, ci0 = cit * 64;
  const bool src1 = a.c1 && ci0 >= a.c0;  // the tile's X source (block-uniform), its row stride, channel base
  const float* const xsrc = src1 ? a.x1 : a.x0;
  const int xst = src1 ? a.c1 : a.c0, xc0 = src1 ? ci0 - a.c0 : ci0;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5;
  const int quad = wave & 3;  // quadrant
  const int wr = 32 * (quad & 1), wc = 32 * (quad >> 1);
  const int Wc = a.W < 32 ? a.W : 32, R = WX_PX / Wc;
  const int HWc = Wc + 2 * HALO, HP = (R + 2 * HALO) * HWc;
  const int lwc = __builtin_ctz(Wc);
  const int segs = a.W / Wc, rows_per_img = a.H / R;
  const int64_t nch = (int64_t)a.N * rows_per_img * segs;
  const int64_t c_beg = (int64_t)zs * a.chunks_per_split;
  const int64_t c_end = c_beg + a.chunks_per_split < nch ? c_beg + a.chunks_per_split : nch;
  f32x16 acc[NTMAX];
#pragma unroll
  for (int t = 0; t < NTMAX; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  float gmax = 0.f;
  const bool do_cs = colpart && cit == 0;
  f32x4 csum = {0.f, 0.f, 0.f, 0.f};
  if (c_beg < c_end) {
    // staging items: (pixel i >> 4, channel quad i & 15), i = tid + NT k; quad fixed per thread
    const int cq = tid & 15;
    const bool co_ok = co0 + 4 * cq + 3 < a.cout, ci_ok = ci0 + 4 * cq + 3 < cin;
    // two register sets (chunk parity): a chunk's loads go out two chunks before its staging
    f32x4 dvs[2][WX_DI], xvs[2][WX_XI];
    int xhy[WX_XI], xhx[WX_XI], ld_x[WX_XI], ld_d[WX_DI];
#pragma unroll
    for (int k = 0; k < WX_XI; ++k) {
      const int hp = (tid + NT * k) >> 4;
      xhy[k] = hp < HP ? hp / HWc - HALO : -1000000;  // halo row / column relative to the chunk origin
      xhx[k] = hp % HWc - HALO;
      ld_x[k] = hp < HP ? ((xhy[k] * a.W + xhx[k]) * xst + xc0 + 4 * cq) * 4 : 0;  // bytes from the chunk origin
    }
#pragma unroll
    for (int k = 0; k < WX_DI; ++k) {
      const int m = (tid + NT * k) >> 4;
      ld_d[k] = (((m >> lwc) * a.W + (m & (Wc - 1))) * a.cout + co0 + 4 * cq) * 4;
    }
    // (every count here is a power of two: H, W and the chunk shape are; shifts, no 64-bit division)
    const int lpi = __builtin_ctz(rows_per_img * segs), lsg = __builtin_ctz(segs);
    auto chunk_origin = [&](int64_t c, int& n, int& y0, int& x0) {
      const int ci = (int)c;
      n = ci >> lpi;
      const int rem = ci & ((1 << lpi) - 1);
      y0 = (rem >> lsg) * R;
      x0 = (rem & (segs - 1)) * Wc;
    };
    auto load = [&](int64_t c, auto SETc) __attribute__((always_inline)) {
      f32x4(&dv)[WX_DI] = dvs[decltype(SETc)::value];
      f32x4(&xv)[WX_XI] = xvs[decltype(SETc)::value];
      if (WX_ABL == 2 && c != c_beg) return;
      int n, y0, x0;
      chunk_origin(c, n, y0, x0);
      // buffer loads from the chunk's image (SGPR descriptors, one add per load for the chunk origin);
      // a padding / out-of-tile lane reads at an offset past the descriptor's range, which returns zeros
      const rsrc_t rd = mkrsrc(a.dy + (size_t)n * a.H * a.W * a.cout);
      const rsrc_t rx = mkrsrc(xsrc + (size_t)n * a.H * a.W * xst);
      const int od = __builtin_amdgcn_readfirstlane((y0 * a.W + x0) * a.cout * 4);
      const int ox = __builtin_amdgcn_readfirstlane((y0 * a.W + x0) * xst * 4);
#pragma unroll
      for (int k = 0; k < WX_DI; ++k) dv[k] = bld4(rd, co_ok ? ld_d[k] + od : WX_OOB, 0);
#pragma unroll
      for (int k = 0; k < WX_XI; ++k) {
        const int y = y0 + xhy[k], x = x0 + xhx[k];
        const bool ok = ci_ok & ((unsigned)y < (unsigned)a.H) & ((unsigned)x < (unsigned)a.W);  // (no branches)
        xv[k] = bld4(rx, ok ? ld_x[k] + ox : WX_OOB, 0);
      }
    };
    // staging of one chunk in WX_PARTS slices (items: the WX_DI dY quads, then the WX_XI halo quads), so
    // that chunk c + 1's split and LDS writes run between chunk c's k-steps
    constexpr int WX_ITEMS = WX_DI + WX_XI, WX_PARTS = WX_PX / 16, WX_PER = (WX_ITEMS + WX_PARTS - 1) / WX_PARTS;
    auto store_item = [&](_Float16* L, int it, auto SETc) __attribute__((always_inline)) {
      const f32x4(&dv)[WX_DI] = dvs[decltype(SETc)::value];
      const f32x4(&xv)[WX_XI] = xvs[decltype(SETc)::value];
      _Float16* X = L + WX_D;
      {
        if (it >= WX_ITEMS) return;
        const bool isd = it < WX_DI;
        const int k = isd ? it : it - WX_DI;
        const f32x4 v = isd ? dv[k] : xv[k];
        const int row = (tid + NT * k) >> 4;
        if (!isd && row >= HP) return;
        if (isd && do_cs) csum += v;
        unsigned h0, l0, h1, l1;
        wx_split2(v[0], v[1], h0, l0);
        wx_split2(v[2], v[3], h1, l1);
        const wx_u2 hi = {h0, h1}, lo = {l0, l1};
        // (v_max3 with |.| modifiers: two values per instruction)
        asm("v_max3_f32 %0, %0, |%1|, |%2|\n\tv_max3_f32 %0, %0, |%3|, |%4|"
            : "+v"(gmax)
            : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));
        const int o = wx_off(row, 4 * cq);
        if (isd) {
          *(wx_lds_u2*)(L + o) = hi;
          if (NPROD == 3) *(wx_lds_u2*)(L + WX_PX * WX_P + o) = lo;
        } else {
          *(wx_lds_u2*)(X + o) = hi;
          if (NPROD == 3) *(wx_lds_u2*)(X + WX_HMAX * WX_P + o) = lo;
        }
      }
    };
    auto store_part = [&](_Float16* L, int part, auto SETc) __attribute__((always_inline)) {
#pragma unroll
      for (int q = 0; q < WX_PER; ++q) store_item(L, part * WX_PER + q, SETc);
    };
    // transposed-read lane roles: group G = lane >> 4 (G & 1: which 16 of the wave's 32 columns, G >> 1 = h:
    // which 8 of the k-step's 16 pixels); lane 4q + p of the group addresses row q, columns 4p .. 4p + 3
    const int G = lane >> 4, q = (lane & 15) >> 2, pcol = 4 * (lane & 3);
    const int cA = wr + 16 * (G & 1) + pcol, cB = wc + 16 * (G & 1) + pcol;
    // MFMAs of one staged chunk for taps T0 .. T0 + NTAP - 1 into acc[0 .. NTAP - 1] (compile-time, so the
    // accumulators stay registers; the two tap groups are two copies of this code, selected per wave)
    auto mfma_chunk = [&](auto T0c, auto NTc, const _Float16* L, _Float16* Ln, bool nxt, auto SETc) __attribute__((always_inline)) {
      constexpr int T0 = decltype(T0c)::value, NTAP = decltype(NTc)::value;
      // the lane's row / column roles laundered per chunk: the fragment addresses are then computed next
      // to their reads instead of ~80 of them being hoisted out of the chunk loop into registers (the
      // round-2 kernel held 392 VGPRs at one wave per SIMD; two waves per SIMD leave 256 each)
      int cAl = cA, cBl = cB, ql = q, hl = h;
      asm volatile("" : "+v"(cAl), "+v"(cBl), "+v"(ql), "+v"(hl));
      const _Float16* Dh = L;
      const _Float16* Xh = L + WX_D;
      // Software-pipelined: taps in pairs whose MFMAs alternate (no back-to-back accumulator
      // dependence), the next pair's B fragments read after the current pair's first MFMAs, the
      // next k-step's A fragments during the last pair (a read the MFMA waits on costs its latency).
      // Fragment addresses = a per-chunk lane base + a wave-uniform row offset + immediates (the 4-row
      // step, the lo plane). A: the k-step's pixels 16 st + 8 hl + (0..7) of the chunk. B: their halo
      // pixels, (16 st + 8 hl) -> halo pixel hb = row (m0 >> lwc) x HWc + column (m0 & (Wc - 1)); for
      // Wc >= 16 the lane half only moves the column (8 hl), for Wc = 8 it moves the row (hl HWc); the
      // tap adds (t / 3) HWc + t % 3.
      const _Float16* pA = Dh + (8 * hl + ql) * WX_P + cAl;
      const _Float16* pB = Xh + ((Wc >= 16 ? 8 * hl : hl * HWc) + ql) * WX_P + cBl;
      auto fetchA = [&](int st, wx_h8& ahi, wx_h8& alo) {
        const _Float16* b = pA + 16 * st * WX_P;
        const wx_h4 ah0 = wx_tr(b, 0), ah1 = wx_tr(b, 4 * WX_P);
        ahi = wx_h8{ah0[0], ah0[1], ah0[2], ah0[3], ah1[0], ah1[1], ah1[2], ah1[3]};
        if (NPROD == 3) {
          const wx_h4 al0 = wx_tr(b, WX_PX * WX_P), al1 = wx_tr(b, WX_PX * WX_P + 4 * WX_P);
          alo = wx_h8{al0[0], al0[1], al0[2], al0[3], al1[0], al1[1], al1[2], al1[3]};
        } else {
          alo = ahi;
        }
      };
      auto fetchB = [&](int st, int t, wx_h8& bhi, wx_h8& blo) {
        const int m0 = 16 * st;  // (wave-uniform part of the k-step's first pixel)
        const int hb = Wc >= 16 ? (m0 >> lwc) * HWc + (m0 & (Wc - 1)) : 2 * st * HWc;
        (void)t;
        const _Float16* b = pB + __builtin_amdgcn_readfirstlane(hb * WX_P);
        const wx_h4 bh0 = wx_tr(b, 0), bh1 = wx_tr(b, 4 * WX_P);
        bhi = wx_h8{bh0[0], bh0[1], bh0[2], bh0[3], bh1[0], bh1[1], bh1[2], bh1[3]};
        if (NPROD == 3) {
          const wx_h4 bl0 = wx_tr(b, WX_HMAX * WX_P), bl1 = wx_tr(b, WX_HMAX * WX_P + 4 * WX_P);
          blo = wx_h8{bl0[0], bl0[1], bl0[2], bl0[3], bl1[0], bl1[1], bl1[2], bl1[3]};
        } else {
          blo = bhi;
        }
      };
      constexpr int NST = WX_PX / 16, NPAIR = (NTAP + 1) / 2;
      wx_h8 ahi, alo, b0h, b0l, b1h, b1l;
      fetchA(0, ahi, alo);
      fetchB(0, T0, b0h, b0l);
      if (NTAP > 1) fetchB(0, T0 + 1, b1h, b1l);
#pragma unroll
      for (int st = 0; st < NST; ++st) {
#pragma unroll
        for (int pp = 0; pp < NPAIR; ++pp) {
          const int l0 = 2 * pp, l1 = 2 * pp + 1;  // local tap indices (accumulators)
          const bool two = l1 < NTAP;
          acc[l0] = WX_MFMA(ahi, b0h, acc[l0], 0, 0, 0);
          if (two) acc[l1] = WX_MFMA(ahi, b1h, acc[l1], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          // next pair (or the next k-step's first pair, and its A fragments)
          wx_h8 n0h, n0l, n1h, n1l, nah, nal;
          const bool last = pp + 1 == NPAIR;
          const int nst = last ? st + 1 : st, nl0 = last ? 0 : l0 + 2;
          const bool more = nst < NST;
          if (more && WX_ABL != 5) {
            fetchB(nst, T0 + nl0, n0h, n0l);
            if (nl0 + 1 < NTAP) fetchB(nst, T0 + nl0 + 1, n1h, n1l);
            if (last) fetchA(nst, nah, nal);
          } else if (more) {
            n0h = b0h; n0l = b0l; n1h = b1h; n1l = b1l; nah = ahi; nal = alo;
          }
          __builtin_amdgcn_sched_barrier(0);
          // chunk c + 1's staging, one item per pair, beside this pair's second MFMA group
          // (the last pair takes the part's remaining items: the 1x1 kernel has one pair per k-step)
          if (WX_IL && nxt && WX_ABL != 3)  // (block-uniform)
#pragma unroll
            for (int q = pp; q < (pp + 1 == NPAIR ? WX_PER : pp + 1); ++q) store_item(Ln, st * WX_PER + q, SETc);
          if (NPROD == 3) {
            acc[l0] = WX_MFMA(ahi, b0l, acc[l0], 0, 0, 0);
            if (two) acc[l1] = WX_MFMA(ahi, b1l, acc[l1], 0, 0, 0);
            acc[l0] = WX_MFMA(alo, b0h, acc[l0], 0, 0, 0);
            if (two) acc[l1] = WX_MFMA(alo, b1h, acc[l1], 0, 0, 0);
          }
          __builtin_amdgcn_sched_barrier(0);
          if (more) {
            b0h = n0h; b0l = n0l;
            if (nl0 + 1 < NTAP) { b1h = n1h; b1l = n1l; }
            if (last) { ahi = nah; alo = nal; }
          }
        }
        if (!WX_IL && nxt && WX_ABL != 3) store_part(Ln, st, SETc);  // (block-uniform)
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    // prologue: chunk c_beg staged, chunks c_beg + 1 (register set 1) and c_beg + 2 (set 0) in flight.
    // Iteration c (k = c - c_beg): MFMAs of chunk c from lds[c & 1] with chunk c + 1's staging slices
    // (set (k + 1) & 1) between its k-steps into lds[(c + 1) & 1] (read by chunk c - 1, whose MFMAs every
    // wave finished before the previous barrier), then chunk c + 3's loads into the set just staged
    // (round 3: one set, loads one chunk ahead, waited on after the chunk's first k-step: 2.36 ms for the
    // 256^2 128 -> 128 layer at B = 32 vs 1.77 ms with the loads ablated)
    const std::integral_constant<int, 0> set0;
    const std::integral_constant<int, 1> set1;
    load(c_beg, set0);
#pragma unroll
    for (int part = 0; part < WX_PARTS; ++part) store_part(lds[c_beg & 1], part, set0);
    __syncthreads();
    // (loads past the block's range re-read its last chunk: every iteration issues the same loads, so
    // the compiler's vmcnt arithmetic waits for one set only - a conditional load made it wait for both)
    auto clampc = [&](int64_t c) { return c < c_end ? c : c_end - 1; };
    load(clampc(c_beg + 1), set1);
    load(clampc(c_beg + 2), set0);
    auto iter = [&](int64_t c, auto SETc) __attribute__((always_inline)) {
      _Float16* L = lds[c & 1];
      _Float16* Ln = lds[(c + 1) & 1];
      const bool nxt = c + 1 < c_end;
      if (c < c_end)  // (block-uniform; the dummy half of an odd count only loads)
        mfma_chunk(std::integral_constant<int, 0>(), std::integral_constant<int, 1>(), L, Ln, nxt, SETc);
      load(clampc(c + 3), SETc);
      __syncthreads();
    };
    // both halves unconditionally: every backedge leaves set 1's loads older than set 0's, so the staging
    // waits for its own set only (wgrad_ws_kernel)
    for (int64_t c = c_beg; c < c_end; c += 2) {
      iter(c, set1);
      iter(c + 1, set0);
    }
  }
  if (gmax >= 65504.0f) atomicOr(guard, 1u);
  if (do_cs) {  // (block-uniform)
    csred[tid] = csum;
    __syncthreads();
    if (tid < 16) {
      f32x4 t = csred[tid];
      for (int r = 1; r < NT / 16; ++r) t += csred[tid + 16 * r];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = co0 + 4 * tid + j;
        if (co < a.cout) colpart[(size_t)zs * a.cout + co] = t[j];
      }
    }
  }
  // C[i][j], i = 8 (r >> 2) + 4 h + (r & 3) (co), j = l32 (ci); slab [z][cout][cin]
  float* slab = a.part + (size_t)zs * a.cout * cin;
  const int ci = ci0 + wc + (lane & 31);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int co = co0 + wr + 8 * (r >> 2) + 4 * h + (r & 3);
    if (co < a.cout && ci < cin) slab[(size_t)co * cin + ci] = acc[0][r];
  }
}

// Wide-tile 1x1 weight gradient (the skip connections, qkv and proj_out: cout and cin multiples of 128):
// dW[co][ci] = sum_p dY[p][co] X[p][ci] for a 128 co x 128 ci tile per block, so a layer's X is read cout / 128
// times and dY cin / 128 times (wgrad_x3_kernel's 64 x 64 tiles read them cout / 64 and cin / 64 times, and staged
// 0.67 KB per MFMA: 1.8 ms for the 256^2 256 -> 128 layer at B = 32, 1.8 TB/s of algorithmic bytes). Same arithmetic per product as wgrad_x3_kernel (split hi / lo, NPROD f16 products into one
// fp32 accumulator per output, k-steps of 16 pixels in pixel order, splits summed by slab_bias_reduce_kernel).
// 4 waves, one 64 co x 64 ci quadrant each (2 x 2 MFMA tiles, one 64-channel LDS plane of each operand);
// chunks of WW_PX consecutive pixels (NHWC rows, never across images: HW % WW_PX == 0), staged pixel-major at
// wgrad_x3_kernel's 96-f16 pitch and read through ds_read_b64_tr_b16. Chunk c + 1 is staged between chunk
// c's k-steps, loads go out two chunks ahead (two register sets, as wgrad_x3_kernel).
constexpr int WW_PX = 16;                    // pixels per chunk (one k-step)
constexpr int WW_K = WW_PX / 8;              // staging rows per thread and operand
constexpr int WW_PL = WW_PX * WX_P;          // one 64-channel plane of one part: WW_PX rows at the 96-f16 pitch
constexpr int WW_OP = 2 * 2 * WW_PL;         // one operand: [part hi / lo][plane 0 / 1]
constexpr int WW_ST = 2 * WW_OP;             // one stage: dY then X
constexpr int WW_NT = 256;
static_assert(2 * WW_ST * 2 <= 160 * 1024, "two stages fit the LDS");
// eligible shapes (the host also needs 128-channel tiles inside one concat source)
__host__ __device__ constexpr bool ww_shape(int cout, int cin) { return cout % 128 == 0 && cin % 128 == 0; }

template <int NPROD>
__global__ __launch_bounds__(WW_NT, 3) void wgrad1x1_wide_kernel(WgArgs a, unsigned* guard, float* colpart) {
  __shared__ __attribute__((aligned(16))) _Float16 lds[2][WW_ST];
  f32x4* const csred = reinterpret_cast<f32x4*>(&lds[0][0]);  // after the chunk loop (its last barrier)
  const int cin = a.c0 + a.c1;
  // (channel tile, pixel split): workgroups go to the 8 XCDs round-robin in launch order, so with a split count
  // divisible by 8 the channel tiles of one split (the same dY chunks) are put 8 launch slots apart, on one XCD,
  // where the second reads dY from that XCD's L2 (wgrad_x3_kernel's map)
  int tile = blockIdx.x, zs = blockIdx.y;
  if ((gridDim.y & 7) == 0) {
    const int L = blockIdx.x + blockIdx.y * gridDim.x, j = L >> 3;
    tile = j % gridDim.x;
    zs = (j / gridDim.x) * 8 + (L & 7);
  }
  const int nci = cin / 128, cit = tile % nci;
  const int ci0 = cit * 128, co0 = (tile / nci) * 128;
  const bool src1 = a.c1 && ci0 >= a.c0;  // the tile's X source (block-uniform; host: 128-channel tiles in one)
  const float* const xsrc = src1 ? a.x1 : a.x0;
  const int xst = src1 ? a.c1 : a.c0, xc0 = src1 ? ci0 - a.c0 : ci0;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5;
  const int HW = a.H * a.W;
  const int64_t nch = a.P / WW_PX;
  const int64_t c_beg = (int64_t)zs * a.chunks_per_split;
  const int64_t c_end = c_beg + a.chunks_per_split < nch ? c_beg + a.chunks_per_split : nch;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  float gmax = 0.f;
  const bool do_cs = colpart && cit == 0;
  f32x4 csum = {0.f, 0.f, 0.f, 0.f};
  // staging items: channel quad cq = tid & 31 (the same for every item of the thread: one co quad of dY, one ci
  // quad of X), pixel rows pr + 8 k, k < WW_K, of each operand
  const int cq = tid & 31, pr = tid >> 5;
  const int pl = cq >> 4, col = 4 * (cq & 15);  // LDS plane (64 channels) and column of the quad
  if (c_beg < c_end) {
    f32x4 dvs[2][WW_K], xvs[2][WW_K];
    auto load = [&](int64_t c, auto SETc) __attribute__((always_inline)) {
      f32x4(&dv)[WW_K] = dvs[decltype(SETc)::value];
      f32x4(&xv)[WW_K] = xvs[decltype(SETc)::value];
      const int64_t p0 = c * WW_PX;
      const int n = (int)(p0 / HW), q0 = (int)(p0 - (int64_t)n * HW);  // image, its first pixel (chunks stay in it)
      const rsrc_t rd = mkrsrc(a.dy + (size_t)n * HW * a.cout);
      const rsrc_t rx = mkrsrc(xsrc + (size_t)n * HW * xst);
      const int od = __builtin_amdgcn_readfirstlane(q0 * a.cout * 4), ox = __builtin_amdgcn_readfirstlane(q0 * xst * 4);
#pragma unroll
      for (int k = 0; k < WW_K; ++k) {
        dv[k] = bld4(rd, ((pr + 8 * k) * a.cout + co0 + 4 * cq) * 4 + od, 0);
        xv[k] = bld4(rx, ((pr + 8 * k) * xst + xc0 + 4 * cq) * 4 + ox, 0);
      }
    };
    auto store_item = [&](_Float16* L, int it, auto SETc) __attribute__((always_inline)) {
      const f32x4(&dv)[WW_K] = dvs[decltype(SETc)::value];
      const f32x4(&xv)[WW_K] = xvs[decltype(SETc)::value];
      const bool isd = it < WW_K;
      const int k = isd ? it : it - WW_K;
      const f32x4 v = isd ? dv[k] : xv[k];
      if (isd && do_cs) csum += v;
      unsigned h0, l0, h1, l1;
      wx_split2(v[0], v[1], h0, l0);
      wx_split2(v[2], v[3], h1, l1);
      asm("v_max3_f32 %0, %0, |%1|, |%2|\n\tv_max3_f32 %0, %0, |%3|, |%4|"
          : "+v"(gmax)
          : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));
      _Float16* O = L + (isd ? 0 : WW_OP) + pl * WW_PL + wx_off(pr + 8 * k, col);
      *(wx_lds_u2*)O = wx_u2{h0, h1};
      if (NPROD == 3) *(wx_lds_u2*)(O + 2 * WW_PL) = wx_u2{l0, l1};
    };
    // fragment roles (wgrad_x3_kernel's transposed reads): group G = lane >> 4, lane 4q + p of the group
    // addresses row q, columns 4p .. 4p + 3; the wave's quadrant is plane (wave & 1) of dY, (wave >> 1) of X
    const int G = lane >> 4, q = (lane & 15) >> 2, pcol = 4 * (lane & 3);
    const int cf = 16 * (G & 1) + pcol;
    auto mfma_chunk = [&](const _Float16* L, _Float16* Ln, bool nxt, auto SETc) __attribute__((always_inline)) {
      int cfl = cf, ql = q, hl = h;
      asm volatile("" : "+v"(cfl), "+v"(ql), "+v"(hl));
      const _Float16* pA = L + (wave & 1) * WW_PL + (8 * hl + ql) * WX_P + cfl;
      const _Float16* pB = L + WW_OP + (wave >> 1) * WW_PL + (8 * hl + ql) * WX_P + cfl;
      auto frag = [&](const _Float16* p0, int st, int t, wx_h8& hi, wx_h8& lo) {
        const _Float16* b = p0 + 16 * st * WX_P + 32 * t;
        const wx_h4 h0v = wx_tr(b, 0), h1v = wx_tr(b, 4 * WX_P);
        hi = wx_h8{h0v[0], h0v[1], h0v[2], h0v[3], h1v[0], h1v[1], h1v[2], h1v[3]};
        if (NPROD == 3) {
          const wx_h4 l0v = wx_tr(b, 2 * WW_PL), l1v = wx_tr(b, 2 * WW_PL + 4 * WX_P);
          lo = wx_h8{l0v[0], l0v[1], l0v[2], l0v[3], l1v[0], l1v[1], l1v[2], l1v[3]};
        } else {
          lo = hi;
        }
      };
#pragma unroll
      for (int st = 0; st < WW_PX / 16; ++st) {
        wx_h8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          frag(pA, st, t, ah[t], al[t]);
          frag(pB, st, t, bh[t], bl[t]);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = WX_MFMA(ah[i], bh[j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (nxt)  // (block-uniform) chunk c + 1's staging, half of it per k-step
#pragma unroll
          for (int it = 4 * st; it < 4 * st + 4; ++it) store_item(Ln, it, SETc);  // (2 WW_K items over WW_PX / 16 k-steps)
        __builtin_amdgcn_sched_barrier(0);
        if (NPROD == 3) {
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = WX_MFMA(ah[i], bl[j], acc[i][j], 0, 0, 0);
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = WX_MFMA(al[i], bh[j], acc[i][j], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    const std::integral_constant<int, 0> set0;
    const std::integral_constant<int, 1> set1;
    load(c_beg, set0);
#pragma unroll
    for (int it = 0; it < 2 * WW_K; ++it) store_item(lds[c_beg & 1], it, set0);
    __syncthreads();
    // (loads past the block's range re-read its last chunk: every iteration issues the same loads)
    auto clampc = [&](int64_t c) { return c < c_end ? c : c_end - 1; };
    load(clampc(c_beg + 1), set1);
    load(clampc(c_beg + 2), set0);
    auto iter = [&](int64_t c, auto SETc) __attribute__((always_inline)) {
      const bool nxt = c + 1 < c_end;
      if (c < c_end) mfma_chunk(lds[c & 1], lds[(c + 1) & 1], nxt, SETc);
      load(clampc(c + 3), SETc);
      __syncthreads();
    };
    for (int64_t c = c_beg; c < c_end; c += 2) {
      iter(c, set1);
      iter(c + 1, set0);
    }
  }
  if (gmax >= 65504.0f) atomicOr(guard, 1u);
  if (do_cs) {  // (block-uniform) the bias gradient's column sums: the 8 pixel rows of each co quad, in order
    csred[tid] = csum;
    __syncthreads();
    if (tid < 32) {
      f32x4 t = csred[tid];
      for (int r = 1; r < WW_NT / 32; ++r) t += csred[tid + 32 * r];
#pragma unroll
      for (int j = 0; j < 4; ++j) colpart[(size_t)zs * a.cout + co0 + 4 * tid + j] = t[j];
    }
  }
  // C[i][j] of MFMA tile (ti, tj): co = 64 (wave & 1) + 32 ti + 8 (r >> 2) + 4 h + (r & 3), ci = ci0 + 64 (wave >> 1)
  // + 32 tj + l32; slab [z][cout][cin]
  float* slab = a.part + (size_t)zs * a.cout * cin;
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < 2; ++tj) {
      const int ci = ci0 + 64 * (wave >> 1) + 32 * tj + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = co0 + 64 * (wave & 1) + 32 * ti + 8 * (r >> 2) + 4 * h + (r & 3);
        slab[(size_t)co * cin + ci] = acc[ti][tj][r];
      }
    }
}

// Warp-specialised 3x3 weight gradient (3xf16 / f16): wgrad_x3_kernel<9, ..>'s arithmetic, LDS image and
// fragment reads, with the roles split. 8 waves, two per SIMD: waves 0-3 are consumers (quadrant w:
// 32 co x 32 ci of all 9 taps, 144 accumulator registers), waves 4-7 producers (global loads, the
// GroupNorm prologue, the split and the LDS writes). In wgrad_x3_kernel every wave carried a share of the
// staging inside its own MFMA stream, and the two serialised: at the 256^2 128 -> 128 layer (B = 32) the
// kernel ran 1.95 ms while its staging alone (MFMAs ablated) took 1.19 ms and its MFMAs alone ~0.84 ms
// (profiles/r03k/wgrad_abl*.txt). Here a consumer's instruction stream holds only fragment reads and
// MFMAs; the producer wave on the same SIMD issues in the MFMAs' shadow.
// One s_barrier per chunk (both roles): the consumers' fragment reads of stage c & 1 and the producers'
// writes of stage (c + 1) & 1 are complete (lgkmcnt(0)) before it; the producers' global loads stay in
// flight across it (chunk c + 3's, two chunks ahead of their staging).
constexpr int WS_NTP = 256;                                  // producer threads
#ifndef WS_PD
#define WS_PD 3  // consumer fragment-read distance, in (k-step, tap) steps of 3 MFMAs
#endif
#ifndef WS_REP
#define WS_REP 1  // development: consumers run each staged chunk's MFMAs WS_REP times (timing only)
#endif
#ifndef WS_PRIO
#define WS_PRIO 0  // consumer wave priority (s_setprio)
#endif
#ifndef WS_ABL
#define WS_ABL 0  // development timing ablations (garbage results): 1 producers idle after the first chunk,
                  // 2 consumers without MFMAs, 3 no range-guard max, 4 the split without the lo part, 5 no LDS
                  // writes, 6 no split / max (raw bits written), 7 no global loads after the first chunk
#endif
#ifndef WS_WC
// widest chunk row of the 64-pixel chunks: 8 x 8 pixels (X halo 10 x 10 = 100 pixels to stage and activate) since
// round 6; 2 x 32 (halo 4 x 34 = 136) before: 240.4 vs 236.9 training images/s, 4 x 16 239.1 (profiles/r06c)
#define WS_WC 8
#endif
#define WS_BARRIER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")
#if WS_ABL == 2
#define WS_MFMA(a, b, c, x, y, z) ([&]() { asm volatile("" ::"v"(a), "v"(b)); return (c); }())
#else
#define WS_MFMA __builtin_amdgcn_mfma_f32_32x32x16_f16
#endif
template <int NPROD, bool GNA>
__global__ __launch_bounds__(512, 1) void wgrad_ws_kernel(WgArgs a, unsigned* guard, float* colpart) {
  constexpr int DI = WX_PX * 16 / WS_NTP;                    // dY 16-B items per producer thread (4)
  // X halo items per producer thread: the largest halo of a chunk shape the kernel can take (a map narrower than
  // WS_WC takes its own width): 8 x 8 chunks 100 pixels (7 items), 4 x 16 108 (7), 2 x 32 136 (9)
  constexpr int HPMAX = WS_WC >= 32 ? 136 : (WS_WC >= 16 ? 108 : 100);
  static_assert(HPMAX <= WX_HMAX, "halo fits the stage");
  constexpr int XI = (HPMAX * 16 + WS_NTP - 1) / WS_NTP;
  constexpr int NTAP = 9;
  __shared__ __attribute__((aligned(16))) _Float16 lds[2][WX_D + WX_X];
  f32x4* const csred = reinterpret_cast<f32x4*>(&lds[0][0]);  // after the chunk loop
  const int cin = a.c0 + a.c1;  // (X = concat(x0[c0], x1[c1]): a 64-channel tile never straddles them)
  const int nci = (cin + 63) / 64;
  int tile = blockIdx.x, zs = blockIdx.y;
  if ((gridDim.y & 7) == 0) {  // the tiles of one z on one XCD (wgrad_x3_kernel)
    const int L = blockIdx.x + blockIdx.y * gridDim.x, j = L >> 3;
    tile = j % gridDim.x;
    zs = (j / gridDim.x) * 8 + (L & 7);
  }
  const int cit = tile % nci, cot = tile / nci;
  const int co0 = cot * 64, ci0 = cit * 64;
  const bool src1 = a.c1 && ci0 >= a.c0;  // the tile's X source (block-uniform), its row stride, channel base
  const float* const xsrc = src1 ? a.x1 : a.x0;
  const int xst = src1 ? a.c1 : a.c0, xc0 = src1 ? ci0 - a.c0 : ci0;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool producer = wave >= 4;
  const int Wc = a.W < WS_WC ? a.W : WS_WC, R = WX_PX / Wc;
  const int HWc = Wc + 2, HP = (R + 2) * HWc;
  const int lwc = __builtin_ctz(Wc);
  const int segs = a.W / Wc, rows_per_img = a.H / R;
  const int64_t nch = (int64_t)a.N * rows_per_img * segs;
  const int64_t c_beg = (int64_t)zs * a.chunks_per_split;
  const int64_t c_end = c_beg + a.chunks_per_split < nch ? c_beg + a.chunks_per_split : nch;
  const int lpi = __builtin_ctz(rows_per_img * segs), lsg = __builtin_ctz(segs);
  auto chunk_origin = [&](int64_t c, int& n, int& y0, int& x0) {
    const int ci = (int)c;
    n = ci >> lpi;
    const int rem = ci & ((1 << lpi) - 1);
    y0 = (rem >> lsg) * R;
    x0 = (rem & (segs - 1)) * Wc;
  };
  auto clampc = [&](int64_t c) { return c < c_end ? c : c_end - 1; };
  const bool do_cs = colpart && cit == 0;

  if (producer) {
    const int ptid = tid - 256;
    float gmax = 0.f;
    f32x4 csum = {0.f, 0.f, 0.f, 0.f};
    if (c_beg < c_end) {
      const int cq = ptid & 15;
      const bool co_ok = co0 + 4 * cq + 3 < a.cout, ci_ok = ci0 + 4 * cq + 3 < cin;
      f32x4 dvs[3][DI], xvs[3][XI];
      f32x4 gas[GNA ? 3 : 1], gbs[GNA ? 3 : 1];
      unsigned okm[GNA ? 3 : 1];
      int xhy[XI], xhx[XI], ld_x[XI], ld_d[DI];
#pragma unroll
      for (int k = 0; k < XI; ++k) {
        const int hp = (ptid + WS_NTP * k) >> 4;
        xhy[k] = hp < HP ? hp / HWc - 1 : -1000000;
        xhx[k] = hp % HWc - 1;
        ld_x[k] = hp < HP ? ((xhy[k] * a.W + xhx[k]) * xst + xc0 + 4 * cq) * 4 : 0;
      }
#pragma unroll
      for (int k = 0; k < DI; ++k) {
        const int m = (ptid + WS_NTP * k) >> 4;
        ld_d[k] = (((m >> lwc) * a.W + (m & (Wc - 1))) * a.cout + co0 + 4 * cq) * 4;
      }
      auto load = [&](int64_t c, auto SETc) __attribute__((always_inline)) {
        constexpr int S = decltype(SETc)::value;
        if (WS_ABL == 7 && c != c_beg) return;
        int n, y0, x0;
        chunk_origin(c, n, y0, x0);
        const rsrc_t rd = mkrsrc(a.dy + (size_t)n * a.H * a.W * a.cout);
        const rsrc_t rx = mkrsrc(xsrc + (size_t)n * a.H * a.W * xst);
        const int od = __builtin_amdgcn_readfirstlane((y0 * a.W + x0) * a.cout * 4);
        const int ox = __builtin_amdgcn_readfirstlane((y0 * a.W + x0) * xst * 4);
#pragma unroll
        for (int k = 0; k < DI; ++k) dvs[S][k] = bld4(rd, co_ok ? ld_d[k] + od : WX_OOB, 0);
        unsigned m = 0;
#pragma unroll
        for (int k = 0; k < XI; ++k) {
          const int y = y0 + xhy[k], x = x0 + xhx[k];
          const bool ok = ci_ok & ((unsigned)y < (unsigned)a.H) & ((unsigned)x < (unsigned)a.W);
          xvs[S][k] = bld4(rx, ok ? ld_x[k] + ox : WX_OOB, 0);
          m |= ok ? 1u << k : 0u;
        }
        if constexpr (GNA) {
          okm[S] = m;
          const int oc = ci_ok ? (ci0 + 4 * cq) * 4 : WX_OOB;
          gas[S] = bld4(mkrsrc(a.actA + (size_t)n * cin), oc, 0);
          gbs[S] = bld4(mkrsrc(a.actB + (size_t)n * cin), oc, 0);
        }
      };
      auto stage = [&](_Float16* L, auto SETc) __attribute__((always_inline)) {
        constexpr int S = decltype(SETc)::value;
        _Float16* X = L + WX_D;
#pragma unroll
        for (int it = 0; it < DI + XI; ++it) {
          const bool isd = it < DI;
          const int k = isd ? it : it - DI;
          f32x4 v = isd ? dvs[S][k] : xvs[S][k];
          const int row = (ptid + WS_NTP * k) >> 4;
          if (!isd && row >= HP) continue;
          if constexpr (GNA) {
            if (!isd) {  // conv_x3.hip's prologue: padding rides in the exponent (2^+inf -> rcp -> 0)
              const float pinf = (okm[S] >> k) & 1u ? 0.f : __builtin_inff();
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                const float t = fmaf(gas[S][j], v[j], gbs[S][j]);
                v[j] = t * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(fmaf(t, -1.4426950408889634f, pinf)));
              }
            }
          }
          if (isd && do_cs) csum += v;
          if (WS_ABL != 3 && WS_ABL != 6)
            asm("v_max3_f32 %0, %0, |%1|, |%2|\n\tv_max3_f32 %0, %0, |%3|, |%4|"
                : "+v"(gmax)
                : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));
          const int o = wx_off(row, 4 * cq);
          _Float16* base = isd ? L : X;
          const int lo_off = isd ? WX_PX * WX_P : WX_HMAX * WX_P;
          if (WS_ABL == 5) {
            asm volatile("" ::"v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(o));
          } else if (WS_ABL == 6) {
            const wx_u2 r0 = {__builtin_bit_cast(unsigned, v[0]), __builtin_bit_cast(unsigned, v[1])};
            *(wx_lds_u2*)(base + o) = r0;
            *(wx_lds_u2*)(base + lo_off + o) = r0;
          } else if (NPROD == 3 && WS_ABL == 4) {
            typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
            typedef float f2_t __attribute__((ext_vector_type(2)));
            const unsigned h0 = __builtin_bit_cast(unsigned, __builtin_convertvector(f2_t{v[0], v[1]}, h2_t));
            const unsigned h1 = __builtin_bit_cast(unsigned, __builtin_convertvector(f2_t{v[2], v[3]}, h2_t));
            *(wx_lds_u2*)(base + o) = wx_u2{h0, h1};
            *(wx_lds_u2*)(base + lo_off + o) = wx_u2{h0, h1};
          } else if (NPROD == 3) {
            unsigned h0, l0, h1, l1;
            wx_split2(v[0], v[1], h0, l0);
            wx_split2(v[2], v[3], h1, l1);
            *(wx_lds_u2*)(base + o) = wx_u2{h0, h1};
            *(wx_lds_u2*)(base + lo_off + o) = wx_u2{l0, l1};
          } else {
            typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
            typedef float f2_t __attribute__((ext_vector_type(2)));
            float v0 = v[0], v1 = v[1], v2 = v[2], v3 = v[3];
            asm volatile("" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));
            const unsigned h0 = __builtin_bit_cast(unsigned, __builtin_convertvector(f2_t{v0, v1}, h2_t));
            const unsigned h1 = __builtin_bit_cast(unsigned, __builtin_convertvector(f2_t{v2, v3}, h2_t));
            *(wx_lds_u2*)(base + o) = wx_u2{h0, h1};
          }
        }
      };
      // three register sets: chunk j's loads go to set j % 3, issued at the START of iteration j - 3 (into
      // the set chunk j - 3 was staged from), so they have three chunk-times to arrive before chunk j's
      // staging in iteration j - 1 (with two sets issued after each staging, the producers waited on
      // them: 1.48 ms at 256^2 without global loads vs 1.88 ms with, profiles/r04b/wgrad_*.txt)
      const std::integral_constant<int, 0> set0;
      const std::integral_constant<int, 1> set1;
      const std::integral_constant<int, 2> set2;
      load(c_beg, set0);
      stage(lds[c_beg & 1], set0);
      load(clampc(c_beg + 1), set1);
      load(clampc(c_beg + 2), set2);
      WS_BARRIER();
      auto iter = [&](int64_t c, auto LSETc, auto SSETc) __attribute__((always_inline)) {
        if (WS_ABL != 1) {
          load(clampc(c + 3), LSETc);
          if (c + 1 < c_end) stage(lds[(c + 1) & 1], SSETc);  // (block-uniform)
        }
        WS_BARRIER();
      };
      // all three thirds unconditionally (a count that is not a multiple of 3 ends with dummy iterations
      // whose barriers the consumers match): every backedge leaves the sets' loads in the same age order,
      // so each staging waits for its own set only
      for (int64_t c = c_beg; c < c_end; c += 3) {
        iter(c, set0, set1);
        iter(c + 1, set1, set2);
        iter(c + 2, set2, set0);
      }
    }
    if (gmax >= 65504.0f) atomicOr(guard, 1u);
    // two block-wide barriers, matched by the consumers': the stages are free, then the partial sums are in
    if (do_cs) {  // (block-uniform)
      WS_BARRIER();
      csred[ptid] = csum;
      WS_BARRIER();
      if (ptid < 16) {
        f32x4 t = csred[ptid];
        for (int r = 1; r < WS_NTP / 16; ++r) t += csred[ptid + 16 * r];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int co = co0 + 4 * ptid + j;
          if (co < a.cout) colpart[(size_t)zs * a.cout + co] = t[j];
        }
      }
    }
    return;
  }
  // consumers
  f32x16 acc[NTAP];
#pragma unroll
  for (int t = 0; t < NTAP; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  const int h = lane >> 5, quad = wave;
  const int wr = 32 * (quad & 1), wc = 32 * (quad >> 1);
  if (WS_PRIO) __builtin_amdgcn_s_setprio(WS_PRIO);
  if (c_beg < c_end) {
    const int G = lane >> 4, q = (lane & 15) >> 2, pcol = 4 * (lane & 3);
    const int cA = wr + 16 * (G & 1) + pcol, cB = wc + 16 * (G & 1) + pcol;
    WS_BARRIER();  // the first stage
    for (int64_t c = c_beg; c < c_end; ++c) {
      const _Float16* L = lds[c & 1];
      int cAl = cA, cBl = cB, ql = q, hl = h;
      asm volatile("" : "+v"(cAl), "+v"(cBl), "+v"(ql), "+v"(hl));
      const _Float16* pA = L + (8 * hl + ql) * WX_P + cAl;
      const _Float16* pB = L + WX_D + ((Wc >= 16 ? 8 * hl : hl * HWc) + ql) * WX_P + cBl;
      auto fetchA = [&](int st, wx_h8& ahi, wx_h8& alo) {
        const _Float16* b = pA + 16 * st * WX_P;
        const wx_h4 ah0 = wx_tr(b, 0), ah1 = wx_tr(b, 4 * WX_P);
        ahi = wx_h8{ah0[0], ah0[1], ah0[2], ah0[3], ah1[0], ah1[1], ah1[2], ah1[3]};
        if (NPROD == 3) {
          const wx_h4 al0 = wx_tr(b, WX_PX * WX_P), al1 = wx_tr(b, WX_PX * WX_P + 4 * WX_P);
          alo = wx_h8{al0[0], al0[1], al0[2], al0[3], al1[0], al1[1], al1[2], al1[3]};
        } else {
          alo = ahi;
        }
      };
      auto fetchB = [&](int st, int t, wx_h8& bhi, wx_h8& blo) {
        const int m0 = 16 * st;
        const int hb = Wc >= 16 ? (m0 >> lwc) * HWc + (m0 & (Wc - 1)) : 2 * st * HWc;
        const int r0 = hb + (t / 3) * HWc + (t % 3);
        const _Float16* b = pB + __builtin_amdgcn_readfirstlane(r0 * WX_P);
        const wx_h4 bh0 = wx_tr(b, 0), bh1 = wx_tr(b, 4 * WX_P);
        bhi = wx_h8{bh0[0], bh0[1], bh0[2], bh0[3], bh1[0], bh1[1], bh1[2], bh1[3]};
        if (NPROD == 3) {
          const wx_h4 bl0 = wx_tr(b, WX_HMAX * WX_P), bl1 = wx_tr(b, WX_HMAX * WX_P + 4 * WX_P);
          blo = wx_h8{bl0[0], bl0[1], bl0[2], bl0[3], bl1[0], bl1[1], bl1[2], bl1[3]};
        } else {
          blo = bhi;
        }
      };
      // The chunk's 36 (k-step, tap) steps in one unrolled sequence, 3 MFMAs each into acc[tap]; the B
      // fragments WS_PD steps ahead (one consumer wave per SIMD: nothing else covers a read's latency),
      // the next k-step's A fragments with the first read of that k-step
      constexpr int NST = WX_PX / 16, NS = NST * NTAP, PD = WS_PD;
      wx_h8 bh[PD + 1], bl[PD + 1], ah[2], al[2];
      for (int rep = 0; rep < WS_REP; ++rep) {
      fetchA(0, ah[0], al[0]);
#pragma unroll
      for (int i = 0; i < PD; ++i) fetchB(i / NTAP, i % NTAP, bh[i], bl[i]);
#pragma unroll
      for (int i = 0; i < NS; ++i) {
        const int st = i / NTAP, t = i % NTAP, sl = i % (PD + 1);
        const int j = i + PD;  // the step whose fragments are read now
        if (j < NS) {
          if (j % NTAP == 0) fetchA(j / NTAP, ah[(j / NTAP) & 1], al[(j / NTAP) & 1]);
          fetchB(j / NTAP, j % NTAP, bh[j % (PD + 1)], bl[j % (PD + 1)]);
        }
        __builtin_amdgcn_sched_barrier(0);
        acc[t] = WS_MFMA(ah[st & 1], bh[sl], acc[t], 0, 0, 0);
        if (NPROD == 3) {
          acc[t] = WS_MFMA(ah[st & 1], bl[sl], acc[t], 0, 0, 0);
          acc[t] = WS_MFMA(al[st & 1], bh[sl], acc[t], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      }
      WS_BARRIER();
    }
    for (int64_t d = (c_end - c_beg) % 3; d && d < 3; ++d) WS_BARRIER();  // (the producers' dummy iterations)
  }
  if (do_cs) {  // (the producers' two column-sum barriers)
    WS_BARRIER();
    WS_BARRIER();
  }
  float* slab = a.part + (size_t)zs * a.cout * cin * NTAP;
  const int ci = ci0 + wc + (lane & 31);
#pragma unroll
  for (int t = 0; t < NTAP; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = co0 + wr + 8 * (r >> 2) + 4 * h + (r & 3);
      if (co < a.cout && ci < cin) slab[((size_t)co * cin + ci) * NTAP + t] = acc[t][r];
    }
}

// sum of the S slabs of element i in slab order; the loads go out 8 at a time ahead of their adds (a sequential
// load-add loop kept one load in flight per thread: the wide weight gradients' 256-384 slabs took ~30 us)
template <typename T>
__device__ __forceinline__ T slab_sum(const float* __restrict__ part, int S, int64_t n, int64_t i) {
  T s = (T)part[i];
  int z = 1;
  for (; z + 8 <= S; z += 8) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = part[(size_t)(z + k) * n + i];
#pragma unroll
    for (int k = 0; k < 8; ++k) s += (T)v[k];
  }
  for (; z < S; ++z) s += (T)part[(size_t)z * n + i];
  return s;
}

__global__ void slab_reduce_kernel(const float* __restrict__ part, int S, int64_t n, float* __restrict__ out,
                                   int accumulate) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float s = slab_sum<float>(part, S, n, i);
  out[i] = accumulate ? out[i] + s : s;
}
// slab_reduce_kernel over the weight slabs and, in the threads past them, colsum_final_kernel's bias sums
// (float64 over the split rows in order): one launch instead of two (84 per training step)
__global__ void slab_bias_reduce_kernel(const float* __restrict__ part, int S, int64_t n, float* __restrict__ out,
                                        const float* __restrict__ colpart, int C, float* __restrict__ db) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    out[i] += slab_sum<float>(part, S, n, i);
  } else if (i < n + C) {
    const int c = (int)(i - n);
    db[c] += (float)slab_sum<double>(colpart, S, C, c);  // (0.0 + first row: the same float64 sum as before)
  }
}

// Column sums of an [P][C] tensor in a fixed order: stage 1 per (pixel slice, column) — a block is
// 64 columns x 4 row lanes (each row lane strides the slice's pixels, coalesced along the columns),
// merged in LDS in lane order; stage 2 adds the slices in order (float64).
constexpr int CS_SLICE = 1024;  // the smallest slice; large tensors use multiples (<= 256 slices)
inline int64_t colsum_slice(int64_t P) {
  int64_t sl = CS_SLICE;
  while ((P + sl - 1) / sl > 256) sl *= 2;
  return sl;
}
__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* __restrict__ x, int64_t P, int C,
                                                             int64_t slice, float* __restrict__ part) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int64_t p0 = (int64_t)blockIdx.y * slice;
  const int64_t p1 = p0 + slice < P ? p0 + slice : P;
  float s = 0.f;
  if (c < C)
    for (int64_t p = p0 + rl; p < p1; p += 4) s += x[p * C + c];
  red[rl][cl] = s;
  __syncthreads();
  if (rl == 0 && c < C) part[(int64_t)blockIdx.y * C + c] = ((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl];
}
__global__ void colsum_final_kernel(const float* __restrict__ part, int S, int C, float* __restrict__ out,
                                    int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0;
  for (int z = 0; z < S; ++z) s += part[(int64_t)z * C + c];
  out[c] = accumulate ? out[c] + (float)s : (float)s;
}

// ---------------------------------------------------------------------------------------------
// GroupNorm(32) forward for training (code/nn.py:46-48, + scale/shift nn.py:203-206, + SiLU):
//   stats[n][g] = (mean, rstd), rstd = 1/sqrt(var + 1e-5), biased var, accumulated in float64;
//   out = act((x - mean) * rstd * gamma + beta) [ * (1 + scale) + shift ]
// ss (optional): [N][ss_stride], scale at [0, C), shift at [C, 2C) (the emb projection's chunk order).
constexpr int GN_SL = 256;  // pixels per partial block (at most; gn_nsl)
// Slices per image of the GroupNorm passes: 256-pixel slices, halved (down to 16 pixels, not below the
// block's pixel-row count 1024 / C) while the grid has fewer than 1024 blocks — at 16x16 and B = 32 one
// slice per image gave 32 blocks for the whole chip (the 16^2 backward passes ran ~57 us for 17 MB).
// The kernels take their slice length from the grid: sl = ceil(HW / gridDim.x).
static int gn_nsl(int HW, int N, int C) {
  int sl = GN_SL;
  const int R = C >= 4 ? 1024 / C : 256;
  while (sl > 16 && sl / 2 >= R && (int64_t)((HW + sl - 1) / sl) * N < 1024) sl /= 2;
  return (HW + sl - 1) / sl;
}
__device__ __forceinline__ int gn_sl(int HW) { return (HW + (int)gridDim.x - 1) / (int)gridDim.x; }
// grid (slices, N), 256 threads. Thread = (row r, channel quad q): Q = C/4 quads side by side and
// R = 256/Q rows striding the slice's pixels, so each 16-B load belongs to a wave that covers whole
// pixel rows. Per-thread float64 sums are combined over the rows in LDS in a fixed order.
__global__ __launch_bounds__(256) void gn_stat_partial_kernel(const float* __restrict__ x, int HW, int C,
                                                              double* __restrict__ part) {
  __shared__ double s1[1024], s2[1024];  // [row][C] (R * C <= 1024), then per channel in row 0
  const int n = blockIdx.y;
  const int sl = gn_sl(HW), p0 = blockIdx.x * sl, p1 = min(p0 + sl, HW);
  const int Q = C >> 2, R = 256 / Q;
  const int q = threadIdx.x % Q, r = threadIdx.x / Q;
  if (r < R) {
    double a[4] = {0.0, 0.0, 0.0, 0.0}, b[4] = {0.0, 0.0, 0.0, 0.0};
    const float* xs = x + (int64_t)n * HW * C + 4 * q;
    for (int p = p0 + r; p < p1; p += R) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(xs + (int64_t)p * C);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const double d = v[j];
        a[j] += d;
        b[j] += d * d;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s1[r * C + 4 * q + j] = a[j];
      s2[r * C + 4 * q + j] = b[j];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {  // column c is read and written by thread c only
    double a = 0.0, b = 0.0;
    for (int k = 0; k < R; ++k) {
      a += s1[k * C + c];
      b += s2[k * C + c];
    }
    s1[c] = a;
    s2[c] = b;
  }
  __syncthreads();
  const int cg = C / 32;
  if (threadIdx.x < 32) {
    double a = 0.0, b = 0.0;
    for (int k = 0; k < cg; ++k) {
      a += s1[threadIdx.x * cg + k];
      b += s2[threadIdx.x * cg + k];
    }
    double* o = part + (((int64_t)n * gridDim.x + blockIdx.x) * 32 + threadIdx.x) * 2;
    o[0] = a;
    o[1] = b;
  }
}
// (mean, rstd) per (n, g) from equal-count granule statistics of cnt values each (the conv epilogue's /
// split-K reduction's): channels [0, C0) from g0[n][C0/4][E], [C0, C) from g1[n][(C-C0)/4][E] (a
// concat's two sources) as (mean, M2). One wave per (n, g), float64 merges in a fixed order (mean of
// the means, then M2 = sum M2_i + cnt sum (mean_i - mean)^2)
// Optional per-channel coefficients of the GroupNorm apply (GnCoef::A non-null): A = rstd gamma (1 + s),
// B = (beta - mean rstd gamma)(1 + s) + shift, so that act(A x + B) is the normalised activation the
// convs' prologues (and the split weight gradient's staging) compute on load; the arithmetic of
// norm.hip's gn_finalize2 (the sampler's coefficients).
struct GnCoef {
  const float* gamma; const float* beta; const float* ss; int ss_stride;
  float* A; float* B;  // [N][C]
};
__device__ __forceinline__ void gn_coef_write(const GnCoef& k, int n, int g, int C, float meanf, float rstd) {
  const int cpg = C / 32;
  for (int j = threadIdx.x; j < cpg; j += 64) {
    const int c = g * cpg + j;
    const float a = rstd * k.gamma[c];
    const float b = k.beta[c] - meanf * a;
    float A = a, B = b;
    if (k.ss) {
      const float sc = 1.0f + k.ss[(int64_t)n * k.ss_stride + c];
      A = a * sc;
      B = b * sc + k.ss[(int64_t)n * k.ss_stride + C + c];
    }
    k.A[(int64_t)n * C + c] = A;
    k.B[(int64_t)n * C + c] = B;
  }
}
__global__ __launch_bounds__(64) void gn_granule_final_kernel(const float* __restrict__ g0, int C0,
                                                              const float* __restrict__ g1, int E, float cnt, int C,
                                                              float* __restrict__ stats, GnCoef coef) {
  const int i = blockIdx.x;  // (n, g)
  const int n = i / 32, g = i % 32;
  const int qpg = C / 128;   // channel quads per group
  const int K = qpg * E;
  const int Q0 = C0 / 4, Q1 = (C - C0) / 4;
  auto at = [&](int k) -> const float* {  // granule k of the group: quad g*qpg + k/E, entry k%E
    const int qq = g * qpg + k / E, e = k % E;
    return qq < Q0 ? g0 + (((int64_t)n * Q0 + qq) * E + e) * 2 : g1 + (((int64_t)n * Q1 + qq - Q0) * E + e) * 2;
  };
  double a = 0.0;
  for (int k = threadIdx.x; k < K; k += 64) a += at(k)[0];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) a += __shfl_xor(a, off);
  const double mean = a / K;
  double q = 0.0;
  for (int k = threadIdx.x; k < K; k += 64) {
    const float* v = at(k);
    const double d = v[0] - mean;
    q += v[1] + (double)cnt * d * d;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) q += __shfl_xor(q, off);
  double var = q / ((double)K * cnt);
  if (var < 0) var = 0;
  // (lane 0's values everywhere: the butterflies' sums can differ between lanes in the last bit)
  const float meanf = __shfl((float)mean, 0), rstd = __shfl((float)(1.0 / sqrt(var + 1e-5)), 0);
  if (coef.A) gn_coef_write(coef, n, g, C, meanf, rstd);
  if (threadIdx.x) return;
  stats[i * 2] = meanf;
  stats[i * 2 + 1] = rstd;
}
// one wave per (n, g): the lanes stride the slices, then a fixed butterfly (deterministic)
__global__ __launch_bounds__(64) void gn_stat_final_kernel(const double* __restrict__ part, int nsl, int HW, int C,
                                                           int N, float* __restrict__ stats, GnCoef coef) {
  const int i = blockIdx.x;  // (n, g)
  const int n = i / 32, g = i % 32;
  double a = 0.0, b = 0.0;
  for (int s = threadIdx.x; s < nsl; s += 64) {
    a += part[(((int64_t)n * nsl + s) * 32 + g) * 2];
    b += part[(((int64_t)n * nsl + s) * 32 + g) * 2 + 1];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    a += __shfl_xor(a, off);
    b += __shfl_xor(b, off);
  }
  const double cnt = (double)HW * (C / 32);
  const double mean = a / cnt;
  double var = b / cnt - mean * mean;
  if (var < 0) var = 0;
  // (lane 0's values everywhere: the butterflies' sums can differ between lanes in the last bit)
  const float meanf = __shfl((float)mean, 0), rstd = __shfl((float)(1.0 / sqrt(var + 1e-5)), 0);
  if (coef.A) gn_coef_write(coef, n, g, C, meanf, rstd);
  if (threadIdx.x) return;
  stats[i * 2] = meanf;
  stats[i * 2 + 1] = rstd;
}

__device__ __forceinline__ float sigm(float z) { return 1.0f / (1.0f + expf(-z)); }

// grid (slices, N), 256 threads in gn_stat_partial_kernel's (row, channel quad) layout: a thread keeps
// its four channels' statistics, affine and scale/shift in registers and streams 16-B pixel quads
__global__ __launch_bounds__(256) void gn_apply_kernel(const float* __restrict__ x, int HW, int C,
                                                       const float* __restrict__ stats, const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, const float* __restrict__ ss,
                                                       int ss_stride, int act_silu, float* __restrict__ out) {
  const int n = blockIdx.y;
  const int sl = gn_sl(HW), p0 = blockIdx.x * sl, p1 = min(p0 + sl, HW);
  const int Q = C >> 2, R = 256 / Q;
  const int q = threadIdx.x % Q, r = threadIdx.x / Q;
  if (r >= R) return;
  const int c0 = 4 * q, cpg = C / 32;
  float mean[4], rstd[4], gam[4], bet[4], sc[4], sh[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = c0 + j, g = c / cpg;
    mean[j] = stats[(n * 32 + g) * 2];
    rstd[j] = stats[(n * 32 + g) * 2 + 1];
    gam[j] = gamma[c];
    bet[j] = beta[c];
    sc[j] = ss ? 1.0f + ss[(int64_t)n * ss_stride + c] : 1.0f;
    sh[j] = ss ? ss[(int64_t)n * ss_stride + C + c] : 0.0f;
  }
  const int64_t base = (int64_t)n * HW * C + c0;
#pragma unroll 2
  for (int p = p0 + r; p < p1; p += R) {
    const f32x4 xv = *reinterpret_cast<const f32x4*>(x + base + (int64_t)p * C);
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float z = (xv[j] - mean[j]) * rstd[j] * gam[j] + bet[j];
      if (ss) z = z * sc[j] + sh[j];
      o[j] = act_silu ? z * sigm(z) : z;
    }
    *reinterpret_cast<f32x4*>(out + base + (int64_t)p * C) = o;
  }
}

// GroupNorm(+ scale/shift)(+ SiLU) backward. With xhat = (x - mean) rstd, nrm = xhat gamma + beta,
// z = nrm (1 + s) + sh (or nrm), a = silu(z) (or z), given da:
//   dz = da silu'(z); dnrm = dz (1 + s); dsh = sum_p dz; ds = sum_p dz nrm;
//   dgamma = sum dnrm xhat; dbeta = sum dnrm; dxhat = dnrm gamma;
//   dx = rstd (dxhat - mean_g(dxhat) - xhat mean_g(dxhat xhat))
// Pass 1 (per image n, pixel slice, channel): A1 = sum dz, A2 = sum dz nrm, A3 = sum dnrm xhat.
struct GnBwdArgs {
  const float* dout; const float* x; int N, HW, C;
  const float* gamma; const float* beta; const float* ss; int ss_stride; int act_silu;
  const float* stats;
  // x = concat(x[C0], x1[C - C0]) (the output blocks' skip concat, read by channel range); C0 = C: one tensor
  const float* x1; int C0;
  // optional addend of dx, [N][HW] pixels with add_stride floats each (a channel range of a wider tensor: the
  // skip part of an output block's concat gradient, added into the encoder chain where dx is written)
  const float* add = nullptr; int add_stride = 0;
  // the resampling ResBlocks (rmode 1: nearest-up x2, 2: AvgPool2d(2); W = the GroupNorm input's width): dout is
  // the gradient at the block's output resolution, read through the resample adjoint (resample4_bwd_kernel's
  // arithmetic), and radd (optional, same resolution: the skip path's gradient) joins dx through it as well
  int rmode = 0, W = 0;
  const float* radd = nullptr;
  // optional split output (concat inputs): dx gets channels [0, C0) as [N][HW][C0] and dx1 channels [C0, C) as
  // [N][HW][C - C0] - the gradient of each concat source in its own tensor (no channel copy out of a C-wide one)
  float* dx1 = nullptr;
};
// the resample adjoint of t (at the output resolution) at GroupNorm-input pixel p of image n, channels c0..c0+3
__device__ __forceinline__ f32x4 gn_radj(const GnBwdArgs& a, const float* t, int n, int p, int c0) {
  const int y = p / a.W, x = p - y * a.W, C = a.C;
  f32x4 v;
  if (a.rmode == 1) {
    const int Ho = 2 * a.W;
    const int64_t b0 = (((int64_t)n * Ho + 2 * y) * Ho + 2 * x) * C + c0;
    const int64_t rs = (int64_t)Ho * C;
    const f32x4 a0 = *reinterpret_cast<const f32x4*>(t + b0), a1 = *reinterpret_cast<const f32x4*>(t + b0 + C);
    const f32x4 a2 = *reinterpret_cast<const f32x4*>(t + b0 + rs), a3 = *reinterpret_cast<const f32x4*>(t + b0 + rs + C);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = ((a0[j] + a1[j]) + a2[j]) + a3[j];
  } else {
    const int Ho = a.W / 2;
    const f32x4 u = *reinterpret_cast<const f32x4*>(t + (((int64_t)n * Ho + y / 2) * Ho + x / 2) * C + c0);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = u[j] / 4.0f;
  }
  return v;
}
// the thread's x quad (channels c0 .. c0 + 3 of image n): base pointer and pixel stride in its source
__device__ __forceinline__ const float* gn_xsrc(const GnBwdArgs& a, int n, int c0, int& stride) {
  if (c0 < a.C0) {
    stride = a.C0;
    return a.x + (int64_t)n * a.HW * a.C0 + c0;
  }
  stride = a.C - a.C0;
  return a.x1 + (int64_t)n * a.HW * stride + (c0 - a.C0);
}
// grid (slices, N), 256 threads laid out as gn_stat_partial_kernel's (row, channel quad); a thread's
// per-channel coefficients stay in registers
__global__ __launch_bounds__(256) void gn_bwd_partial_kernel(GnBwdArgs a, float* __restrict__ part) {
  // part [N][nsl][C][3]
  __shared__ float red[3][1024];  // [row][C] (R * C <= 1024), then per channel in row 0
  const int n = blockIdx.y, C = a.C;
  const int sl = gn_sl(a.HW), p0 = blockIdx.x * sl, p1 = min(p0 + sl, a.HW);
  const int Q = C >> 2, R = 256 / Q;
  const int q = threadIdx.x % Q, r = threadIdx.x / Q;
  if (r < R) {
    const int c0 = 4 * q, cpg = C / 32;
    float mean[4], rstd[4], gam[4], bet[4], onep[4], sh[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = c0 + j, g = c / cpg;
      mean[j] = a.stats[(n * 32 + g) * 2];
      rstd[j] = a.stats[(n * 32 + g) * 2 + 1];
      gam[j] = a.gamma[c];
      bet[j] = a.beta[c];
      onep[j] = a.ss ? 1.0f + a.ss[(int64_t)n * a.ss_stride + c] : 1.0f;
      sh[j] = a.ss ? a.ss[(int64_t)n * a.ss_stride + C + c] : 0.0f;
    }
    float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f}, s3[4] = {0.f, 0.f, 0.f, 0.f};
    const int64_t base = (int64_t)n * a.HW * C + c0;
    int xs;
    const float* const xb = gn_xsrc(a, n, c0, xs);
    for (int p = p0 + r; p < p1; p += R) {
      const f32x4 xv = *reinterpret_cast<const f32x4*>(xb + (int64_t)p * xs);
      const f32x4 dv = a.rmode ? gn_radj(a, a.dout, n, p, c0) : *reinterpret_cast<const f32x4*>(a.dout + base + (int64_t)p * C);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float xhat = (xv[j] - mean[j]) * rstd[j];
        const float nrm = xhat * gam[j] + bet[j];
        const float z = a.ss ? nrm * onep[j] + sh[j] : nrm;
        float dz = dv[j];
        if (a.act_silu) {
          const float sg = sigm(z);
          dz = dv[j] * (sg * (1.0f + z * (1.0f - sg)));
        }
        s1[j] += dz;
        s2[j] += dz * nrm;
        s3[j] += dz * onep[j] * xhat;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      red[0][r * C + c0 + j] = s1[j];
      red[1][r * C + c0 + j] = s2[j];
      red[2][r * C + c0 + j] = s3[j];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float t1 = 0.f, t2 = 0.f, t3 = 0.f;
    for (int k = 0; k < R; ++k) {
      t1 += red[0][k * C + c];
      t2 += red[1][k * C + c];
      t3 += red[2][k * C + c];
    }
    float* o = part + (((int64_t)n * gridDim.x + blockIdx.x) * C + c) * 3;
    o[0] = t1;
    o[1] = t2;
    o[2] = t3;
  }
}
// Per (n, c): A1..A3 (float64 over slices) -> nc, dss; per (n, g): the group means -> red[n][g][2]. One launch,
// a block per (group, image) (round 5; was two launches): each of the group's channels is summed over the
// slices by SL lanes in float64 (lane l takes slices l, l + SL, ...), the lanes combined by a fixed pairwise
// tree, then the group's means from the float-rounded per-channel sums, in channel order. (A serial
// per-channel loop over up to 256 slices took ~18 us a call.)
__global__ __launch_bounds__(256) void gn_bwd_reduce_group_kernel(GnBwdArgs a, const float* __restrict__ part, int nsl,
                                                                  int SL, float* __restrict__ nc,
                                                                  float* __restrict__ dss, float* __restrict__ red) {
  __shared__ double sh[3][256];
  __shared__ float ncs[2][32];
  const int g = blockIdx.x, n = blockIdx.y, C = a.C, cg = C / 32;
  const int k = threadIdx.x / SL, l = threadIdx.x % SL;  // blockDim.x = cg * SL
  const int c = g * cg + k;
  double s1 = 0, s2 = 0, s3 = 0;
  for (int s = l; s < nsl; s += SL) {
    const float* o = part + (((int64_t)n * nsl + s) * C + c) * 3;
    s1 += o[0];
    s2 += o[1];
    s3 += o[2];
  }
  sh[0][threadIdx.x] = s1;
  sh[1][threadIdx.x] = s2;
  sh[2][threadIdx.x] = s3;
  for (int w = SL / 2; w >= 1; w >>= 1) {
    __syncthreads();
    if (l < w) {
      sh[0][threadIdx.x] += sh[0][threadIdx.x + w];
      sh[1][threadIdx.x] += sh[1][threadIdx.x + w];
      sh[2][threadIdx.x] += sh[2][threadIdx.x + w];
    }
  }
  __syncthreads();
  if (l == 0) {
    s1 = sh[0][threadIdx.x];
    s2 = sh[1][threadIdx.x];
    s3 = sh[2][threadIdx.x];
    const int i = n * C + c;
    const float onep = a.ss ? 1.0f + a.ss[(int64_t)n * a.ss_stride + c] : 1.0f;
    const float v1 = (float)(s1 * onep), v2 = (float)s3;
    nc[i * 3] = (float)s1;  // sum dz
    nc[i * 3 + 1] = v1;     // sum dnrm
    nc[i * 3 + 2] = v2;     // sum dnrm xhat
    ncs[0][k] = v1;
    ncs[1][k] = v2;
    if (dss) {  // d scale, d shift (accumulated into the emb-projection gradient)
      dss[(int64_t)n * a.ss_stride + c] += (float)s2;
      dss[(int64_t)n * a.ss_stride + C + c] += (float)s1;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double m1 = 0, m2 = 0;
    for (int kk = 0; kk < cg; ++kk) {
      m1 += (double)a.gamma[g * cg + kk] * ncs[0][kk];
      m2 += (double)a.gamma[g * cg + kk] * ncs[1][kk];
    }
    const double cnt = (double)cg * a.HW;
    red[(n * 32 + g) * 2] = (float)(m1 / cnt);
    red[(n * 32 + g) * 2 + 1] = (float)(m2 / cnt);
  }
}
// slice lanes per channel: a power of two with cg * SL <= 256
static int gn_reduce_lanes(int C) {
  const int cg = C / 32;
  int SL = 1;
  while (2 * SL * cg <= 256) SL *= 2;
  return SL;
}
// grid (nsl + ceil(C / 256), N), the (row, channel quad) layout with per-channel coefficients in registers.
// The blocks past the nsl slices of image 0 are gn_bwd_param_kernel's (dgamma, dbeta += the image sums of nc):
// both need only the reduce kernel's output, so the parameter gradients ride in this launch (was one more
// launch per GroupNorm, 65 a training step).
__global__ __launch_bounds__(256) void gn_bwd_dx_kernel(GnBwdArgs a, const float* __restrict__ red,
                                                        float* __restrict__ dx, int accumulate, int nsl,
                                                        const float* __restrict__ nc, float* __restrict__ dgamma,
                                                        float* __restrict__ dbeta) {
  const int n = blockIdx.y, C = a.C;
  if ((int)blockIdx.x >= nsl) {
    const int c = ((int)blockIdx.x - nsl) * 256 + (int)threadIdx.x;
    if (n != 0 || c >= C) return;
    double g = 0, b = 0;
#pragma unroll 8
    for (int i = 0; i < a.N; ++i) {
      b += nc[((int64_t)i * C + c) * 3 + 1];
      g += nc[((int64_t)i * C + c) * 3 + 2];
    }
    dgamma[c] += (float)g;
    dbeta[c] += (float)b;
    return;
  }
  const int sl = (a.HW + nsl - 1) / nsl, p0 = blockIdx.x * sl, p1 = min(p0 + sl, a.HW);
  const int Q = C >> 2, R = 256 / Q;
  const int q = threadIdx.x % Q, r = threadIdx.x / Q;
  if (r >= R) return;
  const int c0 = 4 * q, cpg = C / 32;
  float mean[4], rstd[4], gam[4], bet[4], onep[4], sh[4], r0[4], r1[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = c0 + j, g = c / cpg;
    mean[j] = a.stats[(n * 32 + g) * 2];
    rstd[j] = a.stats[(n * 32 + g) * 2 + 1];
    gam[j] = a.gamma[c];
    bet[j] = a.beta[c];
    onep[j] = a.ss ? 1.0f + a.ss[(int64_t)n * a.ss_stride + c] : 1.0f;
    sh[j] = a.ss ? a.ss[(int64_t)n * a.ss_stride + C + c] : 0.0f;
    r0[j] = red[(n * 32 + g) * 2];
    r1[j] = red[(n * 32 + g) * 2 + 1];
  }
  const int64_t base = (int64_t)n * a.HW * C + c0;
  int xs;
  const float* const xb = gn_xsrc(a, n, c0, xs);
#pragma unroll 2
  for (int p = p0 + r; p < p1; p += R) {
    const int64_t i = base + (int64_t)p * C;
    const f32x4 xv = *reinterpret_cast<const f32x4*>(xb + (int64_t)p * xs);
    const f32x4 dv = a.rmode ? gn_radj(a, a.dout, n, p, c0) : *reinterpret_cast<const f32x4*>(a.dout + i);
    f32x4 prev = {0.f, 0.f, 0.f, 0.f};
    if (accumulate) prev = *reinterpret_cast<const f32x4*>(dx + i);  // (never with a split output: host-checked)
    if (a.add) prev += *reinterpret_cast<const f32x4*>(a.add + ((int64_t)n * a.HW + p) * a.add_stride + c0);
    if (a.radd) prev += gn_radj(a, a.radd, n, p, c0);
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // gn_bwd_partial_kernel's per-point arithmetic
      const float xhat = (xv[j] - mean[j]) * rstd[j];
      const float nrm = xhat * gam[j] + bet[j];
      const float z = a.ss ? nrm * onep[j] + sh[j] : nrm;
      float dz = dv[j];
      if (a.act_silu) {
        const float sg = sigm(z);
        dz = dv[j] * (sg * (1.0f + z * (1.0f - sg)));
      }
      const float dxhat = dz * onep[j] * gam[j];
      const float v = rstd[j] * (dxhat - r0[j] - xhat * r1[j]);
      o[j] = accumulate || a.add || a.radd ? prev[j] + v : v;
    }
    float* dst = dx + i;
    if (a.dx1) {  // (uniform per thread: its channel quad sits in one source)
      const int64_t px = (int64_t)n * a.HW + p;
      dst = c0 < a.C0 ? dx + px * a.C0 + c0 : a.dx1 + px * (C - a.C0) + (c0 - a.C0);
    }
    *reinterpret_cast<f32x4*>(dst) = o;
  }
}

// ---------------------------------------------------------------------------------------------
// nearest-up x2 / avg-pool 2x2 (code/nn.py:92-133) and their adjoints, NHWC.
__global__ void resample_kernel(const float* __restrict__ x, int N, int Hin, int C, int mode, float* __restrict__ out) {
  const int Ho = mode == 1 ? 2 * Hin : Hin / 2;
  const int64_t tot = (int64_t)N * Ho * Ho * C;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= tot) return;
  const int c = (int)(i % C);
  int64_t r = i / C;
  const int xo = (int)(r % Ho);
  r /= Ho;
  const int yo = (int)(r % Ho);
  const int n = (int)(r / Ho);
  if (mode == 1) {
    out[i] = x[(((int64_t)n * Hin + yo / 2) * Hin + xo / 2) * C + c];
  } else {
    const int64_t b0 = (((int64_t)n * Hin + 2 * yo) * Hin + 2 * xo) * C + c;
    const int64_t rs = (int64_t)Hin * C;
    float s = x[b0];
    s = s + x[b0 + C];
    s = s + x[b0 + rs];
    s = s + x[b0 + rs + C];
    out[i] = s / 4.0f;
  }
}
// 4 channels per thread (C % 4 == 0): one index decode per 4 values
__global__ void resample4_kernel(const float* __restrict__ x, int N, int Hin, int C, int mode, float* __restrict__ out) {
  const int Ho = mode == 1 ? 2 * Hin : Hin / 2;
  const int64_t tot = (int64_t)N * Ho * Ho * C;
  const int64_t i = 4 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= tot) return;
  int64_t r = i / C;
  const int c = (int)(i - r * C);
  const int64_t r2 = r / Ho;
  const int xo = (int)(r - r2 * Ho);
  const int n = (int)(r2 / Ho);
  const int yo = (int)(r2 - (int64_t)n * Ho);
  if (mode == 1) {
    *reinterpret_cast<f32x4*>(out + i) =
        *reinterpret_cast<const f32x4*>(x + (((int64_t)n * Hin + yo / 2) * Hin + xo / 2) * C + c);
  } else {
    const int64_t b0 = (((int64_t)n * Hin + 2 * yo) * Hin + 2 * xo) * C + c;
    const int64_t rs = (int64_t)Hin * C;
    const f32x4 a0 = *reinterpret_cast<const f32x4*>(x + b0), a1 = *reinterpret_cast<const f32x4*>(x + b0 + C);
    const f32x4 a2 = *reinterpret_cast<const f32x4*>(x + b0 + rs), a3 = *reinterpret_cast<const f32x4*>(x + b0 + rs + C);
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v = a0[j];
      v = v + a1[j];
      v = v + a2[j];
      v = v + a3[j];
      o[j] = v / 4.0f;
    }
    *reinterpret_cast<f32x4*>(out + i) = o;
  }
}
__global__ void resample4_bwd_kernel(const float* __restrict__ dy, int N, int Hin, int C, int mode,
                                     float* __restrict__ dx, int accumulate) {
  const int64_t tot = (int64_t)N * Hin * Hin * C;
  const int64_t i = 4 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= tot) return;
  int64_t r = i / C;
  const int c = (int)(i - r * C);
  const int64_t r2 = r / Hin;
  const int x = (int)(r - r2 * Hin);
  const int n = (int)(r2 / Hin);
  const int y = (int)(r2 - (int64_t)n * Hin);
  f32x4 v;
  if (mode == 1) {
    const int Ho = 2 * Hin;
    const int64_t b0 = (((int64_t)n * Ho + 2 * y) * Ho + 2 * x) * C + c;
    const int64_t rs = (int64_t)Ho * C;
    const f32x4 a0 = *reinterpret_cast<const f32x4*>(dy + b0), a1 = *reinterpret_cast<const f32x4*>(dy + b0 + C);
    const f32x4 a2 = *reinterpret_cast<const f32x4*>(dy + b0 + rs), a3 = *reinterpret_cast<const f32x4*>(dy + b0 + rs + C);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = ((a0[j] + a1[j]) + a2[j]) + a3[j];
  } else {
    const int Ho = Hin / 2;
    const f32x4 a = *reinterpret_cast<const f32x4*>(dy + (((int64_t)n * Ho + y / 2) * Ho + x / 2) * C + c);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = a[j] / 4.0f;
  }
  if (accumulate) v = *reinterpret_cast<const f32x4*>(dx + i) + v;
  *reinterpret_cast<f32x4*>(dx + i) = v;
}
// dx at the input resolution from dy at the output resolution
__global__ void resample_bwd_kernel(const float* __restrict__ dy, int N, int Hin, int C, int mode,
                                    float* __restrict__ dx, int accumulate) {
  const int64_t tot = (int64_t)N * Hin * Hin * C;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= tot) return;
  const int c = (int)(i % C);
  int64_t r = i / C;
  const int x = (int)(r % Hin);
  r /= Hin;
  const int y = (int)(r % Hin);
  const int n = (int)(r / Hin);
  float v;
  if (mode == 1) {  // up: each input pixel feeds a 2x2 block
    const int Ho = 2 * Hin;
    const int64_t b0 = (((int64_t)n * Ho + 2 * y) * Ho + 2 * x) * C + c;
    const int64_t rs = (int64_t)Ho * C;
    v = ((dy[b0] + dy[b0 + C]) + dy[b0 + rs]) + dy[b0 + rs + C];
  } else {  // down: each input pixel gets a quarter of its pooled output's gradient
    const int Ho = Hin / 2;
    v = dy[(((int64_t)n * Ho + y / 2) * Ho + x / 2) * C + c] / 4.0f;
  }
  dx[i] = accumulate ? dx[i] + v : v;
}

__global__ void add_kernel(const float* __restrict__ a, const float* __restrict__ b, float* out, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = a[i] + b[i];
}
__global__ void add4_kernel(const float* __restrict__ a, const float* __restrict__ b, float* out, int64_t n) {
  const int64_t i = 4 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (i < n) *reinterpret_cast<f32x4*>(out + i) = *reinterpret_cast<const f32x4*>(a + i) + *reinterpret_cast<const f32x4*>(b + i);
}
// dst[p][doff + c] (+)= src[p][soff + c], c < nc: concat assembly and the split of its gradient
__global__ void copy_channels_kernel(const float* __restrict__ src, int cs, int soff, float* __restrict__ dst, int cd,
                                     int doff, int nc, int64_t npix, int accumulate) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npix * nc) return;
  const int64_t p = i / nc;
  const int c = (int)(i - p * nc);
  const float v = src[p * cs + soff + c];
  float* d = dst + p * cd + doff + c;
  *d = accumulate ? *d + v : v;
}
// the same, 4 channels per thread (every count and offset a multiple of 4)
__global__ void copy_channels4_kernel(const float* __restrict__ src, int cs, int soff, float* __restrict__ dst, int cd,
                                      int doff, int nc, int64_t npix, int accumulate) {
  const int64_t i = 4 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= npix * nc) return;
  const int64_t p = i / nc;
  const int c = (int)(i - p * nc);
  const f32x4 v = *reinterpret_cast<const f32x4*>(src + p * cs + soff + c);
  f32x4* d = reinterpret_cast<f32x4*>(dst + p * cd + doff + c);
  *d = accumulate ? *d + v : v;
}

// ---------------------------------------------------------------------------------------------
// QKVAttention backward (code/nn.py:222-235, chunk-first heads). Per (n, head): q, k, v [T][64]
// at channel offsets (0, C, 2C) + 64 head of the qkv row; s2 = scale^2; P = softmax(s2 q k^T),
// o = P v. Given do: dv = P^T do; dP = do v^T; dS = P (dP - rowsum(dP P)); dq = s2 dS k; dk = s2 dS^T q.
// Kernel A: one block per (n, head, 32 query rows): recompute P rows, dP, dS; write dq and the
// P / dS rows to scratch [N][H][T][T]. Kernel B: one block per (n, head, 32 key rows): dk, dv.
constexpr int AB_R = 32;
__global__ __launch_bounds__(256) void attn_bwd_rows_kernel(const float* __restrict__ qkv, const float* __restrict__ dout,
                                                            int T, int C, float scale, float* __restrict__ dqkv,
                                                            float* __restrict__ Pm, float* __restrict__ dSm) {
  extern __shared__ float sh[];
  float* S = sh;                    // [AB_R][T]
  float* dP = sh + AB_R * T;        // [AB_R][T]
  const int head = blockIdx.y, n = blockIdx.z, nh = gridDim.y;
  const int r0 = blockIdx.x * AB_R;
  const int64_t row = 3 * (int64_t)C;
  const float* base = qkv + (int64_t)n * T * row;
  const float* dob = dout + (int64_t)n * T * C;
  const int qo = head * 64, ko = C + head * 64, vo = 2 * C + head * 64;
  const float s2 = scale * scale;
  // S = (q scale)(k scale)^T and dP = do v^T: a thread owns key column s (its scaled k row and v row in
  // registers, 16-B loads) and reads the block's q / do rows as LDS broadcasts
  float* Qs = sh + 2 * AB_R * T;  // [AB_R][64] scaled q rows
  float* Ds = Qs + AB_R * 64;     // [AB_R][64] do rows
  for (int e = threadIdx.x; e < AB_R * 64; e += blockDim.x) {
    const int r = e >> 6, d = e & 63, tq = r0 + r;
    Qs[e] = tq < T ? base[(int64_t)tq * row + qo + d] * scale : 0.f;
    Ds[e] = tq < T ? dob[(int64_t)tq * C + head * 64 + d] : 0.f;
  }
  __syncthreads();
  for (int s = threadIdx.x; s < T; s += blockDim.x) {
    float kr[64], vr[64];
#pragma unroll
    for (int d4 = 0; d4 < 16; ++d4) {
      const f32x4 kv = *reinterpret_cast<const f32x4*>(base + (int64_t)s * row + ko + 4 * d4);
      const f32x4 vv = *reinterpret_cast<const f32x4*>(base + (int64_t)s * row + vo + 4 * d4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        kr[4 * d4 + j] = kv[j] * scale;
        vr[4 * d4 + j] = vv[j];
      }
    }
    for (int r = 0; r < AB_R; ++r) {
      float acc = 0.f, accp = 0.f;
#pragma unroll
      for (int d = 0; d < 64; ++d) {
        acc += Qs[r * 64 + d] * kr[d];
        accp += Ds[r * 64 + d] * vr[d];
      }
      S[r * T + s] = acc;
      dP[r * T + s] = accp;
    }
  }
  __syncthreads();
  // softmax rows (fp32, max-subtracted), then dS
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int r = wave; r < AB_R; r += 4) {
    if (r0 + r >= T) continue;
    float m = -INFINITY;
    for (int s = lane; s < T; s += 64) m = fmaxf(m, S[r * T + s]);
    for (int o = 32; o; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    float sum = 0.f;
    for (int s = lane; s < T; s += 64) {
      const float e = expf(S[r * T + s] - m);
      S[r * T + s] = e;
      sum += e;
    }
    for (int o = 32; o; o >>= 1) sum += __shfl_xor(sum, o);
    const float inv = 1.0f / sum;
    float dd = 0.f;
    for (int s = lane; s < T; s += 64) {
      const float p = S[r * T + s] * inv;
      S[r * T + s] = p;
      dd += dP[r * T + s] * p;
    }
    for (int o = 32; o; o >>= 1) dd += __shfl_xor(dd, o);
    for (int s = lane; s < T; s += 64) dP[r * T + s] = S[r * T + s] * (dP[r * T + s] - dd);
  }
  __syncthreads();
  const int64_t mo = (((int64_t)n * nh + head) * T + r0) * T;
  for (int e = threadIdx.x; e < AB_R * T; e += blockDim.x) {
    if (r0 + e / T < T) {
      Pm[mo + e] = S[e];
      dSm[mo + e] = dP[e];
    }
  }
  // dq[tq][d] = s2 sum_s dS[tq][s] k[s][d]: wave w takes rows w, w + 4, ..., lane = d, one k load per s
  {
    float acc[AB_R / 4];
#pragma unroll
    for (int i = 0; i < AB_R / 4; ++i) acc[i] = 0.f;
    for (int s = 0; s < T; ++s) {
      const float kv = base[(int64_t)s * row + ko + lane];
#pragma unroll
      for (int i = 0; i < AB_R / 4; ++i) acc[i] += dP[(wave + 4 * i) * T + s] * kv;
    }
#pragma unroll
    for (int i = 0; i < AB_R / 4; ++i) {
      const int tq = r0 + wave + 4 * i;
      if (tq < T) dqkv[((int64_t)n * T + tq) * row + qo + lane] = s2 * acc[i];
    }
  }
}
__global__ __launch_bounds__(256) void attn_bwd_cols_kernel(const float* __restrict__ qkv, const float* __restrict__ dout,
                                                            int T, int C, float scale, float* __restrict__ dqkv,
                                                            const float* __restrict__ Pm, const float* __restrict__ dSm) {
  const int head = blockIdx.y, n = blockIdx.z, nh = gridDim.y;
  const int s0 = blockIdx.x * AB_R;
  const int64_t row = 3 * (int64_t)C;
  const float* base = qkv + (int64_t)n * T * row;
  const float* dob = dout + (int64_t)n * T * C;
  const int qo = head * 64, ko = C + head * 64, vo = 2 * C + head * 64;
  const float s2 = scale * scale;
  const int64_t mo = ((int64_t)n * nh + head) * T * T;
  // wave w takes key rows s0 + w, s0 + w + 4, ..., lane = d: one q / do load per t serves them all
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float dk[AB_R / 4], dv[AB_R / 4];
#pragma unroll
  for (int i = 0; i < AB_R / 4; ++i) dk[i] = dv[i] = 0.f;
  for (int t = 0; t < T; ++t) {
    const float qv = base[(int64_t)t * row + qo + lane];
    const float dov = dob[(int64_t)t * C + head * 64 + lane];
#pragma unroll
    for (int i = 0; i < AB_R / 4; ++i) {
      const int s = min(s0 + wave + 4 * i, T - 1);
      dk[i] += dSm[mo + (int64_t)t * T + s] * qv;
      dv[i] += Pm[mo + (int64_t)t * T + s] * dov;
    }
  }
#pragma unroll
  for (int i = 0; i < AB_R / 4; ++i) {
    const int s = s0 + wave + 4 * i;
    if (s >= T) continue;
    dqkv[((int64_t)n * T + s) * row + ko + lane] = s2 * dk[i];
    dqkv[((int64_t)n * T + s) * row + vo + lane] = dv[i];
  }
}

// The same backward on fp32 MFMAs (round 5; v_mfma_f32_32x32x2_f32, T = 32 KT <= 256): the VALU kernels above
// ran the five T x T x 64 products at ~16 TFLOP/s (0.69 ms per 16x16 attention layer at B = 32).
// Rows kernel: a block per (n, head, 128 queries), wave w takes 32 queries; K (x scale) and V in LDS as in the
// forward (misc.hip attention_mfma_kernel). Per wave, S^T and dP^T tiles by MFMA (lane = query: its softmax,
// rowsum(dP P) and dS = P (dP - rowsum) stay within the lane and its lane ^ 32 partner), dQ = scale (dS (k scale))
// by MFMA, and P^T, dS^T to scratch KEY-major [n][head][key][query] (each half-wave stores 32 consecutive
// queries of one key: coalesced). Cols kernel: a block per (n, head, 128 keys), wave w takes 32 keys; per
// 32-query chunk the wave stages its [32 keys][32 queries] of dS^T and P^T in LDS (stride 33: the A-operand
// reads, one key per lane, hit distinct banks) and the block the chunk's q and do rows; dK = s2 (dS^T q) and
// dV = P^T do by MFMA. Summation orders differ from the VALU kernels (fp32 MFMA accumulation); the training
// tests' tolerances hold (tests/test_gpu_blocks.py, tests/test_gpu_train*.py).
constexpr int ABM_KS = 68, ABM_VS = 68;  // K / V row strides in the rows kernel (ds_read_b128 of 32 rows)
constexpr int ABM_CS = 33;               // dS^T / P^T chunk row stride in the cols kernel

template <int KT>
__global__ __launch_bounds__(256, 1) void attn_bwd_rows_mfma_kernel(const float* __restrict__ qkv,
                                                                   const float* __restrict__ dout, int C, float scale,
                                                                   float* __restrict__ dqkv, float* __restrict__ Pm,
                                                                   float* __restrict__ dSm) {
  constexpr int T = 32 * KT;
  extern __shared__ __attribute__((aligned(16))) float abm[];
  float* Ks = abm;                 // [T][ABM_KS] k * scale
  float* Vs = abm + T * ABM_KS;    // [T][ABM_VS] v
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int head = blockIdx.y, n = blockIdx.z, nh = gridDim.y;
  const size_t rs = 3 * (size_t)C;
  const float* base = qkv + (size_t)n * T * rs + head * 64;
  for (int i = tid; i < T * 16; i += 256) {
    const int row = i >> 4, c4 = 4 * (i & 15);
    f32x4 kv = *(const f32x4*)(base + (size_t)row * rs + C + c4);
#pragma unroll
    for (int j = 0; j < 4; ++j) kv[j] = kv[j] * scale;
    *(f32x4*)(Ks + row * ABM_KS + c4) = kv;
    *(f32x4*)(Vs + row * ABM_VS + c4) = *(const f32x4*)(base + (size_t)row * rs + 2 * C + c4);
  }
  __syncthreads();
  const int q0 = blockIdx.x * 128 + 32 * w;
  if (q0 >= T) return;
  float qv[32], dv[32];  // q (x scale) and do of query q0 + l32, channels 32 h .. 32 h + 31
  const float* dob = dout + ((size_t)n * T + q0 + l32) * C + head * 64 + 32 * h;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const f32x4 v = *(const f32x4*)(base + (size_t)(q0 + l32) * rs + 32 * h + 4 * j);
    const f32x4 d = *(const f32x4*)(dob + 4 * j);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      qv[4 * j + c] = v[c] * scale;
      dv[4 * j + c] = d[c];
    }
  }
  // S^T and dP^T tiles: register r of tile kt = key kt 32 + 8 (r >> 2) + 4 h + (r & 3), query q0 + l32
  f32x16 s[KT], dp[KT];
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
#pragma unroll
    for (int r = 0; r < 16; ++r) s[kt][r] = dp[kt][r] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const f32x4 kf = *(const f32x4*)(Ks + (kt * 32 + l32) * ABM_KS + 32 * h + 4 * j);
      const f32x4 vf = *(const f32x4*)(Vs + (kt * 32 + l32) * ABM_VS + 32 * h + 4 * j);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        s[kt] = __builtin_amdgcn_mfma_f32_32x32x2f32(kf[c], qv[4 * j + c], s[kt], 0, 0, 0);
        dp[kt] = __builtin_amdgcn_mfma_f32_32x32x2f32(vf[c], dv[4 * j + c], dp[kt], 0, 0, 0);
      }
    }
  }
  // softmax over the query's keys (this lane and lane ^ 32), rowsum(dP P), dS = P (dP - rowsum)
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
  float dd = 0.f;
#pragma unroll
  for (int kt = 0; kt < KT; ++kt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s[kt][r] = s[kt][r] * inv;
      dd += dp[kt][r] * s[kt][r];
    }
  dd += __shfl_xor(dd, 32);
  const size_t mo = ((size_t)n * nh + head) * T * T + q0 + l32;
#pragma unroll
  for (int kt = 0; kt < KT; ++kt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      dp[kt][r] = s[kt][r] * (dp[kt][r] - dd);
      const size_t key = kt * 32 + 8 * (r >> 2) + 4 * h + (r & 3);
      Pm[mo + key * T] = s[kt][r];
      dSm[mo + key * T] = dp[kt][r];
    }
  // dQ[q][d] = scale sum_key dS[q][key] (k scale)[key][d]: A = dS (lane = query, k = the lane half's key), B = K
  f32x16 o0, o1;
#pragma unroll
  for (int r = 0; r < 16; ++r) o0[r] = o1[r] = 0.f;
#pragma unroll
  for (int kt = 0; kt < KT; ++kt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float* kr = Ks + (kt * 32 + 8 * (r >> 2) + 4 * h + (r & 3)) * ABM_KS + l32;
      o0 = __builtin_amdgcn_mfma_f32_32x32x2f32(dp[kt][r], kr[0], o0, 0, 0, 0);
      o1 = __builtin_amdgcn_mfma_f32_32x32x2f32(dp[kt][r], kr[32], o1, 0, 0, 0);
    }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int q = q0 + 8 * (r >> 2) + 4 * h + (r & 3);
    float* o = dqkv + ((size_t)n * T + q) * rs + head * 64 + l32;
    o[0] = scale * o0[r];
    o[32] = scale * o1[r];
  }
}

template <int KT>
__global__ __launch_bounds__(256, 1) void attn_bwd_cols_mfma_kernel(const float* __restrict__ qkv,
                                                                   const float* __restrict__ dout, int C, float scale,
                                                                   float* __restrict__ dqkv,
                                                                   const float* __restrict__ Pm,
                                                                   const float* __restrict__ dSm) {
  constexpr int T = 32 * KT;
  __shared__ float qs[32][64], ds_[32][64];        // the chunk's q and do rows (block)
  __shared__ float dst[4][32 * ABM_CS], pt[4][32 * ABM_CS];  // per wave: [32 keys][32 queries] of dS^T, P^T
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int head = blockIdx.y, n = blockIdx.z, nh = gridDim.y;
  const size_t rs = 3 * (size_t)C;
  const float* base = qkv + (size_t)n * T * rs + head * 64;
  const float* dob = dout + (size_t)n * T * C + head * 64;
  const int k0 = blockIdx.x * 128 + 32 * w;
  const bool act = k0 < T;
  const size_t mo = ((size_t)n * nh + head) * T * T;
  f32x16 dk0, dk1, dv0, dv1;
#pragma unroll
  for (int r = 0; r < 16; ++r) dk0[r] = dk1[r] = dv0[r] = dv1[r] = 0.f;
  float* dsw = dst[w];
  float* ptw = pt[w];
  for (int qc = 0; qc < T; qc += 32) {
    __syncthreads();  // the previous chunk's reads are done
    for (int i = tid; i < 32 * 16; i += 256) {
      const int row = i >> 4, c4 = 4 * (i & 15);
      *(f32x4*)&qs[row][c4] = *(const f32x4*)(base + (size_t)(qc + row) * rs + c4);
      *(f32x4*)&ds_[row][c4] = *(const f32x4*)(dob + (size_t)(qc + row) * C + c4);
    }
    if (act) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int idx = e * 64 + lane, row = idx >> 3, c4 = 4 * (idx & 7);
        const size_t g = mo + (size_t)(k0 + row) * T + qc + c4;
        const f32x4 a = *(const f32x4*)(dSm + g), b = *(const f32x4*)(Pm + g);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          dsw[row * ABM_CS + c4 + c] = a[c];
          ptw[row * ABM_CS + c4 + c] = b[c];
        }
      }
    }
    __syncthreads();
    if (act) {
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) {
        const int qq = 2 * kk + h;  // this lane half's query of the step
        const float a_ds = dsw[l32 * ABM_CS + qq], a_p = ptw[l32 * ABM_CS + qq];
        dk0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a_ds, qs[qq][l32], dk0, 0, 0, 0);
        dk1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a_ds, qs[qq][l32 + 32], dk1, 0, 0, 0);
        dv0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a_p, ds_[qq][l32], dv0, 0, 0, 0);
        dv1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a_p, ds_[qq][l32 + 32], dv1, 0, 0, 0);
      }
    }
  }
  if (!act) return;
  const float s2 = scale * scale;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int key = k0 + 8 * (r >> 2) + 4 * h + (r & 3);
    float* o = dqkv + ((size_t)n * T + key) * rs + head * 64 + l32;
    o[C] = s2 * dk0[r];
    o[C + 32] = s2 * dk1[r];
    o[2 * C] = dv0[r];
    o[2 * C + 32] = dv1[r];
  }
}

template <int KT>
static void launch_attn_bwd_mfma(const float* qkv, const float* dout, int N, int C, float scale, float* dqkv, float* Pm,
                                 float* dSm, hipStream_t s) {
  constexpr int T = 32 * KT;
  const size_t lds = (size_t)T * (ABM_KS + ABM_VS) * sizeof(float);
  static bool attr[kMaxDevices] = {};
  (void)set_lds_attr_once(attr, reinterpret_cast<const void*>(&attn_bwd_rows_mfma_kernel<KT>), (int)lds);
  dim3 g((T + 127) / 128, C / 64, N);
  hipLaunchKernelGGL(attn_bwd_rows_mfma_kernel<KT>, g, dim3(256), lds, s, qkv, dout, C, scale, dqkv, Pm, dSm);
  hipLaunchKernelGGL(attn_bwd_cols_mfma_kernel<KT>, g, dim3(256), 0, s, qkv, dout, C, scale, dqkv, Pm, dSm);
}

// ---------------------------------------------------------------------------------------------
// Linear layers of the embedding path (code/unet.py:44-48, code/nn.py:167-170): y = pre(x) W^T + b,
// W [N][K] (torch), pre = identity | SiLU. M (the batch) is small; one thread per output.
__device__ __forceinline__ float pre_f(float v, int pre_silu) { return pre_silu ? v * sigm(v) : v; }
// one wave per (output column j, row m): lanes stride k (the weight row read coalesced), then a
// fixed-order shuffle tree
__global__ __launch_bounds__(256) void linear_kernel(const float* __restrict__ x, int M, int K,
                                                     const float* __restrict__ w, const float* __restrict__ b, int N,
                                                     int pre_silu, int post_silu, float* __restrict__ y) {
  const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wid >= (int64_t)M * N) return;
  const int m = (int)(wid / N), j = (int)(wid % N);
  float acc = 0.f;
  for (int k = lane; k < K; k += 64) acc = fmaf(pre_f(x[(int64_t)m * K + k], pre_silu), w[(int64_t)j * K + k], acc);
  for (int o = 32; o; o >>= 1) acc += __shfl_xor(acc, o);
  if (lane == 0) {
    const float v = acc + (b ? b[j] : 0.f);
    y[wid] = post_silu ? v * sigm(v) : v;
  }
}
// dx[m][k] (+)= (sum_j dy[m][j] W[j][k]) * pre'(x[m][k]); block = 64 k x LDX_Q j-slices (merged in order)
constexpr int LDX_Q = 16;
__global__ __launch_bounds__(64 * LDX_Q) void linear_dx_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                               int M, int K, const float* __restrict__ w, int N,
                                                               int pre_silu, float* __restrict__ dx, int accumulate) {
  __shared__ float red[LDX_Q][64];
  const int kl = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int kblocks = (K + 63) / 64;
  const int m = blockIdx.x / kblocks, k = (blockIdx.x % kblocks) * 64 + kl;
  float part = 0.f;
  if (k < K)
    for (int j = q; j < N; j += LDX_Q) part = fmaf(dy[(int64_t)m * N + j], w[(int64_t)j * K + k], part);
  red[q][kl] = part;
  __syncthreads();
  if (q != 0 || k >= K) return;
  const int64_t i = (int64_t)m * K + k;
  float acc = red[0][kl];
#pragma unroll
  for (int t = 1; t < LDX_Q; ++t) acc += red[t][kl];
  if (pre_silu) {
    const float v = x[i], sg = sigm(v);
    acc *= sg * (1.0f + v * (1.0f - sg));
  }
  dx[i] = accumulate ? dx[i] + acc : acc;
}
// dW[j][k] += sum_m dy[m][j] pre(x[m][k]); db[j] += sum_m dy[m][j]
__global__ void linear_dw_kernel(const float* __restrict__ dy, const float* __restrict__ x, int M, int K, int N,
                                 int pre_silu, float* __restrict__ dw, float* __restrict__ db) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)N * K) return;
  const int j = (int)(i / K), k = (int)(i % K);
  float acc = 0.f, accb = 0.f;
  for (int m = 0; m < M; ++m) {
    const float g = dy[(int64_t)m * N + j];
    acc = fmaf(g, pre_f(x[(int64_t)m * K + k], pre_silu), acc);
    accb += g;
  }
  dw[i] += acc;
  if (db && k == 0) db[j] += accb;
}
// y = silu'(z) * dy for the time-MLP's hidden layer (z stored pre-activation)
__global__ void silu_bwd_kernel(const float* __restrict__ z, const float* __restrict__ dy, float* __restrict__ dz,
                                int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = z[i], sg = sigm(v);
  dz[i] = dy[i] * (sg * (1.0f + v * (1.0f - sg)));
}
// timestep_embedding(t, dim) (code/nn.py:51-61): [cos(t f) | sin(t f)] with the fp32 frequency
// table f (computed on the host exactly as the reference does)
__global__ void temb_kernel(const int64_t* __restrict__ t, const float* __restrict__ freqs, int N, int dim,
                            float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * dim) return;
  const int n = i / dim, k = i % dim, half = dim / 2;
  const int j = k < half ? k : k - half;
  const float arg = (float)t[n] * freqs[j];
  out[i] = k < half ? cosf(arg) : sinf(arg);
}

// ---------------------------------------------------------------------------------------------
// training_losses (code/gaussian_diffusion.py:540-614), fused elementwise parts.
// x_t = q_sample(x0, t, noise) (:172-189); injection (:114-157 via :572-582, injection_schedule
// "all", cumulative noise): x_t = keep q_sample(x0, t[0], cached) + (1 - keep) x_t, keep = 1 - mask.
// Coefficients come from fp32 tables (_extract_into_tensor gathers float64, then .float()).
__global__ void q_sample_inject_kernel(const float* __restrict__ x0, const float* __restrict__ noise,
                                       const float* __restrict__ cached, const float* __restrict__ mask,
                                       const int64_t* __restrict__ t, const float* __restrict__ sa,
                                       const float* __restrict__ s1m, int N, int HW, int inject,
                                       float* __restrict__ xt) {
#pragma clang fp contract(off)
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)N * 3 * HW) return;
  const int n = (int)(i / (3 * (int64_t)HW));
  const int64_t p = i % HW;
  const int64_t tn = t[n];
  float v = sa[tn] * x0[i] + s1m[tn] * noise[i];
  if (inject) {
    const int64_t t0 = t[0];
    const float w = sa[t0] * x0[i] + s1m[t0] * cached[i];
    const float keep = 1.0f - mask[(int64_t)n * HW + p];
    v = keep * w + (1.0f - keep) * v;
  }
  xt[i] = v;
}
// masked eps-MSE: per (n, c): S = sum_p (noise - eps)^2 mask, area = max(sum_p mask, 1);
// loss = mean over (n, c) of S / area; d eps = -2 (noise - eps) mask / area / (N * 3), written
// into the NHWC gradient of the 6-channel model output (variance channels: 0).
__global__ void mse_partial_kernel(const float* __restrict__ out6, int cs, const float* __restrict__ noise,
                                   const float* __restrict__ mask, int HW, float* __restrict__ part) {
  // grid (N * 3); block reduces over HW
  __shared__ double r1[256], r2[256];
  const int nc = blockIdx.x, n = nc / 3, c = nc % 3;
  double a = 0.0, b = 0.0;
  for (int p = threadIdx.x; p < HW; p += blockDim.x) {
    const float m = mask[(int64_t)n * HW + p];
    const float d = noise[((int64_t)n * 3 + c) * HW + p] - out6[((int64_t)n * HW + p) * cs + c];
    a += (double)(d * d * m);
    b += m;
  }
  r1[threadIdx.x] = a;
  r2[threadIdx.x] = b;
  __syncthreads();
  for (int s = 128; s; s >>= 1) {
    if (threadIdx.x < s) {
      r1[threadIdx.x] += r1[threadIdx.x + s];
      r2[threadIdx.x] += r2[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[nc * 2] = (float)r1[0];
    part[nc * 2 + 1] = (float)(r2[0] < 1.0 ? 1.0 : r2[0]);
  }
}
__global__ void mse_final_kernel(const float* __restrict__ part, int NC, float* __restrict__ loss) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double s = 0.0;
  for (int i = 0; i < NC; ++i) s += (double)part[i * 2] / part[i * 2 + 1];
  loss[0] = (float)(s / NC);
}
__global__ void mse_grad_kernel(const float* __restrict__ out6, int cs, const float* __restrict__ noise,
                                const float* __restrict__ mask, const float* __restrict__ part, int N, int HW,
                                float* __restrict__ dout6) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)N * HW * cs) return;
  const int c = (int)(i % cs);
  const int64_t pix = i / cs;
  const int n = (int)(pix / HW);
  const int64_t p = pix % HW;
  float g = 0.f;
  if (c < 3) {
    const float m = mask[(int64_t)n * HW + p];
    const float d = noise[((int64_t)n * 3 + c) * HW + p] - out6[i];
    g = -2.0f * d * m / part[(n * 3 + c) * 2 + 1] / (float)(N * 3);
  }
  dout6[i] = g;
}

// ---------------------------------------------------------------------------------------------
// clip_grad_norm_(max_norm) + AdamW (code/train_inpainting.py:64-66, :394-399; torch semantics):
//   coef = min(1, max_norm / (||g|| + 1e-6)); g *= coef
//   p *= 1 - lr wd; m = b1 m + (1 - b1) g; v = b2 v + (1 - b2) g^2
//   p -= (lr / (1 - b1^k)) m / (sqrt(v) / sqrt(1 - b2^k) + eps)
constexpr int SQ_BLOCKS = 1024;
__global__ void sumsq_partial_kernel(const float* __restrict__ g, int64_t n, double* __restrict__ part) {
  __shared__ double r[256];
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = g[i];
    s += v * v;
  }
  r[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k; k >>= 1) {
    if (threadIdx.x < k) r[threadIdx.x] += r[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = r[0];
}
__global__ void clip_coef_kernel(const double* __restrict__ part, int nb, float max_norm, float* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double s = 0.0;
  for (int i = 0; i < nb; ++i) s += part[i];
  const float norm = (float)sqrt(s);
  const float coef = max_norm / (norm + 1e-6f);
  out[0] = norm;
  out[1] = coef < 1.0f ? coef : 1.0f;
}
// scalars pre-formed on the host in double and rounded once (torch's AdamW: Python-float arithmetic,
// then a float scalar per tensor op): decay = 1 - lr wd, w1 = 1 - b1, b2, w2 = 1 - b2, step = lr / bc1
__global__ void adamw_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
                             int64_t n, const float* __restrict__ clip, float decay, float w1, float b2, float w2,
                             float step, float eps, float bc2s) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float gi = g[i] * clip[1];
  g[i] = gi;
  float pi = p[i] * decay;
  const float mi = m[i] + (gi - m[i]) * w1;  // torch lerp_ (weight < 0.5 branch)
  const float vi = v[i] * b2 + w2 * gi * gi;
  m[i] = mi;
  v[i] = vi;
  const float denom = sqrtf(vi) / bc2s + eps;
  pi = pi - step * (mi / denom);
  p[i] = pi;
}


// 3xf16 split packing of a 3x3 conv weight on the device (unet.hip pack_conv_x3's layout and
// arithmetic): one thread per (ct, chunk, tap, h, col, j) writes both parts.
__device__ __forceinline__ void pack3x3_elem(const float* __restrict__ w, int cout, int cin, int cin_pad16,
                                             int transpose, _Float16* __restrict__ dst, unsigned* guard, int64_t i) {
#pragma clang fp contract(off)
  const int nch = cin_pad16 / 16;
  const int j = (int)(i & 7);
  int64_t r = i >> 3;
  const int col = (int)(r & 63);
  r >>= 6;
  const int hh = (int)(r & 1);
  r >>= 1;
  const int tap = (int)(r % 9);
  r /= 9;
  const int chk = (int)(r % nch);
  const int ct = (int)(r / nch);
  const int o = ct * 64 + col, c = chk * 16 + hh * 8 + j;  // packed (out, in) channel
  float v = 0.f;
  if (transpose == 0) {
    if (o < cout && c < cin) v = w[((size_t)o * cin + c) * 9 + tap];
  } else {
    if (o < cin && c < cout) v = w[((size_t)c * cin + o) * 9 + (8 - tap)];
  }
  const _Float16 hi = (_Float16)v;
  const float s = (float)hi * 2048.0f;
  if (!(fabsf(s) <= 65504.0f)) atomicOr(guard, 2u);
  const _Float16 lo = (_Float16)((v - (float)hi) * 2048.0f);
  const size_t base = ((((size_t)ct * nch + chk) * 9 + tap) * 2) * 2;  // part 0
  dst[((base + hh) * 64 + col) * 8 + j] = (_Float16)s;
  dst[((base + 2 + hh) * 64 + col) * 8 + j] = lo;
}
__device__ __forceinline__ int64_t pack3x3_count(int cin_pad16, int cout_pad) {
  return (int64_t)(cout_pad / 64) * (cin_pad16 / 16) * 9 * 2 * 64 * 8;
}
__global__ void pack_conv_x3_kernel(const float* __restrict__ w, int cout, int cin, int cin_pad16, int cout_pad,
                                    int transpose, _Float16* __restrict__ dst, unsigned* guard) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < pack3x3_count(cin_pad16, cout_pad)) pack3x3_elem(w, cout, cin, cin_pad16, transpose, dst, guard, i);
}

// 3xf16 packing of a 1x1 conv weight for the split kernel's 1x1 chunks (unet.hip pack_skip_x3's layout:
// [cout_pad/64][cin/32][q][part][h][64][8] f16, element (q, part, h, col, j) of chunk s = split part of
// W[64 ct + col][32 s + 16 h + 8 q + j]); transpose=1 packs the dgrad conv (out = cin, in = cout).
__device__ __forceinline__ void pack1x1_elem(const float* __restrict__ w, int cout, int cin, int cs_pad,
                                             int transpose, _Float16* __restrict__ dst, unsigned* guard, int64_t i) {
#pragma clang fp contract(off)
  const int ns = cs_pad / 32;
  const int j = (int)(i & 7);
  int64_t r = i >> 3;
  const int col = (int)(r & 63);
  r >>= 6;
  const int hh = (int)(r & 1);
  r >>= 1;
  const int qq = (int)(r & 1);
  r >>= 1;
  const int sk = (int)(r % ns);
  const int ct = (int)(r / ns);
  const int o = ct * 64 + col, c = sk * 32 + hh * 16 + qq * 8 + j;
  float v = 0.f;
  if (transpose == 0) {
    if (o < cout && c < cin) v = w[(size_t)o * cin + c];
  } else {
    if (o < cin && c < cout) v = w[(size_t)c * cin + o];
  }
  const _Float16 hi = (_Float16)v;
  const float sc = (float)hi * 2048.0f;
  if (!(fabsf(sc) <= 65504.0f)) atomicOr(guard, 2u);
  const _Float16 lo = (_Float16)((v - (float)hi) * 2048.0f);
  const size_t base = ((((size_t)ct * ns + sk) * 2 + qq) * 2) * 2;  // [ct][s][q][part][h]
  dst[((base + 0 + hh) * 64 + col) * 8 + j] = (_Float16)sc;
  dst[((base + 2 + hh) * 64 + col) * 8 + j] = lo;
}
__device__ __forceinline__ int64_t pack1x1_count(int cs_pad, int cout_pad) {
  return (int64_t)(cout_pad / 64) * (cs_pad / 32) * 2 * 2 * 64 * 8;  // without the part index
}
__global__ void pack_conv1x1_x3_kernel(const float* __restrict__ w, int cout, int cin, int cs_pad, int cout_pad,
                                       int transpose, _Float16* __restrict__ dst, unsigned* guard) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < pack1x1_count(cs_pad, cout_pad)) pack1x1_elem(w, cout, cin, cs_pad, transpose, dst, guard, i);
}

// Every split-kernel weight packing of a training step in one launch (round 5; was one launch per conv and
// direction, ~170 a step). Descriptor table (device, built once by the caller): a block's descriptor is found
// by a binary search over the block offsets (uniform per block), then each thread packs PK_EPT elements
// (256 apart) as the single-conv kernels do.
struct PackDesc {
  const float* w;
  void* dst;
  int cout, cin, pad, cout_pad, transpose, taps;
  int64_t block0;  // first block of this descriptor
};
constexpr int PK_EPT = 32;  // elements per thread of the batched packing (amortises the descriptor search)
__global__ __launch_bounds__(256) void pack_x3_batch_kernel(const PackDesc* __restrict__ d, int nd, unsigned* guard) {
  const int64_t b = blockIdx.x;
  int lo = 0, hi = nd - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (d[mid].block0 <= b) lo = mid; else hi = mid - 1;
  }
  const PackDesc e = d[lo];
  const int64_t i0 = (b - e.block0) * 256 * PK_EPT + threadIdx.x;
  if (e.taps == 9) {
    const int64_t n = pack3x3_count(e.pad, e.cout_pad);
    for (int k = 0; k < PK_EPT; ++k) {
      const int64_t i = i0 + 256 * k;
      if (i < n) pack3x3_elem(e.w, e.cout, e.cin, e.pad, e.transpose, (_Float16*)e.dst, guard, i);
    }
  } else {
    const int64_t n = pack1x1_count(e.pad, e.cout_pad);
    for (int k = 0; k < PK_EPT; ++k) {
      const int64_t i = i0 + 256 * k;
      if (i < n) pack1x1_elem(e.w, e.cout, e.cin, e.pad, e.transpose, (_Float16*)e.dst, guard, i);
    }
  }
}

__global__ void scale_kernel(float* __restrict__ x, int64_t n, float s) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = x[i] * s;
}
}  // namespace
}  // namespace ifd

using namespace ifd;

#define TR_LAST() IFD_LAUNCH_STATUS()

extern "C" {

int ifd_tr_pack_conv(const float* w, int cout, int cin, int taps, int bn, int cin_pad, int cout_pad, int transpose,
                     float* wpack, void* stream) {
  const int64_t tot = (int64_t)cout_pad * cin_pad * taps;
  if (!w || !wpack || cin_pad % 8 || cout_pad % bn || (taps != 1 && taps != 9)) {
    set_error("ifd_tr_pack_conv: bad arguments");
    return 2;
  }
  hipLaunchKernelGGL(pack_conv_kernel, dim3(grid1(tot)), dim3(TB), 0, (hipStream_t)stream, w, cout, cin, taps, bn,
                     cin_pad, cout_pad, transpose, wpack);
  return TR_LAST();
}

static void conv_params(ConvParams& p, const float* x0, int c0, const float* x1, int c1, int N, int H,
                        const float* wpack, const float* bias, int cin_pad, int cout, int cout_pad, int bn, int taps,
                        const float* res, float* out) {
  std::memset(&p, 0, sizeof(p));
  p.in0 = x0; p.c0 = c0; p.in1 = x1; p.c1 = c1;
  p.N = N; p.Hin = p.Win = p.H = p.W = H;
  p.act = ACT_NONE;
  p.wpack = wpack; p.bias = bias;
  p.cin_pad = cin_pad; p.cout = cout; p.cout_pad = cout_pad;
  p.res = res; p.res_xform = XF_NONE; p.res_H = p.res_W = H;
  p.out = out;
  p.epi = EPI_NHWC;
  p.opt_bm128 = taps == 1;  // the 256-pixel tiles are instantiated for 3x3 only
  conv_geometry(p, H, H, N, bn, cin_pad / 8);
}

int64_t ifd_tr_conv_part_floats(int N, int H, int cin_pad, int cout, int cout_pad, int bn, int taps) {
  ConvParams p;
  conv_params(p, nullptr, cin_pad, nullptr, 0, N, H, nullptr, nullptr, cin_pad, cout, cout_pad, bn, taps, nullptr,
              nullptr);
  return p.ksplit > 1 ? (int64_t)p.ksplit * N * H * H * cout : 0;
}

int ifd_tr_conv(const float* x0, int c0, const float* x1, int c1, int N, int H, const float* wpack, const float* bias,
                int cin_pad, int cout, int cout_pad, int bn, int taps, const float* res, float* out, float* part,
                int64_t part_floats, void* stream) {
  // cout % 4: the NHWC epilogue stores channel quads
  if ((H & (H - 1)) || c0 % 8 || c1 % 8 || c0 + c1 != cin_pad || (bn != 32 && bn != 64) || cout_pad % bn ||
      cout % 4 || cout > cout_pad || (taps != 1 && taps != 9) || !x0 || !out || !wpack || !bias) {
    set_error("ifd_tr_conv: unsupported arguments");
    return 2;
  }
  ConvParams p;
  conv_params(p, x0, c0, c1 ? x1 : nullptr, c1, N, H, wpack, bias, cin_pad, cout, cout_pad, bn, taps, res, out);
  if (p.ksplit > 1) {
    if (!part || (int64_t)p.ksplit * N * H * H * cout > part_floats) {
      set_error("ifd_tr_conv: split-K workspace too small (ifd_tr_conv_part_floats)");
      return 2;
    }
    p.part = part;
  }
  int e = launch_conv(p, taps, XF_NONE, bn, (hipStream_t)stream);
  if (!e && p.ksplit > 1) e = launch_splitk_reduce(p, (hipStream_t)stream);
  if (e) set_error(std::string("ifd_tr_conv: ") + hipGetErrorString((hipError_t)e));
  return e;
}

int ifd_tr_conv_gn(const float* x0, int c0, const float* x1, int c1, int N, int H, const float* wpack,
                   const float* bias, int cin_pad, int cout, int cout_pad, int bn, int taps, const float* actA,
                   const float* actB, const float* res, float* out, float* part, int64_t part_floats, void* stream) {
  if ((H & (H - 1)) || c0 % 8 || c1 % 8 || c0 + c1 != cin_pad || (bn != 32 && bn != 64) || cout_pad % bn ||
      cout % 4 || cout > cout_pad || (taps != 1 && taps != 9) || !x0 || !out || !wpack || !bias || !actA || !actB) {
    set_error("ifd_tr_conv_gn: unsupported arguments");
    return 2;
  }
  ConvParams p;
  conv_params(p, x0, c0, c1 ? x1 : nullptr, c1, N, H, wpack, bias, cin_pad, cout, cout_pad, bn, taps, res, out);
  p.act = ACT_AFFINE_SILU;
  p.actA = actA;
  p.actB = actB;
  if (p.ksplit > 1) {
    if (!part || (int64_t)p.ksplit * N * H * H * cout > part_floats) {
      set_error("ifd_tr_conv_gn: split-K workspace too small (ifd_tr_conv_part_floats)");
      return 2;
    }
    p.part = part;
  }
  int e = launch_conv(p, taps, XF_NONE, bn, (hipStream_t)stream);
  if (!e && p.ksplit > 1) e = launch_splitk_reduce(p, (hipStream_t)stream);
  if (e) set_error(std::string("ifd_tr_conv_gn: ") + hipGetErrorString((hipError_t)e));
  return e;
}

int64_t ifd_tr_head_x3_pack_floats(int cin) { return (int64_t)conv_head_x3_pack_floats(cin); }

int ifd_tr_conv_head_x3(const float* x, int cin, int N, int H, const float* w, int cout, float* wpack,
                        const float* bias8, const float* actA, const float* actB, float* out, unsigned* guard,
                        void* stream) {
  ConvParams p;
  std::memset(&p, 0, sizeof(p));
  p.in0 = x; p.c0 = cin;
  p.N = N; p.Hin = p.Win = p.H = p.W = H;
  p.act = ACT_AFFINE_SILU; p.actA = actA; p.actB = actB;
  p.bias = bias8;
  p.cin_pad = cin; p.cout = 8; p.cout_pad = 8;
  p.out = out;
  p.epi = EPI_NHWC;
  p.guard = guard;
  if (!x || !w || !wpack || !bias8 || !actA || !actB || !out || !guard || cout < 1 || cout > 8 ||
      !conv_head_x3_nhwc_eligible(p)) {
    set_error("ifd_tr_conv_head_x3: shape not eligible (cin % 32 == 0, cin <= 128, H % 16 == 0, cout <= 8)");
    return 3;
  }
  hipStream_t s = (hipStream_t)stream;
  int e = launch_pack_head_x3(w, cout, cin, wpack, guard, s);
  if (!e) e = launch_conv_head_x3(p, wpack, s);
  if (e) set_error(std::string("ifd_tr_conv_head_x3: ") + hipGetErrorString((hipError_t)e));
  return e;
}

int ifd_tr_pack_conv_x3(const float* w, int cout, int cin, int taps, int cin_pad16, int cout_pad, int transpose,
                        void* wx3, unsigned* guard, void* stream) {
  if (!w || !wx3 || !guard || (taps != 9 && taps != 1) || cin_pad16 % (taps == 1 ? 32 : 16) || cout_pad % 64) {
    set_error("ifd_tr_pack_conv_x3: bad arguments");
    return 2;
  }
  if (taps == 1) {
    const int64_t tot = (int64_t)(cout_pad / 64) * (cin_pad16 / 32) * 2 * 2 * 64 * 8;
    hipLaunchKernelGGL(pack_conv1x1_x3_kernel, dim3(grid1(tot)), dim3(TB), 0, (hipStream_t)stream, w, cout, cin,
                       cin_pad16, cout_pad, transpose, (_Float16*)wx3, guard);
    return TR_LAST();
  }
  const int64_t tot = (int64_t)(cout_pad / 64) * (cin_pad16 / 16) * 9 * 2 * 64 * 8;
  hipLaunchKernelGGL(pack_conv_x3_kernel, dim3(grid1(tot)), dim3(TB), 0, (hipStream_t)stream, w, cout, cin, cin_pad16,
                     cout_pad, transpose, (_Float16*)wx3, guard);
  return TR_LAST();
}

int64_t ifd_tr_pack_desc_bytes() { return (int64_t)sizeof(PackDesc); }

int ifd_tr_pack_x3_batch(const void* desc, int ndesc, int64_t nblocks, unsigned* guard, void* stream) {
  if (!desc || ndesc <= 0 || nblocks <= 0 || !guard) {
    set_error("ifd_tr_pack_x3_batch: bad arguments");
    return 2;
  }
  hipLaunchKernelGGL(pack_x3_batch_kernel, dim3((unsigned)nblocks), dim3(TB), 0, (hipStream_t)stream,
                     (const PackDesc*)desc, ndesc, guard);
  return TR_LAST();
}

// taps = 1: the split kernel's 1x1-only launch (the operand as 32-channel skip chunks, no main
// segment); a residual then goes through the split-K reduction (ksplit >= 2), as unet.hip does
static void conv_x3_params(ConvParams& p, const float* x0, int c0, const float* x1, int c1, int N, int H,
                           const void* wx3, const float* bias, int cin_pad, int cout, const float* res, float* out,
                           int taps = 9) {
  conv_params(p, x0, c0, x1, c1, N, H, (const float*)wx3, bias, cin_pad, cout, cout, 64, 9, res, out);
  p.opt_bm128 = 0;
  p.x3_nprod = 3;
  p.opt_img8_partial = 1;  // four-image 8 x 8 tiles at any N (every tile-origin-derived read stays in the batch)
  if (taps == 1) {  // (two sources: the output blocks' concat, read by channel range)
    p.s0 = x0; p.sc0 = c0; p.s1 = c1 ? x1 : nullptr; p.sc1 = c1;
    p.wskip = (const float*)wx3; p.cs_pad = cin_pad;
    p.in0 = nullptr; p.c0 = 0; p.in1 = nullptr; p.c1 = 0; p.cin_pad = 0;
    conv_geometry(p, H, H, N, 64, cin_pad / 32, true);
    if (res && p.ksplit == 1 && (cin_pad / 32) % 2 == 0) p.ksplit = 2;
    return;
  }
  conv_geometry(p, H, H, N, 64, cin_pad / 16, true);
}

int64_t ifd_tr_conv_x3_part_floats(int N, int H, int cin_pad, int cout) {
  ConvParams p;
  conv_x3_params(p, nullptr, cin_pad, nullptr, 0, N, H, nullptr, nullptr, cin_pad, cout, nullptr, nullptr);
  ConvParams q;  // the 1x1 geometry with a residual (the larger of the two)
  conv_x3_params(q, nullptr, cin_pad, nullptr, 0, N, H, nullptr, nullptr, cin_pad, cout, (const float*)1, nullptr, 1);
  const int S = p.ksplit > q.ksplit ? p.ksplit : q.ksplit;
  return S > 1 ? (int64_t)S * N * H * H * cout : 0;
}

int ifd_tr_conv_x3(const float* x0, int c0, const float* x1, int c1, int N, int H, const void* wx3, const float* bias,
                   int cin_pad, int cout, const float* res, float* out, float* part, int64_t part_floats,
                   unsigned* guard, void* stream) {
  return ifd_tr_conv_x3_taps(x0, c0, x1, c1, N, H, wx3, bias, cin_pad, cout, res, out, part, part_floats, guard, 9,
                             3, stream);
}

static int conv_x3_run(const float* x0, int c0, const float* x1, int c1, int N, int H, const void* wx3,
                       const float* bias, int cin_pad, int cout, const float* res, float* out, float* part,
                       int64_t part_floats, unsigned* guard, int wx3_taps, float* gstat, int64_t gstat_floats,
                       int* gstat_E, float* gstat_cnt, int nprod, void* stream, const float* actA = nullptr,
                       const float* actB = nullptr, GnbParams* gnb = nullptr, int* gnb_nsl = nullptr) {
  if (gstat_E) *gstat_E = 0;
  if (gnb_nsl) *gnb_nsl = 0;
  if ((H & (H - 1)) || c0 + c1 != cin_pad || !x0 || !out || !wx3 || !bias || !guard || (nprod != 1 && nprod != 3)) {
    set_error("ifd_tr_conv_x3: unsupported arguments");
    return 2;
  }
  ConvParams p;
  const int taps = wx3_taps;
  if (taps == 1 && (c0 % 32 || c1 % 32 || (c1 && !x1))) {
    set_error("ifd_tr_conv_x3: 1x1 needs input channel counts % 32 == 0");
    return 3;
  }
  if (actA && (taps != 9 || !actB)) {  // (the 1x1 operand goes to LDS by DMA, unactivated)
    set_error("ifd_tr_conv_x3_gn: the GroupNorm prologue needs a 3x3 conv and both coefficient arrays");
    return 3;
  }
  conv_x3_params(p, x0, c0, c1 ? x1 : nullptr, c1, N, H, wx3, bias, cin_pad, cout, res, out, taps);
  p.guard = guard;
  p.x3_nprod = nprod;
  if (actA) {
    p.act = ACT_AFFINE_SILU;
    p.actA = actA;
    p.actB = actB;
  }
  const int nct = cout / 64;  // the non-SKIP split kernel decodes channel tiles by shifts
  if (cout % 64 || (taps == 9 && (nct & (nct - 1))) || !conv_x3_eligible(p, taps, XF_NONE, 64)) {
    set_error("ifd_tr_conv_x3: shape not eligible for the split kernel (use ifd_tr_conv)");
    return 3;
  }
  if (p.ksplit > 1) {
    if (!part || (int64_t)p.ksplit * N * H * H * cout > part_floats) {
      set_error("ifd_tr_conv_x3: split-K workspace too small (ifd_tr_conv_x3_part_floats)");
      return 2;
    }
    p.part = part;
  }
  // GroupNorm granule statistics of the output (when asked for and the geometry has them): from the
  // epilogue of single-image 256-pixel tiles (E = 4 wave entries per tile, 256 values each), or from
  // the split-K reduction (E = HW / min(HW, 64))
  const int HW = H * H;
  const int64_t skE = HW / (HW < 64 ? HW : 64);
  const bool want = gstat && gstat_E && gstat_cnt && cout % 128 == 0;
  if (want && p.ksplit == 1 && p.IMGS == 1 && p.TW * p.TH == 256 &&
      (int64_t)N * (cout / 4) * p.tiles_x * p.tiles_y * 4 * 2 <= gstat_floats) {
    p.gstat = gstat;
    p.gstat_E = p.tiles_x * p.tiles_y * 4;
  }
  int e;
  if (gnb && gnb_nsl && p.ksplit == 1 && p.IMGS == 1 && (p.TW == 32 || p.TW == 16) && !res && taps == 9 && !p.gstat) {
    // the dgrad + its GroupNorm backward's pass-1 partial sums in the epilogue (conv.h GnbParams)
    gnb->nsl = p.tiles_x * p.tiles_y * 4;
    e = launch_conv_x3_gnb(p, *gnb, (hipStream_t)stream);
    if (!e) *gnb_nsl = gnb->nsl;
  } else {
    e = launch_conv_x3(p, XF_NONE, (hipStream_t)stream);
  }
  if (!e && p.gstat) {
    *gstat_E = p.gstat_E;
    *gstat_cnt = 256.f;
  }
  if (!e && p.ksplit > 1) {
    if (want && HW % (HW < 64 ? HW : 64) == 0 && (int64_t)N * (cout / 4) * skE * 2 <= gstat_floats) {
      p.gstat = gstat;
      int E = 0;
      float cnt = 0.f;
      e = launch_splitk_gstat(p, &E, &cnt, (hipStream_t)stream);
      if (!e) {
        *gstat_E = E;
        *gstat_cnt = cnt;
      }
    } else {
      e = launch_splitk_reduce(p, (hipStream_t)stream);
    }
  }
  if (e) set_error(std::string("ifd_tr_conv_x3: ") + hipGetErrorString((hipError_t)e));
  return e;
}

int ifd_tr_conv_x3_taps(const float* x0, int c0, const float* x1, int c1, int N, int H, const void* wx3,
                        const float* bias, int cin_pad, int cout, const float* res, float* out, float* part,
                        int64_t part_floats, unsigned* guard, int wx3_taps, int nprod, void* stream) {
  return conv_x3_run(x0, c0, x1, c1, N, H, wx3, bias, cin_pad, cout, res, out, part, part_floats, guard, wx3_taps,
                     nullptr, 0, nullptr, nullptr, nprod, stream);
}

int ifd_tr_conv_x3_gn(const float* x0, int c0, const float* x1, int c1, int N, int H, const void* wx3,
                      const float* bias, int cin_pad, int cout, const float* actA, const float* actB, const float* res,
                      float* out, float* part, int64_t part_floats, unsigned* guard, float* gstat,
                      int64_t gstat_floats, int* gstat_E, float* gstat_cnt, int nprod, void* stream) {
  return conv_x3_run(x0, c0, x1, c1, N, H, wx3, bias, cin_pad, cout, res, out, part, part_floats, guard, 9, gstat,
                     gstat_floats, gstat_E, gstat_cnt, nprod, stream, actA, actB);
}

int64_t ifd_tr_gnb_part_floats(int N, int H, int cout) {
  const int64_t HW = (int64_t)H * H;
  return (int64_t)N * (HW >= 64 ? HW / 64 : 1) * cout * 3;
}

int ifd_tr_conv_x3_gnb_act(const float* dy, int cdy, int N, int H, const void* wx3, const float* bias, int cin_pad,
                           int cout, float* out, float* part, int64_t part_floats, unsigned* guard, const float* gx0,
                           int gc0, const float* gx1, const float* stats, const float* gamma, const float* beta,
                           const float* ss, int ss_stride, int act_silu, float* gpart, int64_t gpart_floats,
                           int* gpart_nsl, float* act_out, int nprod, void* stream) {
  if (!gpart_nsl || !gx0 || !stats || !gamma || !beta || gc0 <= 0 || gc0 > cout || (gc0 < cout && !gx1) ||
      cout % 32 || ifd_tr_gnb_part_floats(N, H, cout) > gpart_floats || !gpart) {
    set_error("ifd_tr_conv_x3_gnb: bad GroupNorm arguments or partial-sum buffer too small");
    return 2;
  }
  GnbParams g{};
  g.x0 = gx0; g.x1 = gx1; g.c0 = gc0;
  g.stats = stats; g.gamma = gamma; g.beta = beta;
  g.ss = ss; g.ss_stride = ss_stride; g.silu = act_silu;
  g.part = gpart;
  g.act = act_out;
  return conv_x3_run(dy, cdy, nullptr, 0, N, H, wx3, bias, cin_pad, cout, nullptr, out, part, part_floats, guard, 9,
                     nullptr, 0, nullptr, nullptr, nprod, stream, nullptr, nullptr, &g, gpart_nsl);
}

int ifd_tr_conv_x3_gnb(const float* dy, int cdy, int N, int H, const void* wx3, const float* bias, int cin_pad,
                       int cout, float* out, float* part, int64_t part_floats, unsigned* guard, const float* gx0, int gc0,
                       const float* gx1, const float* stats, const float* gamma, const float* beta, const float* ss,
                       int ss_stride, int act_silu, float* gpart, int64_t gpart_floats, int* gpart_nsl, int nprod,
                       void* stream) {
  return ifd_tr_conv_x3_gnb_act(dy, cdy, N, H, wx3, bias, cin_pad, cout, out, part, part_floats, guard, gx0, gc0, gx1,
                                stats, gamma, beta, ss, ss_stride, act_silu, gpart, gpart_floats, gpart_nsl, nullptr,
                                nprod, stream);
}

// 1x1 conv (forward, or transpose = 1: the dgrad W^T) on the sampler's dedicated split 1x1 kernel (skip_x3.hip,
// HBM-bound, its weight tile resident in LDS), with the weights packed on the device into its layout
// [cout/ntc][K/16][part][h][ntc][8] f16 - unet.hip pack_skip1x1_x3's arithmetic (hi = f16(v), part 0 = f16(hi 2^11),
// part 1 = f16((v - hi) 2^11); a part-0 value outside the f16 range sets the guard). The training step's 1x1
// convs at 256^2 ran ~1 ms each on the split conv kernel's 1x1 chunks.
__global__ void pack_skip1x1_kernel(const float* __restrict__ w, int wcout, int wcin, int transpose, int ntc, int K,
                                    _Float16* __restrict__ dst, unsigned* guard) {
  const int co_n = transpose ? wcin : wcout;  // output channels of the conv
  const int64_t tot = (int64_t)co_n * K * 2;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= tot) return;
  const int j = (int)(i & 7);
  int64_t r = i >> 3;
  const int col = (int)(r % ntc);
  r /= ntc;
  const int hh = (int)(r & 1);
  r >>= 1;
  const int part = (int)(r & 1);
  r >>= 1;
  const int ksn = K / 16;
  const int ks = (int)(r % ksn), nt = (int)(r / ksn);
  const int co = nt * ntc + col, ci = ks * 16 + hh * 8 + j;
  const int kin = transpose ? wcout : wcin;
  const float v = ci < kin ? (transpose ? w[(int64_t)ci * wcin + co] : w[(int64_t)co * wcin + ci]) : 0.f;
  const _Float16 hi = (_Float16)v;
  _Float16 o;
  if (part == 0) {
    const float sc = (float)hi * 2048.0f;
    if (!(fabsf(sc) <= 65504.0f)) atomicOr(guard, 1u);
    o = (_Float16)sc;
  } else {
    o = (_Float16)((v - (float)hi) * 2048.0f);
  }
  dst[i] = o;
}

int64_t ifd_tr_conv1x1_pack_floats(int cout, int cin, int transpose) {
  return (int64_t)(transpose ? cin : cout) * (transpose ? cout : cin);
}

int ifd_tr_conv1x1_x3(const float* x0, int c0, const float* x1, int c1, int N, int H, const float* w, int cout, int cin,
                      int transpose, const float* bias, float* out, void* wpack, int64_t wpack_floats, unsigned* guard,
                      int nprod, void* stream) {
  const int co_n = transpose ? cin : cout, K = c0 + c1;
  Skip1x1Params q{};
  q.s0 = x0; q.sc0 = c0; q.s1 = c1 ? x1 : nullptr; q.sc1 = c1;
  q.npix = N * H * H;
  q.cout = co_n;
  q.wpack = wpack; q.bias = bias; q.out = out; q.guard = guard;
  q.ntc = skip_x3_ntc(K, co_n);
  q.nprod = nprod;
  if (!w || !bias || !out || !wpack || !guard || !x0 || K != (transpose ? cout : cin) || !skip_x3_eligible(q) ||
      ifd_tr_conv1x1_pack_floats(cout, cin, transpose) > wpack_floats) {
    set_error("ifd_tr_conv1x1_x3: shape not eligible for the split 1x1 kernel (use ifd_tr_conv_x3_taps)");
    return 3;
  }
  hipStream_t s = (hipStream_t)stream;
  const int64_t tot = (int64_t)co_n * K * 2;
  hipLaunchKernelGGL(pack_skip1x1_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, w, cout, cin, transpose,
                     q.ntc, K, (_Float16*)wpack, guard);
  const int e = launch_skip_x3(q, s);
  if (e) {
    set_error(std::string("ifd_tr_conv1x1_x3: launch failed: ") + hipGetErrorString((hipError_t)e));
    return 1;
  }
  return TR_LAST();
}

int64_t ifd_tr_gstat_floats(int N, int H, int cout) {
  const int64_t HW = (int64_t)H * H;
  const int64_t E = HW >= 64 ? HW / 64 : 1;
  return (int64_t)N * (cout / 4) * E * 2;
}

int ifd_tr_conv_x3_gstat(const float* x0, int c0, const float* x1, int c1, int N, int H, const void* wx3,
                         const float* bias, int cin_pad, int cout, const float* res, float* out, float* part,
                         int64_t part_floats, unsigned* guard, int taps, float* gstat, int64_t gstat_floats,
                         int* gstat_E, float* gstat_cnt, int nprod, void* stream) {
  return conv_x3_run(x0, c0, x1, c1, N, H, wx3, bias, cin_pad, cout, res, out, part, part_floats, guard, taps,
                     gstat, gstat_floats, gstat_E, gstat_cnt, nprod, stream);
}

int ifd_tr_scale(float* x, int64_t n, float s, void* stream) {
  if (!x || n < 0) {
    set_error("ifd_tr_scale: bad arguments");
    return 2;
  }
  if (n == 0) return 0;
  hipLaunchKernelGGL(scale_kernel, dim3(grid1(n)), dim3(TB), 0, (hipStream_t)stream, x, n, s);
  return TR_LAST();
}

// split-K count of wgrad9_kernel: blocks (tiles x splits) >= ~2 per CU, >= 8 chunks per split
// pixel splits of the 64 x 64-tile weight-gradient kernels
static int wgrad_splits(int cout, int cin, int64_t P) {
  const int tiles = ((cout + 63) / 64) * ((cin + 63) / 64);
  const int64_t nch = P / 32;
  int S = 1;
  while (S < 1024 && (int64_t)tiles * S < 512 && nch / (2 * S) >= 8) S *= 2;
  return S;
}
// pixel splits of wgrad1x1_wide_kernel: three blocks per CU (768) over the (cout / 128) (cin / 128) channel tiles,
// >= 8 chunks each
static int ww_splits(int cout, int cin, int64_t P) {
  const int64_t nch = P / WW_PX;
  int64_t S = 768 / ((cout / 128) * (cin / 128));  // three blocks per CU (48 KB of LDS each)
  if (S > nch / 8) S = nch / 8;
  return S < 1 ? 1 : (int)S;
}

int64_t ifd_tr_wgrad_part_floats(int cout, int cin, int taps, int64_t P, int* splits) {
  int S = wgrad_splits(cout, cin, P);
  if (taps == 1 && ww_shape(cout, cin) && ww_splits(cout, cin, P) > S) S = ww_splits(cout, cin, P);  // (the larger plan)
  if (splits) *splits = S;
  return (int64_t)S * cout * cin * taps;
}

int ifd_tr_conv_wgrad(const float* dy, int cout, const float* x0, int c0, const float* x1, int c1, int N, int H,
                      int taps, float* dw, float* db, float* part, int64_t part_floats, float* colpart,
                      int64_t colpart_floats, void* stream) {
  const int cin = c0 + c1;
  const int64_t P = (int64_t)N * H * H;
  const int S = wgrad_splits(cout, cin, P);
  const int64_t need = (int64_t)S * cout * cin * taps;
  if (!dy || !x0 || !dw || !part || need > part_floats || c0 % 4 || (taps != 1 && taps != 9)) {
    set_error("ifd_tr_conv_wgrad: bad arguments or workspace too small");
    return 2;
  }
  WgArgs a;
  a.dy = dy; a.cout = cout; a.x0 = x0; a.c0 = c0; a.x1 = c1 ? x1 : x0; a.c1 = c1;
  a.N = N; a.H = H; a.W = H; a.taps = taps; a.P = P;
  a.part = part;
  hipStream_t s = (hipStream_t)stream;
  if (H >= 8 && (H & (H - 1)) == 0 && (!c1 || c0 % 4 == 0)) {  // wgrad9's chunking: power-of-two sizes >= 8
    const int64_t nch = P / 32;
    a.chunks_per_split = (int)((nch + S - 1) / S);
    const int tiles = ((cout + 63) / 64) * ((cin + 63) / 64);
    if (taps == 9)
      hipLaunchKernelGGL(wgrad9_kernel<9>, dim3(tiles, S), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL(wgrad9_kernel<1>, dim3(tiles, S), dim3(256), 0, s, a);
  } else {  // small maps: one tap per block (same split count; its slabs hold fewer used chunks)
    const int64_t nch = (P + WG_CH - 1) / WG_CH;
    a.chunks_per_split = (int)((nch + S - 1) / S);
    const int tiles = ((cout + 63) / 64) * ((cin + 63) / 64) * taps;
    hipLaunchKernelGGL(wgrad_kernel, dim3(tiles, S), dim3(256), 0, s, a);
  }
  const int64_t n = (int64_t)cout * cin * taps;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3(grid1(n)), dim3(TB), 0, s, part, S, n, dw, 1);
  if (db) {
    const int64_t slice = colsum_slice(P);
    const int slices = (int)((P + slice - 1) / slice);
    if (!colpart || (int64_t)slices * cout > colpart_floats) {
      set_error("ifd_tr_conv_wgrad: column-sum workspace too small");
      return 2;
    }
    hipLaunchKernelGGL(colsum_partial_kernel, dim3((cout + 63) / 64, slices), dim3(256), 0, s, dy, P, cout, slice,
                       colpart);
    hipLaunchKernelGGL(colsum_final_kernel, dim3((cout + 63) / 64), dim3(64), 0, s, colpart, slices, cout, db, 1);
  }
  return TR_LAST();
}

static int wgrad_x3_run(const float* dy, int cout, const float* x0, int c0, const float* x1, int c1, int N, int H,
                        int taps, const float* actA, const float* actB, float* dw, float* db, float* part,
                        int64_t part_floats, float* colpart, int64_t colpart_floats, unsigned* guard, int nprod,
                        void* stream);
// two sources (the output blocks' concat): the split kernels read a 64-channel input tile from one of them
static bool wgrad_x3_srcs_ok(const float* x1, int c0, int c1) { return !c1 || (x1 && c0 % 64 == 0 && c1 % 4 == 0); }

int ifd_tr_conv_wgrad_x3(const float* dy, int cout, const float* x0, int c0, const float* x1, int c1, int N, int H,
                         int taps, float* dw, float* db, float* part, int64_t part_floats, float* colpart,
                         int64_t colpart_floats, unsigned* guard, int nprod, void* stream) {
  // the split kernel: 3x3 or 1x1, one input tensor, power-of-two maps >= 8, channel counts in 16-B quads
  // (its staging loads four channels at a time); else fp32
  // (and images within a buffer descriptor's 2 GB range: the staging loads address one image each)
  const int cmax = cout > c0 + c1 ? cout : c0 + c1;
  if ((taps != 9 && taps != 1) || !wgrad_x3_srcs_ok(x1, c0, c1) || H < 8 || (H & (H - 1)) || !guard || cout % 4 ||
      c0 % 4 || (int64_t)H * H * cmax * 4 >= 0x7ffffff0)
    return ifd_tr_conv_wgrad(dy, cout, x0, c0, x1, c1, N, H, taps, dw, db, part, part_floats, colpart, colpart_floats,
                             stream);
  return wgrad_x3_run(dy, cout, x0, c0, x1, c1, N, H, taps, nullptr, nullptr, dw, db, part, part_floats, colpart,
                      colpart_floats, guard, nprod, stream);
}

int ifd_tr_conv_wgrad_x3_gn(const float* dy, int cout, const float* x0, int c0, const float* x1, int c1, int N, int H,
                            const float* actA, const float* actB, float* dw, float* db, float* part,
                            int64_t part_floats, float* colpart, int64_t colpart_floats, unsigned* guard, int nprod,
                            void* stream) {
  const int cmax = cout > c0 + c1 ? cout : c0 + c1;
  if (!actA || !actB || !wgrad_x3_srcs_ok(x1, c0, c1) || H < 8 || (H & (H - 1)) || !guard || cout % 4 || c0 % 4 ||
      (int64_t)H * H * cmax * 4 >= 0x7ffffff0) {
    set_error("ifd_tr_conv_wgrad_x3_gn: shape not eligible for the split kernel (materialise the activation)");
    return 3;
  }
  return wgrad_x3_run(dy, cout, x0, c0, x1, c1, N, H, 9, actA, actB, dw, db, part, part_floats, colpart,
                      colpart_floats, guard, nprod, stream);
}

static int wgrad_x3_run(const float* dy, int cout, const float* x0, int c0, const float* x1, int c1, int N, int H,
                        int taps, const float* actA, const float* actB, float* dw, float* db, float* part,
                        int64_t part_floats, float* colpart, int64_t colpart_floats, unsigned* guard, int nprod,
                        void* stream) {
  const int64_t P = (int64_t)N * H * H;
  const int cin = c0 + c1;
  // 1x1 over 128 x 128 channel tiles (each input tile inside one concat source): the wide kernel
  const bool wide = taps == 1 && !actA && ww_shape(cout, cin) && (!c1 || (c0 % 128 == 0 && c1 % 128 == 0)) &&
                    (H * H) % WW_PX == 0;
  const int S = wide ? ww_splits(cout, cin, P) : wgrad_splits(cout, cin, P);
  const int64_t need = (int64_t)S * cout * cin * taps;
  if (!dy || !x0 || !dw || !part || need > part_floats || (nprod != 1 && nprod != 3)) {
    set_error("ifd_tr_conv_wgrad_x3: bad arguments or workspace too small");
    return 2;
  }
  WgArgs a;
  a.dy = dy; a.cout = cout; a.x0 = x0; a.c0 = c0; a.x1 = c1 ? x1 : x0; a.c1 = c1;
  a.N = N; a.H = H; a.W = H; a.taps = taps; a.P = P;
  a.part = part;
  a.actA = actA; a.actB = actB;
  hipStream_t s = (hipStream_t)stream;
  const int64_t nch = P / (wide ? WW_PX : WX_PX);
  a.chunks_per_split = (int)((nch + S - 1) / S);
  const int tiles = ((cout + 63) / 64) * ((cin + 63) / 64);
  // bias gradient fused into the kernel when the column-sum workspace holds one row per split
  const bool fused_db = db && colpart && (int64_t)S * cout <= colpart_floats && cout % 4 == 0;
  float* cp = fused_db ? colpart : nullptr;
  const bool gna = actA != nullptr;
  const dim3 g9(tiles, S), b1(WxCfg<1>::NT);
  const dim3 gw((cout / 128) * (cin / 128), S);
  // 3x3: the warp-specialised kernel (wgrad_x3_kernel<9, ..> measured 1.98 vs 1.79 ms at 256^2 128 -> 128,
  // profiles/r04b/wgrad_exp); 1x1: wgrad_x3_kernel<1, ..>
  if (taps == 9) {
    if (nprod == 3 && gna)
      hipLaunchKernelGGL((wgrad_ws_kernel<3, true>), g9, dim3(512), 0, s, a, guard, cp);
    else if (nprod == 3)
      hipLaunchKernelGGL((wgrad_ws_kernel<3, false>), g9, dim3(512), 0, s, a, guard, cp);
    else if (gna)
      hipLaunchKernelGGL((wgrad_ws_kernel<1, true>), g9, dim3(512), 0, s, a, guard, cp);
    else
      hipLaunchKernelGGL((wgrad_ws_kernel<1, false>), g9, dim3(512), 0, s, a, guard, cp);
  } else if (wide && nprod == 3)
    hipLaunchKernelGGL((wgrad1x1_wide_kernel<3>), gw, dim3(WW_NT), 0, s, a, guard, cp);
  else if (wide)
    hipLaunchKernelGGL((wgrad1x1_wide_kernel<1>), gw, dim3(WW_NT), 0, s, a, guard, cp);
  else if (nprod == 3)
    hipLaunchKernelGGL((wgrad_x3_kernel<3>), g9, b1, 0, s, a, guard, cp);
  else
    hipLaunchKernelGGL((wgrad_x3_kernel<1>), g9, b1, 0, s, a, guard, cp);
  const int64_t n = (int64_t)cout * cin * taps;
  if (fused_db) {
    hipLaunchKernelGGL(slab_bias_reduce_kernel, dim3(grid1(n + cout)), dim3(TB), 0, s, part, S, n, dw, colpart, cout, db);
    return TR_LAST();
  }
  hipLaunchKernelGGL(slab_reduce_kernel, dim3(grid1(n)), dim3(TB), 0, s, part, S, n, dw, 1);
  if (db) {
    const int64_t slice = colsum_slice(P);
    const int slices = (int)((P + slice - 1) / slice);
    if (!colpart || (int64_t)slices * cout > colpart_floats) {
      set_error("ifd_tr_conv_wgrad_x3: column-sum workspace too small");
      return 2;
    }
    hipLaunchKernelGGL(colsum_partial_kernel, dim3((cout + 63) / 64, slices), dim3(256), 0, s, dy, P, cout, slice,
                       colpart);
    hipLaunchKernelGGL(colsum_final_kernel, dim3((cout + 63) / 64), dim3(64), 0, s, colpart, slices, cout, db, 1);
  }
  return TR_LAST();
}

int ifd_tr_gn_fwd(const float* x, int N, int HW, int C, const float* gamma, const float* beta, const float* ss,
                  int ss_stride, int act_silu, float* out, float* stats, double* work, int64_t work_doubles,
                  void* stream) {
  const int nsl = gn_nsl(HW, N, C);
  if (C % 32 || C > 1024 || (int64_t)N * nsl * 64 > work_doubles) {
    set_error("ifd_tr_gn_fwd: C must be a multiple of 32 (<= 1024), work >= N * ifd_tr_gn_slices(HW, N, C) * 64 doubles");
    return 2;
  }
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(gn_stat_partial_kernel, dim3(nsl, N), dim3(256), 0, s, x, HW, C, work);
  hipLaunchKernelGGL(gn_stat_final_kernel, dim3(N * 32), dim3(64), 0, s, work, nsl, HW, C, N, stats, GnCoef{});
  hipLaunchKernelGGL(gn_apply_kernel, dim3(nsl, N), dim3(256), 0, s, x, HW, C, stats, gamma, beta, ss,
                     ss_stride, act_silu, out);
  return TR_LAST();
}

int ifd_tr_gn_fwd_gstat(const float* x, int N, int HW, int C, const float* gamma, const float* beta, const float* ss,
                        int ss_stride, int act_silu, const float* gstat0, int C0, const float* gstat1, int E,
                        float cnt, float* out, float* stats, void* stream) {
  if (C % 128 || C > 1024 || !gstat0 || C0 % 4 || C0 <= 0 || C0 > C || (C0 < C && !gstat1) || E <= 0 ||
      (double)E * cnt != 4.0 * HW) {
    set_error("ifd_tr_gn_fwd_gstat: C must be a multiple of 128 (<= 1024), 0 < C0 <= C in quads, E * cnt == 4 * HW");
    return 2;
  }
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(gn_granule_final_kernel, dim3(N * 32), dim3(64), 0, s, gstat0, C0, gstat1, E, cnt, C, stats,
                     GnCoef{});
  const int nsl = gn_nsl(HW, N, C);
  hipLaunchKernelGGL(gn_apply_kernel, dim3(nsl, N), dim3(256), 0, s, x, HW, C, stats, gamma, beta, ss, ss_stride,
                     act_silu, out);
  return TR_LAST();
}

int64_t ifd_tr_gn_slices(int HW, int N, int C) { return gn_nsl(HW, N, C); }

int ifd_tr_gn_coef(const float* x, int N, int HW, int C, const float* gamma, const float* beta, const float* ss,
                   int ss_stride, const float* gstat0, int C0, const float* gstat1, int E, float cnt, float* stats,
                   float* A, float* B, double* work, int64_t work_doubles, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const GnCoef k{gamma, beta, ss, ss_stride, A, B};
  if (!A || !B || !gamma || !beta || C % 32 || C > 1024) {
    set_error("ifd_tr_gn_coef: C must be a multiple of 32 (<= 1024); A, B, gamma, beta required");
    return 2;
  }
  if (gstat0) {
    if (C % 128 || C0 % 4 || C0 <= 0 || C0 > C || (C0 < C && !gstat1) || E <= 0 || (double)E * cnt != 4.0 * HW) {
      set_error("ifd_tr_gn_coef: granules need C % 128 == 0, 0 < C0 <= C in quads, E * cnt == 4 * HW");
      return 2;
    }
    hipLaunchKernelGGL(gn_granule_final_kernel, dim3(N * 32), dim3(64), 0, s, gstat0, C0, gstat1, E, cnt, C, stats, k);
    return TR_LAST();
  }
  const int nsl = gn_nsl(HW, N, C);
  if (!x || (int64_t)N * nsl * 64 > work_doubles) {
    set_error("ifd_tr_gn_coef: work >= N * ifd_tr_gn_slices(HW, N, C) * 64 doubles");
    return 2;
  }
  hipLaunchKernelGGL(gn_stat_partial_kernel, dim3(nsl, N), dim3(256), 0, s, x, HW, C, work);
  hipLaunchKernelGGL(gn_stat_final_kernel, dim3(N * 32), dim3(64), 0, s, work, nsl, HW, C, N, stats, k);
  return TR_LAST();
}

int ifd_tr_act_apply(const float* x, int N, int HW, int C, const float* A, const float* B, int silu, float* out,
                     void* stream) {
  if (!x || !A || !B || !out || C % 4) {
    set_error("ifd_tr_act_apply: bad arguments");
    return 2;
  }
  return launch_act_apply(x, C, N, HW, silu ? ACT_AFFINE_SILU : ACT_AFFINE, A, B, out, (hipStream_t)stream);
}

// act + nearest-up x2 of an NHWC tensor, and the raw input's nearest-up from the same read: thread = (input pixel,
// channel quad), four 16-B stores of each (code/nn.py:92-133 after nn.py:151-152)
__global__ __launch_bounds__(256) void act_up_kernel(const float* __restrict__ x, int C, int N, int Hin,
                                                     const float* __restrict__ A, const float* __restrict__ B,
                                                     float* __restrict__ out, float* __restrict__ out_raw) {
  const int Q = C / 4, Ho = 2 * Hin;
  const size_t tot = (size_t)N * Hin * Hin * Q;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= tot) return;
  const int q = (int)(i % Q);
  const size_t pix = i / Q;
  const int xi = (int)(pix % Hin), yi = (int)((pix / Hin) % Hin), n = (int)(pix / ((size_t)Hin * Hin));
  const f32x4 v = *(const f32x4*)(x + pix * C + 4 * q);
  const f32x4 a = *(const f32x4*)(A + (size_t)n * C + 4 * q), c = *(const f32x4*)(B + (size_t)n * C + 4 * q);
  f32x4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) r[j] = silu_fast(a[j] * v[j] + c[j]);
  const size_t o = (((size_t)n * Ho + 2 * yi) * Ho + 2 * xi) * C + 4 * q;
  const size_t rs = (size_t)Ho * C;
  *(f32x4*)(out + o) = r;
  *(f32x4*)(out + o + C) = r;
  *(f32x4*)(out + o + rs) = r;
  *(f32x4*)(out + o + rs + C) = r;
  *(f32x4*)(out_raw + o) = v;
  *(f32x4*)(out_raw + o + C) = v;
  *(f32x4*)(out_raw + o + rs) = v;
  *(f32x4*)(out_raw + o + rs + C) = v;
}

int ifd_tr_act_resample(const float* x, int N, int Hin, int C, const float* A, const float* B, int mode, float* out,
                        float* out_raw, void* stream) {
  if (!x || !A || !B || !out || !out_raw || C % 4 || (mode != 1 && mode != 2) || (mode == 2 && Hin % 2)) {
    set_error("ifd_tr_act_resample: bad arguments");
    return 2;
  }
  hipStream_t s = (hipStream_t)stream;
  if (mode == 2) return launch_act_pool(x, C, N, Hin, ACT_AFFINE_SILU, A, B, out, out_raw, s);
  const size_t tot = (size_t)N * Hin * Hin * (C / 4);
  hipLaunchKernelGGL(act_up_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, x, C, N, Hin, A, B, out,
                     out_raw);
  return TR_LAST();
}

int ifd_tr_gn_bwd(const float* dout, const float* x, int N, int HW, int C, const float* gamma, const float* beta,
                  const float* ss, int ss_stride, int act_silu, const float* stats, float* dx, int accumulate,
                  float* dgamma, float* dbeta, float* dss, float* work, int64_t work_floats, void* stream) {
  return ifd_tr_gn_bwd_cat(dout, x, C, nullptr, N, HW, C, gamma, beta, ss, ss_stride, act_silu, stats, dx, accumulate,
                           dgamma, dbeta, dss, work, work_floats, nullptr, 0, nullptr, stream);
}

int ifd_tr_gn_bwd_cat(const float* dout, const float* x0, int C0, const float* x1, int N, int HW, int C,
                      const float* gamma, const float* beta, const float* ss, int ss_stride, int act_silu,
                      const float* stats, float* dx, int accumulate, float* dgamma, float* dbeta, float* dss,
                      float* work, int64_t work_floats, const float* add, int add_stride, float* dx1,
                      void* stream) {
  const int nsl = gn_nsl(HW, N, C);
  const int64_t need = (int64_t)N * nsl * C * 3 + (int64_t)N * C * 3 + (int64_t)N * 64;
  if (C % 32 || C > 1024 || need > work_floats || C0 % 4 || C0 <= 0 || C0 > C || (C0 < C && !x1)) {
    set_error("ifd_tr_gn_bwd: C must be a multiple of 32 (<= 1024), 0 < C0 <= C in quads; work too small");
    return 2;
  }
  if (add && (add_stride < C || add_stride % 4 || ((uintptr_t)add & 15))) {
    set_error("ifd_tr_gn_bwd: addend stride must be >= C, in quads, 16-B aligned");
    return 2;
  }
  if (dx1 && (C0 == C || accumulate || ((uintptr_t)dx1 & 15))) {
    set_error("ifd_tr_gn_bwd: a split output needs a concat input (C0 < C), accumulate 0, 16-B aligned");
    return 2;
  }
  GnBwdArgs a{dout, x0, N, HW, C, gamma, beta, ss, ss_stride, act_silu, stats, x1, C0};
  a.add = add;
  a.add_stride = add_stride;
  a.dx1 = dx1;
  float* part = work;
  float* nc = work + (int64_t)N * nsl * C * 3;
  float* red = nc + (int64_t)N * C * 3;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(gn_bwd_partial_kernel, dim3(nsl, N), dim3(256), 0, s, a, part);
  const int SL = gn_reduce_lanes(C);
  hipLaunchKernelGGL(gn_bwd_reduce_group_kernel, dim3(32, N), dim3(C / 32 * SL), 0, s, a, part, nsl, SL, nc, dss, red);
  hipLaunchKernelGGL(gn_bwd_dx_kernel, dim3(nsl + (C + 255) / 256, N), dim3(256), 0, s, a, red, dx, accumulate, nsl, nc,
                     dgamma, dbeta);
  return TR_LAST();
}

int ifd_tr_gn_bwd_resampled(const float* dout, const float* x, int N, int H, int C, const float* gamma,
                            const float* beta, int act_silu, const float* stats, int mode, const float* radd, float* dx,
                            float* dgamma, float* dbeta, const float* add, int add_stride, float* work,
                            int64_t work_floats, void* stream) {
  const int HW = H * H;
  const int nsl = gn_nsl(HW, N, C);
  const int64_t need = (int64_t)N * nsl * C * 3 + (int64_t)N * C * 3 + (int64_t)N * 64;
  if (C % 32 || C > 1024 || need > work_floats || (mode != 1 && mode != 2) || (mode == 2 && H % 2) ||
      (add && (add_stride < C || add_stride % 4 || ((uintptr_t)add & 15)))) {
    set_error("ifd_tr_gn_bwd_resampled: bad arguments or work too small");
    return 2;
  }
  GnBwdArgs a{dout, x, N, HW, C, gamma, beta, nullptr, 0, act_silu, stats, nullptr, C};
  a.add = add;
  a.add_stride = add_stride;
  a.rmode = mode;
  a.W = H;
  a.radd = radd;
  float* part = work;
  float* nc = work + (int64_t)N * nsl * C * 3;
  float* red = nc + (int64_t)N * C * 3;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(gn_bwd_partial_kernel, dim3(nsl, N), dim3(256), 0, s, a, part);
  const int SL = gn_reduce_lanes(C);
  hipLaunchKernelGGL(gn_bwd_reduce_group_kernel, dim3(32, N), dim3(C / 32 * SL), 0, s, a, part, nsl, SL, nc, nullptr,
                     red);
  hipLaunchKernelGGL(gn_bwd_dx_kernel, dim3(nsl + (C + 255) / 256, N), dim3(256), 0, s, a, red, dx, 0, nsl, nc,
                     dgamma, dbeta);
  return TR_LAST();
}

int ifd_tr_gn_bwd_from_part(const float* dout, const float* x0, int C0, const float* x1, int N, int HW, int C,
                            const float* gamma, const float* beta, const float* ss, int ss_stride, int act_silu,
                            const float* stats, const float* part, int part_nsl, float* dx, int accumulate,
                            float* dgamma, float* dbeta, float* dss, float* work, int64_t work_floats, const float* add,
                            int add_stride, float* dx1, void* stream) {
  const int64_t need = (int64_t)N * C * 3 + (int64_t)N * 64;
  const int nsl = gn_nsl(HW, N, C);  // the dx pass keeps its own pixel slices
  if (C % 32 || C > 1024 || need > work_floats || C0 % 4 || C0 <= 0 || C0 > C || (C0 < C && !x1) || !part ||
      part_nsl <= 0) {
    set_error("ifd_tr_gn_bwd_from_part: bad arguments or work too small");
    return 2;
  }
  if (add && (add_stride < C || add_stride % 4 || ((uintptr_t)add & 15))) {
    set_error("ifd_tr_gn_bwd: addend stride must be >= C, in quads, 16-B aligned");
    return 2;
  }
  if (dx1 && (C0 == C || accumulate || ((uintptr_t)dx1 & 15))) {
    set_error("ifd_tr_gn_bwd: a split output needs a concat input (C0 < C), accumulate 0, 16-B aligned");
    return 2;
  }
  GnBwdArgs a{dout, x0, N, HW, C, gamma, beta, ss, ss_stride, act_silu, stats, x1, C0};
  a.add = add;
  a.add_stride = add_stride;
  a.dx1 = dx1;
  float* nc = work;
  float* red = nc + (int64_t)N * C * 3;
  hipStream_t s = (hipStream_t)stream;
  const int SL = gn_reduce_lanes(C);
  hipLaunchKernelGGL(gn_bwd_reduce_group_kernel, dim3(32, N), dim3(C / 32 * SL), 0, s, a, part, part_nsl, SL, nc, dss,
                     red);
  hipLaunchKernelGGL(gn_bwd_dx_kernel, dim3(nsl + (C + 255) / 256, N), dim3(256), 0, s, a, red, dx, accumulate, nsl, nc,
                     dgamma, dbeta);
  return TR_LAST();
}

int ifd_tr_resample(const float* x, int N, int Hin, int C, int mode, float* out, void* stream) {
  if (mode != 1 && mode != 2) { set_error("ifd_tr_resample: mode 1 (up) or 2 (down)"); return 2; }
  const int Ho = mode == 1 ? 2 * Hin : Hin / 2;
  const int64_t tot = (int64_t)N * Ho * Ho * C;
  if (C % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)out & 15) == 0)
    hipLaunchKernelGGL(resample4_kernel, dim3(grid1(tot / 4)), dim3(TB), 0, (hipStream_t)stream, x, N, Hin, C, mode, out);
  else
    hipLaunchKernelGGL(resample_kernel, dim3(grid1(tot)), dim3(TB), 0, (hipStream_t)stream, x, N, Hin, C, mode, out);
  return TR_LAST();
}

int ifd_tr_resample_bwd(const float* dy, int N, int Hin, int C, int mode, float* dx, int accumulate, void* stream) {
  if (mode != 1 && mode != 2) { set_error("ifd_tr_resample_bwd: mode 1 (up) or 2 (down)"); return 2; }
  const int64_t tot = (int64_t)N * Hin * Hin * C;
  if (C % 4 == 0 && ((uintptr_t)dy & 15) == 0 && ((uintptr_t)dx & 15) == 0)
    hipLaunchKernelGGL(resample4_bwd_kernel, dim3(grid1(tot / 4)), dim3(TB), 0, (hipStream_t)stream, dy, N, Hin, C,
                       mode, dx, accumulate);
  else
    hipLaunchKernelGGL(resample_bwd_kernel, dim3(grid1(tot)), dim3(TB), 0, (hipStream_t)stream, dy, N, Hin, C, mode,
                       dx, accumulate);
  return TR_LAST();
}

int ifd_tr_add(const float* a, const float* b, float* out, int64_t n, void* stream) {
  if (n % 4 == 0 && (((uintptr_t)a | (uintptr_t)b | (uintptr_t)out) & 15) == 0)
    hipLaunchKernelGGL(add4_kernel, dim3(grid1(n / 4)), dim3(TB), 0, (hipStream_t)stream, a, b, out, n);
  else
    hipLaunchKernelGGL(add_kernel, dim3(grid1(n)), dim3(TB), 0, (hipStream_t)stream, a, b, out, n);
  return TR_LAST();
}

int ifd_tr_copy_channels(const float* src, int cs, int soff, float* dst, int cd, int doff, int nc, int64_t npix,
                         int accumulate, void* stream) {
  if (soff + nc > cs || doff + nc > cd) { set_error("ifd_tr_copy_channels: channel range"); return 2; }
  const bool v4 = cs % 4 == 0 && soff % 4 == 0 && cd % 4 == 0 && doff % 4 == 0 && nc % 4 == 0 &&
                  ((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0;
  if (v4)
    hipLaunchKernelGGL(copy_channels4_kernel, dim3(grid1(npix * nc / 4)), dim3(TB), 0, (hipStream_t)stream, src, cs,
                       soff, dst, cd, doff, nc, npix, accumulate);
  else
    hipLaunchKernelGGL(copy_channels_kernel, dim3(grid1(npix * nc)), dim3(TB), 0, (hipStream_t)stream, src, cs, soff,
                       dst, cd, doff, nc, npix, accumulate);
  return TR_LAST();
}

int ifd_tr_attention(const float* qkv, int N, int T, int C, float scale, float* out, void* stream) {
  if (C % 64) { set_error("ifd_tr_attention: 64-channel heads"); return 2; }
  launch_attention(qkv, N, T, C, scale, out, (hipStream_t)stream);
  return TR_LAST();
}

int64_t ifd_tr_attention_bwd_scratch_floats(int N, int T, int C) { return 2 * (int64_t)N * (C / 64) * T * T; }

int ifd_tr_attention_bwd(const float* qkv, const float* dout, int N, int T, int C, float scale, float* dqkv,
                         float* scratch, int64_t scratch_floats, void* stream) {
  const int nh = C / 64;
  if (C % 64 || T > 1024 || ifd_tr_attention_bwd_scratch_floats(N, T, C) > scratch_floats) {
    set_error("ifd_tr_attention_bwd: bad arguments or scratch too small");
    return 2;
  }
  float* Pm = scratch;
  float* dS = scratch + (int64_t)N * nh * T * T;
  hipStream_t s = (hipStream_t)stream;
  if (T == 256 || T == 128 || T == 64 || T == 32) {  // the MFMA kernels (the VALU ones for other T)
    if (T == 256) launch_attn_bwd_mfma<8>(qkv, dout, N, C, scale, dqkv, Pm, dS, s);
    if (T == 128) launch_attn_bwd_mfma<4>(qkv, dout, N, C, scale, dqkv, Pm, dS, s);
    if (T == 64) launch_attn_bwd_mfma<2>(qkv, dout, N, C, scale, dqkv, Pm, dS, s);
    if (T == 32) launch_attn_bwd_mfma<1>(qkv, dout, N, C, scale, dqkv, Pm, dS, s);
    return TR_LAST();
  }
  dim3 g((T + AB_R - 1) / AB_R, nh, N);
  const size_t lds = ((size_t)2 * AB_R * T + 2 * AB_R * 64) * sizeof(float);
  if (lds > 160 * 1024) {
    set_error("ifd_tr_attention_bwd: T too large for the row kernel's LDS");
    return 2;
  }
  static bool attr[kMaxDevices] = {};
  (void)set_lds_attr_once(attr, reinterpret_cast<const void*>(&attn_bwd_rows_kernel), (int)lds);
  hipLaunchKernelGGL(attn_bwd_rows_kernel, g, dim3(256), lds, s, qkv, dout, T, C, scale, dqkv, Pm, dS);
  hipLaunchKernelGGL(attn_bwd_cols_kernel, g, dim3(256), 0, s, qkv, dout, T, C, scale, dqkv, Pm, dS);
  return TR_LAST();
}

int ifd_tr_linear(const float* x, int M, int K, const float* w, const float* b, int N, int pre_silu, int post_silu,
                  float* y, void* stream) {
  hipLaunchKernelGGL(linear_kernel, dim3(grid1((int64_t)M * N * 64)), dim3(TB), 0, (hipStream_t)stream, x, M, K, w, b,
                     N, pre_silu, post_silu, y);
  return TR_LAST();
}

int ifd_tr_linear_bwd(const float* dy, const float* x, int M, int K, const float* w, int N, int pre_silu, float* dx,
                      int dx_accumulate, float* dw, float* db, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (dx)
    hipLaunchKernelGGL(linear_dx_kernel, dim3(M * ((K + 63) / 64)), dim3(64 * LDX_Q), 0, s, dy, x, M, K, w, N, pre_silu, dx,
                       dx_accumulate);
  if (dw)
    hipLaunchKernelGGL(linear_dw_kernel, dim3(grid1((int64_t)N * K)), dim3(TB), 0, s, dy, x, M, K, N, pre_silu, dw, db);
  return TR_LAST();
}

int ifd_tr_silu_bwd(const float* z, const float* dy, float* dz, int64_t n, void* stream) {
  hipLaunchKernelGGL(silu_bwd_kernel, dim3(grid1(n)), dim3(TB), 0, (hipStream_t)stream, z, dy, dz, n);
  return TR_LAST();
}

int ifd_tr_temb(const int64_t* t, const float* freqs, int N, int dim, float* out, void* stream) {
  hipLaunchKernelGGL(temb_kernel, dim3(grid1(N * dim)), dim3(TB), 0, (hipStream_t)stream, t, freqs, N, dim, out);
  return TR_LAST();
}

int ifd_tr_pack_input(const float* x, const float* masked_image, const float* mask, int N, int HW, float* out16,
                      void* stream) {
  launch_pack_input(x, masked_image, mask, 0, N, HW, out16, (hipStream_t)stream);
  return TR_LAST();
}

int ifd_tr_q_sample_inject(const float* x0, const float* noise, const float* cached, const float* mask,
                           const int64_t* t, const float* sqrt_ac, const float* sqrt_1m_ac, int N, int HW, int inject,
                           float* xt, void* stream) {
  const int64_t tot = (int64_t)N * 3 * HW;
  hipLaunchKernelGGL(q_sample_inject_kernel, dim3(grid1(tot)), dim3(TB), 0, (hipStream_t)stream, x0, noise, cached,
                     mask, t, sqrt_ac, sqrt_1m_ac, N, HW, inject, xt);
  return TR_LAST();
}

int ifd_tr_masked_mse(const float* out6_nhwc, int cs, const float* noise, const float* mask, int N, int HW,
                      float* loss, float* dout6_nhwc, float* work, void* stream) {
  if (cs < 3) { set_error("ifd_tr_masked_mse: channel stride < 3"); return 2; }
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(mse_partial_kernel, dim3(N * 3), dim3(256), 0, s, out6_nhwc, cs, noise, mask, HW, work);
  hipLaunchKernelGGL(mse_final_kernel, dim3(1), dim3(64), 0, s, work, N * 3, loss);
  if (dout6_nhwc)
    hipLaunchKernelGGL(mse_grad_kernel, dim3(grid1((int64_t)N * HW * cs)), dim3(TB), 0, s, out6_nhwc, cs, noise, mask,
                       work, N, HW, dout6_nhwc);
  return TR_LAST();
}

int ifd_tr_clip_adamw(float* p, float* g, float* m, float* v, int64_t n, float max_norm, double lr, double b1, double b2,
                      double eps, double wd, int step, double* work, float* norm_coef, void* stream) {
  if (step < 1 || !work || !norm_coef) { set_error("ifd_tr_clip_adamw: bad arguments"); return 2; }
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(sumsq_partial_kernel, dim3(SQ_BLOCKS), dim3(256), 0, s, g, n, work);
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(64), 0, s, work, SQ_BLOCKS, max_norm, norm_coef);
  const double bc1 = 1.0 - std::pow(b1, step);
  const float bc2s = (float)std::sqrt(1.0 - std::pow(b2, step));
  hipLaunchKernelGGL(adamw_kernel, dim3(grid1(n)), dim3(TB), 0, s, p, g, m, v, n, norm_coef, (float)(1.0 - lr * wd),
                     (float)(1.0 - b1), (float)b2, (float)(1.0 - b2), (float)(lr / bc1), (float)eps, bc2s);
  return TR_LAST();
}

}  // extern "C"
