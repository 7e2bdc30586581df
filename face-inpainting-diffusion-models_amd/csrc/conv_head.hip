// Output head of the UNet (code/unet.py:196-200, `out`: GroupNorm -> SiLU -> conv 3x3 ch -> 6):
// fp32 VALU direct convolution with the GroupNorm-apply + SiLU prologue and the NCHW / fused
// sampler-step epilogues of conv.hip.
//
// Why not the MFMA conv kernels: cout = 6 (or 3) fills 6/32 of a 32-wide MFMA tile and the fp32
// MFMA rate equals the fp32 VALU rate on gfx950 (MI355X_MICROARCH.md), so a GEMM tiling wastes
// ~5x. Here each thread owns a column of 4 output pixels and keeps their 4 x 6 accumulators as
// channel pairs; every MAC pair is one v_pk_fma_f32 (the input value broadcast to both halves,
// two output channels' weights from a broadcast LDS read), the packed rate being the full fp32
// VALU rate. Per 8-channel chunk a block stages the activated 34 x 34 halo of its 32 x 32 tile
// (2 quad planes [pixel][4 ch]: a wave's ds_read_b128 of 64 consecutive pixels is conflict-free)
// and the chunk's weights in LDS; a thread reads each halo column of 6 rows once for its
// 3 x 4 (tap row, pixel) uses. The next chunk's halo loads are in flight in registers.
//
// Bound: VALU. Per output pixel 9 * cin * cout FMAs (13.8 kFLOP for cin 128, cout 6) against
// ~0.6 KB of HBM traffic (4 * cin B of input + the step epilogue's 64 B): 23 FLOP/B, above the
// 157 TF/s : 8 TB/s balance point of ~20 FLOP/B. (The first version read the weights by scalar
// loads: at 27 KB they miss the scalar cache and every wait exposed its latency, 39 TFLOP/s.)
#include <hip/hip_runtime.h>

#include <cmath>

#include "conv.h"
#include "conv_dev.h"

namespace ifd {
namespace {

constexpr int HD_TW = 32, HD_TH = 32;                          // output tile (one image)
constexpr int HD_HW = HD_TW + 2, HD_NP = HD_HW * (HD_TH + 2);  // 34 x 34 = 1156 halo pixels
constexpr int HD_NT = 256;                                     // one thread per 4 output pixels
constexpr int HD_PX = 4;                                       // pixels (rows) per thread
constexpr int HD_CH = 8;                                       // channels per chunk
constexpr int HD_ITEMS = (HD_NP * 2 + HD_NT - 1) / HD_NT;      // (pixel, quad) items per thread: 10
typedef float f32x2 __attribute__((ext_vector_type(2)));

// wh: [cin/8][9 taps][8 ci][8] fp32 (co 0..cout-1, zero padded), bias = p.bias
template <int CO>
__global__ __launch_bounds__(HD_NT, 2) void conv_head_kernel(ConvParams p, const float* __restrict__ wh) {
  static_assert(CO % 2 == 0 || CO == 3, "channel pairs");
  constexpr int CP = (CO + 1) / 2;                                 // output channel pairs
  __shared__ __attribute__((aligned(16))) float hal[2][HD_NP][4];  // quad plane q: [pixel][4 channels]
  __shared__ __attribute__((aligned(16))) float wl[9 * HD_CH * 8];  // the chunk's weights
  const int tid = threadIdx.x;
  const int tiles_x = p.W / HD_TW, tiles_y = p.H / HD_TH;
  int b = blockIdx.x;
  const int tx = b % tiles_x;
  b /= tiles_x;
  const int ty = b % tiles_y;
  const int n = b / tiles_y;
  const int x0 = tx * HD_TW, y0 = ty * HD_TH;
  const int cin = p.c0;
  const int nchunk = cin / HD_CH;
  const float* __restrict__ src = p.in0 + (size_t)n * p.H * p.W * cin;

  // staging items: item i = (halo pixel i >> 1, channel quad i & 1); quad = tid & 1 for every item
  const int q = tid & 1;
  int goff[HD_ITEMS];
  bool inb[HD_ITEMS];
#pragma unroll
  for (int k = 0; k < HD_ITEMS; ++k) {
    const int i = tid + k * HD_NT;
    const int pix = i >> 1;
    const int hy = pix / HD_HW, hx = pix - hy * HD_HW;
    const int y = y0 + hy - 1, x = x0 + hx - 1;
    inb[k] = i < 2 * HD_NP && y >= 0 && y < p.H && x >= 0 && x < p.W;
    goff[k] = inb[k] ? (y * p.W + x) * cin + 4 * q : 0;
  }
  f32x4 raw[HD_ITEMS];
  auto load = [&](int ch) {
#pragma unroll
    for (int k = 0; k < HD_ITEMS; ++k)
      raw[k] = inb[k] ? gld4(src + goff[k] + HD_CH * ch) : f32x4{0.f, 0.f, 0.f, 0.f};
  };
  auto stage = [&](int ch) {
    f32x4 ca = {1.f, 1.f, 1.f, 1.f}, cb = {0.f, 0.f, 0.f, 0.f};
    if (p.act != ACT_NONE) {
      ca = gld4(p.actA + (size_t)n * cin + HD_CH * ch + 4 * q);
      cb = gld4(p.actB + (size_t)n * cin + HD_CH * ch + 4 * q);
    }
#pragma unroll
    for (int k = 0; k < HD_ITEMS; ++k) {
      const int i = tid + k * HD_NT;
      if (i < 2 * HD_NP) {
        f32x4 v;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float t = raw[k][c];
          if (p.act != ACT_NONE) {
            t = ca[c] * t + cb[c];
            if (p.act == ACT_AFFINE_SILU) t = silu_fast(t);
          }
          v[c] = inb[k] ? t : 0.f;  // zero padding of the activated input
        }
        *(f32x4*)&hal[q][i >> 1][0] = v;
      }
    }
    for (int i = tid; i < 9 * HD_CH * 2; i += HD_NT)  // 576 weights as float4
      *(f32x4*)&wl[4 * i] = gld4(wh + (size_t)ch * 9 * HD_CH * 8 + 4 * i);
  };

  const int px = tid % HD_TW, py = HD_PX * (tid / HD_TW);  // pixels (py .. py + 3, px)
  const int hp = py * HD_HW + px;                           // halo pixel of tap (0, 0) of the first
  f32x2 acc[HD_PX][CP];
#pragma unroll
  for (int r = 0; r < HD_PX; ++r)
#pragma unroll
    for (int c = 0; c < CP; ++c) acc[r][c] = f32x2{0.f, 0.f};

  load(0);
  for (int ch = 0; ch < nchunk; ++ch) {
    __syncthreads();  // the previous chunk's reads are done
    stage(ch);
    __syncthreads();
    if (ch + 1 < nchunk) load(ch + 1);  // in flight during this chunk's FMAs
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        f32x4 v[HD_PX + 2];  // halo rows py .. py + 5 of column px + dx
#pragma unroll
        for (int hr = 0; hr < HD_PX + 2; ++hr) v[hr] = *(const f32x4*)&hal[qq][hp + hr * HD_HW + dx][0];
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int dy = 0; dy < 3; ++dy) {
            const float* wr = wl + ((dy * 3 + dx) * HD_CH + 4 * qq + c) * 8;
            const f32x4 w03 = *(const f32x4*)wr;
            const f32x4 w47 = *(const f32x4*)(wr + 4);
            const f32x2 wp[4] = {f32x2{w03[0], w03[1]}, f32x2{w03[2], w03[3]}, f32x2{w47[0], w47[1]},
                                 f32x2{w47[2], w47[3]}};
#pragma unroll
            for (int r = 0; r < HD_PX; ++r) {
              const float x = v[dy + r][c];
#pragma unroll
              for (int cp = 0; cp < CP; ++cp)
                acc[r][cp] = __builtin_elementwise_fma(f32x2{x, x}, wp[cp], acc[r][cp]);
            }
          }
      }
    }
  }

  // epilogue (conv.hip's NCHW / DDIM / DDPM paths)
  const int HWp = p.H * p.W;
#pragma unroll
  for (int r = 0; r < HD_PX; ++r) {
    float a[2 * CP];
#pragma unroll
    for (int cp = 0; cp < CP; ++cp) {
      a[2 * cp] = acc[r][cp][0];
      a[2 * cp + 1] = acc[r][cp][1];
    }
    const size_t pix = (size_t)(y0 + py + r) * p.W + (x0 + px);
    if (p.epi == EPI_NCHW) {
#pragma unroll
      for (int co = 0; co < CO; ++co) p.out[((size_t)n * CO + co) * HWp + pix] = a[co] + p.bias[co];
      continue;
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const size_t o3 = ((size_t)n * 3 + c) * HWp + pix;
      const size_t om = (size_t)n * HWp + pix;
      const float eps = a[c] + p.bias[c];
      const float x = p.img[o3];
      const float mk = p.sc.inject ? p.mask[om] : 0.f;
      const float g = p.sc.inject ? p.gt[o3] : 0.f;
      const float kn = p.sc.inject ? p.known[o3] : 0.f;
      float v;
      if (p.epi == EPI_DDIM) {
        const float nz = p.sc.use_noise ? p.noise[o3] : 0.f;
        v = ddim_step_value(p.sc, x, eps, nz, g, mk, kn);
      } else {
        const float var_v = a[CO > 3 ? c + 3 : c] + p.bias[c + 3];
        v = ddpm_step_value(p.sc, x, eps, var_v, p.noise[o3], g, mk, kn);
      }
      p.img[o3] = v;
    }
  }
}


// ---- 3xf16 output head (the 3xf16 precision mode): the same conv on f16 MFMAs with split operands ----
// The VALU head above reaches ~40 TFLOP/s (0.36 ms per eval at B = 16). Here a persistent block per CU keeps
// ALL the head's split weights in LDS ([chunk][tap][part][8 co][32 ch] f16: 36 KiB for 128 channels, co 6, 7
// zero) and walks 16 x 16-pixel tiles in 32-channel chunks, warp-specialised:
// * waves 4-11 (producers, two per SIMD) stage chunk s — the activated, split 18 x 18 halo ([part][px][32 ch]
//   f16, conv_x3.hip's split: the same roundings) — into halo buffer s & 1, with two register sets of loads
//   (chunk s + 2's issued right after chunk s is staged);
// * waves 0-3 (consumers) run chunk s - 1 from the other buffer: wave w computes tile rows 4w..4w+3 as
//   16-pixel M blocks with v_mfma_f32_16x16x32_f16 (N = 16 output channels, 6 used), three split products
//   per MAC as conv_x3.hip (weights x 2^11), hi x hi and the corrections in separate accumulators;
// * one block barrier per chunk step. A finished tile's accumulators go through a transpose buffer (two, by
//   tile parity) to the producers, which run the per-pixel epilogue (bias, NCHW / NHWC store or the fused
//   DDIM / DDPM step) in the next step, its inputs loaded before that step's staging.
// Every producer load is unconditional (padding pixels load a clamped neighbour, the steps past the last
// chunk re-load it): with loads under branches hipcc's waitcnt merge fell back to vmcnt(0) and drained the
// prefetch. (gfx950 counts global stores in vmcnt too.)
// What bounds it (timing ablations): the producers' staging VALU — ~40 issue cycles per
// staged value (affine, exp2, rcp, split) sharing each SIMD's issue with the consumers' MFMAs, which hold it
// 8 of every 16 cycles. Without the staging the head takes 0.13 instead of 0.23 ms per eval; without its
// loads 0.19; without the MFMAs 0.20. The round-2 layout (two 256-thread blocks per CU, staging and MFMAs
// serialised by barriers) ran 0.234 ms; four producer waves 0.25.
constexpr int HX_T = 16;                                  // tile 16 x 16
constexpr int HX_HW = HX_T + 2, HX_NP = HX_HW * HX_HW;  // 324 halo pixels
constexpr int HX_CH = 32;                                 // channels per chunk (one MFMA k-step)
constexpr int HX_MAXCH = 4;                               // chunks held in LDS (cin <= 128)
constexpr int HX_WCO = 8;                                 // packed output channels (6 used; B lanes 8..15 read zeros)
constexpr int HX_WCH = 9 * 2 * HX_WCO * HX_CH;            // f16 per chunk of packed weights
constexpr int HX_Z = 32;                                  // a zero row for the unused B lanes
typedef _Float16 hx_h8 __attribute__((ext_vector_type(8)));
typedef float hx_f4 __attribute__((ext_vector_type(4)));
typedef unsigned hx_u2 __attribute__((ext_vector_type(2)));

#define HX_BARRIER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")
constexpr int HW_PT = 8 * 64;                          // producer threads (two waves per SIMD)
constexpr int HW_NT = 256 + HW_PT;                    // 4 consumer + 8 producer waves
constexpr int HW_ITEMS = (HX_NP * 8 + HW_PT - 1) / HW_PT;  // (pixel, quad) staging items per producer thread
constexpr int HW_NPP = HW_ITEMS * HW_PT / 8;  // halo rows per plane incl. the last items' spill rows
constexpr int HW_A = 2 * HW_NPP * HX_CH;  // f16 per halo stage
constexpr int HW_OB = 256 * HX_WCO;       // floats per transpose buffer
static_assert(HW_NPP >= HX_NP && HW_NPP % 8 == 0, "staging items fit the padded plane");
// weights + zero row + two halo stages + two transpose buffers (150 KiB with 8 producer waves), one block per CU
constexpr size_t HW_LDS = (size_t)(HX_MAXCH * HX_WCH + HX_Z + 2 * HW_A) * 2 + 2 * HW_OB * 4;

// conv_x3.hip's split2: hi = f16(v) for the pair (one v_cvt_pk_f16_f32), lo = f16(v - hi) by v_fma_mix (v - hi
// exact in fp32, rounded once): the values of two casts in 1.5 instead of ~4 VALU ops per value
typedef _Float16 hx_h2 __attribute__((ext_vector_type(2)));
typedef float hx_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void hx_split2(float v0, float v1, unsigned& h, unsigned& l) {
  asm volatile("" : "+v"(v0), "+v"(v1));
  h = __builtin_bit_cast(unsigned, __builtin_convertvector(hx_f2{v0, v1}, hx_h2));
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%3 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %2, 1.0, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(l)
      : "v"(v0), "v"(v1), "v"(h));
}

template <int CO, int ACT, int EPI>
__global__ __launch_bounds__(HW_NT, 1) void conv_head_x3ws_kernel(ConvParams p, const _Float16* __restrict__ wx) {
  extern __shared__ __attribute__((aligned(16))) char hx_smem[];
  _Float16* Wl = reinterpret_cast<_Float16*>(hx_smem);
  _Float16* Zl = Wl + HX_MAXCH * HX_WCH;
  _Float16* Al0 = Zl + HX_Z;                               // halo stage 0; stage 1 follows
  float* Ob0 = reinterpret_cast<float*>(Al0 + 2 * HW_A);  // transpose buffer 0; buffer 1 follows
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cin = p.c0, nch = cin / HX_CH;
  const int tiles_x = p.W / HX_T, tiles_y = p.H / HX_T;
  const int ntiles = p.N * tiles_x * tiles_y;
  {
    const hx_f4* src = reinterpret_cast<const hx_f4*>(wx);
    hx_f4* dst = reinterpret_cast<hx_f4*>(Wl);
    for (int i = tid; i < nch * HX_WCH / 8; i += HW_NT) dst[i] = src[i];
    if (tid < HX_Z / 8) reinterpret_cast<hx_f4*>(Zl)[tid] = hx_f4{0.f, 0.f, 0.f, 0.f};
  }
  auto tile_of = [&](int t, int& n, int& y0, int& x0) {
    x0 = (t % tiles_x) * HX_T;
    t /= tiles_x;
    y0 = (t % tiles_y) * HX_T;
    n = t / tiles_y;
  };
  const int nwork = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;  // >= 1 (grid <= ntiles)
  const int nsteps = nwork * nch;  // chunk steps of this block
  // step s: producers stage chunk s; consumers compute chunk s - 1; producers finish the tile whose last chunk
  // was computed in step s - 1. Every wave runs the same (even) number of steps, one barrier each.
  const int T = (nsteps + 3) & ~1;
  if (wave >= 4) {
    const int ptid = tid - 256;
    const int q = ptid & 7;
    int hyv[HW_ITEMS], hxv[HW_ITEMS], ldo[HW_ITEMS];
#pragma unroll
    for (int k = 0; k < HW_ITEMS; ++k) {
      const int px = (ptid + HW_PT * k) >> 3;  // rows past the halo (the last item) are staged into spill rows
      hyv[k] = px < HX_NP ? px / HX_HW : 0;
      hxv[k] = px < HX_NP ? px % HX_HW : 0;
      ldo[k] = px * HX_CH + 4 * q;
    }
    hx_f4 raw0[HW_ITEMS], raw1[HW_ITEMS], ca0, cb0, ca1, cb1;
    float gmax = 0.f;
    float bias[HX_WCO];  // in registers: read in the epilogue it would be re-read after every store (may alias)
#pragma unroll
    for (int co = 0; co < HX_WCO; ++co) bias[co] = co < (EPI == EPI_NHWC ? HX_WCO : CO) ? p.bias[co] : 0.f;
    auto load = [&](hx_f4 (&raw)[HW_ITEMS], hx_f4& ca, hx_f4& cb, int s) __attribute__((always_inline)) {
      const int se = s < nsteps ? s : nsteps - 1;  // past the end: the last chunk again (unused)
      int n, y0, x0;
      const int c = se % nch;
      tile_of(blockIdx.x + (se / nch) * gridDim.x, n, y0, x0);
      if (ACT != ACT_NONE) {  // the coefficients first: older than the halo loads in the queue
        ca = *reinterpret_cast<const hx_f4*>(p.actA + (size_t)n * cin + HX_CH * c + 4 * q);
        cb = *reinterpret_cast<const hx_f4*>(p.actB + (size_t)n * cin + HX_CH * c + 4 * q);
      }
      const float* src = p.in0 + (size_t)n * p.H * p.W * cin + HX_CH * c + 4 * q;
#pragma unroll
      for (int k = 0; k < HW_ITEMS; ++k) {
        const int y = min(max(y0 + hyv[k] - 1, 0), p.H - 1), x = min(max(x0 + hxv[k] - 1, 0), p.W - 1);
        raw[k] = *reinterpret_cast<const hx_f4*>(src + ((size_t)y * p.W + x) * cin);
      }
    };
    auto stage = [&](const hx_f4 (&raw)[HW_ITEMS], hx_f4 ca, hx_f4 cb, int s) __attribute__((always_inline)) {
      int n, y0, x0;
      tile_of(blockIdx.x + (s / nch) * gridDim.x, n, y0, x0);
      _Float16* Al = Al0 + (s & 1) * HW_A;
#pragma unroll
      for (int k = 0; k < HW_ITEMS; ++k) {
        const int y = y0 + hyv[k] - 1, x = x0 + hxv[k] - 1;
        const bool ok = y >= 0 && y < p.H && x >= 0 && x < p.W;
        float v[4];
        if (ACT == ACT_AFFINE_SILU) {
          // the zero padding rides in the exponent (conv_x3.hip store_act): 2^(+inf) = inf, rcp(1 + inf) = 0
          const float pinf = ok ? 0.f : __builtin_inff();
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float t = fmaf(ca[j], raw[k][j], cb[j]);
            v[j] = t * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(fmaf(t, -1.4426950408889634f, pinf)));
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = ok ? (ACT == ACT_AFFINE ? fmaf(ca[j], raw[k][j], cb[j]) : raw[k][j]) : 0.f;
        }
        gmax = fmaxf(gmax, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
        unsigned h0, l0, h1, l1;
        hx_split2(v[0], v[1], h0, l0);
        hx_split2(v[2], v[3], h1, l1);
        *reinterpret_cast<hx_u2*>(Al + ldo[k]) = hx_u2{h0, h1};
        *reinterpret_cast<hx_u2*>(Al + HW_NPP * HX_CH + ldo[k]) = hx_u2{l0, l1};
      }
    };
    constexpr bool kStep = EPI == EPI_DDIM || EPI == EPI_DDPM;
    const int HWp = p.H * p.W;
    // the step epilogue's optional inputs read a valid stand-in when absent (no branch around the loads)
    const float* gt_p = p.sc.inject ? p.gt : p.img;
    const float* kn_p = p.sc.inject ? p.known : p.img;
    const float* mk_p = p.sc.inject ? p.mask : p.img;
    const float* nz_p = (EPI == EPI_DDPM || p.sc.use_noise) ? p.noise : p.img;
    auto step = [&](hx_f4 (&raw)[HW_ITEMS], hx_f4& ca, hx_f4& cb, int s) __attribute__((always_inline)) {
      // (the first 256 producer threads finish one pixel each)
      const bool epi = s >= 2 && s - 2 < nsteps && (s - 2) % nch == nch - 1 && ptid < 256;
      int je = (s - 2) / nch;
      je = je < 0 ? 0 : (je >= nwork ? nwork - 1 : je);
      int n, y0, x0;
      tile_of(blockIdx.x + je * gridDim.x, n, y0, x0);
      const int pt = ptid & 255;
      const size_t pix = (size_t)(y0 + (pt >> 4)) * p.W + (x0 + (pt & 15));
      float xi[3], gi[3], kn[3], nz[3], mk = 0.f;
      if (kStep) {  // loaded every step (a stand-in tile when no epilogue is due)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const size_t o3 = ((size_t)n * 3 + c) * HWp + pix;
          xi[c] = p.img[o3];
          gi[c] = gt_p[o3];
          kn[c] = kn_p[o3];
          nz[c] = nz_p[o3];
        }
        mk = mk_p[p.sc.inject ? (size_t)n * HWp + pix : ((size_t)n * 3) * HWp + pix];
      }
      if (s < nsteps) stage(raw, ca, cb, s);
      load(raw, ca, cb, s + 2);
      if (epi) {
        const float* Ob = Ob0 + (je & 1) * HW_OB;
        float a[8];
#pragma unroll
        for (int co = 0; co < 8; ++co) a[co] = Ob[pt * 8 + co];
        if (EPI == EPI_NCHW) {
#pragma unroll
          for (int co = 0; co < CO; ++co) p.out[((size_t)n * CO + co) * HWp + pix] = a[co] + bias[co];
        } else if (EPI == EPI_NHWC) {  // the training forward: [N][H][W][8], the padded channels' rows zero
          hx_f4* o = reinterpret_cast<hx_f4*>(p.out + ((size_t)n * HWp + pix) * HX_WCO);
          o[0] = hx_f4{a[0] + bias[0], a[1] + bias[1], a[2] + bias[2], a[3] + bias[3]};
          o[1] = hx_f4{a[4] + bias[4], a[5] + bias[5], a[6] + bias[6], a[7] + bias[7]};
        } else {
          if (!p.sc.inject) mk = 0.f;
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const size_t o3 = ((size_t)n * 3 + c) * HWp + pix;
            const float eps = a[c] + bias[c];
            const float g = p.sc.inject ? gi[c] : 0.f, k = p.sc.inject ? kn[c] : 0.f;
            float v;
            if (EPI == EPI_DDIM) {
              v = ddim_step_value(p.sc, xi[c], eps, p.sc.use_noise ? nz[c] : 0.f, g, mk, k);
            } else {
              const float var_v = a[CO > 3 ? c + 3 : c] + bias[c + 3];
              v = ddpm_step_value(p.sc, xi[c], eps, var_v, nz[c], g, mk, k);
            }
            p.img[o3] = v;
          }
        }
      }
      HX_BARRIER();
    };
    load(raw0, ca0, cb0, 0);
    load(raw1, ca1, cb1, 1);
    // unrolled by two so each register set has one static name
    for (int s = 0; s < T; s += 2) {
      step(raw0, ca0, cb0, s);
      step(raw1, ca1, cb1, s + 1);
    }
    if (p.guard && gmax >= 65504.0f) atomicOr(p.guard, 1u);
    return;
  }
  // consumers. MFMA lane roles (16x16x32): A lane = pixel i (lane & 15) of a tile row, K group kg = lane >> 4
  // (channels 8 kg .. 8 kg + 7); B lane = output channel j (lane & 15), same K group; C lane = channel j,
  // pixels 4 kg .. 4 kg + 3 of the row
  const int li = lane & 15, kg = lane >> 4;
  hx_f4 acc[4], accl[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) acc[r] = accl[r] = hx_f4{0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < T; ++s) {
    if (s >= 1 && s <= nsteps) {
      const int cs = s - 1, c = cs % nch;
      const _Float16* Al = Al0 + (cs & 1) * HW_A;
      const _Float16* Wc = Wl + c * HX_WCH;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        hx_h8 ah[6], al[6];
#pragma unroll
        for (int rr = 0; rr < 6; ++rr) {
          const int hp = (4 * wave + rr) * HX_HW + li + kx;
          ah[rr] = *reinterpret_cast<const hx_h8*>(Al + hp * HX_CH + 8 * kg);
          al[rr] = *reinterpret_cast<const hx_h8*>(Al + HW_NPP * HX_CH + hp * HX_CH + 8 * kg);
        }
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const int tap = 3 * ky + kx;
          const _Float16* bp0 = li < HX_WCO ? Wc + ((tap * 2 + 0) * HX_WCO + li) * HX_CH + 8 * kg : Zl;
          const _Float16* bp1 = li < HX_WCO ? Wc + ((tap * 2 + 1) * HX_WCO + li) * HX_CH + 8 * kg : Zl;
          const hx_h8 bh = *reinterpret_cast<const hx_h8*>(bp0);
          const hx_h8 bl = *reinterpret_cast<const hx_h8*>(bp1);
          // one consumer wave per SIMD: the products grouped by kind, so each accumulator's next MFMA is four
          // MFMAs behind its last
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[r + ky], bh, acc[r], 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 4; ++r) accl[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[r + ky], bl, accl[r], 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 4; ++r) accl[r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[r + ky], bh, accl[r], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (c == nch - 1) {
        // Ob[pixel][channel], pixel = tile row (4 wave + r) x 16 + column (4 kg + e): the producers read it in
        // the next step
        float* Ob = Ob0 + ((cs / nch) & 1) * HW_OB;
        if (li < 8)
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              Ob[((4 * wave + r) * HX_T + 4 * kg + e) * 8 + li] = (acc[r][e] + accl[r][e]) * (1.0f / 2048.0f);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = accl[r] = hx_f4{0.f, 0.f, 0.f, 0.f};
      }
    }
    HX_BARRIER();
  }
}
}  // namespace

bool conv_head_eligible(const ConvParams& p, int taps, int xform) {
  const bool step = p.epi == EPI_DDIM || p.epi == EPI_DDPM;
  return taps == 9 && xform == XF_NONE && !p.in1 && p.c1 == 0 && p.c0 % HD_CH == 0 && p.c0 >= HD_CH && !p.wskip &&
         !p.res && (p.epi == EPI_NCHW || step) && (p.cout == 6 || (p.cout == 3 && p.epi != EPI_DDPM)) &&
         p.H % HD_TH == 0 && p.W % HD_TW == 0 && p.Hin == p.H && p.Win == p.W;
}

size_t conv_head_pack_floats(int cin) { return (size_t)(cin / HD_CH) * 9 * HD_CH * 8; }

// w: torch layout [cout][cin][3][3] -> [cin/8][tap][8][8]
void conv_head_pack(const float* w, int cout, int cin, float* dst) {
  for (int ch = 0; ch < cin / HD_CH; ++ch)
    for (int tap = 0; tap < 9; ++tap)
      for (int c = 0; c < HD_CH; ++c)
        for (int co = 0; co < 8; ++co)
          dst[((size_t)(ch * 9 + tap) * HD_CH + c) * 8 + co] =
              co < cout ? w[((size_t)co * cin + ch * HD_CH + c) * 9 + tap] : 0.f;
}

int launch_conv_head(const ConvParams& p, const float* wh, hipStream_t stream) {
  const int blocks = p.N * (p.H / HD_TH) * (p.W / HD_TW);
  if (p.cout == 6)
    hipLaunchKernelGGL(conv_head_kernel<6>, dim3(blocks), dim3(HD_NT), 0, stream, p, wh);
  else
    hipLaunchKernelGGL(conv_head_kernel<3>, dim3(blocks), dim3(HD_NT), 0, stream, p, wh);
  return IFD_LAUNCH_STATUS();
}

}  // namespace ifd

namespace ifd {

bool conv_head_x3_eligible(const ConvParams& p, int taps, int xform) {
  return conv_head_eligible(p, taps, xform) && p.c0 % HX_CH == 0 && p.c0 <= HX_MAXCH * HX_CH && p.H % HX_T == 0 &&
         p.W % HX_T == 0;
}

size_t conv_head_x3_pack_floats(int cin) { return (size_t)(cin / HX_CH) * HX_WCH / 2; }

// w: [cout][cin][3][3] -> [cin/32][tap][part][8 co][32 ch] f16: part 0 = f16(w) 2^11, part 1 =
// f16((w - f16(w)) 2^11) (conv_x3.hip's weight split); false if |w| >= 32 (the head then stays fp32)
bool conv_head_x3_pack(const float* w, int cout, int cin, float* dst_f) {
  _Float16* dst = reinterpret_cast<_Float16*>(dst_f);
  bool ok = true;
  for (int ch = 0; ch < cin / HX_CH; ++ch)
    for (int tap = 0; tap < 9; ++tap)
      for (int part = 0; part < 2; ++part)
        for (int co = 0; co < HX_WCO; ++co)
          for (int c = 0; c < HX_CH; ++c) {
            const float v = co < cout ? w[((size_t)co * cin + ch * HX_CH + c) * 9 + tap] : 0.f;
            const _Float16 hi = (_Float16)v;
            _Float16 o;
            if (part == 0) {
              const float sc = (float)hi * 2048.0f;
              if (!(std::fabs(sc) <= 65504.0f)) ok = false;
              o = (_Float16)sc;
            } else {
              o = (_Float16)((v - (float)hi) * 2048.0f);
            }
            dst[((((size_t)ch * 9 + tap) * 2 + part) * HX_WCO + co) * HX_CH + c] = o;
          }
  return ok;
}

// The training forward's head (include/ifd_train.h ifd_tr_conv_head_x3): NHWC output of 8 channels (the
// 6 real ones and 2 zero-weight pads), bias padded to 8, GroupNorm + SiLU prologue.
bool conv_head_x3_nhwc_eligible(const ConvParams& p) {
  return !p.in1 && p.c1 == 0 && p.c0 % HX_CH == 0 && p.c0 >= HX_CH && p.c0 <= HX_MAXCH * HX_CH && !p.wskip &&
         !p.res && p.epi == EPI_NHWC && p.cout == HX_WCO && p.H % HX_T == 0 && p.W % HX_T == 0 && p.Hin == p.H &&
         p.Win == p.W;
}

// conv_head_x3_pack on the device (the training step re-packs every step): one thread per packed f16;
// a weight whose split is out of range (|f16(w)| 2^11 > 65504) sets bit 2 of *guard.
__global__ void pack_head_x3_kernel(const float* __restrict__ w, int cout, int cin, _Float16* __restrict__ dst,
                                    unsigned* guard) {
  const int64_t tot = (int64_t)(cin / HX_CH) * 9 * 2 * HX_WCO * HX_CH;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= tot) return;
  const int c = (int)(i % HX_CH);
  int64_t r = i / HX_CH;
  const int co = (int)(r % HX_WCO);
  r /= HX_WCO;
  const int part = (int)(r % 2);
  r /= 2;
  const int tap = (int)(r % 9);
  const int ch = (int)(r / 9);
  const float v = co < cout ? w[((size_t)co * cin + ch * HX_CH + c) * 9 + tap] : 0.f;
  const _Float16 hi = (_Float16)v;
  _Float16 o;
  if (part == 0) {
    const float sc = (float)hi * 2048.0f;
    if (!(fabsf(sc) <= 65504.0f)) atomicOr(guard, 2u);
    o = (_Float16)sc;
  } else {
    o = (_Float16)((v - (float)hi) * 2048.0f);
  }
  dst[i] = o;
}

int launch_pack_head_x3(const float* w, int cout, int cin, float* dst, unsigned* guard, hipStream_t stream) {
  const int64_t tot = (int64_t)(cin / HX_CH) * 9 * 2 * HX_WCO * HX_CH;
  hipLaunchKernelGGL(pack_head_x3_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, w, cout, cin,
                     reinterpret_cast<_Float16*>(dst), guard);
  return IFD_LAUNCH_STATUS();
}

namespace {
template <int CO, int ACT, int EPI>
int launch_head_ws(const ConvParams& p, const float* wx, int grid, hipStream_t stream) {
  static bool attr_set[kMaxDevices] = {};
  const void* fn = reinterpret_cast<const void*>(&conv_head_x3ws_kernel<CO, ACT, EPI>);
  hipError_t e = set_lds_attr_once(attr_set, fn, (int)HW_LDS);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL((conv_head_x3ws_kernel<CO, ACT, EPI>), dim3(grid), dim3(HW_NT), HW_LDS, stream, p,
                     reinterpret_cast<const _Float16*>(wx));
  return IFD_LAUNCH_STATUS();
}
template <int CO, int ACT>
int launch_head_ws_epi(const ConvParams& p, const float* wx, int grid, hipStream_t stream) {
  switch (p.epi) {
    case EPI_NCHW: return launch_head_ws<CO, ACT, EPI_NCHW>(p, wx, grid, stream);
    case EPI_DDIM: return launch_head_ws<CO, ACT, EPI_DDIM>(p, wx, grid, stream);
    case EPI_NHWC: if (CO == 6) return launch_head_ws<CO, ACT, EPI_NHWC>(p, wx, grid, stream); break;
    case EPI_DDPM: if (CO == 6) return launch_head_ws<CO, ACT, EPI_DDPM>(p, wx, grid, stream); break;
  }
  return (int)hipErrorInvalidValue;
}
template <int CO>
int launch_head_ws_act(const ConvParams& p, const float* wx, int grid, hipStream_t stream) {
  if (p.act == ACT_AFFINE_SILU) return launch_head_ws_epi<CO, ACT_AFFINE_SILU>(p, wx, grid, stream);
  if (p.act == ACT_AFFINE) return launch_head_ws_epi<CO, ACT_AFFINE>(p, wx, grid, stream);
  return launch_head_ws_epi<CO, ACT_NONE>(p, wx, grid, stream);
}
}  // namespace

int launch_conv_head_x3(const ConvParams& p, const float* wx, hipStream_t stream) {
  const int ntiles = p.N * (p.H / HX_T) * (p.W / HX_T);
  const int ncu = device_cu_count();  // one block per CU
  const int grid = ntiles < ncu ? ntiles : ncu;
  if (grid <= 0) return 0;
  // (CO only shapes the NCHW / sampler epilogues; the NHWC training head is CO 6 with 8 stored channels)
  if (p.cout == 6 || p.cout == HX_WCO) return launch_head_ws_act<6>(p, wx, grid, stream);
  return launch_head_ws_act<3>(p, wx, grid, stream);
}

}  // namespace ifd
