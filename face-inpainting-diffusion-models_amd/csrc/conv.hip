// Fused implicit-GEMM 3x3 / 1x1 convolution for gfx950 (see conv.h for the operator contract).
//
// GEMM view: M = output pixels (128-pixel tile = IMGS x TH x TW, TW = min(W, 32)),
//            N = output channels (BN tile), K = (tap, input channel) in chunks of 8 channels.
// Per K-chunk the block stages into LDS
//   * the activated input halo  A[q][pixel][4]   (q = channel quad 0/1, (TH+2) x (TW+2) halo per image)
//   * the packed weight slab    W[tap][q][co][4]
// double-buffered.
//
// Warp specialisation (512 threads = 8 waves, 2 per SIMD):
//   * waves 0-3 are CONSUMERS: only ds_read_b128 + v_mfma_f32_32x32x2_f32. Each owns a
//     (32*MR) x (32*NR) sub-tile; per tap it reads one A fragment per 32-pixel block and one B
//     fragment per 32-channel block and issues 4 MFMAs per block pair (MFMA j consumes element j:
//     K = {channel j (lanes 0-31), channel 4+j (lanes 32-63)}).
//   * waves 4-7 are PRODUCERS: global loads of chunk k+1, the prologue (GroupNorm-apply [+ scale/
//     shift] + SiLU, nearest-up / avg-pool resample, zero padding) and the LDS writes.
// A producer and a consumer share each SIMD: the VALU/LDS-write work of the producer issues
// beside the consumer's MFMAs (separate pipes), so the prologue costs no matrix-core time.
// One __syncthreads per chunk hands buffer k&1 to the consumers and (k+1)&1 to the producers.
// fp32 in / fp32 accumulate: the MFMA result is an exact fp32 fma chain (no reduced precision).
#include "conv.h"

#include <cstdlib>

namespace ifd {

// Explicit address spaces: without them the LDS / global accesses compile to flat_* ops, which
// count on BOTH vmcnt and lgkmcnt, so an LDS-read wait would also wait for in-flight global loads.
typedef __attribute__((address_space(3))) float lds_f;
typedef __attribute__((address_space(3))) f32x4 lds_f4;
typedef __attribute__((address_space(1))) const f32x4 glb_f4;
typedef __attribute__((address_space(1))) const float glb_f;

__device__ __forceinline__ f32x4 gld4(const float* p) { return *(glb_f4*)(p); }
__device__ __forceinline__ float gld1(const float* p) { return *(glb_f*)(p); }
__device__ __forceinline__ void gst1(float* p, float v) { *(__attribute__((address_space(1))) float*)(p) = v; }

constexpr int BM = 128;
constexpr int NT = 512;           // threads per block
constexpr int NP_T = 256;         // producer threads (waves 4-7)
constexpr int MAX_HALO_ITEMS = 4;  // 2 * NP <= 1024 (NP = 512 only for 2x2 images)

// SiLU of the GroupNorm-applied value, x / (1 + exp(-x)) with IEEE division and a 1-ulp expf as
// torch's CPU kernel. It runs on the producer waves, beside the MFMAs, so accuracy costs no
// matrix-core time.
__device__ __forceinline__ float silu_fast(float x) { return x / (1.0f + expf(-x)); }

template <int BN, int WGM, int WGN>
struct Tile {
  static constexpr int MR = BM / WGM / 32;
  static constexpr int NR = BN / WGN / 32;
  static_assert(MR >= 1 && NR >= 1, "bad wave grid");
  static_assert(WGM * WGN == 4, "4 consumer waves");
};

template <int BN, int WGM, int WGN>
using AccArr = f32x16[Tile<BN, WGM, WGN>::MR][Tile<BN, WGM, WGN>::NR];
template <int BN, int WGM, int WGN>
using PixArr = int[Tile<BN, WGM, WGN>::MR];

struct SegSrc {
  const float* p0; int c0;
  const float* p1; int c1;
};

// Chunk-invariant per-item staging state: which halo pixel this producer thread stages.
struct HaloItem {
  float valid;  // 1 for an in-bounds pixel of a real image, 0 otherwise (padding / tail)
  int srcpix;   // source pixel index n*Hs*Ws + sy*Ws + sx (top-left for XF_DOWN); 0 if invalid
  int n;        // image index (activation coefficients)
  int ldsoff;   // float offset in the A buffer, -1 if this item slot is unused
  int quad;     // channel quad 0/1
};

template <int TAPS, int XF>
__device__ __forceinline__ void make_items(HaloItem (&it)[MAX_HALO_ITEMS], int ptid, int NP, int HHd, int HWd,
                                           int n0, int y0, int x0, int N, int H, int W, int Hs, int Ws) {
  constexpr int HALO = (TAPS == 9) ? 1 : 0;
#pragma unroll
  for (int k = 0; k < MAX_HALO_ITEMS; ++k) {
    const int idx = ptid + k * NP_T;
    const int q = idx & 1, pix = idx >> 1;
    const int per = HHd * HWd;
    const int img = pix / per, rem = pix - img * per;
    const int hy = rem / HWd, hx = rem - hy * HWd;
    const int n = n0 + img, y = y0 + hy - HALO, x = x0 + hx - HALO;
    const bool inb = idx < 2 * NP && n < N && y >= 0 && y < H && x >= 0 && x < W;
    int sy = y, sx = x;
    if (XF == XF_UP) { sy = y >> 1; sx = x >> 1; }
    if (XF == XF_DOWN) { sy = 2 * y; sx = 2 * x; }
    it[k].valid = inb ? 1.f : 0.f;
    it[k].srcpix = inb ? (n * Hs + sy) * Ws + sx : 0;
    it[k].n = inb ? n : 0;
    it[k].ldsoff = idx < 2 * NP ? (q * NP + pix) * 4 : -1;
    it[k].quad = q;
  }
}

template <int BN, int TAPS, int XF>
struct Producer {
  static constexpr int NSRC = (XF == XF_DOWN) ? 4 : 1;
  static constexpr int WITEMS = (TAPS * 2 * BN + NP_T - 1) / NP_T;
  static constexpr bool WEXACT = (TAPS * 2 * BN) % NP_T == 0;

  f32x4 raw[MAX_HALO_ITEMS][NSRC];
  f32x4 ca[MAX_HALO_ITEMS], cb[MAX_HALO_ITEMS];
  f32x4 wr[WITEMS];

  // Issue the global loads of chunk k into registers (branch-free: invalid items read pixel 0).
  __device__ __forceinline__ void load(const HaloItem (&it)[MAX_HALO_ITEMS], int nitems, int ptid, const SegSrc& s,
                                       int k, int act, const float* actA, const float* actB, int ctot,
                                       const float* wslab, int Ws) {
    const int cb0 = 8 * k;
    const bool first = cb0 < s.c0;
    const float* src = first ? s.p0 : s.p1;
    const int cs = first ? s.c0 : s.c1;
    const int coff = first ? cb0 : cb0 - s.c0;
#pragma unroll
    for (int i = 0; i < MAX_HALO_ITEMS; ++i) {
      if (i < nitems) {
        const float* base = src + (size_t)it[i].srcpix * cs + coff + 4 * it[i].quad;
        raw[i][0] = gld4(base);
        if (XF == XF_DOWN) {
          raw[i][1] = gld4(base + cs);
          raw[i][2] = gld4(base + (size_t)Ws * cs);
          raw[i][3] = gld4(base + (size_t)Ws * cs + cs);
        }
        if (act != ACT_NONE) {
          const int ci = it[i].n * ctot + cb0 + 4 * it[i].quad;
          ca[i] = gld4(actA + ci);
          cb[i] = gld4(actB + ci);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < WITEMS; ++i) {
      const int idx = ptid + i * NP_T;
      if (WEXACT || idx < TAPS * 2 * BN) wr[i] = gld4(wslab + 4 * idx);
    }
  }

  __device__ __forceinline__ static float act1(float v, float a, float b, int act) {
    if (act == ACT_NONE) return v;
    const float t = a * v + b;
    return act == ACT_AFFINE_SILU ? silu_fast(t) : t;
  }

  // Apply the prologue (act, resample, zero padding) and write the chunk into LDS.
  __device__ __forceinline__ void store(const HaloItem (&it)[MAX_HALO_ITEMS], int nitems, int ptid, int act,
                                        lds_f* As, lds_f* Ws_) {
#pragma unroll
    for (int i = 0; i < MAX_HALO_ITEMS; ++i) {
      if (i < nitems && it[i].ldsoff >= 0) {
        f32x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float r;
          if (XF == XF_DOWN) {
            // AvgPool2d(2,2) of the activated tensor: ((v00 + v01) + v10) + v11, then / 4
            float s = act1(raw[i][0][j], ca[i][j], cb[i][j], act);
            s = s + act1(raw[i][1][j], ca[i][j], cb[i][j], act);
            s = s + act1(raw[i][2][j], ca[i][j], cb[i][j], act);
            s = s + act1(raw[i][3][j], ca[i][j], cb[i][j], act);
            r = s * 0.25f;
          } else {
            r = act1(raw[i][0][j], ca[i][j], cb[i][j], act);
          }
          v[j] = r * it[i].valid;  // zero padding after the activation (and for tail images)
        }
        *(lds_f4*)(As + it[i].ldsoff) = v;
      }
    }
#pragma unroll
    for (int i = 0; i < WITEMS; ++i) {
      const int idx = ptid + i * NP_T;
      if (WEXACT || idx < TAPS * 2 * BN) *(lds_f4*)(Ws_ + 4 * idx) = wr[i];
    }
  }
};

// MFMAs over one staged chunk (consumer waves).
template <int BN, int WGM, int WGN, int TAPS>
__device__ __forceinline__ void consume(AccArr<BN, WGM, WGN>& acc, const lds_f* As, const lds_f* Ws_, int NP, int HWd,
                                        const PixArr<BN, WGM, WGN>& pb, int wn0) {
  using T = Tile<BN, WGM, WGN>;
  const int lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
#pragma unroll
  for (int tap = 0; tap < TAPS; ++tap) {
    const int toff = (TAPS == 9) ? ((tap / 3) * HWd + (tap % 3)) : 0;
    f32x4 a[T::MR], b[T::NR];
#pragma unroll
    for (int mr = 0; mr < T::MR; ++mr) a[mr] = *(const lds_f4*)(As + 4 * (h * NP + pb[mr] + toff));
#pragma unroll
    for (int nr = 0; nr < T::NR; ++nr) b[nr] = *(const lds_f4*)(Ws_ + 4 * ((tap * 2 + h) * BN + wn0 + nr * 32 + l32));
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int mr = 0; mr < T::MR; ++mr)
#pragma unroll
        for (int nr = 0; nr < T::NR; ++nr)
          acc[mr][nr] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[mr][j], b[nr][j], acc[mr][nr], 0, 0, 0);
  }
}

// One K segment (all chunks of one (source, weights) pair) through the specialised pipeline.
// Both roles execute exactly 1 + nchunks barriers.
template <int BN, int WGM, int WGN, int TAPS, int XF>
__device__ __forceinline__ void run_segment(bool consumer, AccArr<BN, WGM, WGN>& acc, lds_f* smem, int npA,
                                            const SegSrc& src, int nchunks, int act, const float* actA,
                                            const float* actB, const float* wbase, int NP, int HHd, int HWd, int n0,
                                            int y0, int x0, int N, int H, int W, int Hs, int Ws,
                                            const PixArr<BN, WGM, WGN>& pb, int wn0, int k0) {
  lds_f* const A0 = smem;
  lds_f* const A1 = smem + npA * 8;
  lds_f* const W0 = smem + 2 * npA * 8;
  lds_f* const W1 = W0 + 9 * 8 * BN;
  if (consumer) {
    __syncthreads();
    for (int k = 0; k < nchunks; k += 2) {
      consume<BN, WGM, WGN, TAPS>(acc, A0, W0, NP, HWd, pb, wn0);
      __syncthreads();
      if (k + 1 >= nchunks) break;
      consume<BN, WGM, WGN, TAPS>(acc, A1, W1, NP, HWd, pb, wn0);
      __syncthreads();
    }
  } else {
    const int ptid = threadIdx.x - NP_T;
    const int nitems = (2 * NP + NP_T - 1) / NP_T;
    using P = Producer<BN, TAPS, XF>;
    P prod;
    HaloItem items[MAX_HALO_ITEMS];
    make_items<TAPS, XF>(items, ptid, NP, HHd, HWd, n0, y0, x0, N, H, W, Hs, Ws);
    const int slab = TAPS * 8 * BN;
    const int ctot = src.c0 + src.c1;
    prod.load(items, nitems, ptid, src, k0, act, actA, actB, ctot, wbase, Ws);
    prod.store(items, nitems, ptid, act, A0, W0);
    __syncthreads();
    for (int k = 0; k < nchunks; k += 2) {
      if (k + 1 < nchunks) {
        prod.load(items, nitems, ptid, src, k0 + k + 1, act, actA, actB, ctot, wbase + (size_t)(k + 1) * slab, Ws);
        prod.store(items, nitems, ptid, act, A1, W1);
      }
      __syncthreads();
      if (k + 1 >= nchunks) break;
      if (k + 2 < nchunks) {
        prod.load(items, nitems, ptid, src, k0 + k + 2, act, actA, actB, ctot, wbase + (size_t)(k + 2) * slab, Ws);
        prod.store(items, nitems, ptid, act, A0, W0);
      }
      __syncthreads();
    }
  }
}

template <int BN, int WGM, int WGN, int TAPS, int XF>
__global__ __launch_bounds__(NT) void conv_kernel(ConvParams p) {
  using T = Tile<BN, WGM, WGN>;
  extern __shared__ __attribute__((aligned(16))) float smem_raw[];
  lds_f* const smem = (lds_f*)(smem_raw);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool consumer = __builtin_amdgcn_readfirstlane(wave) < 4;
  const int h = lane >> 5, l32 = lane & 31;
  const int cw = wave & 3;
  const int wm = cw / WGN, wn = cw % WGN;
  const int wm0 = wm * (BM / WGM), wn0 = wn * (BN / WGN);

  int bx = blockIdx.x;
  const int tx = bx % p.tiles_x;
  bx /= p.tiles_x;
  const int ty = bx % p.tiles_y;
  const int tn = bx / p.tiles_y;
  const int n0 = tn * p.IMGS, y0 = ty * p.TH, x0 = tx * p.TW;
  const int ct = blockIdx.y;
  const int TPI = p.TH * p.TW;  // pixels per image in the tile

  constexpr int HALO = (TAPS == 9) ? 1 : 0;
  const int HHd = p.TH + 2 * HALO, HWd = p.TW + 2 * HALO;
  const int NP = p.IMGS * HHd * HWd;
  const int npA = NP > BM ? NP : BM;

  f32x16 acc[T::MR][T::NR];
#pragma unroll
  for (int mr = 0; mr < T::MR; ++mr)
#pragma unroll
    for (int nr = 0; nr < T::NR; ++nr)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mr][nr][r] = 0.f;

  int pb[T::MR], pm[T::MR];
#pragma unroll
  for (int mr = 0; mr < T::MR; ++mr) {
    const int m = wm0 + mr * 32 + l32;
    const int img = m >> p.lg_tpi, rem = m & (TPI - 1);
    const int py = rem >> p.lg_tw, px = rem & (p.TW - 1);
    pb[mr] = img * HHd * HWd + py * HWd + px;
    pm[mr] = m;
  }

  const int z = blockIdx.z, S = p.ksplit;
  // main segment: 3x3 (or 1x1) over concat(in0, in1) with fused prologue
  {
    SegSrc src{p.in0, p.c0, p.in1, p.c1};
    const int nch = p.cin_pad / 8;
    const int klo = z * nch / S, khi = (z + 1) * nch / S;
    const float* wbase = p.wpack + ((size_t)ct * nch + klo) * (TAPS * 8 * BN);
    run_segment<BN, WGM, WGN, TAPS, XF>(consumer, acc, smem, npA, src, khi - klo, p.act, p.actA, p.actB, wbase, NP,
                                        HHd, HWd, n0, y0, x0, p.N, p.H, p.W, p.Hin, p.Win, pb, wn0, klo);
  }
  // 1x1 segment: ResBlock skip_connection over the raw block input (output resolution)
  if (p.wskip && z == S - 1) {
    SegSrc src{p.s0, p.sc0, p.s1, p.sc1};
    const int nch = p.cs_pad / 8;
    const float* wbase = p.wskip + (size_t)ct * nch * (8 * BN);
    run_segment<BN, WGM, WGN, 1, XF_NONE>(consumer, acc, smem, npA, src, nch, ACT_NONE, nullptr, nullptr, wbase, BM,
                                          p.TH, p.TW, n0, y0, x0, p.N, p.H, p.W, p.H, p.W, pm, wn0, 0);
  }

  if (p.epi == EPI_NHWC && S > 1) {
    if (!consumer) return;
    float* slab = p.part + (size_t)z * p.N * p.H * p.W * p.cout;
#pragma unroll
    for (int nr = 0; nr < T::NR; ++nr) {
      const int co = ct * BN + wn0 + nr * 32 + l32;
      if (co >= p.cout) continue;
#pragma unroll
      for (int mr = 0; mr < T::MR; ++mr)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = wm0 + mr * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          const int img = m >> p.lg_tpi, rem = m & (TPI - 1);
          const int n = n0 + img, y = y0 + (rem >> p.lg_tw), x = x0 + (rem & (p.TW - 1));
          if (n < p.N) gst1(slab + ((size_t)(n * p.H + y) * p.W + x) * p.cout + co, acc[mr][nr][r]);
        }
    }
    return;
  }

  if (p.epi == EPI_NHWC) {
    if (!consumer) return;
#pragma unroll
    for (int nr = 0; nr < T::NR; ++nr) {
      const int co = ct * BN + wn0 + nr * 32 + l32;
      if (co >= p.cout) continue;
      const float bias = gld1(p.bias + co);
#pragma unroll
      for (int mr = 0; mr < T::MR; ++mr) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = wm0 + mr * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          const int img = m >> p.lg_tpi, rem = m & (TPI - 1);
          const int py = rem >> p.lg_tw, px = rem & (p.TW - 1);
          const int n = n0 + img, y = y0 + py, x = x0 + px;
          if (n >= p.N) continue;
          float v = acc[mr][nr][r] + bias;
          if (p.res) {
            float rv;
            if (p.res_xform == XF_NONE) {
              rv = gld1(p.res + ((size_t)(n * p.H + y) * p.W + x) * p.cout + co);
            } else if (p.res_xform == XF_UP) {
              rv = gld1(p.res + ((size_t)(n * p.res_H + (y >> 1)) * p.res_W + (x >> 1)) * p.cout + co);
            } else {
              const size_t b0 = ((size_t)(n * p.res_H + 2 * y) * p.res_W + 2 * x) * p.cout + co;
              const size_t rs = (size_t)p.res_W * p.cout;
              float s = gld1(p.res + b0);
              s = s + gld1(p.res + b0 + p.cout);
              s = s + gld1(p.res + b0 + rs);
              s = s + gld1(p.res + b0 + rs + p.cout);
              rv = s / 4.0f;
            }
            v = rv + v;
          }
          gst1(p.out + ((size_t)(n * p.H + y) * p.W + x) * p.cout + co, v);
        }
      }
    }
    return;
  }

  // Final-conv epilogues: stage the tile through LDS, then per-pixel NCHW work (coalesced along x).
  constexpr int LDT = BN + 1;
  lds_f* tile = smem;  // all segment buffers are dead after the last __syncthreads
  if (consumer) {
#pragma unroll
    for (int mr = 0; mr < T::MR; ++mr)
#pragma unroll
      for (int nr = 0; nr < T::NR; ++nr)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = wm0 + mr * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          tile[m * LDT + wn0 + nr * 32 + l32] = acc[mr][nr][r];
        }
  }
  __syncthreads();
  const int HWp = p.H * p.W;
  if (p.epi == EPI_NCHW) {
    const int co_lo = ct * BN;
    const int nco = min(BN, p.cout - co_lo);
    for (int idx = tid; idx < BM * nco; idx += NT) {
      const int c = idx / BM, m = idx - c * BM;
      const int img = m >> p.lg_tpi, rem = m & (TPI - 1);
      const int py = rem >> p.lg_tw, px = rem & (p.TW - 1);
      const int n = n0 + img;
      if (n >= p.N) continue;
      const int co = co_lo + c;
      p.out[((size_t)n * p.cout + co) * HWp + (size_t)(y0 + py) * p.W + (x0 + px)] = tile[m * LDT + c] + p.bias[co];
    }
    return;
  }
  // EPI_DDIM / EPI_DDPM: requires cout == 6 within this single channel tile (ct == 0)
  for (int idx = tid; idx < BM * 3; idx += NT) {
    const int c = idx / BM, m = idx - c * BM;
    const int img = m >> p.lg_tpi, rem = m & (TPI - 1);
    const int py = rem >> p.lg_tw, px = rem & (p.TW - 1);
    const int n = n0 + img;
    if (n >= p.N) continue;
    const size_t pix = (size_t)(y0 + py) * p.W + (x0 + px);
    const size_t o3 = ((size_t)n * 3 + c) * HWp + pix;
    const size_t om = (size_t)n * HWp + pix;
    const float eps = tile[m * LDT + c] + p.bias[c];
    const float x = p.img[o3];
    const float mk = p.sc.inject ? p.mask[om] : 0.f;
    const float g = p.sc.inject ? p.gt[o3] : 0.f;
    const float kn = p.sc.inject ? p.known[o3] : 0.f;
    float v;
    if (p.epi == EPI_DDIM) {
      const float nz = p.sc.use_noise ? p.noise[o3] : 0.f;
      v = ddim_step_value(p.sc, x, eps, nz, g, mk, kn);
    } else {
      const float var_v = tile[m * LDT + c + 3] + p.bias[c + 3];
      v = ddpm_step_value(p.sc, x, eps, var_v, p.noise[o3], g, mk, kn);
    }
    p.img[o3] = v;
  }
}

template <int BN, int WGM, int WGN, int TAPS, int XF>
static int launch_one(const ConvParams& p, hipStream_t stream) {
  const int HALO = (TAPS == 9) ? 1 : 0;
  const int NP = p.IMGS * (p.TH + 2 * HALO) * (p.TW + 2 * HALO);
  const int npA = NP > BM ? NP : BM;
  const size_t lds = (size_t)(2 * npA * 8 + 2 * 9 * 8 * BN) * sizeof(float);
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_kernel<BN, WGM, WGN, TAPS, XF>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  const int tiles_n = (p.N + p.IMGS - 1) / p.IMGS;
  dim3 grid(tiles_n * p.tiles_y * p.tiles_x, p.cout_pad / BN, p.ksplit);
  hipLaunchKernelGGL((conv_kernel<BN, WGM, WGN, TAPS, XF>), grid, dim3(NT), lds, stream, p);
  return (int)hipGetLastError();
}

// BN = 64 everywhere it divides Cout: the 49 KB double-buffered LDS footprint admits several
// blocks per CU, which hides each block's prologue/epilogue behind another's main loop (measured
// faster than BN = 128 on every UNet layer once the producer/consumer split removed the staging
// stall). IFD_CONV_BN=128 restores 128-wide tiles for experiments.
int conv_pick_bn(int cout, int taps, int H, int W, int N) {
  (void)taps; (void)H; (void)W; (void)N;
  static const char* ov = getenv("IFD_CONV_BN");
  if (ov && atoi(ov) == 128 && cout % 128 == 0) return 128;
  if (cout % 64 == 0) return 64;
  return 32;
}

void conv_geometry(ConvParams& p, int H, int W, int N, int bn, int nchunks) {
  p.TW = W < 32 ? W : 32;
  p.TH = H < BM / p.TW ? H : BM / p.TW;
  p.IMGS = BM / (p.TH * p.TW);
  p.tiles_x = W / p.TW;
  p.tiles_y = H / p.TH;
  p.lg_tw = __builtin_ctz(p.TW);
  p.lg_tpi = __builtin_ctz(p.TH * p.TW);
  const int tiles_n = (N + p.IMGS - 1) / p.IMGS;
  const long blocks = (long)tiles_n * p.tiles_y * p.tiles_x * (p.cout_pad / bn);
  // split K until the grid covers ~2 blocks per CU, keeping >= 4 chunks per split
  int S = 1;
  while (S < 8 && blocks * S < 512 && nchunks / (2 * S) >= 4) S *= 2;
  p.ksplit = S;
}

__global__ void splitk_reduce_kernel(ConvParams p) {
  const size_t tot = (size_t)p.N * p.H * p.W * p.cout;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= tot) return;
  const int co = (int)(i % p.cout);
  const size_t pix = i / p.cout;
  float acc = p.part[i];
  for (int z = 1; z < p.ksplit; ++z) acc += p.part[(size_t)z * tot + i];
  float v = acc + p.bias[co];
  if (p.res) {
    const int x = (int)(pix % p.W), y = (int)((pix / p.W) % p.H), n = (int)(pix / ((size_t)p.W * p.H));
    float rv;
    if (p.res_xform == XF_NONE) {
      rv = p.res[i];
    } else if (p.res_xform == XF_UP) {
      rv = p.res[((size_t)(n * p.res_H + (y >> 1)) * p.res_W + (x >> 1)) * p.cout + co];
    } else {
      const size_t b0 = ((size_t)(n * p.res_H + 2 * y) * p.res_W + 2 * x) * p.cout + co;
      const size_t rs = (size_t)p.res_W * p.cout;
      float s = p.res[b0];
      s = s + p.res[b0 + p.cout];
      s = s + p.res[b0 + rs];
      s = s + p.res[b0 + rs + p.cout];
      rv = s / 4.0f;
    }
    v = rv + v;
  }
  p.out[i] = v;
}

int launch_splitk_reduce(const ConvParams& p, hipStream_t stream) {
  const size_t tot = (size_t)p.N * p.H * p.W * p.cout;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, p);
  return (int)hipGetLastError();
}

int launch_conv(const ConvParams& p, int taps, int xform, int bn, hipStream_t stream) {
  if (bn == 128) {
    if (taps == 1) return launch_one<128, 2, 2, 1, XF_NONE>(p, stream);
    if (xform == XF_NONE) return launch_one<128, 2, 2, 9, XF_NONE>(p, stream);
    if (xform == XF_UP) return launch_one<128, 2, 2, 9, XF_UP>(p, stream);
    return launch_one<128, 2, 2, 9, XF_DOWN>(p, stream);
  }
  if (bn == 64) {
    if (taps == 1) return launch_one<64, 2, 2, 1, XF_NONE>(p, stream);
    if (xform == XF_NONE) return launch_one<64, 2, 2, 9, XF_NONE>(p, stream);
    if (xform == XF_UP) return launch_one<64, 2, 2, 9, XF_UP>(p, stream);
    return launch_one<64, 2, 2, 9, XF_DOWN>(p, stream);
  }
  if (taps == 9 && xform == XF_NONE) return launch_one<32, 4, 1, 9, XF_NONE>(p, stream);
  return (int)hipErrorInvalidValue;
}

}  // namespace ifd
