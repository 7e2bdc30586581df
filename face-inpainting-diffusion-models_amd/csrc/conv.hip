// Fused implicit-GEMM 3x3 / 1x1 convolution for gfx950 (see conv.h for the operator contract).
//
// GEMM view: M = output pixels (128-pixel tile = IMGS x TH x TW, TW = min(W, 32)),
//            N = output channels (BN tile), K = (tap, input channel) in chunks of 8 channels.
// Per K-chunk the block stages into LDS
//   * the activated input halo  A[q][pixel][4]   (q = channel quad 0/1, (TH+2) x (TW+2) halo per image)
//   * the packed weight slab    W[tap][q][co][4]
// double-buffered with register prefetch of chunk k+1 while chunk k runs on the matrix cores.
// Each wave owns a (32*MR) x (32*NR) sub-tile; per tap it reads one ds_read_b128 A fragment per
// 32-pixel block and one per 32-channel block, and issues 4 v_mfma_f32_32x32x2_f32 per block pair:
// MFMA j consumes element j of the fragments, i.e. K = {channel j (lanes 0-31), channel 4+j (32-63)}.
// fp32 in / fp32 accumulate: the MFMA result is an exact fp32 fma chain (no reduced precision).
#include "conv.h"

namespace ifd {

constexpr int BM = 128;
constexpr int NT = 256;
constexpr int MAX_HALO_ITEMS = 4;  // 2 * NP <= 1024 (NP = 512 only for 2x2 images)

template <int BN, int WGM, int WGN>
struct Tile {
  static constexpr int MR = BM / WGM / 32;
  static constexpr int NR = BN / WGN / 32;
  static_assert(MR >= 1 && NR >= 1, "bad wave grid");
  static_assert(WGM * WGN == 4, "4 waves");
};

template <int BN, int WGM, int WGN>
using AccArr = f32x16[Tile<BN, WGM, WGN>::MR][Tile<BN, WGM, WGN>::NR];
template <int BN, int WGM, int WGN>
using PixArr = int[Tile<BN, WGM, WGN>::MR];

struct SegSrc {
  const float* p0; int c0;
  const float* p1; int c1;
};

// Chunk-invariant per-item staging state: which halo pixel this thread stages and where it reads.
struct HaloItem {
  int valid;   // in-bounds pixel of a real image (else the LDS slot gets 0)
  int srcpix;  // source pixel index n*Hs*Ws + sy*Ws + sx (top-left for XF_DOWN)
  int n;       // image index (activation coefficients)
  int ldsoff;  // float offset in the A buffer
};

template <int TAPS, int XF>
__device__ __forceinline__ void make_items(HaloItem (&it)[MAX_HALO_ITEMS], int NP, int HHd, int HWd, int n0, int y0,
                                           int x0, int N, int H, int W, int Hs, int Ws) {
  constexpr int HALO = (TAPS == 9) ? 1 : 0;
#pragma unroll
  for (int k = 0; k < MAX_HALO_ITEMS; ++k) {
    const int idx = threadIdx.x + k * NT;
    it[k].valid = 0;
    it[k].srcpix = 0;
    it[k].n = 0;
    it[k].ldsoff = -1;
    if (idx < 2 * NP) {
      const int q = idx & 1, pix = idx >> 1;
      const int per = HHd * HWd;
      const int img = pix / per, rem = pix - img * per;
      const int hy = rem / HWd, hx = rem - hy * HWd;
      const int n = n0 + img, y = y0 + hy - HALO, x = x0 + hx - HALO;
      it[k].ldsoff = (q * NP + pix) * 4;
      it[k].n = n < N ? n : 0;
      if (n < N && y >= 0 && y < H && x >= 0 && x < W) {
        int sy = y, sx = x;
        if (XF == XF_UP) { sy = y >> 1; sx = x >> 1; }
        if (XF == XF_DOWN) { sy = 2 * y; sx = 2 * x; }
        it[k].valid = 1;
        it[k].srcpix = (n * Hs + sy) * Ws + sx;
      }
    }
  }
}

template <int BN, int WGM, int WGN, int TAPS, int XF>
struct Segment {
  using T = Tile<BN, WGM, WGN>;
  static constexpr int NSRC = (XF == XF_DOWN) ? 4 : 1;
  static constexpr int WITEMS = (TAPS * 2 * BN + NT - 1) / NT;

  f32x4 raw[MAX_HALO_ITEMS][NSRC];
  f32x4 ca[MAX_HALO_ITEMS], cb[MAX_HALO_ITEMS];
  f32x4 wr[WITEMS];

  // Issue the global loads of chunk k into registers.
  __device__ __forceinline__ void load(const HaloItem (&it)[MAX_HALO_ITEMS], const SegSrc& s, int k, int act,
                                       const float* actA, const float* actB, int ctot, const float* wslab, int Ws) {
    const int cb0 = 8 * k;
    const float* src;
    int cs, coff;
    if (cb0 < s.c0) { src = s.p0; cs = s.c0; coff = cb0; }
    else { src = s.p1; cs = s.c1; coff = cb0 - s.c0; }
#pragma unroll
    for (int i = 0; i < MAX_HALO_ITEMS; ++i) {
      if (it[i].valid) {
        const int quad = (threadIdx.x + i * NT) & 1;
        const float* base = src + (size_t)it[i].srcpix * cs + coff + 4 * quad;
        raw[i][0] = *reinterpret_cast<const f32x4*>(base);
        if (XF == XF_DOWN) {
          raw[i][1] = *reinterpret_cast<const f32x4*>(base + cs);
          raw[i][2] = *reinterpret_cast<const f32x4*>(base + (size_t)Ws * cs);
          raw[i][3] = *reinterpret_cast<const f32x4*>(base + (size_t)Ws * cs + cs);
        }
        if (act != ACT_NONE) {
          const int ci = it[i].n * ctot + cb0 + 4 * quad;
          ca[i] = *reinterpret_cast<const f32x4*>(actA + ci);
          cb[i] = *reinterpret_cast<const f32x4*>(actB + ci);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < WITEMS; ++i) {
      const int idx = threadIdx.x + i * NT;
      if (idx < TAPS * 2 * BN) wr[i] = *reinterpret_cast<const f32x4*>(wslab + 4 * idx);
    }
  }

  __device__ __forceinline__ static float act1(float v, float a, float b, int act) {
    if (act == ACT_NONE) return v;
    float t = a * v + b;
    return act == ACT_AFFINE_SILU ? silu_f(t) : t;
  }

  // Apply the prologue (act, resample, zero padding) and write chunk registers into LDS.
  __device__ __forceinline__ void store(const HaloItem (&it)[MAX_HALO_ITEMS], int act, float* As, float* Ws_) {
#pragma unroll
    for (int i = 0; i < MAX_HALO_ITEMS; ++i) {
      if (it[i].ldsoff >= 0) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (it[i].valid) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (XF == XF_DOWN) {
              // AvgPool2d(2,2) of the activated tensor: ((v00 + v01) + v10) + v11, then / 4
              float s = act1(raw[i][0][j], ca[i][j], cb[i][j], act);
              s = s + act1(raw[i][1][j], ca[i][j], cb[i][j], act);
              s = s + act1(raw[i][2][j], ca[i][j], cb[i][j], act);
              s = s + act1(raw[i][3][j], ca[i][j], cb[i][j], act);
              v[j] = s / 4.0f;
            } else {
              v[j] = act1(raw[i][0][j], ca[i][j], cb[i][j], act);
            }
          }
        }
        *reinterpret_cast<f32x4*>(As + it[i].ldsoff) = v;
      }
    }
#pragma unroll
    for (int i = 0; i < WITEMS; ++i) {
      const int idx = threadIdx.x + i * NT;
      if (idx < TAPS * 2 * BN) *reinterpret_cast<f32x4*>(Ws_ + 4 * idx) = wr[i];
    }
  }

  // MFMAs over one staged chunk.
  __device__ __forceinline__ static void compute(f32x16 (&acc)[T::MR][T::NR], const float* As, const float* Ws_, int NP,
                                                 int HWd, const int (&pb)[T::MR], int wn0) {
    const int lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
#pragma unroll
    for (int tap = 0; tap < TAPS; ++tap) {
      const int toff = (TAPS == 9) ? ((tap / 3) * HWd + (tap % 3)) : 0;
      f32x4 a[T::MR], b[T::NR];
#pragma unroll
      for (int mr = 0; mr < T::MR; ++mr)
        a[mr] = *reinterpret_cast<const f32x4*>(As + 4 * (h * NP + pb[mr] + toff));
#pragma unroll
      for (int nr = 0; nr < T::NR; ++nr)
        b[nr] = *reinterpret_cast<const f32x4*>(Ws_ + 4 * ((tap * 2 + h) * BN + wn0 + nr * 32 + l32));
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int mr = 0; mr < T::MR; ++mr)
#pragma unroll
          for (int nr = 0; nr < T::NR; ++nr)
            acc[mr][nr] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[mr][j], b[nr][j], acc[mr][nr], 0, 0, 0);
    }
  }
};

// Run one K segment (all chunks of one (source, weights) pair) through the double-buffered pipeline.
template <int BN, int WGM, int WGN, int TAPS, int XF>
__device__ __forceinline__ void run_segment(AccArr<BN, WGM, WGN>& acc,
                                            float* smem, int npA, const SegSrc& src, int nchunks, int act,
                                            const float* actA, const float* actB, const float* wbase, int NP,
                                            int HHd, int HWd, int n0, int y0, int x0, int N, int H, int W, int Hs,
                                            int Ws, const PixArr<BN, WGM, WGN>& pb, int wn0) {
  using S = Segment<BN, WGM, WGN, TAPS, XF>;
  S seg;
  HaloItem items[MAX_HALO_ITEMS];
  make_items<TAPS, XF>(items, NP, HHd, HWd, n0, y0, x0, N, H, W, Hs, Ws);
  float* Abuf[2] = {smem, smem + npA * 8};
  float* Wbuf[2] = {smem + 2 * npA * 8, smem + 2 * npA * 8 + 9 * 8 * BN};
  const int slab = TAPS * 8 * BN;
  const int ctot = src.c0 + src.c1;
  seg.load(items, src, 0, act, actA, actB, ctot, wbase, Ws);
  seg.store(items, act, Abuf[0], Wbuf[0]);
  __syncthreads();
  for (int k = 0; k < nchunks; ++k) {
    const int cur = k & 1;
    if (k + 1 < nchunks) seg.load(items, src, k + 1, act, actA, actB, ctot, wbase + (size_t)(k + 1) * slab, Ws);
    S::compute(acc, Abuf[cur], Wbuf[cur], NP, HWd, pb, wn0);
    if (k + 1 < nchunks) seg.store(items, act, Abuf[cur ^ 1], Wbuf[cur ^ 1]);
    __syncthreads();
  }
}

template <int BN, int WGM, int WGN, int TAPS, int XF>
__global__ __launch_bounds__(NT) void conv_kernel(ConvParams p) {
  using T = Tile<BN, WGM, WGN>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int wm = wave / WGN, wn = wave % WGN;
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
    const int img = m / TPI, rem = m - img * TPI;
    const int py = rem / p.TW, px = rem - py * p.TW;
    pb[mr] = img * HHd * HWd + py * HWd + px;
    pm[mr] = m;
  }

  // main segment: 3x3 (or 1x1) over concat(in0, in1) with fused prologue
  {
    SegSrc src{p.in0, p.c0, p.in1, p.c1};
    const int nch = p.cin_pad / 8;
    const float* wbase = p.wpack + (size_t)ct * nch * (TAPS * 8 * BN);
    run_segment<BN, WGM, WGN, TAPS, XF>(acc, smem, npA, src, nch, p.act, p.actA, p.actB, wbase, NP, HHd, HWd, n0, y0,
                                        x0, p.N, p.H, p.W, p.Hin, p.Win, pb, wn0);
  }
  // 1x1 segment: ResBlock skip_connection over the raw block input (output resolution)
  if (p.wskip) {
    SegSrc src{p.s0, p.sc0, p.s1, p.sc1};
    const int nch = p.cs_pad / 8;
    const float* wbase = p.wskip + (size_t)ct * nch * (8 * BN);
    run_segment<BN, WGM, WGN, 1, XF_NONE>(acc, smem, npA, src, nch, ACT_NONE, nullptr, nullptr, wbase, BM, p.TH, p.TW,
                                          n0, y0, x0, p.N, p.H, p.W, p.H, p.W, pm, wn0);
  }

  if (p.epi == EPI_NHWC) {
#pragma unroll
    for (int nr = 0; nr < T::NR; ++nr) {
      const int co = ct * BN + wn0 + nr * 32 + l32;
      if (co >= p.cout) continue;
      const float bias = p.bias[co];
#pragma unroll
      for (int mr = 0; mr < T::MR; ++mr) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = wm0 + mr * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          const int img = m / TPI, rem = m - img * TPI;
          const int py = rem / p.TW, px = rem - py * p.TW;
          const int n = n0 + img, y = y0 + py, x = x0 + px;
          if (n >= p.N) continue;
          float v = acc[mr][nr][r] + bias;
          if (p.res) {
            float rv;
            if (p.res_xform == XF_NONE) {
              rv = p.res[((size_t)(n * p.H + y) * p.W + x) * p.cout + co];
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
          p.out[((size_t)(n * p.H + y) * p.W + x) * p.cout + co] = v;
        }
      }
    }
    return;
  }

  // Final-conv epilogues: stage the tile through LDS, then per-pixel NCHW work (coalesced along x).
  constexpr int LDT = BN + 1;
  float* tile = smem;  // all segment buffers are dead after the last __syncthreads
#pragma unroll
  for (int mr = 0; mr < T::MR; ++mr)
#pragma unroll
    for (int nr = 0; nr < T::NR; ++nr)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = wm0 + mr * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        tile[m * LDT + wn0 + nr * 32 + l32] = acc[mr][nr][r];
      }
  __syncthreads();
  const int HWp = p.H * p.W;
  if (p.epi == EPI_NCHW) {
    const int co_lo = ct * BN;
    const int nco = min(BN, p.cout - co_lo);
    for (int idx = tid; idx < BM * nco; idx += NT) {
      const int c = idx / BM, m = idx - c * BM;
      const int img = m / TPI, rem = m - img * TPI;
      const int py = rem / p.TW, px = rem - py * p.TW;
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
    const int img = m / TPI, rem = m - img * TPI;
    const int py = rem / p.TW, px = rem - py * p.TW;
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
  dim3 grid(tiles_n * p.tiles_y * p.tiles_x, p.cout_pad / BN);
  hipLaunchKernelGGL((conv_kernel<BN, WGM, WGN, TAPS, XF>), grid, dim3(NT), lds, stream, p);
  return (int)hipGetLastError();
}

int conv_pick_bn(int cout, int taps, int H, int W, int N) {
  (void)taps; (void)H; (void)W; (void)N;
  if (cout % 128 == 0) return 128;
  if (cout % 64 == 0) return 64;
  return 32;
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
