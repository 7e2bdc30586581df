// Fused implicit-GEMM 3x3 / 1x1 convolution for gfx950 (see conv.h for the operator contract).
//
// GEMM view: M = output pixels (BM-pixel tile = IMGS x TH x TW, TW = min(W, 32); BM = 256 for the
//            high-resolution layers, 128 otherwise), N = output channels (BN = 64, 32 for the
//            6-channel head), K = (tap, input channel) in chunks of 8 channels.
// Per K-chunk the block stages into LDS
//   * the activated input halo  A[q][pixel][4]   (q = channel quad 0/1, (TH+2) x (TW+2) halo per image)
//   * the packed weight slab    W[tap][q][co][4]
// double-buffered.
//
// Warp specialisation (512 threads = 8 waves, 2 per SIMD):
//   * waves 0-3 are CONSUMERS: only ds_read_b128 + v_mfma_f32_32x32x2_f32. Each owns a
//     (32*MR) x (32*NR) sub-tile; per tap it reads one A fragment per 32-pixel block and one B
//     fragment per 32-channel block and issues 4 MFMAs per block pair (MFMA j consumes element j:
//     K = {channel j (lanes 0-31), channel 4+j (lanes 32-63)}). The next tap's fragment reads are
//     pinned after the first MFMA group (sched_group_barrier) so their latency hides.
//   * waves 4-7 are PRODUCERS: global loads of chunk k+2 (two register sets in flight), the
//     prologue of chunk k+1 (GroupNorm-apply [+ scale/shift] + SiLU, nearest-up / avg-pool
//     resample, zero padding) and its LDS writes.
// A producer and a consumer share each SIMD: the producer's VALU/LDS-write work issues beside the
// consumer's MFMAs (separate pipes). One __syncthreads per chunk hands buffer k&1 to the consumers
// and (k+1)&1 to the producers. Ablation (IFD_ABLATE=1: producers idle) shows the consumer/barrier
// structure alone reaches ~94% of the fp32 MFMA peak; the producer's global-load stream (weights:
// 9*8*BN floats per chunk, reused by BM pixels) is what BM = 256 amortises.
// fp32 in / fp32 accumulate: the MFMA result is an exact fp32 fma chain (no reduced precision).
#include "conv.h"
#include "conv_dev.h"

#include <cstdlib>

// IFD_ABLATE (timing-only ablation builds): see conv_dev.h.
// IFD_TRACE=1: per-block timestamps (s_memrealtime, 100 MHz) into ConvParams::trace (64 slots/block):
//   [0] entry  [1] consumer past the first barrier  [2] consumer main segment done
//   [3] consumer epilogue done  [4] producer first chunk written  [5] HW_ID | XCC_ID << 32
//   [6] producer main segment done  [7] shader cycles entry -> epilogue done (s_memtime)
#ifndef IFD_TRACE
#define IFD_TRACE 0
#endif
// IFD_PRIO=1: producers at s_setprio 1; =2: consumers at s_setprio 1 (timing experiments)
#ifndef IFD_PRIO
#define IFD_PRIO 0
#endif
#if IFD_TRACE
#define TRACE_AT(slot, cond)                                                                     \
  do {                                                                                           \
    if (tr && (cond)) tr[slot] = __builtin_amdgcn_s_memrealtime();                               \
  } while (0)
#else
#define TRACE_AT(slot, cond) \
  do {                       \
  } while (0)
#endif

namespace ifd {


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
};

template <int TAPS, int XF, int MAXI>
__device__ __forceinline__ void make_items(HaloItem (&it)[MAXI], int ptid, int NP, int HHd, int HWd, int n0, int y0,
                                           int x0, int N, int H, int W, int Hs, int Ws) {
  constexpr int HALO = (TAPS == 9) ? 1 : 0;
#pragma unroll
  for (int k = 0; k < MAXI; ++k) {
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
  }
}

// Producer register set for one chunk. Every item of a thread has the same channel quad
// (ptid & 1, since NP_T is even); with ONEIMG (tile = one image) they also share the image, so
// one GroupNorm coefficient pair per thread per chunk replaces one per item.
template <int BN, int TAPS, int XF, int MAXI, bool ONEIMG>
struct Producer {
  static constexpr int NSRC = (XF == XF_DOWN) ? 4 : 1;
  static constexpr int NCO = ONEIMG ? 1 : MAXI;
  static constexpr int WITEMS = (TAPS * 2 * BN + NP_T - 1) / NP_T;
  static constexpr bool WEXACT = (TAPS * 2 * BN) % NP_T == 0;

  f32x4 raw[MAXI][NSRC];
  f32x4 ca[NCO], cb[NCO];
  f32x4 wr[WITEMS];

  // Issue the global loads of chunk k into registers (branch-free: invalid items read pixel 0).
  __device__ __forceinline__ void load(const HaloItem (&it)[MAXI], int nitems, int ptid, const SegSrc& s, int k,
                                       int act, const float* actA, const float* actB, int ctot, const float* wslab,
                                       int Ws, int n0) {
    if (IFD_ABLATE == 1) return;
    const int cb0 = 8 * k;
    const bool first = cb0 < s.c0;
    const float* src = first ? s.p0 : s.p1;
    const int cs = first ? s.c0 : s.c1;
    const int quad = ptid & 1;
    const int coff = (first ? cb0 : cb0 - s.c0) + 4 * quad;
#pragma unroll
    for (int i = 0; i < MAXI; ++i) {
      if (i < nitems) {
        const float* base = src + (size_t)it[i].srcpix * cs + coff;
        raw[i][0] = gld4(base);
        if (XF == XF_DOWN) {
          raw[i][1] = gld4(base + cs);
          raw[i][2] = gld4(base + (size_t)Ws * cs);
          raw[i][3] = gld4(base + (size_t)Ws * cs + cs);
        }
        if (!ONEIMG && act != ACT_NONE) {
          const int ci = it[i].n * ctot + cb0 + 4 * quad;
          ca[i] = gld4(actA + ci);
          cb[i] = gld4(actB + ci);
        }
      }
    }
    if (ONEIMG && act != ACT_NONE) {
      const int ci = n0 * ctot + cb0 + 4 * quad;
      ca[0] = gld4(actA + ci);
      cb[0] = gld4(actB + ci);
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
  __device__ __forceinline__ void store(const HaloItem (&it)[MAXI], int nitems, int ptid, int act, lds_f* As,
                                        lds_f* Ws_) {
    if (IFD_ABLATE == 1) return;
#pragma unroll
    for (int i = 0; i < MAXI; ++i) {
      if (i < nitems && it[i].ldsoff >= 0) {
        const int c = ONEIMG ? 0 : i;
        f32x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float r;
          if (XF == XF_DOWN) {
            // AvgPool2d(2,2) of the activated tensor: ((v00 + v01) + v10) + v11, then / 4
            float s = act1(raw[i][0][j], ca[c][j], cb[c][j], act);
            s = s + act1(raw[i][1][j], ca[c][j], cb[c][j], act);
            s = s + act1(raw[i][2][j], ca[c][j], cb[c][j], act);
            s = s + act1(raw[i][3][j], ca[c][j], cb[c][j], act);
            r = s * 0.25f;
          } else {
            r = act1(raw[i][0][j], ca[c][j], cb[c][j], act);
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

// One K segment (all chunks of one (source, weights) pair) through the specialised pipeline.
// Both roles execute exactly 1 + nchunks barriers.
template <int BM, int BN, int WGM, int WGN, int TAPS, int XF, int MAXI, bool ONEIMG>
__device__ __forceinline__ void run_segment(bool consumer, AccArr<BM, BN, WGM, WGN>& acc, lds_f* smem, int npA,
                                            const SegSrc& src, int nchunks, int act, const float* actA,
                                            const float* actB, const float* wbase, int NP, int HHd, int HWd, int n0,
                                            int y0, int x0, int N, int H, int W, int Hs, int Ws,
                                            const PixArr<BM, BN, WGM, WGN>& pb, int wn0, int k0,
                                            unsigned long long* tr) {
  (void)tr;
  lds_f* const A0 = smem;
  lds_f* const A1 = smem + npA * 8;
  lds_f* const W0 = smem + 2 * npA * 8;
  lds_f* const W1 = W0 + 9 * 8 * BN;
  if (consumer) {
    __syncthreads();
    TRACE_AT(1, threadIdx.x == 0);
    for (int k = 0; k < nchunks; k += 2) {
      consume<BM, BN, WGM, WGN, TAPS>(acc, A0, W0, NP, HWd, pb, wn0);
      __syncthreads();
      if (k + 1 >= nchunks) break;
      consume<BM, BN, WGM, WGN, TAPS>(acc, A1, W1, NP, HWd, pb, wn0);
      __syncthreads();
    }
  } else {
    // Producer: two register sets in flight (chunk k+2 loading while chunk k+1 is activated and
    // written), so each global load has a full consumer period to land.
    const int ptid = threadIdx.x - NP_T;
    const int nitems = (2 * NP + NP_T - 1) / NP_T;
    using P = Producer<BN, TAPS, XF, MAXI, ONEIMG>;
    P pa, pbuf;
    HaloItem items[MAXI];
    make_items<TAPS, XF, MAXI>(items, ptid, NP, HHd, HWd, n0, y0, x0, N, H, W, Hs, Ws);
    const int slab = TAPS * 8 * BN;
    const int ctot = src.c0 + src.c1;
    pa.load(items, nitems, ptid, src, k0, act, actA, actB, ctot, wbase, Ws, n0);
    if (nchunks > 1) pbuf.load(items, nitems, ptid, src, k0 + 1, act, actA, actB, ctot, wbase + slab, Ws, n0);
    pa.store(items, nitems, ptid, act, A0, W0);
    TRACE_AT(4, ptid == 0);
    __syncthreads();
    for (int k = 0; k < nchunks; k += 2) {
      if (k + 2 < nchunks)
        pa.load(items, nitems, ptid, src, k0 + k + 2, act, actA, actB, ctot, wbase + (size_t)(k + 2) * slab, Ws, n0);
      if (k + 1 < nchunks) pbuf.store(items, nitems, ptid, act, A1, W1);
      __syncthreads();
      if (k + 1 >= nchunks) break;
      if (k + 3 < nchunks)
        pbuf.load(items, nitems, ptid, src, k0 + k + 3, act, actA, actB, ctot, wbase + (size_t)(k + 3) * slab, Ws,
                  n0);
      if (k + 2 < nchunks) pa.store(items, nitems, ptid, act, A0, W0);
      __syncthreads();
    }
  }
}

// min 4 waves per SIMD (two 8-wave blocks per CU, <= 128 VGPRs) except the avg-pool variant,
// whose producer holds 4 source pixels per halo item.
template <int BM, int BN, int WGM, int WGN, int TAPS, int XF, int MAXI, bool ONEIMG>
__global__ __launch_bounds__(NT, XF == XF_DOWN ? 2 : 4) void conv_kernel(ConvParams p) {
  using T = Tile<BM, BN, WGM, WGN>;
  extern __shared__ __attribute__((aligned(16))) float smem_raw[];
  lds_f* const smem = (lds_f*)(smem_raw);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool consumer = __builtin_amdgcn_readfirstlane(wave) < 4;
  const int h = lane >> 5, l32 = lane & 31;
  const int cw = wave & 3;
  const int wm = cw / WGN, wn = cw % WGN;
  const int wm0 = wm * (BM / WGM), wn0 = wn * (BN / WGN);
  if (IFD_PRIO == 1 && !consumer) __builtin_amdgcn_s_setprio(1);
  if (IFD_PRIO == 2 && consumer) __builtin_amdgcn_s_setprio(1);

  // XCD-aware block -> (pixel tile, channel tile) map. Workgroups are dealt round-robin over the
  // 8 XCDs (blocks b and b+8 share one; MI355X_MICROARCH.md, speed only): the channel tiles of one
  // pixel tile get IDs 8 apart, so they run on one XCD at about the same time and the second one
  // reads the activation halo from that XCD's L2 instead of HBM. Bijective on the padded grid.
  const int nct = p.cout_pad / BN;
  const int L = blockIdx.x;
  const int grp = L / (8 * nct), rr = L - grp * 8 * nct;
  const int ct = rr >> 3;
  int bx = grp * 8 + (rr & 7);
  if (bx >= p.npix_tiles) return;  // padding of the last group of 8 (whole block exits: no barrier)
  const int tx = bx % p.tiles_x;
  bx /= p.tiles_x;
  const int ty = bx % p.tiles_y;
  const int tn = bx / p.tiles_y;
  const int n0 = tn * p.IMGS, y0 = ty * p.TH, x0 = tx * p.TW;
  const int TPI = p.TH * p.TW;  // pixels per image in the tile
#if IFD_TRACE
  unsigned long long* const tr =
      p.trace ? p.trace + 64 * ((size_t)blockIdx.z * gridDim.x + blockIdx.x) : nullptr;
  const unsigned long long cyc0 = __builtin_amdgcn_s_memtime();
  TRACE_AT(0, tid == 0);
  if (tr && tid == 0) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    tr[5] = hw | ((unsigned long long)xcc << 32);
  }
#else
  unsigned long long* const tr = nullptr;
#endif

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
    run_segment<BM, BN, WGM, WGN, TAPS, XF, MAXI, ONEIMG>(consumer, acc, smem, npA, src, khi - klo, p.act, p.actA,
                                                          p.actB, wbase, NP, HHd, HWd, n0, y0, x0, p.N, p.H, p.W,
                                                          p.Hin, p.Win, pb, wn0, klo, tr);
    TRACE_AT(2, tid == 0);
    TRACE_AT(6, tid == NP_T);
  }
  // 1x1 segment: ResBlock skip_connection over the raw block input (output resolution)
  if (p.wskip && z == S - 1) {
    SegSrc src{p.s0, p.sc0, p.s1, p.sc1};
    const int nch = p.cs_pad / 8;
    const float* wbase = p.wskip + (size_t)ct * nch * (8 * BN);
    run_segment<BM, BN, WGM, WGN, 1, XF_NONE, BM / 128, ONEIMG>(consumer, acc, smem, npA, src, nch, ACT_NONE, nullptr,
                                                               nullptr, wbase, BM, p.TH, p.TW, n0, y0, x0, p.N, p.H,
                                                               p.W, p.H, p.W, pm, wn0, 0, nullptr);
  }

  if (p.epi == EPI_NHWC) {
    // Stage the accumulators through LDS, then all 8 waves move 16-byte quads (4 channels of one
    // pixel): 16 lanes cover one pixel's BN channels. Bias, then residual, in torch's order
    // (h = conv + bias; out = x_res + h). Split-K writes raw partial sums (splitk_reduce adds the
    // rest). Residual loads are issued as a batch before any store: on CDNA stores and loads share
    // vmcnt, so a load issued after a store cannot be waited on without waiting for the store.
    constexpr int LDE = BN + 4;
    constexpr int QPP = BN / 4;
    constexpr int ITEMS = BM * QPP / NT;
    static_assert(BM * QPP % NT == 0, "epilogue items");
    lds_f* tile = smem;  // segment buffers are dead after the last barrier
    const bool split = S > 1;
    // every item of a thread has the same channel quad (NT % QPP == 0): one bias load, issued
    // before the LDS round trip so its latency hides behind it
    const int q = tid % QPP;
    const int co = ct * BN + 4 * q;
    const bool co_ok = co < p.cout;
    f32x4 bias4 = {0.f, 0.f, 0.f, 0.f};
    if (!split && co_ok) bias4 = gld4(p.bias + co);
    if (consumer) {
#pragma unroll
      for (int mr = 0; mr < T::MR; ++mr)
#pragma unroll
        for (int nr = 0; nr < T::NR; ++nr)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = wm0 + mr * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            tile[m * LDE + wn0 + nr * 32 + l32] = acc[mr][nr][r];
          }
    }
    __syncthreads();
    float* const dst = split ? p.part + (size_t)z * p.N * p.H * p.W * p.cout : p.out;
    f32x4 v[ITEMS];
    int off[ITEMS];  // float offset within image n (< 2^31: one image's H*W*cout)
    int nimg[ITEMS];
    bool ok[ITEMS];
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
      const int m = tid / QPP + i * (NT / QPP);
      const int img = m >> p.lg_tpi, rem = m & (TPI - 1);
      const int y = y0 + (rem >> p.lg_tw), x = x0 + (rem & (p.TW - 1));
      nimg[i] = n0 + img;
      ok[i] = nimg[i] < p.N && co_ok;
      off[i] = (y * p.W + x) * p.cout + co;
      v[i] = *(const lds_f4*)(tile + m * LDE + 4 * q);
      if (!split) v[i] = v[i] + bias4;
    }
    if (!split && p.res) {
      const size_t img_res = (size_t)p.res_H * p.res_W * p.cout;
      if (p.res_xform == XF_NONE) {
        f32x4 rv[ITEMS];
#pragma unroll
        for (int i = 0; i < ITEMS; ++i)
          if (ok[i]) rv[i] = gld4(p.res + nimg[i] * img_res + off[i]);
#pragma unroll
        for (int i = 0; i < ITEMS; ++i)
          if (ok[i]) v[i] = rv[i] + v[i];
      } else {
        f32x4 rv[ITEMS];
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
          if (!ok[i]) continue;
          const int pix = off[i] / p.cout;
          const int y = pix / p.W, x = pix - y * p.W;
          const float* rb = p.res + nimg[i] * img_res + co;
          if (p.res_xform == XF_UP) {
            rv[i] = gld4(rb + ((size_t)(y >> 1) * p.res_W + (x >> 1)) * p.cout);
          } else {
            const size_t b0 = ((size_t)(2 * y) * p.res_W + 2 * x) * p.cout;
            const size_t rs = (size_t)p.res_W * p.cout;
            f32x4 s = gld4(rb + b0);
            s = s + gld4(rb + b0 + p.cout);
            s = s + gld4(rb + b0 + rs);
            s = s + gld4(rb + b0 + rs + p.cout);
            rv[i] = s / 4.0f;
          }
        }
#pragma unroll
        for (int i = 0; i < ITEMS; ++i)
          if (ok[i]) v[i] = rv[i] + v[i];
      }
    }
    if constexpr (QPP == 16) {
      if (!split && p.gstat) {
        // GroupNorm granule statistics of the tile (single-image tiles only, host-checked): thread
        // = (quad q, ITEMS pixels); merge lanes q, q+16, q+32, q+48, then the 8 waves in order
        GStat g = gstat_xlanes16(gstat_of<ITEMS>(v));
        __syncthreads();  // all reads of the staged tile are done: reuse it
        if (lane < 16) {
          tile[(wave * 16 + lane) * 3 + 0] = g.n;
          tile[(wave * 16 + lane) * 3 + 1] = g.mean;
          tile[(wave * 16 + lane) * 3 + 2] = g.m2;
        }
        __syncthreads();
        if (tid < 16) {
          GStat a = {tile[tid * 3], tile[tid * 3 + 1], tile[tid * 3 + 2]};
#pragma unroll
          for (int w = 1; w < NT / 64; ++w) {
            const int o = (w * 16 + tid) * 3;
            a = gmerge(a, GStat{tile[o], tile[o + 1], tile[o + 2]});
          }
          const int e = ty * p.tiles_x + tx;
          float* o = p.gstat + (((size_t)n0 * (p.cout / 4) + ct * QPP + tid) * p.gstat_E + e) * 2;
          o[0] = a.mean;
          o[1] = a.m2;
        }
      }
    }
    const size_t img_out = (size_t)p.H * p.W * p.cout;
#pragma unroll
    for (int i = 0; i < ITEMS; ++i)
      if (ok[i]) *(__attribute__((address_space(1))) f32x4*)(dst + nimg[i] * img_out + off[i]) = v[i];
#if IFD_TRACE
    if (tr && tid == 0) {
      tr[3] = __builtin_amdgcn_s_memrealtime();
      tr[7] = __builtin_amdgcn_s_memtime() - cyc0;
    }
#endif
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

template <int BM, int BN, int WGM, int WGN, int TAPS, int XF, int MAXI, bool ONEIMG>
static int launch_inst(const ConvParams& p, size_t lds, hipStream_t stream) {
  static bool attr_set[kMaxDevices] = {};
  hipError_t e = set_lds_attr_once(
      attr_set, reinterpret_cast<const void*>(&conv_kernel<BM, BN, WGM, WGN, TAPS, XF, MAXI, ONEIMG>), 160 * 1024);
  if (e != hipSuccess) return (int)e;
  const int ptiles = (p.npix_tiles + 7) / 8 * 8;
  dim3 grid(ptiles * (p.cout_pad / BN), 1, p.ksplit);
  hipLaunchKernelGGL((conv_kernel<BM, BN, WGM, WGN, TAPS, XF, MAXI, ONEIMG>), grid, dim3(NT), lds, stream, p);
  return IFD_LAUNCH_STATUS();
}

template <int BM, int BN, int WGM, int WGN, int TAPS, int XF>
static int launch_one(const ConvParams& p, hipStream_t stream) {
  const int HALO = (TAPS == 9) ? 1 : 0;
  const int NP = p.IMGS * (p.TH + 2 * HALO) * (p.TW + 2 * HALO);
  const int npA = NP > BM ? NP : BM;
  const size_t stage = (size_t)(2 * npA * 8 + 2 * 9 * 8 * BN);
  const size_t epi = (size_t)BM * (BN + 4);  // NHWC epilogue tile (the final-conv tile is smaller)
  const size_t lds = (stage > epi ? stage : epi) * sizeof(float);
  const bool one = p.IMGS == 1;
  if constexpr (BM == 256) {  // only used for W >= 32 (one image per tile, 2*NP <= 1024)
    if (!one || 2 * NP > 4 * NP_T) return (int)hipErrorInvalidValue;
    return launch_inst<BM, BN, WGM, WGN, TAPS, XF, 4, true>(p, lds, stream);
  } else {
    if (2 * NP <= 2 * NP_T) {
      if (one) return launch_inst<BM, BN, WGM, WGN, TAPS, XF, 2, true>(p, lds, stream);
      return launch_inst<BM, BN, WGM, WGN, TAPS, XF, 2, false>(p, lds, stream);
    }
    if (2 * NP > 4 * NP_T) return (int)hipErrorInvalidValue;
    return launch_inst<BM, BN, WGM, WGN, TAPS, XF, 4, false>(p, lds, stream);
  }
}

int conv_pick_bn(int cout, int taps, int H, int W, int N) {
  (void)taps; (void)H; (void)W; (void)N;
  if (cout % 64 == 0) return 64;
  return 32;
}

// Tile geometry + split-K. BM = 256 (8 rows x 32 columns of one image) where the layer is wide and
// the grid still gives >= 2 blocks per CU: it halves the weight-slab loads per MFMA, the producer's
// bottleneck. Otherwise BM = 128, with split-K to cover the chip on the low-resolution layers.
constexpr long kInvBatch = 16;  // the batch-invariant geometry's reference batch (the bench's images per GPU)

void conv_geometry(ConvParams& p, int H, int W, int N, int bn, int nchunks, bool x3) {
  const bool allow256 = !p.opt_bm128;  // (the training 1x1 convs: 256-pixel tiles are instantiated for 3x3 only)
  int bm = 128;
  if (x3) {
    // 3xf16 split kernel (conv_x3.hip): 256-pixel tiles of one image (8 x 32 or 16 x 16) whatever
    // the tile count (persistent grid); nchunks = 16-channel chunks of the whole K stream
    if (bn == 64 && W >= 16 && H >= 256 / (W < 32 ? W : 32)) bm = 256;
    // four whole 8 x 8 images per tile; with opt_img8_partial at any N (a partial last tile recomputes the
    // batch's last image in its spare slots, conv_x3.hip unit_of)
    if (bn == 64 && W == 8 && H == 8 && (N % 4 == 0 || p.opt_img8_partial)) bm = 256;
  } else if (allow256 && bn == 64 && W >= 32 && H >= 8) {
    const long blocks256 = (long)(p.opt_invariant ? kInvBatch : N) * (H / 8) * (W / 32) * (p.cout_pad / bn);
    if (blocks256 >= 512) bm = 256;
  }
  p.bm = bm;
  p.TW = W < 32 ? W : 32;
  p.TH = H < bm / p.TW ? H : bm / p.TW;
  p.IMGS = bm / (p.TH * p.TW);
  p.tiles_x = W / p.TW;
  p.tiles_y = H / p.TH;
  p.lg_tw = __builtin_ctz(p.TW);
  p.lg_tpi = __builtin_ctz(p.TH * p.TW);
  const int tiles_n = (N + p.IMGS - 1) / p.IMGS;
  p.npix_tiles = tiles_n * p.tiles_y * p.tiles_x;
  // batch-invariant option: the geometry of a fixed reference batch (kInvBatch images), whatever the launch
  // holds, so an image's arithmetic (split-K factor, tile shape) does not depend on its batch (round 5: was one
  // image, which over-split the bench's 16- and 64-image launches: 13-14 % slower, profiles/r05b)
  const long inv_tiles = (p.npix_tiles / tiles_n) * ((kInvBatch + p.IMGS - 1) / p.IMGS);  // tiles of kInvBatch images
  const long blocks = (long)(p.opt_invariant ? inv_tiles : p.npix_tiles) * (p.cout_pad / bn);
  int S = 1;
  if (x3 && bm == 256) {
    // persistent units: split K until the units cover the 256 CUs, keeping >= 4 chunks per unit
    const int minch = W == 8 ? 2 : 4;  // the 8x8 layers: few units, split down to 2 chunks
    while (S < 8 && blocks * S < 256 && nchunks % (2 * S) == 0 && nchunks / (2 * S) >= minch) S *= 2;
  } else {
    // split K until the grid covers ~2 blocks per CU, keeping >= 4 chunks per split
    while (S < 8 && blocks * S < 512 && nchunks / (2 * S) >= 4) S *= 2;
  }
  p.ksplit = S;
}

__global__ void splitk_reduce_kernel(ConvParams p) {
  const size_t tot = (size_t)p.N * p.H * p.W * p.cout;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= tot) return;
  const int co = (int)(i % p.cout);
  const size_t pix = i / p.cout;
  float sl[8];
#pragma unroll
  for (int z = 0; z < 8; ++z)
    if (z < p.ksplit) sl[z] = p.part[(size_t)z * tot + i];
  float acc = sl[0];
#pragma unroll
  for (int z = 1; z < 8; ++z)
    if (z < p.ksplit) acc += sl[z];
  for (int z = 8; z < p.ksplit; ++z) acc += p.part[(size_t)z * tot + i];
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

// Split-K reduction that also writes the GroupNorm granule statistics of its output (a split
// kernel's units end in raw slabs, so it has no per-tile statistics epilogue). Block = (slice of
// SKG_SL pixels x 64 channel quads, image n); thread = (quad, pixel lane of 4). Per pixel: the slabs
// summed in slab order, + bias, + residual - splitk_reduce_kernel's arithmetic - stored, and folded
// into shifted sums (K = the lane's first value); the quad's 4 channels and the 4 pixel lanes merge
// in a fixed order (Chan) into granule entry (n, slice) of the quad: the entry layout of the conv
// epilogues (gstat[n][cout/4][e] = (mean, M2), e = slice, cnt = 4 * SKG_SL values). 8 quads x
// 32 pixel lanes per block: enough blocks even for the 8x8 layers (one slice per image).
constexpr int SKG_SL = 64;
constexpr int SKG_MAXS = 8;  // split-K counts conv_geometry produces (S <= 8)
constexpr int SKG_Q = 8, SKG_PL = 256 / SKG_Q;
__global__ __launch_bounds__(256) void splitk_gstat_kernel(ConvParams p) {
  __shared__ float red[SKG_PL][SKG_Q][3];
  const int q = threadIdx.x % SKG_Q, pl = threadIdx.x / SKG_Q;
  const int QP = p.cout / 4;
  const int nqb = (QP + SKG_Q - 1) / SKG_Q;
  const int e = blockIdx.x / nqb, qq = (blockIdx.x % nqb) * SKG_Q + q;
  const int n = blockIdx.y;
  const int HW = p.H * p.W;
  const int slice = HW < SKG_SL ? HW : SKG_SL;
  const bool act = qq < QP;
  const size_t tot = (size_t)p.N * HW * p.cout;
  f32x4 K = {0.f, 0.f, 0.f, 0.f}, s1 = K, s2 = K;
  float cnt = 0.f;
  if (act) {
    const f32x4 b = gld4(p.bias + 4 * qq);
    for (int i = pl; i < slice; i += SKG_PL) {
      const int px = e * slice + i;
      const size_t idx = ((size_t)n * HW + px) * p.cout + 4 * qq;
      // all slabs' loads in flight together (a runtime-bounded loop issued them one latency apart),
      // summed in slab order as before
      f32x4 sl[SKG_MAXS];
#pragma unroll
      for (int z = 0; z < SKG_MAXS; ++z)
        if (z < p.ksplit) sl[z] = gld4(p.part + (size_t)z * tot + idx);
      f32x4 acc = sl[0];
#pragma unroll
      for (int z = 1; z < SKG_MAXS; ++z)
        if (z < p.ksplit) acc += sl[z];
      for (int z = SKG_MAXS; z < p.ksplit; ++z) acc += gld4(p.part + (size_t)z * tot + idx);
      f32x4 v = acc + b;
      if (p.res) {
        const int x = px % p.W, y = px / p.W;
        f32x4 rv;
        if (p.res_xform == XF_NONE) {
          rv = gld4(p.res + idx);
        } else if (p.res_xform == XF_UP) {
          rv = gld4(p.res + ((size_t)(n * p.res_H + (y >> 1)) * p.res_W + (x >> 1)) * p.cout + 4 * qq);
        } else {
          const size_t b0 = ((size_t)(n * p.res_H + 2 * y) * p.res_W + 2 * x) * p.cout + 4 * qq;
          const size_t rs = (size_t)p.res_W * p.cout;
          const f32x4 r00 = gld4(p.res + b0), r01 = gld4(p.res + b0 + p.cout);
          const f32x4 r10 = gld4(p.res + b0 + rs), r11 = gld4(p.res + b0 + rs + p.cout);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float s = r00[j];
            s = s + r01[j];
            s = s + r10[j];
            s = s + r11[j];
            rv[j] = s / 4.0f;
          }
        }
        v = rv + v;
      }
      gst4(p.out + idx, v);
      if (cnt == 0.f) K = v;
      const f32x4 d = v - K;
      s1 += d;
      s2 += d * d;
      cnt += 1.f;
    }
  }
  GStat g = {0.f, 0.f, 0.f};  // a lane without pixels (slices smaller than the lanes) stays empty
  if (cnt > 0.f) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      GStat st;
      st.n = cnt;
      st.mean = K[j] + s1[j] / cnt;
      st.m2 = fmaxf(s2[j] - s1[j] * (s1[j] / cnt), 0.f);
      g = j == 0 ? st : gmerge(g, st);
    }
  }
  red[pl][q][0] = g.n;
  red[pl][q][1] = g.mean;
  red[pl][q][2] = g.m2;
  __syncthreads();
  if (pl == 0 && act) {
    GStat a = {red[0][q][0], red[0][q][1], red[0][q][2]};
    for (int l = 1; l < SKG_PL; ++l)
      if (red[l][q][0] > 0.f) a = gmerge(a, GStat{red[l][q][0], red[l][q][1], red[l][q][2]});
    float* o = p.gstat + (((size_t)n * QP + qq) * (HW / slice) + e) * 2;
    o[0] = a.mean;
    o[1] = a.m2;
  }
}

int launch_splitk_gstat(const ConvParams& p, int* E, float* cnt, hipStream_t stream) {
  const int HW = p.H * p.W;
  const int slice = HW < SKG_SL ? HW : SKG_SL;
  if (HW % slice != 0 || p.cout % 4 != 0 || !p.gstat) return (int)hipErrorInvalidValue;
  *E = HW / slice;
  *cnt = 4.0f * slice;
  const int nqb = (p.cout / 4 + SKG_Q - 1) / SKG_Q;
  hipLaunchKernelGGL(splitk_gstat_kernel, dim3(*E * nqb, p.N), dim3(256), 0, stream, p);
  return IFD_LAUNCH_STATUS();
}

int launch_splitk_reduce(const ConvParams& p, hipStream_t stream) {
  const size_t tot = (size_t)p.N * p.H * p.W * p.cout;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, p);
  return IFD_LAUNCH_STATUS();
}

int launch_conv(const ConvParams& p, int taps, int xform, int bn, hipStream_t stream) {
  if (bn == 64 && p.bm == 256) {
    if (taps == 1) return (int)hipErrorInvalidValue;
    if (xform == XF_NONE) return launch_one<256, 64, 4, 1, 9, XF_NONE>(p, stream);
    if (xform == XF_UP) return launch_one<256, 64, 4, 1, 9, XF_UP>(p, stream);
    return launch_one<256, 64, 4, 1, 9, XF_DOWN>(p, stream);
  }
  if (bn == 64) {
    if (taps == 1) return launch_one<128, 64, 2, 2, 1, XF_NONE>(p, stream);
    if (xform == XF_NONE) return launch_one<128, 64, 2, 2, 9, XF_NONE>(p, stream);
    if (xform == XF_UP) return launch_one<128, 64, 2, 2, 9, XF_UP>(p, stream);
    return launch_one<128, 64, 2, 2, 9, XF_DOWN>(p, stream);
  }
  if (taps == 9 && xform == XF_NONE) return launch_one<128, 32, 4, 1, 9, XF_NONE>(p, stream);
  return (int)hipErrorInvalidValue;
}

}  // namespace ifd
