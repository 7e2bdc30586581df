// 3xf16 split-precision fused 3x3 convolution ("3xf16" precision mode) for the wide layers.
//
// Why: gfx950 has no xf32, and v_mfma_f32_32x32x2_f32 runs at the fp32 VECTOR rate (157 TF/s),
// sharing the VALU with the producer waves. The f16 matrix path is 16x faster per K. Each fp32
// operand is split into two f16 parts,
//     a = a_hi + a_lo,           a_hi = f16(a),  a_lo = f16(a - a_hi)              (RNE both)
//     w = w_hi + 2^-11 w_lo',    w_hi = f16(w),  w_lo' = f16((w - w_hi) * 2^11)   (once, at load)
// and the product is rebuilt from three f16 MFMAs into ONE fp32 accumulator carried at scale 2^11,
// with both B operands stored pre-scaled so the consumer waves run no VALU at all:
//     acc += a_hi * (w_hi 2^11)  +  a_hi * w_lo'  +  a_lo * (w_hi 2^11)        (then out = acc * 2^-11)
// Every f16 x f16 product is exact in fp32; the dropped a_lo w_lo term and the roundings bound the
// error per product by ~2^-21 relative (a_lo goes subnormal below |a| ~ 2^-3, adding <= 2^-25
// absolute), below fp32's own accumulation rounding over K = 9 * Cin terms. Measured on the reduced and full UNet (tests/
// test_cpu_split_numerics.py emulates this exact arithmetic on CPU): max-abs vs an fp64 UNet is
// the same as the fp32 UNet's (8.3e-7 vs 9.6e-7 at 256^2). Cost: 3 MFMAs at the f16 rate =
// 5.3x the fp32 MFMA rate for the same K. The 2^11 weight scale needs |w| < 32 (host-checked;
// a layer outside that range stays on the fp32 kernel).
//
// Structure (one persistent workgroup per CU; the LDS footprint forces it): the conv_stream.hip
// design with K-chunks of 16 channels.
//   * waves 0-3 consumers (one per SIMD): per tap 4 A-fragment (hi/lo x 2 pixel blocks) and 4
//     B-fragment ds_read_b128, 12 v_mfma_f32_32x32x16_f16; next tap's fragments pinned after the
//     first MFMA group; after a tile's last chunk the epilogue straight from the accumulators
//     (x 2^-11, bias, residual prefetched during the last chunk, GroupNorm granule statistics,
//     fire-and-forget dword stores that drain behind the next tile).
//   * waves 4-7 producers: halo of chunk j+2 in registers (buffer descriptors, no per-chunk VALU
//     address work), weights of chunk j+2 by LDS-DMA, prologue of chunk j+1 (GroupNorm-apply
//     [+ scale/shift] + SiLU, nearest-up, zero padding) + the f16 split, LDS writes.
// LDS: A = 4 planes [part hi/lo][channel half h][340 halo px][8 f16] (21.25 KiB) double-buffered,
// W = [tap][part][h][64 co][8 f16] (36 KiB) in a 3-slot ring (DMA two chunks ahead).
#include "conv.h"
#include "conv_dev.h"

// Timing-only ablation builds (never shipped; outputs are garbage): X3_ABLATE=
//   1 producers skip the halo loads and LDS writes (weights DMA + barriers only)
//   2 producers load the halo but skip the prologue / split / LDS writes
//   3 consumers skip the MFMAs (fragment reads kept)   4 consumers idle (barriers only)
//   5 no weight DMA                                    7 producers store without act / split VALU
//   8 producers idle (no DMA, no halo)   9 = 8 + no consumer epilogue   10 = 9 + no barriers
#ifndef X3_ABLATE
#define X3_ABLATE 0
#endif

namespace ifd {

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) f16x8 lds_h8;

constexpr int XBN = 64, XTW = 32, XTH = 8;
constexpr int XHW = XTW + 2, XHH = XTH + 2;            // halo 34 x 10
constexpr int XNP = XHW * XHH;                         // 340 halo pixels
constexpr int XITEMS = (2 * XNP + NP_T - 1) / NP_T;    // 3 (pixel, channel half) items per producer thread
constexpr int XA = 4 * XNP * 4;                        // floats per A stage (4 planes x 340 x 16 B)
constexpr int XW = 9 * 2 * 2 * XBN * 4;                // floats per W stage (36 KiB)
constexpr int XWDMA = XW / 4 / NP_T;                   // 16-B LDS-DMA rounds per producer thread (9)
constexpr int X_LDS_FLOATS = 2 * XA + 3 * XW;          // 38528 floats = 150.5 KiB
constexpr float kLo = 2048.0f;                         // 2^11
static_assert(XW % (4 * NP_T) == 0, "weight slab must be whole DMA rounds");

// LDS-DMA ops and register loads issued per producer interval (the barrier's vmcnt arithmetic)
constexpr int X_LOADS_PER_CHUNK = 2 * XITEMS + 4;

#define XBARRIER_CONSUMER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")
#define XBARRIER_PRODUCER(N) asm volatile("s_waitcnt vmcnt(" #N ") lgkmcnt(0)\n\ts_barrier" ::: "memory")

template <int XF>
struct XSet {
  f32x4 raw[XITEMS][2];
  f32x4 ca[2], cb[2];
  float vld[XITEMS];
};

template <int XF, bool SKIP>
struct XProducer {
  int ptid, hh;  // hh: channel half (8 of the chunk's 16 channels) this thread stages
  int hy[XITEMS], hx[XITEMS], ldso[XITEMS];  // ldso: 16-B slot of the pixel in the hi plane; -1 unused
  int cur_tile = -1;
  rsrc_t r0, r1, ra, rb;
  int off0[XITEMS], off1[XITEMS], so[XITEMS];  // so: output-resolution pixel (skip segment)
  int tn0;
  float valid[XITEMS];

  __device__ __forceinline__ void init(int t) {
    ptid = t;
    hh = t & 1;
#pragma unroll
    for (int i = 0; i < XITEMS; ++i) {
      const int idx = t + i * NP_T, pix = idx >> 1;
      hy[i] = pix / XHW;
      hx[i] = pix - hy[i] * XHW;
      ldso[i] = idx < 2 * XNP ? hh * XNP + pix : -1;
    }
  }

  __device__ __forceinline__ void tile_setup(const ConvParams& p, const STile& t) {
    const size_t img = (size_t)p.Hin * p.Win;
    r0 = mkrsrc(p.in0 + (size_t)t.n0 * img * p.c0);
    r1 = mkrsrc(p.in1 ? p.in1 + (size_t)t.n0 * img * p.c1 : p.in0);
    const int ctot = p.c0 + p.c1;
    // act == ACT_NONE: the coefficient loads still issue (fixed vmcnt arithmetic) from the input
    ra = p.actA ? mkrsrc(p.actA + (size_t)t.n0 * ctot) : r0;
    rb = p.actB ? mkrsrc(p.actB + (size_t)t.n0 * ctot) : r0;
    tn0 = t.n0;
#pragma unroll
    for (int i = 0; i < XITEMS; ++i) {
      const int y = t.y0 + hy[i] - 1, x = t.x0 + hx[i] - 1;
      const bool inb = ldso[i] >= 0 && y >= 0 && y < p.H && x >= 0 && x < p.W;
      int sy = y, sx = x;
      if (XF == XF_UP) { sy = y >> 1; sx = x >> 1; }
      const int sp = inb ? sy * p.Win + sx : 0;
      so[i] = inb ? y * p.W + x : 0;
      valid[i] = inb ? 1.f : 0.f;
      off0[i] = (sp * p.c0 + 8 * hh) * 4;
      off1[i] = (sp * p.c1 + 8 * hh) * 4;
    }
  }

  // Global loads of chunk k (16 channels) of tile t into set s; chunks >= nmain belong to the 1x1
  // skip segment. Exactly X_LOADS_PER_CHUNK loads on every path (see conv_stream.hip
  // SProducer::load for why).
  __device__ __forceinline__ void load(XSet<XF>& s, const ConvParams& p, const STile& t, int ti, int k, int nmain) {
    if (ti != cur_tile) {
      tile_setup(p, t);
      cur_tile = ti;
    }
    const int cb0 = 16 * k;
#pragma unroll
    for (int i = 0; i < XITEMS; ++i) s.vld[i] = valid[i];
    if (X3_ABLATE == 1 || X3_ABLATE >= 8) return;
    if (SKIP && k >= nmain) {
      // 1x1 skip segment: raw block input at output resolution (the consumer reads only the
      // centre tap, i.e. the tile's own pixels; the halo ring loads are unused)
      const int cs = 16 * (k - nmain);
      const bool first = cs < p.sc0;
      const int sc = first ? p.sc0 : p.sc1;
      const rsrc_t rs = mkrsrc((first ? p.s0 : p.s1) + (size_t)tn0 * p.H * p.W * sc);
      const int cso = (first ? cs : cs - p.sc0) * 4;
#pragma unroll
      for (int i = 0; i < XITEMS; ++i) {
        const int o = (so[i] * sc + 8 * hh) * 4;
        s.raw[i][0] = bld4(rs, o, cso);
        s.raw[i][1] = bld4(rs, o + 16, cso);
      }
      s.ca[0] = bld4(ra, 0, 0);  // unused (act NONE): keeps the per-chunk load count fixed
      s.ca[1] = bld4(ra, 0, 0);
      s.cb[0] = bld4(rb, 0, 0);
      s.cb[1] = bld4(rb, 0, 0);
      return;
    }
    if (cb0 < p.c0) {
#pragma unroll
      for (int i = 0; i < XITEMS; ++i) {
        s.raw[i][0] = bld4(r0, off0[i], cb0 * 4);
        s.raw[i][1] = bld4(r0, off0[i] + 16, cb0 * 4);
      }
    } else {
#pragma unroll
      for (int i = 0; i < XITEMS; ++i) {
        s.raw[i][0] = bld4(r1, off1[i], (cb0 - p.c0) * 4);
        s.raw[i][1] = bld4(r1, off1[i] + 16, (cb0 - p.c0) * 4);
      }
    }
    s.ca[0] = bld4(ra, 32 * hh, cb0 * 4);
    s.ca[1] = bld4(ra, 32 * hh + 16, cb0 * 4);
    s.cb[0] = bld4(rb, 32 * hh, cb0 * 4);
    s.cb[1] = bld4(rb, 32 * hh + 16, cb0 * 4);
  }

  // Weight slab of chunk k of channel tile ct into W stage `Wslot` by LDS-DMA: 9 rounds of 1 KiB
  // per producer wave for a 3x3 chunk, 1 round for a 1x1 skip chunk ([1 tap][part][h][64][8]).
  __device__ __forceinline__ void dma_weights(const ConvParams& p, int ct, int k, int nmain, int nskip,
                                              lds_f* Wslot) const {
    if (X3_ABLATE == 5 || X3_ABLATE >= 8) return;
    const int pw = __builtin_amdgcn_readfirstlane(ptid >> 6);
    if (SKIP && k >= nmain) {
      const rsrc_t r = mkrsrc(p.wskip + ((size_t)ct * nskip + (k - nmain)) * (XW / 9));
      const int qb = pw * 64;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(Wslot + 4 * qb), 16,
                                               16 * (qb + (ptid & 63)), 0, 0, 0);
      return;
    }
    const rsrc_t r = mkrsrc(p.wpack + ((size_t)ct * nmain + k) * XW);
#pragma unroll
    for (int i = 0; i < XWDMA; ++i) {
      const int qb = (i * 4 + pw) * 64;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(Wslot + 4 * qb), 16,
                                               16 * (qb + (ptid & 63)), 0, 0, 0);
    }
  }

  // GroupNorm-apply [+ SiLU] per value in SCALAR fp32: beside f16 MFMAs, packed-fp32 VALU ops
  // (v_pk_fma/mul/add_f32) cost ~22-26 issue cycles each (MI355X_MICROARCH.md, filler prices),
  // scalar ones fit the MFMA gaps. silu(t) = t * rcp(1 + 2^(-t log2 e)), as conv_stream.hip.
  __device__ __forceinline__ static float act1(float v, float a, float b, int act) {
    if (act == ACT_NONE) return v;
    const float t = a * v + b;
    if (act != ACT_AFFINE_SILU) return t;
    return t * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(t * -1.4426950408889634f));
  }

  // prologue + split: hi plane at slot ldso, lo plane 2 planes further
  __device__ __forceinline__ void store(const XSet<XF>& s, int act, lds_f* As) const {
    if (X3_ABLATE == 1 || X3_ABLATE == 2 || X3_ABLATE >= 8) return;
#pragma unroll
    for (int i = 0; i < XITEMS; ++i) {
      if (X3_ABLATE == 7 && ldso[i] >= 0) {
        f16x8 h8;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          h8[j] = (_Float16)s.raw[i][0][j];
          h8[4 + j] = (_Float16)s.raw[i][1][j];
        }
        *(lds_h8*)(As + 4 * ldso[i]) = h8;
        *(lds_h8*)(As + 4 * (ldso[i] + 2 * XNP)) = h8;
      } else if (ldso[i] >= 0) {
        f16x8 h8, l8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int g = j >> 2, c = j & 3;
          const float v = act1(s.raw[i][g][c], s.ca[g][c], s.cb[g][c], act) * s.vld[i];
          const _Float16 hv = (_Float16)v;
          h8[j] = hv;
          l8[j] = (_Float16)(v - (float)hv);  // exact difference, rounded once
        }
        *(lds_h8*)(As + 4 * ldso[i]) = h8;
        *(lds_h8*)(As + 4 * (ldso[i] + 2 * XNP)) = l8;
      }
    }
  }
};

// MFMAs over one staged chunk: TAPS taps x (3 split products x 2 x 2 fragment blocks). TAPS = 1
// is the skip segment's 1x1 chunk: centre tap of the halo layout, weight slab [1][part][h][64][8].
__device__ __forceinline__ f32x16 xmfma(f16x8 a, f16x8 b, f32x16 c) {
  if (X3_ABLATE == 3) {
    asm volatile("" : "+v"(c) : "v"(a), "v"(b));
    return c;
  }
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

template <int TAPS>
__device__ __forceinline__ void consume_x3(f32x16 (&acc)[2][2], const lds_f* As, const lds_f* Ws, const int (&pb)[2]) {
  const int lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
  const lds_f* Ah = As + 4 * (h * XNP);
  const lds_f* Al = As + 4 * ((2 + h) * XNP);
  const lds_f* Wb = Ws + 4 * (h * XBN + l32);
  f16x8 ah[2][2], al[2][2], bs[2][2], bl[2][2];
  auto fetch = [&](int tap, int slot) {
    const int toff = TAPS == 9 ? (tap / 3) * XHW + (tap % 3) : XHW + 1;
#pragma unroll
    for (int mr = 0; mr < 2; ++mr) {
      ah[slot][mr] = *(const lds_h8*)(Ah + 4 * (pb[mr] + toff));
      al[slot][mr] = *(const lds_h8*)(Al + 4 * (pb[mr] + toff));
    }
#pragma unroll
    for (int nr = 0; nr < 2; ++nr) {
      bs[slot][nr] = *(const lds_h8*)(Wb + 4 * (tap * 4 * XBN + nr * 32));
      bl[slot][nr] = *(const lds_h8*)(Wb + 4 * (tap * 4 * XBN + 2 * XBN + nr * 32));
    }
  };
  fetch(0, 0);
#pragma unroll
  for (int tap = 0; tap < TAPS; ++tap) {
    const int cur = tap & 1;
#pragma unroll
    for (int mr = 0; mr < 2; ++mr)
#pragma unroll
      for (int nr = 0; nr < 2; ++nr)
        acc[mr][nr] = xmfma(ah[cur][mr], bs[cur][nr], acc[mr][nr]);
    __builtin_amdgcn_sched_barrier(0);
    if (tap + 1 < TAPS) fetch(tap + 1, cur ^ 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int mr = 0; mr < 2; ++mr)
#pragma unroll
      for (int nr = 0; nr < 2; ++nr)
        acc[mr][nr] = xmfma(ah[cur][mr], bl[cur][nr], acc[mr][nr]);
#pragma unroll
    for (int mr = 0; mr < 2; ++mr)
#pragma unroll
      for (int nr = 0; nr < 2; ++nr)
        acc[mr][nr] = xmfma(al[cur][mr], bs[cur][nr], acc[mr][nr]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int XF, bool SKIP>
__global__ __launch_bounds__(NT, 2) void conv_x3_kernel(ConvParams p) {
  extern __shared__ __attribute__((aligned(16))) float smem_raw[];
  lds_f* const smem = (lds_f*)(smem_raw);
  lds_f* const A0 = smem;                 // stage s at A0 + s * XA
  lds_f* const W0 = smem + 2 * XA;        // ring slot s at W0 + s * XW

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool consumer = __builtin_amdgcn_readfirstlane(wave) < 4;
  const int nct = p.cout_pad / XBN;
  const int nvirt = p.npix_tiles * nct;
  const int G = gridDim.x;
  const int ntile = (nvirt - (int)blockIdx.x + G - 1) / G;  // host guarantees >= 1
  const int nmain = p.cin_pad / 16;
  const int nskip = SKIP ? p.cs_pad / 16 : 0;
  const int nch = nmain + nskip;  // chunks per tile: 3x3 segment, then the 1x1 skip segment
  const int J = ntile * nch;
  auto tile_of = [&](int ti) { return decode_tile(p, (int)blockIdx.x + ti * G, nct); };

  if (consumer) {
    const int h = lane >> 5, l32 = lane & 31;
    const int wm0 = wave * 64;
    f32x16 acc[2][2];
    int pb[2];
#pragma unroll
    for (int mr = 0; mr < 2; ++mr) {
      const int m = wm0 + mr * 32 + l32;
      pb[mr] = (m >> 5) * XHW + (m & 31);
    }
    auto zero = [&]() {
#pragma unroll
      for (int mr = 0; mr < 2; ++mr)
#pragma unroll
        for (int nr = 0; nr < 2; ++nr)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[mr][nr][r] = 0.f;
    };
    // Epilogue straight from the accumulators. Lane (h, l32) holds channel 32 nr + l32 of pixels
    // (row 2 wave + mr, column (r & 3) + 8 (r >> 2) + 4 h) of the 8 x 32 tile: one dword store per
    // register = two 128-B row segments. Bias and residual are loaded in the same layout while the
    // tile's last chunk is on the MFMAs, so the epilogue waits on nothing and its stores drain
    // behind the next tile's chunks.
    float rv[2][2][16];
    float bias2[2];
    auto col_soff = [&](int r) { return ((r & 3) + 8 * (r >> 2)) * p.cout * 4; };  // wave-uniform
    auto prefetch = [&](const STile& t) {
#pragma unroll
      for (int nr = 0; nr < 2; ++nr) bias2[nr] = gld1(p.bias + t.ct * XBN + 32 * nr + l32);
      if (!p.res) return;
      const rsrc_t rr = mkrsrc(p.res + (size_t)t.n0 * p.res_H * p.res_W * p.cout);
      if (p.res_xform == XF_NONE) {
        const int vb = (((t.y0 + 2 * wave) * p.W + t.x0 + 4 * h) * p.cout + t.ct * XBN + l32) * 4;
#pragma unroll
        for (int mr = 0; mr < 2; ++mr)
#pragma unroll
          for (int nr = 0; nr < 2; ++nr)
#pragma unroll
            for (int r = 0; r < 16; ++r)
              rv[mr][nr][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                            rr, vb + mr * p.W * p.cout * 4 + nr * 128, col_soff(r), 0));
      } else {  // XF_UP: nearest-upsampled residual (XF_DOWN residuals arrive pre-pooled)
#pragma unroll
        for (int mr = 0; mr < 2; ++mr)
#pragma unroll
          for (int nr = 0; nr < 2; ++nr)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int y = (t.y0 + 2 * wave + mr) >> 1, x = (t.x0 + 4 * h + (r & 3) + 8 * (r >> 2)) >> 1;
              const int o = ((y * p.res_W + x) * p.cout + t.ct * XBN + 32 * nr + l32) * 4;
              rv[mr][nr][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr, o, 0, 0));
            }
      }
    };
    auto epilogue = [&](const STile& t) {
      const rsrc_t ro = mkrsrc(p.out + (size_t)t.n0 * p.H * p.W * p.cout);
      const int vb = (((t.y0 + 2 * wave) * p.W + t.x0 + 4 * h) * p.cout + t.ct * XBN + l32) * 4;
#pragma unroll
      for (int nr = 0; nr < 2; ++nr) {
        float v[2][16];
#pragma unroll
        for (int mr = 0; mr < 2; ++mr)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            float x = acc[mr][nr][r] * (1.0f / kLo);  // exact rescale
            x = x + bias2[nr];
            if (p.res) x = rv[mr][nr][r] + x;  // torch order: x_res + (conv + bias)
            v[mr][r] = x;
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, x), ro,
                                                  vb + mr * p.W * p.cout * 4 + nr * 128, col_soff(r), 0);
          }
        if (p.gstat) {
          // GroupNorm granule statistics: channel over this lane's 32 pixels (two-pass), merged
          // with the other column half (lane ^ 32), then over the channel quad (lanes ^ 1, ^ 2)
          float sm = 0.f;
#pragma unroll
          for (int mr = 0; mr < 2; ++mr)
#pragma unroll
            for (int r = 0; r < 16; ++r) sm += v[mr][r];
          const float mean = sm * (1.0f / 32);
          float m2 = 0.f;
#pragma unroll
          for (int mr = 0; mr < 2; ++mr)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const float d = v[mr][r] - mean;
              m2 += d * d;
            }
          GStat g = {32.f, mean, m2};
          auto xmerge = [&](GStat a, int off) {
            GStat b;
            b.n = __shfl_xor(a.n, off);
            b.mean = __shfl_xor(a.mean, off);
            b.m2 = __shfl_xor(a.m2, off);
            return (lane & off) == 0 ? gmerge(a, b) : gmerge(b, a);
          };
          g = xmerge(g, 32);
          g = xmerge(g, 1);
          g = xmerge(g, 2);
          if (h == 0 && (l32 & 3) == 0) {
            const int e = ((t.y0 / XTH) * p.tiles_x + t.x0 / XTW) * 4 + wave;
            float* o = p.gstat + (((size_t)t.n0 * p.gstat_E + e) * (p.cout / 4) + t.ct * 16 + nr * 8 + (l32 >> 2)) * 2;
            o[0] = g.mean;
            o[1] = g.m2;
          }
        }
      }
    };
    zero();
    XBARRIER_CONSUMER();  // chunk 0 staged
    int k = 0, ti = 0;
    for (int j = 0; j < J; ++j) {
      const lds_f* Ws = W0 + (j % 3) * XW;
      if (k == nch - 1 && X3_ABLATE < 9) prefetch(tile_of(ti));
      if (X3_ABLATE == 4) {
      } else if (!SKIP || k < nmain) {
        consume_x3<9>(acc, A0 + (j & 1) * XA, Ws, pb);
      } else {
        consume_x3<1>(acc, A0 + (j & 1) * XA, Ws, pb);
      }
      if (++k == nch) {
        k = 0;
        if (X3_ABLATE < 9)
          epilogue(tile_of(ti));
        else
          asm volatile("" ::"v"(acc[0][0]), "v"(acc[0][1]), "v"(acc[1][0]), "v"(acc[1][1]));
        ++ti;
        zero();
      }
      if (X3_ABLATE != 10) XBARRIER_CONSUMER();
    }
    return;
  }

  // ---- producers: halo two chunks ahead in registers, weights two chunks ahead by LDS-DMA into
  // a 3-slot ring (chunk c in slot c % 3) ----
  const int ptid = tid - NP_T;
  XProducer<XF, SKIP> P;
  P.init(ptid);
  XSet<XF> s0, s1;
  auto load_chunk = [&](XSet<XF>& s, int c) {
    c = min(c, J - 1);
    const int ti = c / nch, kk = c - ti * nch;
    P.load(s, p, tile_of(ti), ti, kk, nmain);
  };
  // prologue of chunk c: the main segment's activation, none for the skip segment
  auto act_of = [&](int c) { return !SKIP || (c % nch) < nmain ? p.act : (int)ACT_NONE; };
  auto dma_chunk = [&](int c) {
    c = min(c, J - 1);  // past the end: re-copies the last chunk's identical bytes
    const int ti = c / nch, kk = c - ti * nch;
    P.dma_weights(p, tile_of(ti).ct, kk, nmain, nskip, W0 + (c % 3) * XW);
  };
  dma_chunk(0);
  dma_chunk(1);
  load_chunk(s0, 0);
  load_chunk(s1, 1);
  P.store(s0, act_of(0), A0);  // waits for chunk 0's loads, hence for both older DMAs
  XBARRIER_PRODUCER(10);
  static_assert(X_LOADS_PER_CHUNK == 10, "barrier vmcnt literals");
  // interval j: weights of chunk j+2 (DMA), halo of chunk j+2, LDS writes of chunk j+1, barrier
  // once chunk j+1's DMA (issued in interval j-1) has landed: younger than it are the 10 halo
  // loads of chunk j+1, the DMA of chunk j+2 (9 ops; 1 for a skip chunk) and its 10 halo loads
#define X3_PRODUCER_BARRIER()            \
  do {                                   \
    if constexpr (SKIP)                  \
      XBARRIER_PRODUCER(21);             \
    else                                 \
      XBARRIER_PRODUCER(29);             \
  } while (0)
  if (X3_ABLATE == 10) return;
  for (int j = 0; j < J; j += 2) {
    dma_chunk(j + 2);
    load_chunk(s0, j + 2);
    if (j + 1 < J) P.store(s1, act_of(j + 1), A0 + XA);
    X3_PRODUCER_BARRIER();
    if (j + 1 >= J) break;
    dma_chunk(j + 3);
    load_chunk(s1, j + 3);
    if (j + 2 < J) P.store(s0, act_of(j + 2), A0);
    X3_PRODUCER_BARRIER();
  }
#undef X3_PRODUCER_BARRIER
}

template <int XF, bool SKIP>
static int launch_x3_inst(const ConvParams& p, hipStream_t stream) {
  static bool attr_set = false;
  const size_t lds = (size_t)X_LDS_FLOATS * sizeof(float);
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_x3_kernel<XF, SKIP>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (ncu <= 0) ncu = 256;
  }
  const int nvirt = p.npix_tiles * (p.cout_pad / XBN);
  const int grid = nvirt < ncu ? nvirt : ncu;  // one workgroup per CU (LDS-bound)
  hipLaunchKernelGGL((conv_x3_kernel<XF, SKIP>), dim3(grid), dim3(NT), lds, stream, p);
  return (int)hipGetLastError();
}

}  // namespace

// Eligible: 3x3, BN = 64, BM = 256 geometry (8 x 32 tiles of one image, whole groups of 8 pixel
// tiles so the XCD map is a bijection), NHWC epilogue without split-K, cout a multiple of 64,
// 16-channel chunks on every source (main and skip), no avg-pool prologue (run_conv feeds those
// layers a pooled activation instead) nor avg-pool residual (pooled likewise). Any act, identity
// or nearest-up residual, 1x1 skip segment.
bool conv_x3_eligible(const ConvParams& p, int taps, int xform, int bn) {
  return taps == 9 && xform != XF_DOWN && bn == XBN && p.bm == 256 && p.TW == XTW && p.TH == XTH && p.IMGS == 1 &&
         p.epi == EPI_NHWC && p.ksplit == 1 && p.cout % XBN == 0 && p.cout_pad == p.cout && p.npix_tiles % 8 == 0 &&
         p.c0 % 16 == 0 && p.c1 % 16 == 0 && (!p.wskip || (p.sc0 % 16 == 0 && p.sc1 % 16 == 0)) &&
         (!p.res || p.res_xform != XF_DOWN);
}

int launch_conv_x3(const ConvParams& p, int xform, hipStream_t stream) {
  if (p.wskip) {
    if (xform == XF_NONE) return launch_x3_inst<XF_NONE, true>(p, stream);
    return (int)hipErrorInvalidValue;  // the skip segment comes with XF_NONE only (ResBlock conv2)
  }
  if (xform == XF_NONE) return launch_x3_inst<XF_NONE, false>(p, stream);
  if (xform == XF_UP) return launch_x3_inst<XF_UP, false>(p, stream);
  return (int)hipErrorInvalidValue;
}

}  // namespace ifd
