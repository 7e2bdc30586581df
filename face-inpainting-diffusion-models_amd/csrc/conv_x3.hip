// 3xf16 split-precision fused 3x3 convolution ("3xf16" precision mode) for the wide layers.
//
// Why: gfx950 has no xf32, and v_mfma_f32_32x32x2_f32 runs at the fp32 VECTOR rate (157 TF/s),
// sharing the VALU with the producer waves. The f16 matrix path is 16x faster per K. Each fp32
// operand is split into two f16 parts,
//     a = a_hi + 2^-11 a_lo',   a_hi = f16(a),  a_lo' = f16((a - a_hi) * 2^11)     (RNE both)
// (weights likewise, once at load time), and the product is rebuilt from three f16 MFMAs into ONE
// fp32 accumulator carried at scale 2^11:
//     acc += a_hi * (w_hi 2^11)  +  a_hi * w_lo'  +  a_lo' * w_hi          (then out = acc * 2^-11)
// Every f16 x f16 product is exact in fp32; the dropped a_lo' w_lo' 2^-22 term and the two
// roundings bound the relative error per product by ~2^-21, below fp32's own accumulation
// rounding over K = 9 * Cin terms. Measured on the reduced and full UNet (tests/
// test_cpu_split_numerics.py emulates this exact arithmetic on CPU): max-abs vs an fp64 UNet is
// the same as the fp32 UNet's (8.3e-7 vs 9.6e-7 at 256^2). Cost: 3 MFMAs at the f16 rate =
// 5.3x the fp32 MFMA rate for the same K. The 2^11 weight scale needs |w| < 32 (host-checked;
// a layer outside that range stays on the fp32 kernel).
//
// Structure (one persistent workgroup per CU; the LDS footprint forces it): the conv_stream.hip
// design with K-chunks of 16 channels.
//   * waves 0-3 consumers (one per SIMD): per tap 4 A-fragment (hi/lo x 2 pixel blocks) and 4
//     B-fragment ds_read_b128, 12 v_mfma_f32_32x32x16_f16; next tap's fragments pinned after the
//     first MFMA group; after a tile's last chunk the wave-private epilogue (x 2^-11, bias,
//     residual, GroupNorm granule statistics, 16-byte NHWC stores) through an LDS strip.
//   * waves 4-7 producers: halo of chunk j+2 in registers (buffer descriptors, no per-chunk VALU
//     address work), weights of chunk j+1 by LDS-DMA, prologue of chunk j+1 (GroupNorm-apply
//     [+ scale/shift] + SiLU, nearest-up, zero padding) + the f16 split, LDS writes.
// LDS per chunk stage: A = 4 planes [part hi/lo][channel half h][340 halo px][8 f16] (21.25 KiB),
// W = [tap][part][h][64 co][8 f16] (36 KiB); both double-buffered, plus 4 epilogue strips.
#include "conv.h"
#include "conv_dev.h"

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
constexpr int XLDE = XBN + 4;                          // epilogue strip row stride (floats)
constexpr int XSTRIP = 16 * XLDE;
constexpr int X_LDS_FLOATS = 2 * XA + 2 * XW + 4 * XSTRIP;  // 33664 floats = 131.5 KiB
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

template <int XF>
struct XProducer {
  int ptid, hh;  // hh: channel half (8 of the chunk's 16 channels) this thread stages
  int hy[XITEMS], hx[XITEMS], ldso[XITEMS];  // ldso: 16-B slot of the pixel in the hi plane; -1 unused
  int cur_tile = -1;
  rsrc_t r0, r1, ra, rb;
  int off0[XITEMS], off1[XITEMS];
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
    ra = mkrsrc(p.actA + (size_t)t.n0 * ctot);
    rb = mkrsrc(p.actB + (size_t)t.n0 * ctot);
#pragma unroll
    for (int i = 0; i < XITEMS; ++i) {
      const int y = t.y0 + hy[i] - 1, x = t.x0 + hx[i] - 1;
      const bool inb = ldso[i] >= 0 && y >= 0 && y < p.H && x >= 0 && x < p.W;
      int sy = y, sx = x;
      if (XF == XF_UP) { sy = y >> 1; sx = x >> 1; }
      const int sp = inb ? sy * p.Win + sx : 0;
      valid[i] = inb ? 1.f : 0.f;
      off0[i] = (sp * p.c0 + 8 * hh) * 4;
      off1[i] = (sp * p.c1 + 8 * hh) * 4;
    }
  }

  // Global loads of chunk k (16 channels) of tile t into set s; issued on every path (see
  // conv_stream.hip SProducer::load for why).
  __device__ __forceinline__ void load(XSet<XF>& s, const ConvParams& p, const STile& t, int ti, int k) {
    if (ti != cur_tile) {
      tile_setup(p, t);
      cur_tile = ti;
    }
    const int cb0 = 16 * k;
#pragma unroll
    for (int i = 0; i < XITEMS; ++i) s.vld[i] = valid[i];
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

  // Weight slab of chunk k of channel tile ct into W stage `Wslot` by LDS-DMA (9 rounds of 1 KiB
  // per producer wave).
  __device__ __forceinline__ void dma_weights(const ConvParams& p, int ct, int k, int nch, lds_f* Wslot) const {
    const rsrc_t r = mkrsrc(p.wpack + ((size_t)ct * nch + k) * XW);
    const int pw = __builtin_amdgcn_readfirstlane(ptid >> 6);
#pragma unroll
    for (int i = 0; i < XWDMA; ++i) {
      const int qb = (i * 4 + pw) * 64;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(Wslot + 4 * qb), 16,
                                               16 * (qb + (ptid & 63)), 0, 0, 0);
    }
  }

  __device__ __forceinline__ static f32x2 act2(f32x2 v, f32x2 a, f32x2 b, int act) {
    const f32x2 t = a * v + b;
    if (act != ACT_AFFINE_SILU) return t;
    const f32x2 m = t * -1.4426950408889634f;
    f32x2 d;
    d.x = __builtin_amdgcn_exp2f(m.x);
    d.y = __builtin_amdgcn_exp2f(m.y);
    d = d + 1.0f;
    f32x2 r;
    r.x = __builtin_amdgcn_rcpf(d.x);
    r.y = __builtin_amdgcn_rcpf(d.y);
    return t * r;
  }

  // prologue + split: hi plane at slot ldso, lo plane 2 planes further
  __device__ __forceinline__ void store(const XSet<XF>& s, int act, lds_f* As) const {
#pragma unroll
    for (int i = 0; i < XITEMS; ++i) {
      if (ldso[i] >= 0) {
        float v[8];
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          const f32x2 lo = act2(s.raw[i][g].xy, s.ca[g].xy, s.cb[g].xy, act) * s.vld[i];
          const f32x2 hi = act2(s.raw[i][g].zw, s.ca[g].zw, s.cb[g].zw, act) * s.vld[i];
          v[4 * g + 0] = lo.x;
          v[4 * g + 1] = lo.y;
          v[4 * g + 2] = hi.x;
          v[4 * g + 3] = hi.y;
        }
        f16x8 h8, l8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const _Float16 hv = (_Float16)v[j];
          h8[j] = hv;
          l8[j] = (_Float16)((v[j] - (float)hv) * kLo);
        }
        *(lds_h8*)(As + 4 * ldso[i]) = h8;
        *(lds_h8*)(As + 4 * (ldso[i] + 2 * XNP)) = l8;
      }
    }
  }
};

// MFMAs over one staged chunk: 9 taps x (3 split products x 2 x 2 fragment blocks).
__device__ __forceinline__ void consume_x3(f32x16 (&acc)[2][2], const lds_f* As, const lds_f* Ws, const int (&pb)[2]) {
  const int lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
  const lds_f* Ah = As + 4 * (h * XNP);
  const lds_f* Al = As + 4 * ((2 + h) * XNP);
  const lds_f* Wb = Ws + 4 * (h * XBN + l32);
  f16x8 ah[2][2], al[2][2], bs[2][2], bl[2][2];
  auto fetch = [&](int tap, int slot) {
    const int toff = (tap / 3) * XHW + (tap % 3);
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
  for (int tap = 0; tap < 9; ++tap) {
    const int cur = tap & 1;
#pragma unroll
    for (int mr = 0; mr < 2; ++mr)
#pragma unroll
      for (int nr = 0; nr < 2; ++nr)
        acc[mr][nr] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[cur][mr], bs[cur][nr], acc[mr][nr], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    if (tap + 1 < 9) fetch(tap + 1, cur ^ 1);
    f16x8 bh[2];
#pragma unroll
    for (int nr = 0; nr < 2; ++nr) bh[nr] = bs[cur][nr] * (_Float16)(1.0f / kLo);  // exact: w_hi
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int mr = 0; mr < 2; ++mr)
#pragma unroll
      for (int nr = 0; nr < 2; ++nr)
        acc[mr][nr] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[cur][mr], bl[cur][nr], acc[mr][nr], 0, 0, 0);
#pragma unroll
    for (int mr = 0; mr < 2; ++mr)
#pragma unroll
      for (int nr = 0; nr < 2; ++nr)
        acc[mr][nr] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[cur][mr], bh[nr], acc[mr][nr], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int XF>
__global__ __launch_bounds__(NT, 2) void conv_x3_kernel(ConvParams p) {
  extern __shared__ __attribute__((aligned(16))) float smem_raw[];
  lds_f* const smem = (lds_f*)(smem_raw);
  lds_f* const A0 = smem;                 // stage s at A0 + s * XA
  lds_f* const W0 = smem + 2 * XA;        // stage s at W0 + s * XW
  lds_f* const ST = smem + 2 * XA + 2 * XW;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool consumer = __builtin_amdgcn_readfirstlane(wave) < 4;
  const int nct = p.cout_pad / XBN;
  const int nvirt = p.npix_tiles * nct;
  const int G = gridDim.x;
  const int ntile = (nvirt - (int)blockIdx.x + G - 1) / G;  // host guarantees >= 1
  const int nch = p.cin_pad / 16;
  const int J = ntile * nch;
  auto tile_of = [&](int ti) { return decode_tile(p, (int)blockIdx.x + ti * G, nct); };

  if (consumer) {
    const int h = lane >> 5, l32 = lane & 31;
    const int wm0 = wave * 64;
    lds_f* const strip = ST + wave * XSTRIP;
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
    const int q = lane & 15, prow = lane >> 4;
    // wave-private epilogue (as conv_stream2_kernel), accumulators rescaled by 2^-11 (exact)
    auto epilogue = [&](const STile& t) {
      const rsrc_t ro = mkrsrc(p.out + (size_t)t.n0 * p.H * p.W * p.cout);
      const rsrc_t rr = mkrsrc(p.res ? p.res + (size_t)t.n0 * p.res_H * p.res_W * p.cout : p.out);
      const int co = t.ct * XBN + 4 * q;
      const f32x4 bias4 = gld4(p.bias + co);
      GStat gs = {0.f, 0.f, 0.f};
#pragma unroll
      for (int piece = 0; piece < 4; ++piece) {
        const int mr = piece >> 1, half = piece & 1;
        int goff[4];
        f32x4 rv[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int m = wm0 + 32 * mr + 16 * half + prow + 4 * v;
          const int y = t.y0 + (m >> 5), x = t.x0 + (m & 31);
          goff[v] = ((y * p.W + x) * p.cout + co) * 4;
          if (p.res) {
            const int ro_ = p.res_xform == XF_NONE ? goff[v]
                                                   : (((y >> 1) * p.res_W + (x >> 1)) * p.cout + co) * 4;
            rv[v] = bld4(rr, ro_, 0);
          }
        }
#pragma unroll
        for (int nr = 0; nr < 2; ++nr)
#pragma unroll
          for (int rr8 = 0; rr8 < 8; ++rr8) {
            const int r = 8 * half + rr8;
            const int pp = (r & 3) + 8 * ((r >> 2) & 1) + 4 * h;
            strip[pp * XLDE + nr * 32 + l32] = acc[mr][nr][r] * (1.0f / kLo);
          }
        f32x4 vals[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          f32x4 val = *(const lds_f4*)(strip + (prow + 4 * v) * XLDE + 4 * q);
          val = val + bias4;
          if (p.res) val = rv[v] + val;
          bst4(ro, goff[v], val);
          vals[v] = val;
        }
        if (p.gstat) {
          const GStat g = gstat_of<4>(vals);
          gs = piece == 0 ? g : gmerge(gs, g);
        }
      }
      if (p.gstat) {
        gs = gstat_xlanes16(gs);
        if (lane < 16) {
          const int e = ((t.y0 / XTH) * p.tiles_x + t.x0 / XTW) * 4 + wave;
          float* o = p.gstat + (((size_t)t.n0 * p.gstat_E + e) * (p.cout / 4) + t.ct * 16 + q) * 2;
          o[0] = gs.mean;
          o[1] = gs.m2;
        }
      }
    };
    zero();
    XBARRIER_CONSUMER();  // chunk 0 staged
    int k = 0, ti = 0;
    for (int j = 0; j < J; ++j) {
      consume_x3(acc, A0 + (j & 1) * XA, W0 + (j & 1) * XW, pb);
      if (++k == nch) {
        k = 0;
        epilogue(tile_of(ti++));
        zero();
      }
      XBARRIER_CONSUMER();
    }
    return;
  }

  // ---- producers: halo two chunks ahead in registers, weights one chunk ahead by LDS-DMA ----
  const int ptid = tid - NP_T;
  XProducer<XF> P;
  P.init(ptid);
  XSet<XF> s0, s1;
  auto load_chunk = [&](XSet<XF>& s, int c) {
    c = min(c, J - 1);
    const int ti = c / nch, kk = c - ti * nch;
    P.load(s, p, tile_of(ti), ti, kk);
  };
  auto dma_chunk = [&](int c) {
    c = min(c, J - 1);
    const int ti = c / nch, kk = c - ti * nch;
    P.dma_weights(p, tile_of(ti).ct, kk, nch, W0 + (c & 1) * XW);
  };
  dma_chunk(0);
  load_chunk(s0, 0);
  load_chunk(s1, 1);
  P.store(s0, p.act, A0);
  XBARRIER_PRODUCER(10);  // chunk 0's weights landed (younger: chunk 1's 10 halo/coef loads)
  static_assert(X_LOADS_PER_CHUNK == 10, "barrier vmcnt literal");
  for (int j = 0; j < J; j += 2) {
    dma_chunk(j + 1);
    load_chunk(s0, j + 2);
    if (j + 1 < J) P.store(s1, p.act, A0 + XA);
    XBARRIER_PRODUCER(10);
    if (j + 1 >= J) break;
    dma_chunk(j + 2);
    load_chunk(s1, j + 3);
    if (j + 2 < J) P.store(s0, p.act, A0);
    XBARRIER_PRODUCER(10);
  }
}

template <int XF>
static int launch_x3_inst(const ConvParams& p, hipStream_t stream) {
  static bool attr_set = false;
  const size_t lds = (size_t)X_LDS_FLOATS * sizeof(float);
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_x3_kernel<XF>),
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
  hipLaunchKernelGGL((conv_x3_kernel<XF>), dim3(grid), dim3(NT), lds, stream, p);
  return (int)hipGetLastError();
}

}  // namespace

// Same eligibility as the fp32 streaming kernel plus 16-channel chunks on both concat sources.
bool conv_x3_eligible(const ConvParams& p, int taps, int xform, int bn) {
  return conv_stream_eligible(p, taps, xform, bn) && p.c0 % 16 == 0 && p.c1 % 16 == 0;
}

int launch_conv_x3(const ConvParams& p, int xform, hipStream_t stream) {
  if (xform == XF_NONE) return launch_x3_inst<XF_NONE>(p, stream);
  if (xform == XF_UP) return launch_x3_inst<XF_UP>(p, stream);
  return (int)hipErrorInvalidValue;
}

}  // namespace ifd
