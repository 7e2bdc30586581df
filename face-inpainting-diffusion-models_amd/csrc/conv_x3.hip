// 3xf16 split-precision fused 3x3 convolution ("3xf16" precision mode).
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
// absolute), below fp32's own accumulation rounding over K = 9 * Cin terms. Measured on the
// reduced and full UNet (tests/test_cpu_split_numerics.py emulates this exact arithmetic on CPU):
// max-abs vs an fp64 UNet is the same as the fp32 UNet's (8.7e-7 vs 9.6e-7 at 256^2). Cost: 3
// MFMAs at the f16 rate = 5.3x the fp32 MFMA rate for the same K. The 2^11 weight scale needs
// |w| < 32 (host-checked; a layer outside that range stays on the fp32 kernel).
//
// Structure: one persistent workgroup per CU (the LDS footprint forces it) walks a strided list
// of work units = (256-pixel tile of one image: 8 x 32 or 16 x 16 pixels, 64-channel tile, K split
// z); K runs in chunks of 16 channels and the chunk stream continues across units without a break.
// Low-resolution layers split K over S units so the grid covers the chip; their partial sums go
// to slabs that splitk_reduce (conv.hip) finishes with bias and residual.
//   * waves 0-3 consumers (one per SIMD): per tap 4 A-fragment (hi/lo x 2 pixel blocks) and 4
//     B-fragment ds_read_b128, 12 v_mfma_f32_32x32x16_f16; next tap's fragments pinned after the
//     first MFMA group; after a unit's last chunk the epilogue straight from the accumulators
//     (x 2^-11, bias, residual prefetched during the last chunk, GroupNorm granule statistics,
//     fire-and-forget dword stores that drain behind the next unit).
//   * waves 4-7 producers: halo of chunk j+2 in registers (buffer descriptors, no per-chunk VALU
//     address work), weights of chunk j+2 by LDS-DMA, prologue of chunk j+1 (GroupNorm-apply
//     [+ scale/shift] + SiLU, nearest-up, zero padding) + the f16 split, LDS writes.
//   * a ResBlock's 1x1 skip segment (the chunks after the 3x3 ones, XSK channels each): the
//     producers LDS-DMA only the chunk's weight slab into the ring; the raw fp32 operand goes
//     straight from HBM into the consumer waves' registers (no wave shares a pixel row of the 1x1
//     operand, so LDS staging buys no reuse), two chunks deep: the two lanes of a pixel load its
//     XSK x 4 B as whole cache lines, the first chunks during the unit's last 3x3 chunk, then chunk
//     s + 2 while chunk s is split and consumed.
// LDS: A = 4 planes [part hi/lo][channel half h][halo px][8 f16] (<= 21.25 KiB) double-buffered,
// W = [tap][part][h][64 co][8 f16] (36 KiB) in a 3-slot ring (DMA two chunks ahead).
#include "conv.h"
#include "conv_dev.h"

// Timing-only ablation builds (never shipped; outputs are garbage): X3_ABLATE=
//   1 producers skip the halo loads and LDS writes (weights DMA + barriers only)
//   2 producers load the halo but skip the prologue / split / LDS writes
//   4 consumers skip the 3x3 MFMAs        5 no weight DMA
//   8 producers idle (no DMA, no halo)   12 skip operands all read from one tile (cache-resident)
//   13 no epilogue (accumulators discarded)   14 epilogue without stores   15 epilogue without GN statistics
#ifndef X3_ABLATE
#define X3_ABLATE 0
#endif
// Cache policy of the epilogue's output stores: nontemporal (NT). A layer's output is read by the next
// launch, long after it has left the 4 MiB L2 at the 128^2 / 256^2 sizes that dominate; same-box
// interleaved +0.4 % per UNet eval (17.7 vs 17.8 ms, profiles/r04b/lds/nt.txt). The residual loads'
// policy (NT as well) measured the same, so they keep the default.
#ifndef X3_STORE_AUX
#define X3_STORE_AUX 2
#endif
// Deferred output stores (X3_DEFER = phases, 0 = off): a unit whose successor on the block has at least
// X3_DEFER chunks before its residual prefetch leaves its outputs (+ bias + residual) in the residual
// registers and issues the 64 stores per lane as side work of the successor's first X3_DEFER chunks, so
// that the consumer's MFMA stream does not wait behind the chip-wide store burst at every unit end
// (profiles/r05a: the epilogue is store-drain-bound, ~6k of the +7.5k cycles a unit transition costs).
#ifndef X3_DEFER
#define X3_DEFER 4
#endif
#ifndef X3_DEFER1_OFF  // (development A/B: 1 = no deferral for one-chunk units)
#define X3_DEFER1_OFF 0
#endif
#ifndef X3_RES_AUX
#define X3_RES_AUX 0
#endif
// IFD_TRACE=1 builds: shader-cycle stamps (s_memtime) of the first 16 chunk intervals into
// ConvParams::trace, 64 slots per block: [j] consumer wave 0 at interval start, [16 + j] after
// its MFMAs are issued; producer wave 4: [48 + j] after the LDS writes of interval j, [32 + j]
// after its DMA + loads are issued (just before its barrier).
#ifndef IFD_TRACE
#define IFD_TRACE 0
#endif

namespace ifd {

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) f16x8 lds_h8;
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_u4;

// The f16 split of two values: hi = f16(v) (one v_cvt_pk_f16_f32 for the pair), lo = f16(v - hi)
// by v_fma_mix{lo,hi}_f16 reading hi's halves as f16 (v - hi is exact in fp32, rounded once). The
// empty asm pins v as an fp32 register value: the compiler would otherwise fold the product that
// makes v into a v_fma_mix conversion — a single rounding for one use of hi and a double one for
// the other.
__device__ __forceinline__ void split2(float v0, float v1, unsigned& h, unsigned& l) {
  asm volatile("" : "+v"(v0), "+v"(v1));
  const f16x2 h2 = __builtin_convertvector(f32x2{v0, v1}, f16x2);
  h = __builtin_bit_cast(unsigned, h2);
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%3 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %2, 1.0, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(l)
      : "v"(v0), "v"(v1), "v"(h));
}


constexpr int XBN = 64;
constexpr int XNPMAX = 400;                    // halo pixels of the largest tile (4 images x 10 x 10)
constexpr int XA = 4 * XNPMAX * 4;             // floats per A stage (4 planes x 400 px x 16 B)
constexpr int XW = 9 * 2 * 2 * XBN * 4;        // floats per weight-ring slot (36 KiB)
constexpr int XWDMA = XW / 4 / NP_T;           // 16-B LDS-DMA rounds per producer thread (9)
constexpr int X_LDS_FLOATS = 2 * XA + 3 * XW;  // 40448 floats = 158 KiB
constexpr int XSK = 32;                        // channels per 1x1 skip chunk
constexpr int XSQ = XSK / 16;                  // k = 16 MFMA steps (sub-chunks) per skip chunk
constexpr int XSL = XSQ * 2;                   // operand quads per lane (channel half: XSK / 2 channels)
constexpr int XWS = XSQ * 2 * 2 * XBN * 4;     // floats per skip weight slab [q][part][h][64 co][8 f16]
constexpr float kLo = 2048.0f;                 // 2^11
static_assert(XW % (4 * NP_T) == 0 && XWS % (4 * NP_T) == 0, "weight slabs must be whole DMA rounds");
static_assert(XWS <= XW, "skip slab fits a ring slot");

#define XBARRIER_CONSUMER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")
#define XBARRIER_PRODUCER(N) asm volatile("s_waitcnt vmcnt(" #N ") lgkmcnt(0)\n\ts_barrier" ::: "memory")

// Tile of 256 output pixels: TW x TH of one image (TW = 32, 16), or TW = 8: four whole 8 x 8
// images (the 8x8 layers), one per consumer wave; halo (TW + 2) x (TH + 2) per image.
template <int TW>
struct XGeo {
  static constexpr int IMG = TW == 8 ? 4 : 1;               // images per tile
  static constexpr int TH = 256 / (TW * IMG);
  static constexpr int HW = TW + 2;
  static constexpr int HP = HW * (TH + 2);                  // halo pixels per image
  static constexpr int NP = IMG * HP;                       // 340 (8 x 32), 324 (16 x 16), 400 (4 x 8 x 8)
  static constexpr int ITEMS = (2 * NP + NP_T - 1) / NP_T;  // (pixel, channel half) items per producer thread
  static constexpr int LOADS = 2 * ITEMS + 4;               // register loads per 3x3 chunk (vmcnt arithmetic)
  static_assert(NP <= XNPMAX && (ITEMS == 3 || (IMG == 4 && ITEMS == 4)), "halo staging items");
};
// vmcnt ops per chunk of a producer thread, in issue order: a 3x3 chunk = XDMA3 weight DMAs then
// XGeo::LOADS halo / coefficient register loads; a skip chunk = XDMA1 weight DMAs and no register
// load (the barrier's vmcnt arithmetic).
constexpr int XDMA3 = 9, XDMA1 = XWS / 4 / NP_T;

// Work unit L -> (tile, split z). The S splits of a tile are consecutive L; pixel tiles in groups
// of 8 get channel-tile IDs 8 apart (conv.hip's XCD-aware map) when the tile count allows: block b
// runs units L = b + u G, and blocks b and b + 8 sit on the same XCD (workgroups are dealt to the 8
// XCDs round robin), so the channel tiles of a pixel tile run at the same time on one XCD and fetch
// their shared input (halo, skip operand) from HBM once. (Round 3's alternative, a block running the
// channel tiles of one pixel tile back to back, measured 1 % slower per eval: profiles/r04a.) Every
// divisor is a power of two (run_conv requires power-of-two sizes; S, cout / 64 in {1, 2, 4, 8}),
// so the decode is shifts and masks on log2 values taken once per kernel.
struct XDec {
  int lks, lnct, ltx, lty, limg;
  bool xcd;  // conv.hip's XCD-aware map (pixel tiles in groups of 8)
  int nct;   // channel tiles; not a power of two (the 1536-wide qkv 1x1): decoded by division
  bool pow2;
};
__device__ __forceinline__ XDec x3_dec(const ConvParams& p, int nct) {
  const bool pow2 = (nct & (nct - 1)) == 0;
  return {__builtin_ctz(p.ksplit), __builtin_ctz(nct), __builtin_ctz(p.tiles_x), __builtin_ctz(p.tiles_y),
          __builtin_ctz(p.IMGS), pow2 && p.npix_tiles % 8 == 0, nct, pow2};
}
// Unit u of block b. NP2: non-power-of-two channel-tile counts allowed (the 1x1-only launches, which
// use the SKIP instantiations; the others keep the shift-only decode and its register budget)
template <bool NP2>
__device__ __forceinline__ STile x3_unit(const ConvParams& p, const XDec& d, int b, int u, int& z) {
  STile t;
  int bx;
  {
    const int L = b + u * (int)gridDim.x;
    z = L & ((1 << d.lks) - 1);
    const int v = L >> d.lks;
    if (NP2 && !d.pow2) {
      bx = v / d.nct;
      t.ct = v - bx * d.nct;
    } else if (d.xcd) {
      const int rr = v & ((8 << d.lnct) - 1);
      t.ct = rr >> 3;
      bx = ((v >> (3 + d.lnct)) << 3) + (rr & 7);
    } else {
      t.ct = v & ((1 << d.lnct) - 1);
      bx = v >> d.lnct;
    }
  }
  t.x0 = (bx & ((1 << d.ltx) - 1)) * p.TW;
  bx >>= d.ltx;
  t.y0 = (bx & ((1 << d.lty) - 1)) * p.TH;
  t.n0 = (bx >> d.lty) << d.limg;
  return t;
}

#ifndef X3_PINF
#define X3_PINF 1
#endif

template <int ITEMS>
struct XSet {
  f32x4 raw[ITEMS][2];
  f32x4 ca[2], cb[2];
  float vld[ITEMS];
};

template <int XF, bool SKIP, int TW, int NPROD>
struct XProducer {
  using Geo = XGeo<TW>;
  static constexpr int IT = Geo::ITEMS;
  using Set = XSet<IT>;
  int ptid, hh;  // hh: channel half (8 of the chunk's 16 channels) this thread stages
  int pimg;      // four-image tiles: the image of the tile this thread stages (= its wave): one
                 // image per thread, so one set of GroupNorm coefficients per thread
  int lane16;    // 16 * lane: the weight DMA's per-lane byte offset
  int hi[IT], hy[IT], hx[IT], ldso[IT];  // image of the tile, halo row / column; ldso: 16-B slot of
                                         // the pixel in the hi plane, -1 unused
  int cur_unit = -1;
  rsrc_t r0, r1, ra, rb;
  int off0[IT], off1[IT];
  // Skip chunks issue their weight DMA only - no register load, no per-chunk VALU: a dead
  // placeholder load would free its VGPRs for VALU temporaries, the compiler would then wait (vmcnt)
  // for it, and as its vmcnt model omits LDS-DMA ops, that wait would also drain the DMA in flight.
  float valid[IT];
  float gmax = 0.f;  // range guard: largest |operand| this thread split

  __device__ __forceinline__ void init(int t) {
    ptid = t;
    hh = t & 1;
    lane16 = 16 * (t & 63);
    pimg = Geo::IMG > 1 ? t >> 6 : 0;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      if (Geo::IMG > 1) {  // items (lane + 64 i) of the wave's image: 2 x 100 per image
        const int idx = (t & 63) + 64 * i, pix = idx >> 1;
        hi[i] = pimg;
        hy[i] = pix / Geo::HW;
        hx[i] = pix - hy[i] * Geo::HW;
        ldso[i] = idx < 2 * Geo::HP ? hh * Geo::NP + pimg * Geo::HP + pix : -1;
      } else {
        const int idx = t + i * NP_T, pix = idx >> 1;
        hi[i] = 0;
        hy[i] = pix / Geo::HW;
        hx[i] = pix - hy[i] * Geo::HW;
        ldso[i] = idx < 2 * Geo::NP ? hh * Geo::NP + pix : -1;
      }
    }
  }

  __device__ __forceinline__ void tile_setup(const ConvParams& p, const STile& t) {
    const size_t img = (size_t)p.Hin * p.Win;
    r0 = mkrsrc(p.in0 + (size_t)t.n0 * img * p.c0);
    r1 = mkrsrc(p.in1 ? p.in1 + (size_t)t.n0 * img * p.c1 : p.in0);
    const int ctot = p.c0 + p.c1;
    // act == ACT_NONE: the coefficient loads still issue (fixed vmcnt arithmetic), from the start of this thread's
    // own image of the input (offsets < ctot * 4 B). Not from r0: a partial four-image tile moves the tile origin
    // n0 of its spare slots below image 0 (unit_of), and r0's offset 0 then lies below the tensor (the status-700
    // fault of the training step's dgrad convs, profiles/r05r/repro4_async.txt).
    const rsrc_t rself = mkrsrc(p.in0 + ((size_t)t.n0 + pimg) * img * p.c0);
    ra = p.actA ? mkrsrc(p.actA + ((size_t)t.n0 + pimg) * ctot) : rself;
    rb = p.actB ? mkrsrc(p.actB + ((size_t)t.n0 + pimg) * ctot) : rself;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int y = t.y0 + hy[i] - 1, x = t.x0 + hx[i] - 1;
      const bool inb = ldso[i] >= 0 && y >= 0 && y < p.H && x >= 0 && x < p.W;
      int sy = y, sx = x;
      if (XF == XF_UP) { sy = y >> 1; sx = x >> 1; }
      // a padding pixel reads its own image's first pixel (times valid = 0): the base is the tile origin n0, which
      // a partial four-image tile moves below 0 for its spare slots (unit_of), so offset 0 is not in the batch
      const int sp = inb ? (hi[i] * p.Hin + sy) * p.Win + sx : hi[i] * p.Hin * p.Win;
      valid[i] = inb ? 1.f : 0.f;
      off0[i] = (sp * p.c0 + 8 * hh) * 4;
      off1[i] = (sp * p.c1 + 8 * hh) * 4;
    }
  }

  // Global loads of 3x3 chunk c of the entered unit into set s: Geo::LOADS loads.
  // per-unit state (descriptors, pixel offsets): before the unit's first DMA or load
  __device__ __forceinline__ void enter(const ConvParams& p, const STile& t, int u) {
    if (u != cur_unit) {
      tile_setup(p, t);
      cur_unit = u;
    }
  }

  // ism: a 3x3 chunk (idx = its 16-channel chunk of the main input) or a 1x1 skip chunk (idx =
  // its 64-channel chunk of the skip input)
  __device__ __forceinline__ void load(Set& s, const ConvParams& p, bool ism, int idx) {
#pragma unroll
    for (int i = 0; i < IT; ++i) s.vld[i] = valid[i];
    if (X3_ABLATE == 1 || X3_ABLATE == 8) return;
    if (SKIP && !ism) return;  // operand by DMA (see dma)
    const int cb0 = 16 * idx;
    if (cb0 < p.c0) {
#pragma unroll
      for (int i = 0; i < IT; ++i) {
        s.raw[i][0] = bld4(r0, off0[i], cb0 * 4);
        s.raw[i][1] = bld4(r0, off0[i] + 16, cb0 * 4);
      }
    } else {
#pragma unroll
      for (int i = 0; i < IT; ++i) {
        s.raw[i][0] = bld4(r1, off1[i], (cb0 - p.c0) * 4);
        s.raw[i][1] = bld4(r1, off1[i] + 16, (cb0 - p.c0) * 4);
      }
    }
    s.ca[0] = bld4(ra, 32 * hh, cb0 * 4);
    s.ca[1] = bld4(ra, 32 * hh + 16, cb0 * 4);
    s.cb[0] = bld4(rb, 32 * hh, cb0 * 4);
    s.cb[1] = bld4(rb, 32 * hh + 16, cb0 * 4);
  }

  // LDS-DMA of chunk idx of channel tile ct into ring slot `Wslot`: the 3x3 weight slab (XDMA3
  // rounds of 1 KiB per producer wave) or the 1x1 skip slab (XDMA1 rounds).
  __device__ __forceinline__ void dma(const ConvParams& p, int ct, bool ism, int idx, int nmain, int nskip,
                                      lds_f* Wslot) const {
    if (X3_ABLATE == 5 || X3_ABLATE == 8) return;
    const int pw = __builtin_amdgcn_readfirstlane(ptid >> 6);
    if (SKIP && !ism) {
      const rsrc_t r = mkrsrc(p.wskip + ((size_t)ct * nskip + idx) * XWS);
#pragma unroll
      for (int i = 0; i < XDMA1; ++i) {
        const int qb = (i * 4 + pw) * 64;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(Wslot + 4 * qb), 16,
                                                 lane16, 16 * qb, 0, 0);
      }
      return;
    }
    // per-lane offset = the loop-invariant 16 * lane (lane16), the round in the scalar offset: a
    // per-round VALU temporary would share VGPRs with in-flight halo loads and make the compiler
    // wait for them (vmcnt) before the DMA issues
    const rsrc_t r = mkrsrc(p.wpack + ((size_t)ct * nmain + idx) * XW);
#pragma unroll
    for (int i = 0; i < XWDMA; ++i) {
      const int qb = (i * 4 + pw) * 64;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(Wslot + 4 * qb), 16,
                                               lane16, 16 * qb, 0, 0);
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

  // prologue + split: hi plane at slot ldso, lo plane 2 planes further. The activation kind is
  // uniform: one branch per store, not two v_cndmask per value (13 % of the producer's VALU).
  __device__ __forceinline__ void store(const Set& s, int act, lds_f* As) {
    if (act == ACT_AFFINE_SILU)
      store_act<ACT_AFFINE_SILU>(s, As);
    else if (act == ACT_NONE)
      store_act<ACT_NONE>(s, As);
    else
      store_act<ACT_AFFINE>(s, As);
  }
  template <int ACT>
  __device__ __forceinline__ void store_act(const Set& s, lds_f* As) {
    if (X3_ABLATE == 1 || X3_ABLATE == 2 || X3_ABLATE == 8) return;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      if (ldso[i] >= 0) {
        // SiLU: the zero padding rides in the exponent — 2^(+inf) = inf, rcp(1 + inf) = 0, t * 0 = 0
        // for the finite t of a padding pixel — instead of a multiply by the validity per value
        const float pinf = s.vld[i] != 0.f ? 0.f : __builtin_inff();
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int g = j >> 2, c = j & 3;
          if (ACT == ACT_AFFINE_SILU && X3_PINF) {
            const float t = fmaf(s.ca[g][c], s.raw[i][g][c], s.cb[g][c]);
            v[j] = t * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(fmaf(t, -1.4426950408889634f, pinf)));
          } else {
            v[j] = act1(s.raw[i][g][c], s.ca[g][c], s.cb[g][c], ACT) * s.vld[i];
          }
        }
        // range guard: |v| >= 65504 would split into an f16 inf (max3 chains: ~0.6 VALU op per value)
        gmax = fmaxf(gmax, fmaxf(fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))),
                                 fmaxf(fmaxf(fabsf(v[4]), fabsf(v[5])), fmaxf(fabsf(v[6]), fabsf(v[7])))));
        unsigned h[4], l[4];
        if (NPROD == 1) {  // f16 mode: the hi part only (one conversion per pair), no lo plane
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            float a0 = v[2 * k], a1 = v[2 * k + 1];
            asm volatile("" : "+v"(a0), "+v"(a1));
            h[k] = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a0, a1}, f16x2));
          }
          *(lds_u4*)(As + 4 * ldso[i]) = u32x4{h[0], h[1], h[2], h[3]};
          continue;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) split2(v[2 * k], v[2 * k + 1], h[k], l[k]);
        *(lds_u4*)(As + 4 * ldso[i]) = u32x4{h[0], h[1], h[2], h[3]};
        *(lds_u4*)(As + 4 * (ldso[i] + 2 * Geo::NP)) = u32x4{l[0], l[1], l[2], l[3]};
      }
    }
  }
};

// The lower and the upper wave half's value of v, in every lane (the lane ^ 32 exchange of the
// GroupNorm merges), by two v_permlane32_swap against zero: [v_lo, 0] | [0, v_lo] and [v_hi, 0] |
// [0, v_hi]. (hipcc miscompiles the builtin given the same value twice: both results come back in
// one register.)
__device__ __forceinline__ void wave_halves(float v, float& lo, float& hi) {
  const unsigned x = __builtin_bit_cast(unsigned, v);
  const auto a = __builtin_amdgcn_permlane32_swap(x, 0u, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(0u, x, false, false);
  lo = __builtin_bit_cast(float, a[0] | b[0]);
  hi = __builtin_bit_cast(float, a[1] | b[1]);
}

__device__ __forceinline__ f32x16 xmfma(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// MFMAs over one staged 3x3 chunk: 9 taps x (3 split products x 2 x 2 fragment blocks);
// operand = the halo stage (planes of Geo::NP pixels, pb = halo pixel).
// NPROD = 1 (the f16 precision mode): the hi x hi product only.
struct NoSide {
  template <int K>
  __device__ __forceinline__ void step() {}
};

// side.step<k>() runs after MFMA group k (k = 3 tap + group, 27 per chunk): work interleaved into the
// MFMA stream (the residual prefetch of a unit's last chunks)
template <int TW, int NPROD, class Side = NoSide>
__device__ __forceinline__ void consume_x3(f32x16 (&acc)[2][2], f32x16 (&accl)[2][2], const lds_f* As, const lds_f* Ws,
                                           const int (&pb)[2], Side&& side = Side()) {
  using Geo = XGeo<TW>;
  const int lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
  const lds_f* Ah = As + 4 * (h * Geo::NP);
  const lds_f* Al = As + 4 * ((2 + h) * Geo::NP);
  const lds_f* Wb = Ws + 4 * (h * XBN + l32);
  // hi fragments double-buffered (the next tap's are read right after the current tap's first MFMA
  // group); lo fragments single-buffered, each re-read as soon as the group that uses it is issued,
  // eight MFMAs before its next use (16 registers fewer: the residual prefetch fits beside both
  // accumulator sets' successors)
  f16x8 ah[2][2], bs[2][2], al[2], bl[2];
  auto toff = [&](int tap) { return (tap / 3) * Geo::HW + (tap % 3); };
  auto fetch_hi = [&](int tap, int slot) {
#pragma unroll
    for (int mr = 0; mr < 2; ++mr) ah[slot][mr] = *(const lds_h8*)(Ah + 4 * (pb[mr] + toff(tap)));
#pragma unroll
    for (int nr = 0; nr < 2; ++nr) bs[slot][nr] = *(const lds_h8*)(Wb + 4 * (tap * 4 * XBN + nr * 32));
  };
  auto fetch_bl = [&](int tap) {
#pragma unroll
    for (int nr = 0; nr < 2; ++nr) bl[nr] = *(const lds_h8*)(Wb + 4 * (tap * 4 * XBN + 2 * XBN + nr * 32));
  };
  auto fetch_al = [&](int tap) {
#pragma unroll
    for (int mr = 0; mr < 2; ++mr) al[mr] = *(const lds_h8*)(Al + 4 * (pb[mr] + toff(tap)));
  };
  fetch_hi(0, 0);
  if (NPROD == 3) {
    fetch_bl(0);
    fetch_al(0);
  }
  auto tap_step = [&](auto tapc) __attribute__((always_inline)) {
    constexpr int tap = decltype(tapc)::value;
    constexpr int cur = tap & 1;
#pragma unroll
    for (int mr = 0; mr < 2; ++mr)
#pragma unroll
      for (int nr = 0; nr < 2; ++nr)
        acc[mr][nr] = xmfma(ah[cur][mr], bs[cur][nr], acc[mr][nr]);
    __builtin_amdgcn_sched_barrier(0);
    if (tap + 1 < 9) fetch_hi(tap + 1, cur ^ 1);
    side.template step<3 * tap>();
    if (NPROD == 1) {  // one group per tap: all of the tap's side work here
      side.template step<3 * tap + 1>();
      side.template step<3 * tap + 2>();
      __builtin_amdgcn_sched_barrier(0);
      return;
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int mr = 0; mr < 2; ++mr)
#pragma unroll
      for (int nr = 0; nr < 2; ++nr)
        accl[mr][nr] = xmfma(ah[cur][mr], bl[nr], accl[mr][nr]);
    __builtin_amdgcn_sched_barrier(0);
    if (tap + 1 < 9) fetch_bl(tap + 1);
    side.template step<3 * tap + 1>();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int mr = 0; mr < 2; ++mr)
#pragma unroll
      for (int nr = 0; nr < 2; ++nr)
        accl[mr][nr] = xmfma(al[mr], bs[cur][nr], accl[mr][nr]);
    __builtin_amdgcn_sched_barrier(0);
    if (tap + 1 < 9) fetch_al(tap + 1);
    side.template step<3 * tap + 2>();
    __builtin_amdgcn_sched_barrier(0);
  };
  tap_step(std::integral_constant<int, 0>{});
  tap_step(std::integral_constant<int, 1>{});
  tap_step(std::integral_constant<int, 2>{});
  tap_step(std::integral_constant<int, 3>{});
  tap_step(std::integral_constant<int, 4>{});
  tap_step(std::integral_constant<int, 5>{});
  tap_step(std::integral_constant<int, 6>{});
  tap_step(std::integral_constant<int, 7>{});
  tap_step(std::integral_constant<int, 8>{});
}

// The residual prefetch of a unit (identity or nearest-up residual) as side work of the MFMA stream:
// the 64 loads of a lane's tile (register (mr, nr, r) = channel 32 nr + l32 of tile pixel
// wm0 + 32 mr + 8 (r >> 2) + 4 h + (r & 3)) go out 2-3 per MFMA group over one chunk instead of as one
// 64-load burst ahead of it. Offsets: a per-mr lane base (nr * 128 as the immediate) + a wave-uniform
// scalar part; the kind (identity / nearest-up) is a select, not a branch in the MFMA stream.
template <int TW, int I0, int I1, int KN>  // loads [I0, I1) spread over MFMA groups 0 .. KN-1
struct ResSide {
  float (&rv)[2][2][16];
  rsrc_t rr;
  int vb[2];           // lane base per mr
  int up;              // nearest-up residual
  int W4, cout4;       // XF_NONE: output row width x cout x 4 B, cout x 4 B
  int wm0, y0, x0, res_W;
  template <int K>
  __device__ __forceinline__ void step() const {
    constexpr int lo = K < KN ? I0 + K * (I1 - I0) / KN : I1, hi = K < KN ? I0 + (K + 1) * (I1 - I0) / KN : I1;
#pragma unroll
    for (int i = lo; i < hi; ++i) {
      const int mr = i >> 5, nr = (i >> 4) & 1, r = i & 15;
      const int lin = 8 * (r >> 2) + (r & 3);
      const int s_none = ((lin / TW) * W4) + (lin % TW) * cout4;
      const int ub = wm0 + 32 * mr + 8 * (r >> 2);
      const int yy = (y0 + ub / TW) >> 1, xx = ((x0 + ub % TW) >> 1) + ((r & 3) >> 1);
      const int s_up = (yy * res_W + xx) * cout4;
      rv[mr][nr][r] = __builtin_bit_cast(
          float, __builtin_amdgcn_raw_buffer_load_b32(rr, vb[mr] + nr * 128, up ? s_up : s_none, X3_RES_AUX));
    }
  }
};

// A unit's deferred output stores as side work of the NEXT unit's MFMA stream (X3_DEFER phases, one per
// chunk): phase PH issues stores [PH NS, PH NS + NS) of the 64 per lane, spread over the chunk's 27 MFMA
// groups, from the registers the values were left in (the residual-prefetch set, free until the unit's
// last two chunks). Same addresses and layout as the immediate epilogue's stores.
template <int TW, int NS, int PH>
struct StoreSide {
  const float (&xv)[2][2][16];
  rsrc_t ro;
  int vb[2];       // lane base per mr
  int W4, cout4;   // output row width x cout x 4 B, cout x 4 B
  template <int K>
  __device__ __forceinline__ void step() const {
    constexpr int lo = (K * NS + 26) / 27, hi = ((K + 1) * NS + 26) / 27;
#pragma unroll
    for (int i = PH * NS + lo; i < PH * NS + (hi < NS ? hi : NS); ++i) {
      const int mr = i >> 5, nr = (i >> 4) & 1, r = i & 15;
      const int lin = 8 * (r >> 2) + (r & 3);
      const float x = xv[mr][nr][r];
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, x), ro, vb[mr] + nr * 128,
                                            ((lin / TW) * W4) + (lin % TW) * cout4, X3_STORE_AUX);
    }
  }
};

template <int XF, bool SKIP, int TW, int NPROD, bool GNB>
__device__ __forceinline__ void conv_x3_body(const ConvParams& p, const GnbParams& g) {
  using Geo = XGeo<TW>;
  extern __shared__ __attribute__((aligned(16))) float smem_raw[];
  lds_f* const smem = (lds_f*)(smem_raw);
  lds_f* const A0 = smem;           // stage s at A0 + s * XA
  lds_f* const W0 = smem + 2 * XA;  // ring slot s at W0 + s * XW

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool consumer = wave < 4;
  const int nct = p.cout_pad / XBN;
  const int S = p.ksplit;
  const int nunit = p.npix_tiles * nct * S;
  const int G = gridDim.x;
  const int nu = (nunit - (int)blockIdx.x + G - 1) / G;  // host guarantees >= 1
  const int nmain = p.cin_pad / 16;
  const int nskip = SKIP ? p.cs_pad / XSK : 0;
  const int nchu = (nmain + nskip) / S;  // chunks per unit (host: divisible)
  const int J = nu * nchu;
  const XDec dec = x3_dec(p, nct);
  // Four-image tiles (8 x 8 layers) at N % 4 != 0: image slot w of a tile (consumer wave w, producer wave
  // 4 + w) past the batch recomputes the batch's last image N - 1 - by moving that wave's tile origin n0, so
  // every read stays inside the batch and the spare slots store the very values (same image, same K order)
  // the owning slot stores; an image's arithmetic never depends on its tile-mates (the batch-invariant mode).
  auto unit_of = [&](int u, int& z) {
    STile t = x3_unit<SKIP>(p, dec, (int)blockIdx.x, u, z);
    if constexpr (Geo::IMG > 1) {
      const int slot = wave & (Geo::IMG - 1);
      t.n0 = min(t.n0 + slot, p.N - 1) - slot;
    }
    return t;
  };
  if (IFD_TRACE && p.trace && tid == 0) {  // block entry: real time (100 MHz) and shader cycles
    p.trace[64 * blockIdx.x + 59] = __builtin_amdgcn_s_memrealtime();
    p.trace[64 * blockIdx.x + 61] = __builtin_amdgcn_s_memtime();
  }

  if (consumer) {
    const int h = lane >> 5, l32 = lane & 31;
    const int wm0 = wave * 64;
    f32x16 acc[2][2], accl[2][2];  // hi x hi products; the two correction products (module comment)
    int pb[2];
#pragma unroll
    for (int mr = 0; mr < 2; ++mr) {
      const int m = wm0 + mr * 32 + l32;
      const int mi = m / (Geo::TH * TW), mp = m % (Geo::TH * TW);  // image of the tile, its pixel
      pb[mr] = mi * Geo::HP + (mp / TW) * Geo::HW + (mp % TW);
    }
    // acc at the unit's start; accl just before its first use (after a deferred-epilogue chunk, whose
    // final values need the registers)
    auto zero = [&]() {
#pragma unroll
      for (int mr = 0; mr < 2; ++mr)
#pragma unroll
        for (int nr = 0; nr < 2; ++nr)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[mr][nr][r] = 0.f;
    };
    auto zero_l = [&]() {
#pragma unroll
      for (int mr = 0; mr < 2; ++mr)
#pragma unroll
        for (int nr = 0; nr < 2; ++nr)
#pragma unroll
          for (int r = 0; r < 16; ++r) accl[mr][nr][r] = 0.f;
    };
    // Epilogue straight from the accumulators. Lane (h, l32) holds channel 32 nr + l32 of tile
    // pixel wm0 + 32 mr + 8 (r >> 2) + 4 h + (r & 3) (column offset 4 h + (r & 3) < 8 stays in
    // its row): one dword store per register = two 128-B row segments. Bias and residual are
    // loaded in the same layout while the unit's last chunk is on the MFMAs, so the epilogue
    // waits on nothing and its stores drain behind the next unit's chunks.
    float bias2[2];
    // Register (mr, r) of lane (h, l32) sits at tile pixel wm0 + 32 mr + 8 (r >> 2) + 4 h + (r & 3).
    // Byte offsets: vbase (lane: tile origin, the wave's rows, 4 h, channel) + mr * mstep (lane) +
    // roff(r) (16 wave-uniform scalar offsets).
    auto roff = [&](int r) {
      const int lin = 8 * (r >> 2) + (r & 3);
      return ((lin / TW) * p.W + lin % TW) * p.cout * 4;
    };
    const int mstep = (32 / TW) * p.W * p.cout * 4;
    // the wave's 64 pixels: rows of one image (8x8 tiles: the whole image wm0 / 64 of the tile)
    const int wimg = wm0 / (Geo::TH * TW), wrow = (wm0 % (Geo::TH * TW)) / TW;
    // the lane id re-read where a lane-dependent address is needed once per unit (volatile: not hoisted),
    // so that no such address lives through the chunk loop (they were spilled, and the reloads' vmcnt(0)
    // waited for the loads or stores in flight)
    auto lane_id = [&]() {
      int ln;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
      return ln;
    };
    auto vbase = [&](const STile& t) {
      const int ln = lane_id();
      return (((wimg * p.H + t.y0 + wrow) * p.W + t.x0 + 4 * (ln >> 5)) * p.cout + t.ct * XBN + (ln & 31)) * 4;
    };
    // SKIP kernels have no residual (the host runs a 1x1 conv with a residual, proj_out, split-K: the
    // reduction adds it). Its 64 registers would not fit beside the skip operand buffers.
    auto bias_load = [&](const STile& t) {
#pragma unroll
      for (int nr = 0; nr < 2; ++nr) bias2[nr] = gld1(p.bias + t.ct * XBN + 32 * nr + l32);
    };
    // GroupNorm granule statistics of the unit's outputs V(mr, nr, r) (the epilogue's values): over this
    // lane's 32 pixels (two-pass), then merged with the other column half (lane ^ 32) and over the channel
    // quad (lanes ^ 1, ^ 2). Every merge joins two equal counts, so Chan's update needs no division:
    //   mean = ma + d / 2,  M2 = (M2a + M2b) + d^2 n / 2,  d = mb - ma  (n = one side's count)
    // (bit-identical to gmerge: the factors are powers of two). The partner values come from
    // v_permlane32_swap and DPP quad permutes (VALU) instead of LDS-routed shuffles, and the two channel
    // blocks' chains are interleaved.
    auto gstats = [&](const STile& t, auto&& V) __attribute__((always_inline)) {
      float mean[2], m2[2];
#pragma unroll
      for (int nr = 0; nr < 2; ++nr) {
        float sm = 0.f;
#pragma unroll
        for (int mr = 0; mr < 2; ++mr)
#pragma unroll
          for (int r = 0; r < 16; ++r) sm += V(mr, nr, r);
        mean[nr] = sm * (1.0f / 32);
        float q = 0.f;
#pragma unroll
        for (int mr = 0; mr < 2; ++mr)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float d = V(mr, nr, r) - mean[nr];
            q += d * d;
          }
        m2[nr] = q;
      }
      auto merge = [&](float am, float aq, float bm, float bq, float n, float& om, float& oq) {
        const float d = bm - am;
        om = am + d * 0.5f;
        oq = (aq + bq) + ((d * d) * n) * 0.5f;
      };
#pragma unroll
      for (int nr = 0; nr < 2; ++nr) {  // lane ^ 32
        float ml, mh, ql, qh;
        wave_halves(mean[nr], ml, mh);
        wave_halves(m2[nr], ql, qh);
        merge(ml, ql, mh, qh, 32.f, mean[nr], m2[nr]);
      }
      // lanes ^ 1 then ^ 2 within the quad: quad_perm [0,0,2,2] / [1,1,3,3], then [0,1,0,1] / [2,3,2,3]
#define IFD_QP(v, ctrl) __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), ctrl, 0xf, 0xf, false))
#pragma unroll
      for (int nr = 0; nr < 2; ++nr)
        merge(IFD_QP(mean[nr], 0xA0), IFD_QP(m2[nr], 0xA0), IFD_QP(mean[nr], 0xF5), IFD_QP(m2[nr], 0xF5), 64.f, mean[nr],
              m2[nr]);
#pragma unroll
      for (int nr = 0; nr < 2; ++nr)
        merge(IFD_QP(mean[nr], 0x44), IFD_QP(m2[nr], 0x44), IFD_QP(mean[nr], 0xEE), IFD_QP(m2[nr], 0xEE), 128.f, mean[nr],
              m2[nr]);
#undef IFD_QP
      // through a buffer descriptor (scalar base, lane offset from a fresh lane id): a 64-bit per-lane
      // pointer here was spilled, and its reload's vmcnt(0) waited for the unit's 64 output stores
      const int ln = lane_id();
      if (ln < 32 && (ln & 3) == 0) {
        const int e = Geo::IMG > 1 ? 0 : ((t.y0 / p.TH) * p.tiles_x + t.x0 / p.TW) * 4 + wave;
        const rsrc_t rg = mkrsrc(p.gstat + (size_t)(t.n0 + wimg) * (p.cout / 4) * p.gstat_E * 2);
        const int vo = (ln >> 2) * p.gstat_E * 8;
#pragma unroll
        for (int nr = 0; nr < 2; ++nr) {
          const int so = ((t.ct * 16 + nr * 8) * p.gstat_E + e) * 8;
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, mean[nr]), rg, vo, so, 0);
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, m2[nr]), rg, vo + 4, so, 0);
        }
      }
    };
    auto epilogue = [&](const STile& t, int z, const float (&rv)[2][2][16], bool tstamp = false) {
      if (X3_ABLATE == 13) {  // timing only: no epilogue
        asm volatile("" ::"v"(acc[0][0]), "v"(acc[0][1]), "v"(acc[1][0]), "v"(acc[1][1]));
        return;
      }
      const size_t img = (size_t)p.H * p.W * p.cout;
      const int vb = vbase(t);
      if (S > 1) {  // raw partial sums into slab z (splitk_reduce adds the slabs, bias, residual)
        const rsrc_t rp = mkrsrc(p.part + ((size_t)z * p.N + t.n0) * img);
#pragma unroll
        for (int nr = 0; nr < 2; ++nr)
#pragma unroll
          for (int mr = 0; mr < 2; ++mr)
#pragma unroll
            for (int r = 0; r < 16; ++r)
              __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, acc[mr][nr][r] * (1.0f / kLo)), rp,
                                                    vb + mr * mstep + nr * 128, roff(r), 0);
        return;
      }
      const rsrc_t ro = mkrsrc(p.out + (size_t)t.n0 * img);
      // the outputs replace the accumulators (they are zeroed after the epilogue)
#pragma unroll
      for (int nr = 0; nr < 2; ++nr)
#pragma unroll
        for (int mr = 0; mr < 2; ++mr)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            float x = acc[mr][nr][r] * (1.0f / kLo);  // exact rescale
            x = x + bias2[nr];
            if (!SKIP && p.res) x = rv[mr][nr][r] + x;  // torch order: x_res + (conv + bias)
            acc[mr][nr][r] = x;
            if (X3_ABLATE != 14)
              __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, x), ro, vb + mr * mstep + nr * 128,
                                                    roff(r), X3_STORE_AUX);
          }
      if (IFD_TRACE && p.trace && wave == 0 && lane == 0 && tstamp)
        p.trace[64 * blockIdx.x + 44] = __builtin_amdgcn_s_memtime();  // values + stores issued
      if (X3_ABLATE != 15 && p.gstat) gstats(t, [&](int mr, int nr, int r) { return acc[mr][nr][r]; });
      if (IFD_TRACE && p.trace && wave == 0 && lane == 0 && tstamp)
        p.trace[64 * blockIdx.x + 45] = __builtin_amdgcn_s_memtime();  // statistics done
    };
    // The deferred epilogue (X3_DEFER): the outputs go to the residual registers xv (which hold the residual
    // when there is one: x_res + (conv + bias), torch's order), their statistics are taken now, and the 64
    // stores per lane are left to the next unit's first chunks (StoreSide); pvb / pro keep their addresses.
    bool pend = false;
    STile pt;  // the pending unit's tile (uniform: its store addresses are re-derived per chunk, no VGPR
               // lives from one unit into the next)
    auto epilogue_defer = [&](const STile& t, float (&xv)[2][2][16], bool tstamp = false) {
      const bool hres = !SKIP && p.res;
#pragma unroll
      for (int nr = 0; nr < 2; ++nr)
#pragma unroll
        for (int mr = 0; mr < 2; ++mr)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            float x = acc[mr][nr][r] * (1.0f / kLo);  // exact rescale
            x = x + bias2[nr];
            if (hres) x = xv[mr][nr][r] + x;
            xv[mr][nr][r] = x;
          }
      if (IFD_TRACE && p.trace && wave == 0 && lane == 0 && tstamp)
        p.trace[64 * blockIdx.x + 44] = __builtin_amdgcn_s_memtime();  // values
      if (X3_ABLATE != 15 && p.gstat) gstats(t, [&](int mr, int nr, int r) { return xv[mr][nr][r]; });
      if (IFD_TRACE && p.trace && wave == 0 && lane == 0 && tstamp)
        p.trace[64 * blockIdx.x + 45] = __builtin_amdgcn_s_memtime();  // statistics done
      pt = t;
      pend = true;
    };
    // Training (ConvParams::gnb_*): this conv is the dgrad whose output da feeds a GroupNorm(+ scale/shift)(+ SiLU)
    // backward; x (that GroupNorm's input, prefetched into xr like a residual) gives per value
    //   xhat = (x - mean) rstd, nrm = xhat gamma + beta, z = nrm (1 + s) + sh, dz = da silu'(z) (or da),
    // and the epilogue adds over the wave's 64 pixels, per channel, A1 = sum dz, A2 = sum dz nrm and
    // A3 = (1 + s) sum dz xhat - gn_bwd_partial_kernel's pass 1 (train_ops.hip) without its pass over (da, x).
    // The outputs are then stored as in the other epilogues (deferred from xr, or at once from acc).
    // GNB: the epilogue's per-(image, channel) parameters (mean, rstd, gamma, beta, 1 + scale, shift) of both channel
    // blocks, all twelve loads issued together at the epilogue's start (round 5 loaded nr = 1's after nr = 0's sums:
    // two rounds of global-load latency between every unit's MFMAs and its successor's). Loaded earlier, during the
    // unit's last chunks beside the prefetched x, they spilled 33-98 VGPRs (round 6, -Rpass-analysis)
    float gpf[GNB ? 2 : 1][6];
    auto gnb_params = [&](const STile& t) __attribute__((always_inline)) {
      if constexpr (GNB) {
        const int ll = lane_id() & 31;
        const int n = t.n0 + wimg, C = p.cout, cpg = C / 32;
#pragma unroll
        for (int nr = 0; nr < 2; ++nr) {
          const int cc = t.ct * XBN + 32 * nr + ll, grp = cc / cpg;
          gpf[nr][0] = g.stats[(n * 32 + grp) * 2];
          gpf[nr][1] = g.stats[(n * 32 + grp) * 2 + 1];
          gpf[nr][2] = g.gamma[cc];
          gpf[nr][3] = g.beta[cc];
          gpf[nr][4] = g.ss ? 1.0f + g.ss[(size_t)n * g.ss_stride + cc] : 1.0f;
          gpf[nr][5] = g.ss ? g.ss[(size_t)n * g.ss_stride + C + cc] : 0.0f;
        }
      }
    };
    auto epilogue_gnb = [&](const STile& t, float (&xv)[2][2][16], bool dfr) {
#pragma unroll
      for (int nr = 0; nr < 2; ++nr)
#pragma unroll
        for (int mr = 0; mr < 2; ++mr)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            float x = acc[mr][nr][r] * (1.0f / kLo);  // exact rescale
            acc[mr][nr][r] = x + bias2[nr];
          }
      const int ln = lane_id(), ll = ln & 31;
      const int n = t.n0 + wimg, C = p.cout;
      float a1[2], a2[2], a3[2], onep[2];
      // g.act: the GroupNorm's forward output act = silu(z) (or z), the input of the conv whose weight gradient
      // follows, written at the dgrad output's addresses (same [N][H][W][cout] layout) from the values computed here
      // anyway, so that weight gradient runs without re-applying the GroupNorm + SiLU on load
      const bool wact = g.act != nullptr;
      const rsrc_t rac = mkrsrc(wact ? g.act + (size_t)t.n0 * p.H * p.W * p.cout : p.bias);
      const int vba = vbase(t);
#pragma unroll
      for (int nr = 0; nr < 2; ++nr) {
        // the per-(image, channel) GroupNorm parameters, loaded during the unit's last chunks (gnb_params)
        const float mean = gpf[nr][0], rstd = gpf[nr][1], gam = gpf[nr][2], bet = gpf[nr][3];
        onep[nr] = gpf[nr][4];
        const float sh = gpf[nr][5];
        float s1 = 0.f, s2 = 0.f, s3 = 0.f;
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int mr = 0; mr < 2; ++mr)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float xhat = (xv[mr][nr][r] - mean) * rstd;
            const float nrm = xhat * gam + bet;
            const float zz = nrm * onep[nr] + sh;
            float dz = acc[mr][nr][r];
            float av = zz;
            if (g.silu) {
              const float sg = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(zz * -1.4426950408889634f));
              dz = dz * (sg * (1.0f + zz * (1.0f - sg)));
              av = zz * sg;
            }
            if (wact)
              __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, av), rac, vba + mr * mstep + nr * 128,
                                                    roff(r), X3_STORE_AUX);
            s1 += dz;
            s2 += dz * nrm;
            s3 += dz * xhat;
            if ((r & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // (four values at a time: a short live set)
          }
        // + the other column half of the same pixel rows (lane ^ 32), same channel
        float lo, hi;
        wave_halves(s1, lo, hi);
        a1[nr] = lo + hi;
        wave_halves(s2, lo, hi);
        a2[nr] = lo + hi;
        wave_halves(s3, lo, hi);
        a3[nr] = (lo + hi) * onep[nr];
      }
      if (ln < 32) {
        const int e = ((t.y0 / p.TH) * p.tiles_x + t.x0 / p.TW) * 4 + wave;
        float* o = g.part + ((size_t)n * g.nsl + e) * C * 3;
#pragma unroll
        for (int nr = 0; nr < 2; ++nr) {
          const int cc = t.ct * XBN + 32 * nr + ll;
          o[cc * 3] = a1[nr];
          o[cc * 3 + 1] = a2[nr];
          o[cc * 3 + 2] = a3[nr];
        }
      }
      if (dfr) {  // the outputs into the residual registers: their stores go out during the next unit's chunks
#pragma unroll
        for (int nr = 0; nr < 2; ++nr)
#pragma unroll
          for (int mr = 0; mr < 2; ++mr)
#pragma unroll
            for (int r = 0; r < 16; ++r) xv[mr][nr][r] = acc[mr][nr][r];
        pt = t;
        pend = true;
      } else {
        const rsrc_t ro = mkrsrc(p.out + (size_t)t.n0 * p.H * p.W * p.cout);
        const int vb = vbase(t);
#pragma unroll
        for (int nr = 0; nr < 2; ++nr)
#pragma unroll
          for (int mr = 0; mr < 2; ++mr)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const float x = acc[mr][nr][r];
              __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, x), ro, vb + mr * mstep + nr * 128,
                                                    roff(r), X3_STORE_AUX);
            }
      }
    };
    // ---- 1x1 skip chunks: the lane's operand = channels [XSK/2 h, XSK/2 (h + 1)) of the chunk at tile
    // pixels wm0 + 32 mr + l32, loaded into registers two chunks ahead. Sub-chunk q (one k = 16 MFMA
    // step) takes channels XSK/2 h + 8 q + (0..7), quads 2q and 2q+1; the host packs the weights in
    // the same order (unet.hip pack_skip_x3).
    f32x4 sq0[2][XSL], sq1[2][XSL];
    rsrc_t rs0, rs1;
    int so0[2], so1[2];
    auto skip_setup = [&](const STile& t) __attribute__((always_inline)) {
      const size_t img = (size_t)p.H * p.W;
      rs0 = mkrsrc(p.s0 + (X3_ABLATE == 12 ? 0 : (size_t)t.n0 * img * p.sc0));
      rs1 = p.s1 ? mkrsrc(p.s1 + (size_t)t.n0 * img * p.sc1) : rs0;
#pragma unroll
      for (int mr = 0; mr < 2; ++mr) {
        const int m = wm0 + mr * 32 + l32;
        const int mi = m / (Geo::TH * TW), mp = m % (Geo::TH * TW);
        const int pix = X3_ABLATE == 12 ? m : mi * p.H * p.W + (t.y0 + mp / TW) * p.W + t.x0 + mp % TW;
        so0[mr] = (pix * p.sc0 + (XSK / 2) * h) * 4;
        so1[mr] = (pix * p.sc1 + (XSK / 2) * h) * 4;
      }
    };
    auto skip_load = [&](f32x4(&b)[2][XSL], int sk, int q) __attribute__((always_inline)) {  // quads 2q, 2q+1 of skip chunk sk
      const int cs = XSK * sk;
      const bool first = cs < p.sc0;
      const int soff = (first ? cs : cs - p.sc0) * 4 + 32 * q;
#pragma unroll
      for (int mr = 0; mr < 2; ++mr) {
        const int vo = first ? so0[mr] : so1[mr];
        b[mr][2 * q] = bld4(first ? rs0 : rs1, vo, soff);
        b[mr][2 * q + 1] = bld4(first ? rs0 : rs1, vo, soff + 16);
      }
    };
    auto skip_load_all = [&](f32x4(&b)[2][XSL], int sk) __attribute__((always_inline)) {
#pragma unroll
      for (int q = 0; q < XSQ; ++q) skip_load(b, sk, q);
    };
    float gmax = 0.f;
    // one skip chunk from registers b (weights at Ws: [q][part][h][64 co][8 f16]); with `reload`, sub-chunk
    // q's quads are reloaded with skip chunk `next` as soon as they are split. `reload` is a constant at
    // every call site: a run-time test per sub-chunk would make each quad a branch merge of two values.
    auto skip_chunk = [&](f32x4(&b)[2][XSL], const lds_f* Ws, bool reload, int next) __attribute__((always_inline)) {
      const lds_f* Wb = Ws + 4 * (h * XBN + l32);
      f16x8 ah[2], al[2], bs[2], bl[2];
#pragma unroll
      for (int q = 0; q < XSQ; ++q) {
#pragma unroll
        for (int mr = 0; mr < 2; ++mr) {
          float v[8];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            v[i] = b[mr][2 * q][i];
            v[4 + i] = b[mr][2 * q + 1][i];
          }
          // range guard (the raw residual stream is not normalised)
          gmax = fmaxf(gmax, fmaxf(fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))),
                                   fmaxf(fmaxf(fabsf(v[4]), fabsf(v[5])), fmaxf(fabsf(v[6]), fabsf(v[7])))));
          unsigned hw[4], lw[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            if (NPROD == 1) {
              float a0 = v[2 * k], a1 = v[2 * k + 1];
              asm volatile("" : "+v"(a0), "+v"(a1));
              hw[k] = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a0, a1}, f16x2));
            } else {
              split2(v[2 * k], v[2 * k + 1], hw[k], lw[k]);
            }
          }
          ah[mr] = __builtin_bit_cast(f16x8, u32x4{hw[0], hw[1], hw[2], hw[3]});
          if (NPROD == 3) al[mr] = __builtin_bit_cast(f16x8, u32x4{lw[0], lw[1], lw[2], lw[3]});
        }
        if (reload) skip_load(b, next, q);
#pragma unroll
        for (int nr = 0; nr < 2; ++nr) {
          bs[nr] = *(const lds_h8*)(Wb + 4 * (q * 4 * XBN + nr * 32));
          if (NPROD == 3) bl[nr] = *(const lds_h8*)(Wb + 4 * (q * 4 * XBN + 2 * XBN + nr * 32));
        }
#pragma unroll
        for (int mr = 0; mr < 2; ++mr)
#pragma unroll
          for (int nr = 0; nr < 2; ++nr) acc[mr][nr] = xmfma(ah[mr], bs[nr], acc[mr][nr]);
        // one sub-chunk at a time: unconstrained, the scheduler hoists every sub-chunk's split and
        // fragment reads to the top and the live set no longer fits beside the two operand buffers
        __builtin_amdgcn_sched_barrier(0);
        if (NPROD == 1) continue;
#pragma unroll
        for (int mr = 0; mr < 2; ++mr)
#pragma unroll
          for (int nr = 0; nr < 2; ++nr) acc[mr][nr] = xmfma(ah[mr], bl[nr], acc[mr][nr]);
#pragma unroll
        for (int mr = 0; mr < 2; ++mr)
#pragma unroll
          for (int nr = 0; nr < 2; ++nr) acc[mr][nr] = xmfma(al[mr], bs[nr], acc[mr][nr]);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    auto stamp = [&](int j, int slot = 0) {  // slot 0: chunk start, 16: its MFMAs issued
      if (IFD_TRACE && p.trace && wave == 0 && lane == 0 && j < 16)
        p.trace[64 * blockIdx.x + slot + j] = __builtin_amdgcn_s_memtime();
    };
    if (IFD_TRACE && p.trace && wave == 0 && lane == 0) p.trace[64 * blockIdx.x + 58] = __builtin_amdgcn_s_memtime();
    XBARRIER_CONSUMER();  // chunk 0 staged
    int j = 0;  // position in the block's chunk stream: ring slot j % 3, A stage j & 1
    // xr: the residual prefetch of a unit's last two chunks (declared out here with the epilogue's values
    // in the same registers; a per-unit declaration gave the allocator two homes and copies between them)
    float xr[2][2][16];
    for (int u = 0; u < nu; ++u) {
      int z;
      const STile t = unit_of(u, z);
      zero();  // (here, not after the epilogue: the zeros of the next unit are then not live through this one)
      // the unit's K range [c0, c1): 3x3 chunks [c0, me), then skip chunks [sb, se) of the 1x1 segment
      const int c0 = z * nchu, c1 = c0 + nchu;
      const int me = c1 < nmain ? c1 : nmain;
      const int sb = (c0 > nmain ? c0 : nmain) - nmain, se = c1 - nmain;
      const bool has_skip = SKIP && sb < se;
      // sep: the correction products into accl; otherwise into acc (after fold)
      auto main_chunk = [&](bool sep) __attribute__((always_inline)) {
        stamp(j);
        if (X3_ABLATE != 4) {
          if (sep)
            consume_x3<TW, NPROD>(acc, accl, A0 + (j & 1) * XA, W0 + (j % 3) * XW, pb);
          else
            consume_x3<TW, NPROD>(acc, acc, A0 + (j & 1) * XA, W0 + (j % 3) * XW, pb);
        }
        stamp(j, 16);
        ++j;
        XBARRIER_CONSUMER();
      };
      auto main_chunk_side = [&](bool sep, auto&& side) __attribute__((always_inline)) {
        stamp(j);
        if (X3_ABLATE != 4) {
          if (sep)
            consume_x3<TW, NPROD>(acc, accl, A0 + (j & 1) * XA, W0 + (j % 3) * XW, pb, side);
          else
            consume_x3<TW, NPROD>(acc, acc, A0 + (j & 1) * XA, W0 + (j % 3) * XW, pb, side);
        }
        stamp(j, 16);
        ++j;
        XBARRIER_CONSUMER();
      };
      // the correction sum joins the main one (one rounding per output) before the unit's last 3x3
      // chunk: from there on accl is dead and its registers hold the residual / skip-operand prefetch
      auto fold = [&]() __attribute__((always_inline)) {
        if (NPROD == 1) return;
#pragma unroll
        for (int mr = 0; mr < 2; ++mr)
#pragma unroll
          for (int nr = 0; nr < 2; ++nr) {
            acc[mr][nr] += accl[mr][nr];
            // pinned here: hipcc otherwise sinks the adds past the residual prefetch (both sets live)
            asm volatile("" : "+v"(acc[mr][nr])::"memory");
          }
      };
      // The unit's last 3x3 chunk is peeled: what it prefetches (residual, first skip operands) is then
      // not a loop-carried value. The two cases are separate branches so that the operand buffers are
      // defined on every path to their use (otherwise they would stay live across all 3x3 chunks).
      if (!has_skip) {
        // The residual (64 loads per lane) goes out during the unit's last two 3x3 chunks, interleaved
        // into their MFMA groups: the mr = 0 half spread over the whole of chunk me - 2 (which still
        // accumulates the corrections in accl), then the fold, then the mr = 1 half over the first third
        // of chunk me - 1 (its correction products go to acc). Peak: acc + accl + fragments + half the
        // residual, or acc + fragments + the residual.
        // gnb (training): the last two chunks prefetch the GroupNorm input x instead of a residual (the host
        // never sets both)
        const bool gnb = GNB && !SKIP && S == 1 && g.part;
        const bool rpf = !SKIP && S == 1 && (p.res || gnb);
        zero_l();
        int c = c0;
        if constexpr (X3_DEFER > 0 && !SKIP) {
          if (pend && nmain - 2 >= X3_DEFER) {  // the previous unit's 64 stores per lane, over this unit's first
                                                // X3_DEFER chunks (a one-chunk unit carries them below)
            constexpr int NS = 64 / (X3_DEFER > 0 ? X3_DEFER : 1);
            const int W4 = p.W * p.cout * 4, c4 = p.cout * 4;
            auto ss = [&](auto ph) __attribute__((always_inline)) {
              const int vb0 = vbase(pt);
              main_chunk_side(true, StoreSide<TW, NS, decltype(ph)::value>{
                                        xr, mkrsrc(p.out + (size_t)pt.n0 * p.H * p.W * p.cout), {vb0, vb0 + mstep}, W4, c4});
            };
            ss(std::integral_constant<int, 0>{});
            if constexpr (X3_DEFER > 1) ss(std::integral_constant<int, 1>{});
            if constexpr (X3_DEFER > 2) {
              ss(std::integral_constant<int, 2>{});
              ss(std::integral_constant<int, 3>{});
            }
            c += X3_DEFER;
            pend = false;
          }
        }
        for (; c < me - 2; ++c) main_chunk(true);
        if (me > c0) {
          // the lane's id re-read here (volatile: not hoisted, so no per-lane address lives through the
          // whole unit loop for these loads: such values were spilled, and the reload's vmcnt(0) waited
          // on the loads in flight)
          const int ln = lane_id();
          const int lh = ln >> 5, ll = ln & 31;
          if (!SKIP && S == 1) {
            const rsrc_t rb = mkrsrc(p.bias);
#pragma unroll
            for (int nr = 0; nr < 2; ++nr)
              bias2[nr] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rb, 4 * ll, 4 * (t.ct * XBN + 32 * nr), 0));
          }
          const int up = p.res_xform != XF_NONE;
          const int cu = t.ct * XBN;
          // the prefetched tensor's channels: the residual's (cout), or (GNB) the 64-channel tile's concat source
          int Cx = p.cout, cux = cu;
          const float* xsrc = p.res ? p.res + (size_t)t.n0 * p.res_H * p.res_W * p.cout : p.bias;
          if constexpr (GNB) {
            const bool xs1 = cu >= g.c0;
            Cx = xs1 ? p.cout - g.c0 : g.c0;
            cux = xs1 ? cu - g.c0 : cu;
            xsrc = (xs1 ? g.x1 : g.x0) + (size_t)t.n0 * p.H * p.W * Cx;
          }
          const int vn = (((wimg * p.H + t.y0 + wrow) * p.W + t.x0 + 4 * lh) * Cx + cux + ll) * 4;
          const int vu = (2 * lh * p.cout + cu + ll) * 4;
          const rsrc_t rr = mkrsrc(xsrc);
          const int vb0 = up ? vu : vn, vb1 = up ? vu : vn + (GNB ? (32 / TW) * p.W * Cx * 4 : mstep);
          const int W4 = p.W * p.cout * 4, c4 = p.cout * 4;
          const int W4r = GNB ? p.W * Cx * 4 : W4, c4r = GNB ? Cx * 4 : c4;  // (residual / x strides)
          if (me - c0 >= 2) {
            if (rpf)
              main_chunk_side(true, ResSide<TW, 0, 32, 27>{xr, rr, {vb0, vb1}, up, W4r, c4r, wm0, t.y0, t.x0, p.res_W});
            else
              main_chunk(true);
            fold();
            if (rpf)
              main_chunk_side(false, ResSide<TW, 32, 64, 9>{xr, rr, {vb0, vb1}, up, W4r, c4r, wm0, t.y0, t.x0, p.res_W});
            else
              main_chunk(false);
          } else {  // a one-chunk unit: all of the residual in its first third
            fold();
            if (rpf) {
              main_chunk_side(false, ResSide<TW, 0, 64, 9>{xr, rr, {vb0, vb1}, up, W4r, c4r, wm0, t.y0, t.x0, p.res_W});
            } else if (X3_DEFER > 0 && !SKIP && pend) {  // (the 16 -> 128 input conv) the previous unit's
              const int vp = vbase(pt);                    // stores, all 64 in this unit's one chunk
              main_chunk_side(false, StoreSide<TW, 64, 0>{xr, mkrsrc(p.out + (size_t)pt.n0 * p.H * p.W * p.cout),
                                                          {vp, vp + mstep}, W4, c4});
              pend = false;
            } else {
              main_chunk(false);
            }
          }
        }
      } else {
        skip_setup(t);
        zero_l();
        for (int c = c0; c < me - 1; ++c) main_chunk(true);
        fold();
        // one definition point per operand buffer on every path (a buffer defined in two branches
        // gets register copies at the merge, and a copy of a load in flight is a vmcnt wait)
        const int sb1 = sb + 1 < se ? sb + 1 : sb;  // (a one-chunk segment reloads its chunk: harmless)
        skip_load_all(sq0, sb);                      // a whole 3x3 chunk ahead of its use
        if (me > c0) main_chunk(false);
        skip_load_all(sq1, sb1);
        auto skip_step = [&](f32x4(&b)[2][XSL], bool reload, int next) __attribute__((always_inline)) {
          stamp(j);
          skip_chunk(b, W0 + (j % 3) * XW, reload, next);
          stamp(j, 16);
          ++j;
          XBARRIER_CONSUMER();
        };
        int sk = sb;
        for (; sk + 3 < se; sk += 2) {  // pairs whose chunks both have a successor two ahead
          skip_step(sq0, true, sk + 2);
          skip_step(sq1, true, sk + 3);
        }
        // the last 1 to 3 chunks
        if (sk + 2 < se) {
          skip_step(sq0, true, sk + 2);
          skip_step(sq1, false, 0);
          skip_step(sq0, false, 0);
        } else {
          skip_step(sq0, false, 0);
          if (sk + 1 < se) skip_step(sq1, false, 0);
        }
      }
      if (SKIP && S == 1) bias_load(t);  // (SKIP kernels have no residual)
      if (IFD_TRACE && p.trace && wave == 0 && lane == 0 && u == 0)
        p.trace[64 * blockIdx.x + 43] = __builtin_amdgcn_s_memtime();  // first epilogue: start
      // deferred when the block's next unit has X3_DEFER chunks ahead of its residual prefetch to carry the stores,
      // or is a single chunk without a residual (its chunk carries all 64)
      const bool gnbu = GNB && !SKIP && S == 1 && g.part;
      const bool dfr = X3_DEFER > 0 && !SKIP && S == 1 && u + 1 < nu &&
                       (nmain - 2 >= X3_DEFER || (!X3_DEFER1_OFF && nmain == 1 && !p.res && !gnbu));
      if constexpr (GNB) {  // (launched only with gnb_part set and S == 1)
        (void)gnbu;
        gnb_params(t);
        epilogue_gnb(t, xr, dfr);
      } else {
        if (dfr)
          epilogue_defer(t, xr, u == 0);
        else
          epilogue(t, z, xr, u == 0);
      }
      if (IFD_TRACE && p.trace && wave == 0 && lane == 0 && u == 0)
        p.trace[64 * blockIdx.x + 63] = __builtin_amdgcn_s_memtime();  // first epilogue: end (no store drain wait)
    }
    if (SKIP && p.guard && gmax >= 65504.0f) atomicOr(p.guard, 1u);
    if (IFD_TRACE && p.trace && wave == 0 && lane == 0) {  // consumer done (stores issued)
      p.trace[64 * blockIdx.x + 60] = __builtin_amdgcn_s_memrealtime();
      p.trace[64 * blockIdx.x + 62] = __builtin_amdgcn_s_memtime();
    }
    return;
  }

  // ---- producers: halo two chunks ahead in registers, weights two chunks ahead by LDS-DMA into a
  // 3-slot ring (chunk j in slot j % 3) ----
  const int ptid = tid - NP_T;
  XProducer<XF, SKIP, TW, NPROD> P;
  P.init(ptid);
  typename XProducer<XF, SKIP, TW, NPROD>::Set s0, s1;
  // Lookahead cursor over the chunk stream: position jl = (unit ul, chunk kl of the unit), the
  // unit's tile decoded once per unit; past the end it stays on the last chunk (re-issued loads /
  // DMA of identical bytes keep the op counts fixed).
  // lastmain: the last issued chunk is a 3x3 chunk (an int kept in an SGPR: a bool array here was
  // materialised through a VGPR that aliased an in-flight load, i.e. a vmcnt wait every interval).
  int jl = 0, ul = 0, kl = 0, zl = 0;
  STile tl = unit_of(0, zl);
  int lastmain = 1, prevmain = 1;  // the last / the previous issued chunk is a 3x3 chunk
  int cmain = 1, cidx = 0;  // kind / index of the cursor's chunk (kept for the clamped repeats)
  auto issue = [&](typename XProducer<XF, SKIP, TW, NPROD>::Set& s) {  // DMA + register loads of the cursor's chunk, then advance
    if (jl < J) {
      const int c = __builtin_amdgcn_readfirstlane(zl * nchu + kl);  // 3x3 chunks, then the skip chunks
      cmain = c < nmain ? 1 : 0;
      cidx = cmain ? c : c - nmain;
    }
    prevmain = lastmain;
    lastmain = (!SKIP || cmain) ? 1 : 0;
    P.enter(p, tl, ul);
    P.dma(p, tl.ct, cmain, cidx, nmain, nskip, W0 + (jl % 3) * XW);
    P.load(s, p, cmain, cidx);
    if (jl + 1 < J) {
      ++jl;
      if (++kl == nchu) {
        kl = 0;
        tl = unit_of(++ul, zl);
      }
    } else {
      jl += 3;  // parity / ring slot of the clamped repeats: keep writing slot (J - 1) % 3
    }
  };
  // Barrier once chunk q's DMA has landed, chunk q+1 being the last issued: younger are chunk q's
  // register loads (L = Geo::LOADS, none for a skip chunk), then all of chunk q+1 (9 + L, or XDMA1).
  static_assert(XWDMA == XDMA3 && XDMA1 == 2 && (Geo::LOADS == 10 || Geo::LOADS == 12), "barrier vmcnt literals");
  auto barrier = [&]() {
    if constexpr (Geo::LOADS == 10) {
      if (!SKIP || (prevmain && lastmain))
        XBARRIER_PRODUCER(29);
      else if (prevmain)
        XBARRIER_PRODUCER(12);
      else if (lastmain)
        XBARRIER_PRODUCER(19);
      else
        XBARRIER_PRODUCER(2);
    } else {
      if (!SKIP || (prevmain && lastmain))
        XBARRIER_PRODUCER(33);
      else if (prevmain)
        XBARRIER_PRODUCER(14);
      else if (lastmain)
        XBARRIER_PRODUCER(21);
      else
        XBARRIER_PRODUCER(2);
    }
  };
  auto fstamp = [&](int slot) {  // (trace builds: the pipeline fill)
    if (IFD_TRACE && p.trace && ptid == 0) p.trace[64 * blockIdx.x + slot] = __builtin_amdgcn_s_memtime();
  };
  issue(s0);  // chunk 0
  fstamp(46);
  const int main0 = lastmain;
  issue(s1);  // chunk 1
  fstamp(47);
  if (main0) P.store(s0, p.act, A0);  // (a split-K unit may start in the skip segment)
  fstamp(56);
  barrier();
  fstamp(57);
  // interval j: LDS writes of chunk j+1 (its loads were issued one interval ago), then the DMA and
  // halo loads of chunk j+2, then the barrier once chunk j+1's DMA (issued in interval j-1) has
  // landed. Writes BEFORE issue: hipcc's vmcnt model does not count LDS-DMA ops, so a wait for
  // chunk j+1's registers placed after chunk j+2's DMA would also wait for that DMA.
  auto stamp = [&](int slot, int j) {
    // (slots of j >= 8 hold the fill and the consumer's first-epilogue stamps)
    if (IFD_TRACE && p.trace && ptid == 0 && j < 8) p.trace[64 * blockIdx.x + slot + j] = __builtin_amdgcn_s_memtime();
  };
  for (int j = 0; j < J; j += 2) {
    if (j + 1 < J && lastmain) P.store(s1, p.act, A0 + XA);  // last issued = chunk j+1
    stamp(48, j);
    issue(s0);  // chunk j+2
    stamp(32, j);
    barrier();
    if (j + 1 >= J) break;
    if (j + 2 < J && lastmain) P.store(s0, p.act, A0);
    stamp(48, j + 1);
    issue(s1);  // chunk j+3
    stamp(32, j + 1);
    barrier();
  }
  if (p.guard && P.gmax >= 65504.0f) atomicOr(p.guard, 1u);
}

template <int XF, bool SKIP, int TW, int NPROD>
__global__ __launch_bounds__(NT, 2) void conv_x3_kernel(ConvParams p) {
  conv_x3_body<XF, SKIP, TW, NPROD, false>(p, GnbParams{});
}
template <int TW, int NPROD>
__global__ __launch_bounds__(NT, 2) void conv_x3_gnb_kernel(ConvParams p, GnbParams g) {
  conv_x3_body<XF_NONE, false, TW, NPROD, true>(p, g);
}

template <int XF, bool SKIP, int TW, int NPROD>
static int launch_x3_inst(const ConvParams& p, hipStream_t stream) {
  static bool attr_set[kMaxDevices] = {};
  const size_t lds = (size_t)X_LDS_FLOATS * sizeof(float);
  hipError_t e = set_lds_attr_once(attr_set, reinterpret_cast<const void*>(&conv_x3_kernel<XF, SKIP, TW, NPROD>), (int)lds);
  if (e != hipSuccess) return (int)e;
  const int ncu = device_cu_count();
  const int nunit = p.npix_tiles * (p.cout_pad / XBN) * p.ksplit;
  const int grid = nunit < ncu ? nunit : ncu;  // one workgroup per CU (LDS-bound)
  hipLaunchKernelGGL((conv_x3_kernel<XF, SKIP, TW, NPROD>), dim3(grid), dim3(NT), lds, stream, p);
  return IFD_LAUNCH_STATUS();
}

template <int TW, int NPROD>
static int launch_x3_gnb_inst(const ConvParams& p, const GnbParams& g, hipStream_t stream) {
  static bool attr_set[kMaxDevices] = {};
  const size_t lds = (size_t)X_LDS_FLOATS * sizeof(float);
  hipError_t e = set_lds_attr_once(attr_set, reinterpret_cast<const void*>(&conv_x3_gnb_kernel<TW, NPROD>), (int)lds);
  if (e != hipSuccess) return (int)e;
  const int ncu = device_cu_count();
  const int nunit = p.npix_tiles * (p.cout_pad / XBN) * p.ksplit;
  const int grid = nunit < ncu ? nunit : ncu;
  hipLaunchKernelGGL((conv_x3_gnb_kernel<TW, NPROD>), dim3(grid), dim3(NT), lds, stream, p, g);
  return IFD_LAUNCH_STATUS();
}

template <int TW, int NPROD>
static int launch_x3_tw(const ConvParams& p, int xform, hipStream_t stream) {
  if (p.wskip) {
    if (xform == XF_NONE) return launch_x3_inst<XF_NONE, true, TW, NPROD>(p, stream);
    return (int)hipErrorInvalidValue;  // the skip segment comes with XF_NONE only (ResBlock conv2)
  }
  if (xform == XF_NONE) return launch_x3_inst<XF_NONE, false, TW, NPROD>(p, stream);
  if (xform == XF_UP) return launch_x3_inst<XF_UP, false, TW, NPROD>(p, stream);
  return (int)hipErrorInvalidValue;
}

}  // namespace

// Eligible: 3x3, BN = 64, 256-pixel tiles of one image (8 x 32 or 16 x 16), NHWC epilogue, cout a
// multiple of 64, 16-channel chunks on the main sources and 64-channel chunks on the skip sources,
// K chunks divisible by the split, no avg-pool prologue (run_conv feeds those layers a pooled activation instead) nor
// avg-pool residual without split-K (pooled likewise). Any act, identity or nearest-up residual,
// 1x1 skip segment.
bool conv_x3_eligible(const ConvParams& p, int taps, int xform, int bn) {
  const int nch = p.cin_pad / 16 + (p.wskip ? p.cs_pad / XSK : 0);
  const bool one_img = (p.TW == 32 || p.TW == 16) && p.TH * p.TW == 256 && p.IMGS == 1;
  const bool img8 = p.TW == 8 && p.TH == 8 && p.H == 8 && p.W == 8 && p.IMGS == 4 &&
                    xform == XF_NONE && (!p.res || p.res_xform == XF_NONE);
  const bool only1x1 = taps == 1 && p.cin_pad == 0 && p.wskip;  // a 1x1 conv: 1x1 chunks only
  return (taps == 9 || only1x1) && xform != XF_DOWN && bn == XBN && p.bm == 256 && (one_img || img8) &&
         p.epi == EPI_NHWC && p.cout % XBN == 0 && p.cout_pad == p.cout &&
         p.c0 % 16 == 0 && p.c1 % 16 == 0 &&
         (!p.wskip || (p.sc0 % XSK == 0 && p.sc1 % XSK == 0 && p.cs_pad == p.sc0 + p.sc1)) &&
         p.ksplit >= 1 && nch % p.ksplit == 0 && (!p.res || p.res_xform != XF_DOWN || p.ksplit > 1) &&
         (!p.wskip || !p.res || p.ksplit > 1);  // a SKIP kernel's residual goes through the split-K reduction
}

// Eligible as conv_x3_eligible plus: single-image 256-pixel tiles (TW 32 or 16), no split-K, no residual, no
// 1x1 segment, XF_NONE (the host checks with conv_x3_eligible first).
int launch_conv_x3_gnb(const ConvParams& p, const GnbParams& g, hipStream_t stream) {
  if (p.ksplit != 1 || p.IMGS != 1 || p.res || p.wskip || !g.part || !g.x0 || !g.stats || (p.TW != 32 && p.TW != 16))
    return (int)hipErrorInvalidValue;
  if (p.x3_nprod == 1) return p.TW == 32 ? launch_x3_gnb_inst<32, 1>(p, g, stream) : launch_x3_gnb_inst<16, 1>(p, g, stream);
  return p.TW == 32 ? launch_x3_gnb_inst<32, 3>(p, g, stream) : launch_x3_gnb_inst<16, 3>(p, g, stream);
}

int launch_conv_x3(const ConvParams& p, int xform, hipStream_t stream) {
  if (p.x3_nprod == 1) {
    if (p.TW == 32) return launch_x3_tw<32, 1>(p, xform, stream);
    if (p.TW == 16) return launch_x3_tw<16, 1>(p, xform, stream);
    if (p.TW == 8) return launch_x3_tw<8, 1>(p, xform, stream);
    return (int)hipErrorInvalidValue;
  }
  if (p.TW == 32) return launch_x3_tw<32, 3>(p, xform, stream);
  if (p.TW == 16) return launch_x3_tw<16, 3>(p, xform, stream);
  if (p.TW == 8) return launch_x3_tw<8, 3>(p, xform, stream);
  return (int)hipErrorInvalidValue;
}

}  // namespace ifd
