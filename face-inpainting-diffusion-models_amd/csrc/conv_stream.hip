// Persistent streaming variant of the fused 3x3 convolution for the wide layers (BM = 256-pixel
// tiles of one image = 8 rows x 32 columns, BN = 64 output channels, no 1x1 skip segment).
//
// Why: with one tile per workgroup, per-block traces (IFD_TRACE builds, tools/conv_trace.py)
// showed the MFMA pipe at ~99 % of its shared rate inside the K loop but idle for ~12 us of
// pipeline fill (the first chunk's loads queue behind every other block's prefetch), ~5 us of
// epilogue and ~5 us of dispatch gap per 140 us tile: the two co-resident blocks of a CU run in
// lockstep, so neither covers the other's boundary.
//
// Here ONE workgroup per CU (the LDS footprint forces it) walks a strided list of tiles
// (tile L = blockIdx.x + i * gridDim.x, XCD-aware L -> (pixel tile, channel tile) map as in
// conv.hip), and the chunk stream runs across tile boundaries without a break:
//   * waves 0-3 (consumers, one per SIMD, alone on the matrix pipe): ds_read + MFMA over each
//     staged chunk; after a tile's last chunk they dump the 256x64 accumulator tile into the
//     epilogue buffer E in LDS, clear the accumulators and continue with the next tile;
//   * waves 4-7 (producers): global loads two chunks ahead (two register sets), prologue
//     (GroupNorm-apply [+ scale/shift] + SiLU, resample, zero padding) and LDS writes, exactly
//     as conv.hip; in the first four chunk intervals of tile T+1 they also retire tile T's
//     epilogue from E (bias, residual, 16-byte NHWC stores), one 64-pixel piece per interval,
//     with each piece's residual loads issued one interval ahead.
// One workgroup barrier per chunk interval, as in conv.hip, but issued as a bare s_barrier with
// explicit waits (see BARRIER_* below). Arithmetic (MFMA order, bias then
// residual) is identical to conv.hip, so outputs match it bit for bit.
#include "conv.h"
#include "conv_dev.h"

#include <cstdlib>

#ifndef IFD_TRACE
#define IFD_TRACE 0
#endif
// IFD_TRACE=1: shader-cycle stamps (s_memtime) of chunk intervals 8..15 into ConvParams::trace,
// 64 slots per block: [8*i + 0..3] producer wave 4 lane 0 at interval start / loads issued /
// LDS writes done / epilogue done, [8*i + 6] after a full vmcnt drain at interval start;
// [8*i + 4..5] consumer wave 0 lane 0 at interval start / MFMAs issued; [63] HW_ID | XCC_ID << 32.

namespace ifd {

namespace {

constexpr int SBM = 256, SBN = 64, STW = 32, STH = 8;
constexpr int SHW = STW + 2, SHH = STH + 2;       // halo 34 x 10
constexpr int SNP = SHW * SHH;                    // 340 halo pixels
constexpr int SITEMS = (2 * SNP + NP_T - 1) / NP_T;  // 3 halo quads per producer thread
constexpr int SWQ = 9 * 2 * SBN;                  // weight quads per chunk (1152)
constexpr int SWITEMS = (SWQ + NP_T - 1) / NP_T;  // 5
constexpr int SA = SNP * 8;                       // floats per A stage
constexpr int SW = 9 * 8 * SBN;                   // floats per W stage
constexpr int SLDE = SBN + 4;                     // epilogue tile row stride (floats)
constexpr int SE = SBM * SLDE;
constexpr int SWP = 20 * 64 * 4;                  // W ring slot: 1280 quads (5 LDS-DMA rounds of 256)
constexpr int NWS = 3;                            // W ring slots (chunk c in slot c % 3)
constexpr int SLDS_FLOATS = 2 * SA + NWS * SWP + SE;  // 38208 floats = 149.25 KiB
constexpr int EPI_PIECES = 4;                     // 64-pixel pieces, one per consumer wave's rows

// __syncthreads() would make the compiler drain vmcnt to 0 before every barrier once LDS-DMA
// (an LDS write counted by vmcnt) is in flight, killing the prefetch. The barriers are therefore
// bare s_barrier in asm (a compiler memory barrier too) with the waits each role needs:
//   consumers: their LDS reads / E writes done (lgkmcnt(0));
//   producers: their A-stage ds_writes done (lgkmcnt(0)) and the weight DMA of the chunk the
//              consumers read next landed (vmcnt(N), N = memory ops issued after it).
#define BARRIER_CONSUMER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")
#define BARRIER_PRODUCER(N) asm volatile("s_waitcnt vmcnt(" #N ") lgkmcnt(0)\n\ts_barrier" ::: "memory")

template <int XF>
struct SSet {
  f32x4 raw[SITEMS];
  f32x4 ca, cb;
  float vld[SITEMS];
};

template <int XF>
struct SProducer {
  int ptid, quad;
  int hy[SITEMS], hx[SITEMS], ldso[SITEMS];
  // load-cursor tile: descriptors (image bases of the two concat sources, GroupNorm coefficient
  // rows, the channel tile's weight slabs) and per-lane byte offsets within them
  int cur_tile = -1;
  rsrc_t r0, r1, ra, rb;
  int off0[SITEMS], off1[SITEMS];
  float valid[SITEMS];

  __device__ __forceinline__ void init(int t) {
    ptid = t;
    quad = t & 1;
#pragma unroll
    for (int i = 0; i < SITEMS; ++i) {
      const int idx = t + i * NP_T, pix = idx >> 1;
      hy[i] = pix / SHW;
      hx[i] = pix - hy[i] * SHW;
      ldso[i] = idx < 2 * SNP ? ((idx & 1) * SNP + pix) * 4 : -1;
    }
  }

  __device__ __forceinline__ void tile_setup(const ConvParams& p, const STile& t, int nch) {
    const size_t img = (size_t)p.Hin * p.Win;
    r0 = mkrsrc(p.in0 + (size_t)t.n0 * img * p.c0);
    r1 = mkrsrc(p.in1 ? p.in1 + (size_t)t.n0 * img * p.c1 : p.in0);
    const int ctot = p.c0 + p.c1;
    ra = mkrsrc(p.actA + (size_t)t.n0 * ctot);
    rb = mkrsrc(p.actB + (size_t)t.n0 * ctot);
#pragma unroll
    for (int i = 0; i < SITEMS; ++i) {
      const int y = t.y0 + hy[i] - 1, x = t.x0 + hx[i] - 1;
      const bool inb = ldso[i] >= 0 && y >= 0 && y < p.H && x >= 0 && x < p.W;
      int sy = y, sx = x;
      if (XF == XF_UP) { sy = y >> 1; sx = x >> 1; }
      const int sp = inb ? sy * p.Win + sx : 0;
      valid[i] = inb ? 1.f : 0.f;
      off0[i] = (sp * p.c0 + 4 * quad) * 4;
      off1[i] = (sp * p.c1 + 4 * quad) * 4;
    }
  }

  // Global loads of chunk k of tile `t` (tile index ti in this block's list) into set s. Every
  // load is issued on every path (a load skipped on some path would force the compiler's vmcnt
  // bookkeeping down to vmcnt(0) at the next wait, draining the following chunk's prefetch).
  __device__ __forceinline__ void load(SSet<XF>& s, const ConvParams& p, const STile& t, int ti, int k, int nch) {
    if (ti != cur_tile) {
      tile_setup(p, t, nch);
      cur_tile = ti;
    }
    const int cb0 = 8 * k;
#pragma unroll
    for (int i = 0; i < SITEMS; ++i) s.vld[i] = valid[i];
    if (IFD_ABLATE == 10) {  // timing experiment: no halo / coefficient loads
    } else if (IFD_ABLATE == 11) {  // timing experiment: same loads, contiguous 1 KB per wave
#pragma unroll
      for (int i = 0; i < SITEMS; ++i) s.raw[i] = bld4(r0, 16 * ptid + 4096 * i, cb0 * 4);
    } else if (cb0 < p.c0) {
#pragma unroll
      for (int i = 0; i < SITEMS; ++i) s.raw[i] = bld4(r0, off0[i], cb0 * 4);
    } else {
#pragma unroll
      for (int i = 0; i < SITEMS; ++i) s.raw[i] = bld4(r1, off1[i], (cb0 - p.c0) * 4);
    }
    if (IFD_ABLATE != 10) {
      s.ca = bld4(ra, 16 * quad, cb0 * 4);  // act != ACT_NONE (eligibility)
      s.cb = bld4(rb, 16 * quad, cb0 * 4);
    }
  }

  // Weight slab of chunk k of channel tile ct straight into W ring slot `Wslot` by LDS-DMA
  // (buffer_load ... lds: no VGPR staging, no ds_write). 5 rounds of 256 quads; the tail of the
  // last round reads past the 1152-quad slab into padding of the slot.
  __device__ __forceinline__ void dma_weights(const ConvParams& p, int ct, int k, int nch, lds_f* Wslot) const {
    const rsrc_t r = mkrsrc(p.wpack + ((size_t)ct * nch + k) * SW);
    const int pw = __builtin_amdgcn_readfirstlane(ptid >> 6);
#pragma unroll
    for (int i = 0; i < SWITEMS; ++i) {
      const int qb = (i * 4 + pw) * 64;  // first quad of this wave's round-i piece
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(Wslot + 4 * qb), 16,
                                               16 * (qb + (ptid & 63)), 0, 0, 0);
    }
  }

  // GroupNorm-apply [+ SiLU] on packed f32 pairs (v_pk_fma / v_pk_mul / v_pk_add: half the
  // issue slots of the scalar form; transcendentals stay per value). Bit-identical to
  // silu_fast(a * v + b): exp2(t * -log2 e) == __expf(-t).
  __device__ __forceinline__ static f32x2 act2(f32x2 v, f32x2 a, f32x2 b, int act) {
    if (IFD_ABLATE == 8) return v;  // timing experiment: no activation math
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

  __device__ __forceinline__ void store(const SSet<XF>& s, int act, lds_f* As) const {
#pragma unroll
    for (int i = 0; i < SITEMS; ++i) {
      if (ldso[i] >= 0) {
        const f32x2 lo = act2(s.raw[i].xy, s.ca.xy, s.cb.xy, act) * s.vld[i];
        const f32x2 hi = act2(s.raw[i].zw, s.ca.zw, s.cb.zw, act) * s.vld[i];
        *(lds_f4*)(As + ldso[i]) = f32x4{lo.x, lo.y, hi.x, hi.y};
      }
    }
  }
};

// Producer-side epilogue of one tile, retired in EPI_PIECES 64-pixel pieces. Thread t owns
// channel quad q = t % 16 of pixels 64u + t/16 + 16v (v = 0..3) in piece u. Residuals of piece u
// are loaded at the end of the interval before the one that retires it.
struct SEpilogue {
  int q, prow;
  f32x4 bias4;
  STile t;
  rsrc_t ro, rr;

  __device__ __forceinline__ int pix(int u, int v) const { return 64 * u + prow + 16 * v; }

  __device__ __forceinline__ void begin(const ConvParams& p, const STile& tile) {
    t = tile;
    bias4 = gld4(p.bias + t.ct * SBN + 4 * q);
    ro = mkrsrc(p.out + (size_t)t.n0 * p.H * p.W * p.cout);
    rr = mkrsrc(p.res ? p.res + (size_t)t.n0 * p.res_H * p.res_W * p.cout : p.out);
  }

  // byte offset of (pixel (y, x), this thread's quad) in an NHWC image of width w
  __device__ __forceinline__ int boff(const ConvParams& p, int y, int x, int w) const {
    return ((y * w + x) * p.cout + t.ct * SBN + 4 * q) * 4;
  }

  __device__ __forceinline__ void prefetch(const ConvParams& p, int u, f32x4 (&rv)[4]) const {
    if (!p.res) return;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int m = pix(u, v);
      const int y = t.y0 + (m >> 5), x = t.x0 + (m & 31);
      if (p.res_xform == XF_NONE)
        rv[v] = bld4(rr, boff(p, y, x, p.W), 0);
      else  // XF_UP (XF_DOWN residuals are not stream-eligible)
        rv[v] = bld4(rr, boff(p, y >> 1, x >> 1, p.res_W), 0);
    }
  }

  __device__ __forceinline__ void retire(const ConvParams& p, const lds_f* E, int u, const f32x4 (&rv)[4]) const {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int m = pix(u, v);
      const int y = t.y0 + (m >> 5), x = t.x0 + (m & 31);
      f32x4 val = *(const lds_f4*)(E + m * SLDE + 4 * q);
      val = val + bias4;
      if (p.res) val = rv[v] + val;
      bst4(ro, boff(p, y, x, p.W), val);
    }
  }
};

// CW consumer waves (4: one per SIMD; 8: two per SIMD, each 32 pixels x 64 channels) + 4
// producer waves.
template <int XF, int CW>
__global__ __launch_bounds__(64 * CW + NP_T, CW == 4 ? 2 : 3) void conv_stream_kernel(ConvParams p) {
  using T = Tile<SBM, SBN, CW, 1>;
  constexpr int PT0 = 64 * CW;  // first producer thread
  extern __shared__ __attribute__((aligned(16))) float smem_raw[];
  lds_f* const smem = (lds_f*)(smem_raw);
  lds_f* const A0 = smem;
  lds_f* const W0 = smem + 2 * SA;  // W ring: slot c % NWS at W0 + (c % NWS) * SWP
  lds_f* const E = smem + 2 * SA + NWS * SWP;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool consumer = __builtin_amdgcn_readfirstlane(wave) < CW;
  const int nct = p.cout_pad / SBN;
  const int nvirt = p.npix_tiles * nct;
  const int G = gridDim.x;
  const int ntile = (nvirt - (int)blockIdx.x + G - 1) / G;  // host guarantees >= 1
  const int nch = p.cin_pad / 8;
  const int J = ntile * nch;  // chunk intervals of this block
#if IFD_TRACE
  // stamps go to LDS during the loop (a global store would sit in vmcnt and distort the waits)
  // and are copied out at the end
  unsigned long long* const tr = p.trace ? p.trace + 64 * (size_t)blockIdx.x : nullptr;
  __attribute__((address_space(3))) unsigned long long* const trl =
      (__attribute__((address_space(3))) unsigned long long*)(smem + SLDS_FLOATS);
  if (tr && tid == 0) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    tr[63] = hw | ((unsigned long long)xcc << 32);
  }
#define STAMP(j, slot, who)                                                         \
  do {                                                                               \
    if (tr && tid == (who) && (j) >= 8 && (j) < 16) trl[8 * ((j)-8) + (slot)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#define TRACE_FLUSH(who)                                                            \
  do {                                                                               \
    if (tr && tid == (who))                                                          \
      for (int i_ = 0; i_ < 8; ++i_)                                                 \
        for (int s_ = 0; s_ < 8; ++s_)                                               \
          if (((who) == 0) == (s_ == 4 || s_ == 5)) tr[8 * i_ + s_] = trl[8 * i_ + s_]; \
  } while (0)
#else
#define STAMP(j, slot, who) \
  do {                      \
  } while (0)
#define TRACE_FLUSH(who) \
  do {                   \
  } while (0)
#endif

  if (consumer) {
    const int h = lane >> 5, l32 = lane & 31;
    const int wm0 = wave * (SBM / CW);
    f32x16 acc[T::MR][T::NR];
    int pb[T::MR];
#pragma unroll
    for (int mr = 0; mr < T::MR; ++mr) {
      const int m = wm0 + mr * 32 + l32;
      pb[mr] = (m >> 5) * SHW + (m & 31);
    }
    auto zero = [&]() {
#pragma unroll
      for (int mr = 0; mr < T::MR; ++mr)
#pragma unroll
        for (int nr = 0; nr < T::NR; ++nr)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[mr][nr][r] = 0.f;
    };
    zero();
    BARRIER_CONSUMER();  // chunk 0 staged
    int k = 0;
    for (int j = 0; j < J; ++j) {
      const int b = j & 1;
      STAMP(j, 4, 0);
      if (IFD_ABLATE != 7)  // timing experiment 7: consumers idle (barriers only)
        consume<SBM, SBN, CW, 1, 9>(acc, A0 + b * SA, W0 + (j % NWS) * SWP, SNP, SHW, pb, 0);
      STAMP(j, 5, 0);
      if (++k == nch) {
        k = 0;
#pragma unroll
        for (int mr = 0; mr < T::MR; ++mr)
#pragma unroll
          for (int nr = 0; nr < T::NR; ++nr)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int m = wm0 + mr * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
              E[m * SLDE + nr * 32 + l32] = acc[mr][nr][r];
            }
        zero();
      }
      BARRIER_CONSUMER();
    }
    TRACE_FLUSH(0);
    return;
  }

  // ---- producers ----
#ifndef IFD_SPRIO
#define IFD_SPRIO 0
#endif
  if (IFD_SPRIO > 0) __builtin_amdgcn_s_setprio(IFD_SPRIO);
  const int ptid = tid - PT0;
  SProducer<XF> P;
  P.init(ptid);
  // chunk c lives in sets[c % NS]: loads run NS chunks ahead (3 when the register budget allows)
  constexpr int NS = CW == 4 ? 3 : 2;
  SSet<XF> sets[NS];
  SEpilogue ep;
  ep.q = ptid & 15;
  ep.prow = ptid >> 4;
  f32x4 rv[4];

  auto tile_of = [&](int ti) { return decode_tile(p, (int)blockIdx.x + ti * G, nct); };
  // load chunk c (block-local stream index, clamped so the load is unconditional)
  auto load_chunk = [&](SSet<XF>& s, int c) {
    c = min(c, J - 1);
    const int ti = c / nch, kk = c - ti * nch;
    P.load(s, p, tile_of(ti), ti, kk, nch);
  };

  // weights of chunk c (clamped: the DMA is issued on every path, see SProducer::load)
  auto dma_chunk = [&](int c) {
    c = min(c, J - 1);
    const int ti = c / nch, kk = c - ti * nch;
    P.dma_weights(p, tile_of(ti).ct, kk, nch, W0 + (c % NWS) * SWP);
  };

#pragma unroll
  for (int i = 0; i < NS; ++i) load_chunk(sets[i], i);
  dma_chunk(0);
  dma_chunk(1);
  P.store(sets[0], p.act, A0);
  BARRIER_PRODUCER(5);  // chunk 0's weights landed (younger: chunk 1's five DMA pieces)

  // Interval j: loads of chunk j+NS (unconditional) -> LDS writes of chunk j+1 -> retire epilogue
  // piece kk of the previous tile (kk < 4) -> conditional residual prefetch of the next piece
  // (or, at kk = nch-1, piece 0 of the tile just finished) -> barrier. The conditional loads
  // come last so every wait on a chunk's registers still counts the next chunk's loads.
  auto interval = [&](int j, SSet<XF>& sl, const SSet<XF>& ss) {
    const int ti = j / nch, kk = j - ti * nch;
    STAMP(j, 0, PT0);
#if IFD_TRACE
    if (tr) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // diagnostic: drain, then time the issue alone
    STAMP(j, 6, PT0);
#endif
    load_chunk(sl, j + NS);
    dma_chunk(j + 2);
    STAMP(j, 1, PT0);
    if (j + 1 < J) P.store(ss, p.act, A0 + ((j + 1) & 1) * SA);
    STAMP(j, 2, PT0);
    if (IFD_ABLATE != 9 && ti >= 1 && kk < EPI_PIECES) ep.retire(p, E, kk, rv);
    if (IFD_ABLATE != 9 && kk == nch - 1) {
      ep.begin(p, tile_of(ti));
      ep.prefetch(p, 0, rv);
    } else if (ti >= 1 && kk + 1 < EPI_PIECES) {
      ep.prefetch(p, kk + 1, rv);
    }
    STAMP(j, 3, PT0);
    // chunk j+1's weights (DMA'd in interval j-1) must have landed before the barrier: at least
    // this interval's halo/coefficient loads (5) and weight DMA (5) are younger than them
    BARRIER_PRODUCER(10);
  };
  int j = 0;
  if constexpr (NS == 3) {
    for (; j + 3 <= J; j += 3) {
      interval(j, sets[0], sets[1]);
      interval(j + 1, sets[1], sets[2]);
      interval(j + 2, sets[2], sets[0]);
    }
    if (j < J) interval(j, sets[0], sets[1]);
    if (j + 1 < J) interval(j + 1, sets[1], sets[2]);
  } else {
    for (; j + 2 <= J; j += 2) {
      interval(j, sets[0], sets[1]);
      interval(j + 1, sets[1], sets[0]);
    }
    if (j < J) interval(j, sets[0], sets[1]);
  }
  // last tile's epilogue (piece 0 was prefetched in the last interval)
#pragma unroll
  for (int u = 0; u < EPI_PIECES; ++u) {
    ep.retire(p, E, u, rv);
    if (u + 1 < EPI_PIECES) ep.prefetch(p, u + 1, rv);
  }
  TRACE_FLUSH(PT0);
}

// ---------------------------------------------------------------------------------------------
// Mode 2: TWO persistent workgroups per CU (<= 80 KiB LDS each). The two pipelines on a CU are
// independent, so one workgroup's latency tails (producer load waits, the epilogue) overlap the
// other's MFMAs — what the one-tile-per-workgroup kernel gets from two co-resident blocks —
// while the chunk stream still runs across tiles without a fill. LDS: A stages (2 x 10.6 KiB),
// W ring of 2 slots (weights of chunk j+1 DMA'd during interval j, 2 x 20 KiB), and a 4.25 KiB
// staging strip per consumer wave for the epilogue, which the consumers do themselves.
constexpr int S2_STRIP = 16 * SLDE;                          // 16 pixels x 68 floats
constexpr int S2_LDS_FLOATS = 2 * SA + 2 * SWP + 4 * S2_STRIP;  // 19952 floats = 77.9 KiB

template <int XF>
__global__ __launch_bounds__(NT, 4) void conv_stream2_kernel(ConvParams p) {
  using T = Tile<SBM, SBN, 4, 1>;
  extern __shared__ __attribute__((aligned(16))) float smem_raw[];
  lds_f* const smem = (lds_f*)(smem_raw);
  lds_f* const A0 = smem;
  lds_f* const W0 = smem + 2 * SA;  // slot c & 1 at W0 + (c & 1) * SWP
  lds_f* const ST = smem + 2 * SA + 2 * SWP;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool consumer = __builtin_amdgcn_readfirstlane(wave) < 4;
  const int nct = p.cout_pad / SBN;
  const int nvirt = p.npix_tiles * nct;
  const int G = gridDim.x;
  const int ntile = (nvirt - (int)blockIdx.x + G - 1) / G;  // host guarantees >= 1
  const int nch = p.cin_pad / 8;
  const int J = ntile * nch;
  auto tile_of = [&](int ti) { return decode_tile(p, (int)blockIdx.x + ti * G, nct); };

  if (consumer) {
    const int h = lane >> 5, l32 = lane & 31;
    const int wm0 = wave * (SBM / 4);
    lds_f* const strip = ST + wave * S2_STRIP;
    f32x16 acc[T::MR][T::NR];
    int pb[T::MR];
#pragma unroll
    for (int mr = 0; mr < T::MR; ++mr) {
      const int m = wm0 + mr * 32 + l32;
      pb[mr] = (m >> 5) * SHW + (m & 31);
    }
    auto zero = [&]() {
#pragma unroll
      for (int mr = 0; mr < T::MR; ++mr)
#pragma unroll
        for (int nr = 0; nr < T::NR; ++nr)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[mr][nr][r] = 0.f;
    };
    // epilogue lane map: channel quad q = lane & 15 of piece pixels (lane >> 4) + 4 v
    const int q = lane & 15, prow = lane >> 4;
    // Wave-private epilogue of one tile: 4 pieces of 16 pixels (half of one 32-pixel MFMA row
    // block each) through the strip; bias then residual (torch order), 16-byte stores.
    auto epilogue = [&](const STile& t) {
      const rsrc_t ro = mkrsrc(p.out + (size_t)t.n0 * p.H * p.W * p.cout);
      const rsrc_t rr = mkrsrc(p.res ? p.res + (size_t)t.n0 * p.res_H * p.res_W * p.cout : p.out);
      const int co = t.ct * SBN + 4 * q;
      const f32x4 bias4 = gld4(p.bias + co);
      GStat gs = {0.f, 0.f, 0.f};
#pragma unroll
      for (int piece = 0; piece < 2 * T::MR; ++piece) {
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
        for (int nr = 0; nr < T::NR; ++nr)
#pragma unroll
          for (int rr8 = 0; rr8 < 8; ++rr8) {
            const int r = 8 * half + rr8;
            const int pp = (r & 3) + 8 * ((r >> 2) & 1) + 4 * h;  // pixel within the piece
            strip[pp * SLDE + nr * 32 + l32] = acc[mr][nr][r];
          }
        f32x4 vals[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          f32x4 val = *(const lds_f4*)(strip + (prow + 4 * v) * SLDE + 4 * q);
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
        // GroupNorm granule statistics: this wave's 64 pixels x quad q, one entry per wave
        gs = gstat_xlanes16(gs);
        if (lane < 16) {
          const int e = ((t.y0 / STH) * p.tiles_x + t.x0 / STW) * 4 + wave;
          float* o = p.gstat + (((size_t)t.n0 * (p.cout / 4) + t.ct * 16 + q) * p.gstat_E + e) * 2;
          o[0] = gs.mean;
          o[1] = gs.m2;
        }
      }
    };
    zero();
    BARRIER_CONSUMER();  // chunk 0 staged
    int k = 0, ti = 0;
    for (int j = 0; j < J; ++j) {
      consume<SBM, SBN, 4, 1, 9>(acc, A0 + (j & 1) * SA, W0 + (j & 1) * SWP, SNP, SHW, pb, 0);
      if (++k == nch) {
        k = 0;
        epilogue(tile_of(ti++));
        zero();
      }
      BARRIER_CONSUMER();
    }
    return;
  }

  // ---- producers: halo two chunks ahead in registers, weights one chunk ahead by LDS-DMA ----
  const int ptid = tid - NP_T;
  SProducer<XF> P;
  P.init(ptid);
  SSet<XF> s0, s1;
  auto load_chunk = [&](SSet<XF>& s, int c) {
    c = min(c, J - 1);
    const int ti = c / nch, kk = c - ti * nch;
    P.load(s, p, tile_of(ti), ti, kk, nch);
  };
  auto dma_chunk = [&](int c) {
    c = min(c, J - 1);
    const int ti = c / nch, kk = c - ti * nch;
    P.dma_weights(p, tile_of(ti).ct, kk, nch, W0 + (c & 1) * SWP);
  };
  dma_chunk(0);
  load_chunk(s0, 0);
  load_chunk(s1, 1);
  P.store(s0, p.act, A0);
  BARRIER_PRODUCER(5);  // chunk 0's weights landed (younger: chunk 1's five halo/coef loads)
  // interval j: weights of chunk j+1 (DMA, first so a vmcnt can single them out), halo of chunk
  // j+2, LDS writes of chunk j+1, barrier once the DMA has landed
  for (int j = 0; j < J; j += 2) {
    dma_chunk(j + 1);
    load_chunk(s0, j + 2);
    if (j + 1 < J) P.store(s1, p.act, A0 + SA);
    BARRIER_PRODUCER(5);
    if (j + 1 >= J) break;
    dma_chunk(j + 2);
    load_chunk(s1, j + 3);
    if (j + 2 < J) P.store(s0, p.act, A0);
    BARRIER_PRODUCER(5);
  }
}

}  // namespace

size_t conv_stream_lds_bytes() { return (size_t)SLDS_FLOATS * sizeof(float) + (IFD_TRACE ? 512 : 0); }

// Eligible: BM = 256 geometry (8 x 32 tiles of one image), BN = 64, 3x3 without a 1x1 segment,
// NHWC epilogue without split-K, >= EPI_PIECES + 1 chunks (the epilogue buffer is reused once
// per tile), cout a multiple of 64, whole
// groups of 8 pixel tiles (the XCD-aware map is then a bijection onto real tiles), a GroupNorm
// prologue and no avg-pool residual.
bool conv_stream_eligible(const ConvParams& p, int taps, int xform, int bn) {
  return taps == 9 && xform != XF_DOWN && bn == SBN && p.bm == SBM && p.TW == STW && p.TH == STH && p.IMGS == 1 && !p.wskip &&
         p.epi == EPI_NHWC && p.ksplit == 1 && p.cin_pad / 8 >= EPI_PIECES + 1 && p.cout % SBN == 0 &&
         p.cout_pad == p.cout && p.npix_tiles % 8 == 0 && p.act != ACT_NONE &&
         (!p.res || p.res_xform != XF_DOWN);
}

template <int XF, int CW>
static int launch_stream_inst(const ConvParams& p, hipStream_t stream) {
  static bool attr_set[kMaxDevices] = {};
  hipError_t e = set_lds_attr_once(attr_set, reinterpret_cast<const void*>(&conv_stream_kernel<XF, CW>), 160 * 1024);
  if (e != hipSuccess) return (int)e;
  const int ncu = device_cu_count();
  const int nvirt = p.npix_tiles * (p.cout_pad / SBN);
  const int grid = nvirt < ncu ? nvirt : ncu;  // one workgroup per CU (LDS-bound)
  hipLaunchKernelGGL((conv_stream_kernel<XF, CW>), dim3(grid), dim3(64 * CW + NP_T), conv_stream_lds_bytes(), stream, p);
  return IFD_LAUNCH_STATUS();
}

template <int XF>
static int launch_stream2_inst(const ConvParams& p, hipStream_t stream) {
  static bool attr_set[kMaxDevices] = {};
  const size_t lds = (size_t)S2_LDS_FLOATS * sizeof(float);
  hipError_t e = set_lds_attr_once(attr_set, reinterpret_cast<const void*>(&conv_stream2_kernel<XF>), (int)lds);
  if (e != hipSuccess) return (int)e;
  const int ncu = device_cu_count();
  const int nvirt = p.npix_tiles * (p.cout_pad / SBN);
  const int grid = nvirt < 2 * ncu ? nvirt : 2 * ncu;  // two workgroups per CU
  hipLaunchKernelGGL((conv_stream2_kernel<XF>), dim3(grid), dim3(NT), lds, stream, p);
  return IFD_LAUNCH_STATUS();
}

int launch_conv_stream(const ConvParams& p, int xform, int mode, hipStream_t stream) {
  if (mode == 2) {
    if (xform == XF_NONE) return launch_stream2_inst<XF_NONE>(p, stream);
    if (xform == XF_UP) return launch_stream2_inst<XF_UP>(p, stream);
    return (int)hipErrorInvalidValue;
  }
  if (xform == XF_NONE) return launch_stream_inst<XF_NONE, 8>(p, stream);
  if (xform == XF_UP) return launch_stream_inst<XF_UP, 8>(p, stream);
  return (int)hipErrorInvalidValue;  // avg-pool prologue: conv.hip (its 4-source register sets do not fit 3 deep)
}

}  // namespace ifd
