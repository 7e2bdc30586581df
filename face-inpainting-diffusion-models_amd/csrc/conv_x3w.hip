// 3xf16 fused 3x3 convolution, wide-unit variant: 128 output channels per work unit.
//
// Same arithmetic as conv_x3.hip (operands split into f16 hi + lo, weights pre-split and pre-scaled
// by 2^11, three f16 MFMAs per MAC into one fp32 accumulator; the fused prologue is GroupNorm-apply
// [+ scale/shift] + SiLU, nearest-up, zero padding; the epilogue adds bias and residual and writes
// the output's GroupNorm granule statistics). What changes is who does what per FLOP.
//
// conv_x3's chunk interval is set by its producer waves' prologue VALU (GroupNorm-apply + SiLU +
// split per staged value, issued on the SIMDs beside the consumers' MFMAs): with 64
// output channels per unit, every input value is activated once per channel tile (twice for the
// 128-channel layers) and 340 halo pixels are staged per 256 output pixels. Here a unit is an
// 8 x 16 pixel tile x 128 output channels: per 16-channel chunk the producers stage 180 halo pixels
// (720 quarter-pixel items, 12 values per producer lane against 24) for the same MFMA work.
//
// The 128-channel weight slab of a chunk (72 KiB) would not fit a multi-buffered LDS ring beside the
// halo stages, so the weights do not go through LDS at all: consumer wave w owns output channels
// 32 w .. 32 w + 31 of the unit, and its B fragments are private to it. Each consumer loads them
// from L2 straight into registers (two 1-KiB wave loads per tap, 18 per chunk, 72 VGPRs), one chunk
// ahead: right after a tap's last MFMA group has issued, the same registers are reloaded with the
// next chunk's fragments of that tap. LDS holds the halo stages and the residual; one barrier per
// chunk hands a stage from the producers to the consumers.
//   * waves 0-3 consumers: wave w = 128 pixels (4 blocks of 32, rows 2 mr, 2 mr + 1 of the tile) x
//     32 channels; per tap 8 A-fragment ds_read_b128 (hi / lo x 4 pixel blocks, double-buffered by
//     tap parity) and 12 v_mfma_f32_32x32x16_f16 in three groups of four independent accumulators.
//     The stages are written two chunks ahead, so a chunk's tap-0 fragments are read during the
//     previous chunk's last tap instead of after the barrier. The residual arrives by LDS-DMA during
//     the unit's last chunks (no registers held for it).
//   * waves 4-7 producers: thread t stages channel quarter t & 3 of halo pixels t / 4 + 64 k
//     (k < 3): one 16-B load per item, the GroupNorm coefficients of its quarter (two 16-B loads),
//     registers two intervals ahead, the prologue + split two chunks ahead, 8-B LDS writes.
// LDS: A = [part hi / lo][channel half h][180 halo px][8 f16] (11.25 KiB) x 3 stages + 4 x 16 KiB of
// residual.
#include "conv.h"
#include "conv_dev.h"

namespace ifd {

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) f16x8 lds_h8;
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) u32x2 lds_u2;

constexpr int WTW = 16, WTH = 8;          // output tile
constexpr int WHW = WTW + 2;              // halo row width
constexpr int WNP = WHW * (WTH + 2);      // 180 halo pixels
constexpr int WBN = 128;                  // output channels per unit
constexpr int WA = 4 * WNP * 4;           // floats per A stage (4 planes x 180 px x 16 B)
constexpr int WST = 3;                    // A stages (the consumers read a chunk's tap 0 an interval early)
constexpr int WRES = 64 * 64;             // residual floats per consumer wave (64 registers x 64 lanes)
constexpr int W_LDS_FLOATS = WST * WA + 4 * WRES;  // 34,560 + 65,536 B
constexpr int WIT = 3;                    // quarter-pixel items per producer thread (4 x 180 = 720 <= 3 x 256)
constexpr float kLo = 2048.0f;            // 2^11
constexpr int WPF = 2;                    // residual / bias prefetch: chunks before the unit's end
static_assert(4 * WNP <= WIT * NP_T, "producer items");

#define WBARRIER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")

// Timing-only ablation builds (never shipped; outputs are garbage): X3W_ABLATE=
//   1 producers write the raw bits (no prologue / split VALU)   2 consumers skip the B reloads
//   3 consumers skip the A reads after a chunk's tap 0          4 producers idle (barriers only)
//   5 consumers skip the MFMAs   6 SiLU replaced by the affine value (no exp / rcp)
//   7 lo part not computed (zero) and no range guard   8 no range guard
//   9 exp and rcp replaced by 8-FMA chains each (same dependency depth class, no transcendental)
// IFD_TRACE=1 builds: consumer wave 0 of each block stamps (s_memtime, s_memrealtime) at its start and
// end into ConvParams::trace[64 b + 0..3] (the shader clock over the launch = d memtime / d realtime x 100 MHz)
#ifndef IFD_TRACE
#define IFD_TRACE 0
#endif
#ifndef X3W_ABLATE
#define X3W_ABLATE 0
#endif

// f16 split of a pair (conv_x3.hip split2): hi = f16(v), lo = f16(v - hi); the empty asm keeps v an
// fp32 register value so hipcc cannot fold the producing multiply into a v_fma_mix conversion.
__device__ __forceinline__ void split2w(float v0, float v1, unsigned& h, unsigned& l) {
  asm volatile("" : "+v"(v0), "+v"(v1));
  const f16x2 h2 = __builtin_convertvector(f32x2{v0, v1}, f16x2);
  h = __builtin_bit_cast(unsigned, h2);
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%3 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %2, 1.0, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(l)
      : "v"(v0), "v"(v1), "v"(h));
}

// SiLU of the GroupNorm-applied value t: t * rcp(1 + 2^(-t log2 e)), padding (pinf = +inf) -> 0.
// X3W_SILU selects how the two reciprocal / exponential steps are computed:
//   0 v_exp_f32 + v_rcp_f32 (two transcendentals)
//   1 polynomial 2^x + v_rcp_f32     2 v_exp_f32 + Newton reciprocal     3 neither (full-rate VALU only)
// The polynomial: x clamped to [-126, 126] (a padding value, x = +inf, then gives t * 2^-126, which the
// f16 split rounds to exactly 0, as it does every |v| < 2^-25), n = rint(x) by the 1.5 * 2^23 shifter,
// 2^(x - n) by a degree-6 fit on [-1/2, 1/2] (max rel. error 1.0e-7), 2^n built in the exponent field.
// The Newton reciprocal: seed 0x7EF311C3 - bits(d) (rel. error <= 12 %), three steps r += r (1 - d r)
// (<= 4e-8).
#ifndef X3W_SILU
#define X3W_SILU 0
#endif
__device__ __forceinline__ float exp2_poly(float x) {
  x = __builtin_amdgcn_fmed3f(x, -126.0f, 126.0f);
  const float sh = 12582912.0f;  // 1.5 * 2^23
  const float y = x + sh;
  const float f = x - (y - sh);
  float p = 1.5337577497120947e-04f;
  p = fmaf(p, f, 1.3399859890341759e-03f);
  p = fmaf(p, f, 9.618519805371761e-03f);
  p = fmaf(p, f, 5.550329014658928e-02f);
  p = fmaf(p, f, 2.4022646248340607e-01f);
  p = fmaf(p, f, 6.931471824645996e-01f);
  p = fmaf(p, f, 1.0f);
  // bits(y) = 0x4B400000 + n  ->  bits(2^n) = (n + 127) << 23
  const unsigned sc = (__builtin_bit_cast(unsigned, y) << 23) + ((127u - 0x4B400000u) << 23);
  return p * __builtin_bit_cast(float, sc);
}
__device__ __forceinline__ float rcp_newton(float d) {
  float r = __builtin_bit_cast(float, 0x7EF311C3u - __builtin_bit_cast(unsigned, d));
#pragma unroll
  for (int i = 0; i < 3; ++i) r = fmaf(r, fmaf(-d, r, 1.0f), r);
  return r;
}
__device__ __forceinline__ float silu_w(float t, float pinf) {
  const float x = fmaf(t, -1.4426950408889634f, pinf);
  const float e = (X3W_SILU & 1) ? exp2_poly(x) : __builtin_amdgcn_exp2f(x);
  const float d = 1.0f + e;
  return t * ((X3W_SILU & 2) ? rcp_newton(d) : __builtin_amdgcn_rcpf(d));
}

__device__ __forceinline__ f32x16 wmfma(f16x8 a, f16x8 b, f32x16 c) {
  if (X3W_ABLATE == 5) {
    asm volatile("" ::"v"(a), "v"(b));
    return c;
  }
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// Unit u of block b: pixel tile b + G (u / nct), channel tile u % nct (the channel tiles of a pixel
// tile back to back, so the second one re-reads the halo from L2). Tile dims are powers of two.
struct WUnit {
  int n0, y0, x0, ct, tile;
};
__device__ __forceinline__ WUnit w_unit(const ConvParams& p, int lnct, int ltx, int lty, int b, int u) {
  WUnit t;
  const int q = u >> lnct;
  t.ct = u - (q << lnct);
  int bx = b + (int)gridDim.x * q;
  t.tile = bx;
  t.x0 = (bx & ((1 << ltx) - 1)) * WTW;
  bx >>= ltx;
  t.y0 = (bx & ((1 << lty) - 1)) * WTH;
  t.n0 = bx >> lty;
  return t;
}

template <int XF>
struct WProducer {
  int q;              // channel quarter this thread stages (channels 4 q .. 4 q + 3 of a chunk)
  int px[WIT];        // halo pixel of item k, -1 past the 180
  int hy[WIT], hx[WIT];
  int off0[WIT], off1[WIT];
  float valid[WIT];
  rsrc_t r0, r1, ra, rb;
  int cur_tile = -1;
  float gmax = 0.f;
  struct Set {
    f32x4 raw[WIT];
    f32x4 ca, cb;
    float vld[WIT];
  };

  __device__ __forceinline__ void init(int pt) {
    q = pt & 3;
#pragma unroll
    for (int k = 0; k < WIT; ++k) {
      const int pix = (pt >> 2) + 64 * k;
      px[k] = pix < WNP ? pix : -1;
      hy[k] = pix / WHW;
      hx[k] = pix - hy[k] * WHW;
    }
  }

  __device__ __forceinline__ void enter(const ConvParams& p, const WUnit& t) {
    if (t.tile == cur_tile) return;
    cur_tile = t.tile;
    const size_t img = (size_t)p.Hin * p.Win;
    r0 = mkrsrc(p.in0 + (size_t)t.n0 * img * p.c0);
    r1 = mkrsrc(p.in1 ? p.in1 + (size_t)t.n0 * img * p.c1 : p.in0);
    const int ctot = p.c0 + p.c1;
    // act == ACT_NONE: the coefficient loads still issue (a fixed load count) from the input
    ra = p.actA ? mkrsrc(p.actA + (size_t)t.n0 * ctot) : r0;
    rb = p.actB ? mkrsrc(p.actB + (size_t)t.n0 * ctot) : r0;
#pragma unroll
    for (int k = 0; k < WIT; ++k) {
      const int y = t.y0 + hy[k] - 1, x = t.x0 + hx[k] - 1;
      const bool inb = px[k] >= 0 && y >= 0 && y < p.H && x >= 0 && x < p.W;
      int sy = y, sx = x;
      if (XF == XF_UP) {
        sy = y >> 1;
        sx = x >> 1;
      }
      const int sp = inb ? sy * p.Win + sx : 0;
      valid[k] = inb ? 1.f : 0.f;
      off0[k] = (sp * p.c0 + 4 * q) * 4;
      off1[k] = (sp * p.c1 + 4 * q) * 4;
    }
  }

  // the 16-channel chunk `idx` of the concatenated input: WIT + 2 loads
  __device__ __forceinline__ void load(Set& s, const ConvParams& p, int idx) const {
    if (X3W_ABLATE == 4) return;
    const int cb0 = 16 * idx;
#pragma unroll
    for (int k = 0; k < WIT; ++k) s.vld[k] = valid[k];
    if (cb0 < p.c0) {
#pragma unroll
      for (int k = 0; k < WIT; ++k) s.raw[k] = bld4(r0, off0[k], cb0 * 4);
    } else {
#pragma unroll
      for (int k = 0; k < WIT; ++k) s.raw[k] = bld4(r1, off1[k], (cb0 - p.c0) * 4);
    }
    s.ca = bld4(ra, 16 * q, cb0 * 4);
    s.cb = bld4(rb, 16 * q, cb0 * 4);
  }

  template <int ACT, int NPROD>
  __device__ __forceinline__ void store_act(const Set& s, lds_f* As) {
    const int hh = q >> 1, sub = q & 1;
    if (X3W_ABLATE == 4) return;
#pragma unroll
    for (int k = 0; k < WIT; ++k) {
      if (px[k] < 0) continue;
      if (X3W_ABLATE == 1) {
        lds_f* d1 = As + 4 * (hh * WNP + px[k]) + 2 * sub;
        *(lds_u2*)d1 = u32x2{__builtin_bit_cast(unsigned, s.raw[k][0]), __builtin_bit_cast(unsigned, s.raw[k][1])};
        *(lds_u2*)(d1 + 4 * 2 * WNP) = u32x2{__builtin_bit_cast(unsigned, s.raw[k][2]), __builtin_bit_cast(unsigned, s.raw[k][3])};
        continue;
      }
      float v[4];
      if (ACT == ACT_AFFINE_SILU) {
        // zero padding through the exponent: 2^(+inf) = inf, rcp(1 + inf) = 0, t * 0 = 0
        const float pinf = s.vld[k] != 0.f ? 0.f : __builtin_inff();
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float t = fmaf(s.ca[c], s.raw[k][c], s.cb[c]);
          if (X3W_ABLATE == 6)
            v[c] = fmaf(t, 0.5f, pinf);
          else if (X3W_ABLATE == 9) {
            float e = fmaf(t, -1.4426950408889634f, pinf);
            float a = e;
#pragma unroll
            for (int z = 0; z < 8; ++z) a = fmaf(a, e, 0.3f);
            float d = 1.0f + a, r = d;
#pragma unroll
            for (int z = 0; z < 8; ++z) r = fmaf(r, d, -0.7f);
            v[c] = t * r;
          }
          else
            v[c] = silu_w(t, pinf);
        }
      } else if (ACT == ACT_AFFINE) {
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = (s.ca[c] * s.raw[k][c] + s.cb[c]) * s.vld[k];
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = s.raw[k][c] * s.vld[k];
      }
      // range guard: |v| >= 65504 would split into an f16 inf
      if (X3W_ABLATE != 7 && X3W_ABLATE != 8)
        gmax = fmaxf(gmax, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
      unsigned h0, h1, l0, l1;
      lds_f* dst = As + 4 * (hh * WNP + px[k]) + 2 * sub;
      if (NPROD == 1) {
        float a0 = v[0], a1 = v[1], a2 = v[2], a3 = v[3];
        asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
        h0 = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a0, a1}, f16x2));
        h1 = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a2, a3}, f16x2));
        *(lds_u2*)dst = u32x2{h0, h1};
        continue;
      }
      if (X3W_ABLATE == 7) {
        h0 = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{v[0], v[1]}, f16x2));
        h1 = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{v[2], v[3]}, f16x2));
        l0 = l1 = 0;
      } else {
        split2w(v[0], v[1], h0, l0);
        split2w(v[2], v[3], h1, l1);
      }
      *(lds_u2*)dst = u32x2{h0, h1};
      *(lds_u2*)(dst + 4 * 2 * WNP) = u32x2{l0, l1};
    }
  }
  template <int NPROD>
  __device__ __forceinline__ void store(const Set& s, int act, lds_f* As) {
    if (act == ACT_AFFINE_SILU)
      store_act<ACT_AFFINE_SILU, NPROD>(s, As);
    else if (act == ACT_NONE)
      store_act<ACT_NONE, NPROD>(s, As);
    else
      store_act<ACT_AFFINE, NPROD>(s, As);
  }
};

__device__ __forceinline__ void wave_halves_w(float v, float& lo, float& hi) {
  const unsigned x = __builtin_bit_cast(unsigned, v);
  const auto a = __builtin_amdgcn_permlane32_swap(x, 0u, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(0u, x, false, false);
  lo = __builtin_bit_cast(float, a[0] | b[0]);
  hi = __builtin_bit_cast(float, a[1] | b[1]);
}

template <int XF, int NPROD>
__global__ __launch_bounds__(NT, 2) void conv_x3w_kernel(ConvParams p) {
  extern __shared__ __attribute__((aligned(16))) float smem_raw[];
  lds_f* const A0 = (lds_f*)(smem_raw);  // stage s at A0 + s * WA

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nct = p.cout / WBN;
  const int lnct = __builtin_ctz(nct), ltx = __builtin_ctz(p.tiles_x), lty = __builtin_ctz(p.tiles_y);
  const int G = gridDim.x, b = blockIdx.x;
  const int nu = ((p.npix_tiles - b + G - 1) / G) << lnct;  // host: grid <= npix_tiles
  const int nch = p.cin_pad / 16;                            // host: even
  const int J = nu * nch;

  if (IFD_TRACE && p.trace && tid == 0) {
    p.trace[64 * b + 0] = __builtin_amdgcn_s_memtime();
    p.trace[64 * b + 1] = __builtin_amdgcn_s_memrealtime();
  }
  if (wave < 4) {
    // ---------------- consumers ----------------
    const int h = lane >> 5, l32 = lane & 31;
    int pb[4];
#pragma unroll
    for (int mr = 0; mr < 4; ++mr) {
      const int m = 32 * mr + l32;
      pb[mr] = (m >> 4) * WHW + (m & 15);
    }
    // B fragments: lane (h, l32) of wave w = channel 32 w + l32 of the unit's 128, k = 8 h .. 8 h + 7
    const rsrc_t rw = mkrsrc(p.wpack);
    const int bvo = (h * WBN + 32 * wave + l32) * 16;
    auto bsoff = [&](int ct, int chunk, int tap, int part) { return (((ct * nch + chunk) * 9 + tap) * 2 + part) * (2 * WBN * 16); };
    f16x8 bh[9], bl[9];
    auto bload = [&](int ct, int chunk, int tap) __attribute__((always_inline)) {
      if (X3W_ABLATE == 2 && chunk + ct > 0) return;
      bh[tap] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, bvo, bsoff(ct, chunk, tap, 0), 0));
      if (NPROD == 3)
        bl[tap] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, bvo, bsoff(ct, chunk, tap, 1), 0));
    };
    f32x16 acc[4];
    auto zero = [&]() {
#pragma unroll
      for (int mr = 0; mr < 4; ++mr)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[mr][r] = 0.f;
    };
    // Register (mr, r) of lane (h, l32): channel 32 w + l32 at tile pixel m = 32 mr + 8 (r >> 2) + 4 h + (r & 3),
    // i.e. tile row 2 mr + (r >> 3), column 8 ((r >> 2) & 1) + 4 h + (r & 3).
    auto roff = [&](int r) { return (((r >> 3) * p.W) + 8 * ((r >> 2) & 1) + (r & 3)) * p.cout * 4; };
    const int mstep = 2 * p.W * p.cout * 4;
    auto vbase = [&](const WUnit& t) { return (((t.y0 * p.W) + t.x0 + 4 * h) * p.cout + t.ct * WBN + 32 * wave + l32) * 4; };
    // The residual goes HBM -> LDS by DMA (buffer_load ... lds) during the unit's last chunks: register
    // (mr, r) of every lane lands at Rw[(16 mr + r) * 64 + lane] (64 dword DMAs of 256 B), read back in
    // the epilogue; no registers are held for it across the chunks.
    lds_f* const Rw = A0 + WST * WA + wave * WRES;
    float bias = 0.f;
    auto prefetch = [&](const WUnit& t) {
      bias = gld1(p.bias + t.ct * WBN + 32 * wave + l32);
      if (!p.res) return;
      const rsrc_t rr = mkrsrc(p.res + (size_t)t.n0 * p.res_H * p.res_W * p.cout);
      const int vb = vbase(t);
#pragma unroll
      for (int mr = 0; mr < 4; ++mr)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          auto* dst = (__attribute__((address_space(3))) void*)(Rw + (16 * mr + r) * 64);
          if (p.res_xform == XF_NONE) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rr, dst, 4, vb + mr * mstep, roff(r), 0, 0);
          } else {  // XF_UP: nearest-upsampled residual
            const int y = (t.y0 + 2 * mr + (r >> 3)) >> 1, x = (t.x0 + 8 * ((r >> 2) & 1) + 4 * h + (r & 3)) >> 1;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rr, dst, 4, ((y * p.res_W + x) * p.cout + t.ct * WBN + 32 * wave + l32) * 4,
                                                     0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);  // one address at a time (64 hoisted ones would spill)
          }
        }
    };
    auto epilogue = [&](const WUnit& t) {
      const size_t img = (size_t)p.H * p.W * p.cout;
      const rsrc_t ro = mkrsrc(p.out + (size_t)t.n0 * img);
      const int vb = vbase(t);
      // the residual DMA (not in hipcc's vmcnt model) was issued before the B loads of the unit's last
      // WPF chunks (18 per chunk, 9 in the f16 mode): wait until only those are outstanding
      static_assert(WPF == 2, "vmcnt literal");
      if (p.res) {
        if (NPROD == 3)
          asm volatile("s_waitcnt vmcnt(36)" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
      }
#pragma unroll
      for (int mr = 0; mr < 4; ++mr) {  // one pixel block at a time (bounds the residual values in flight)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float x = acc[mr][r] * (1.0f / kLo);  // exact rescale
          x = x + bias;
          if (p.res) x = Rw[(16 * mr + r) * 64 + lane] + x;  // torch order: x_res + (conv + bias)
          acc[mr][r] = x;
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, x), ro, vb + mr * mstep, roff(r), 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (p.gstat) {
        // granule statistics of 4 channels x the tile's 128 pixels: this lane's 64 (two-pass), the
        // other column half (lane ^ 32), then the channel quad (lanes ^ 1, ^ 2); every merge joins
        // two equal counts (conv_x3.hip)
        float sm = 0.f;
#pragma unroll
        for (int mr = 0; mr < 4; ++mr)
#pragma unroll
          for (int r = 0; r < 16; ++r) sm += acc[mr][r];
        float mean = sm * (1.0f / 64), m2 = 0.f;
#pragma unroll
        for (int mr = 0; mr < 4; ++mr)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float d = acc[mr][r] - mean;
            m2 += d * d;
          }
        auto merge = [&](float am, float aq, float bm, float bq, float n, float& om, float& oq) {
          const float d = bm - am;
          om = am + d * 0.5f;
          oq = (aq + bq) + ((d * d) * n) * 0.5f;
        };
        {
          float ml, mh, ql, qh;
          wave_halves_w(mean, ml, mh);
          wave_halves_w(m2, ql, qh);
          merge(ml, ql, mh, qh, 64.f, mean, m2);
        }
#define IFD_QPW(v, ctrl) __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), ctrl, 0xf, 0xf, false))
        merge(IFD_QPW(mean, 0xA0), IFD_QPW(m2, 0xA0), IFD_QPW(mean, 0xF5), IFD_QPW(m2, 0xF5), 128.f, mean, m2);
        merge(IFD_QPW(mean, 0x44), IFD_QPW(m2, 0x44), IFD_QPW(mean, 0xEE), IFD_QPW(m2, 0xEE), 256.f, mean, m2);
#undef IFD_QPW
        if (h == 0 && (l32 & 3) == 0) {
          const int e = (t.y0 / WTH) * p.tiles_x + t.x0 / WTW;
          float* o = p.gstat + (((size_t)t.n0 * (p.cout / 4) + t.ct * 32 + wave * 8 + (l32 >> 2)) * p.gstat_E + e) * 2;
          o[0] = mean;
          o[1] = m2;
        }
      }
    };
    // A fragments: the hi parts double-buffered by tap parity (the slot sequence runs on across chunks:
    // 9 taps, chunk parity sb = slot of its tap 0), the lo parts single: the next tap's hi reads go out
    // right after the current tap's hi x hi group and its lo reads after the lo x hi group, each 8
    // MFMAs ahead of use. The last tap reads the next chunk's tap 0 from its stage, which the producers
    // completed an interval earlier (three stages).
    f16x8 ah[2][4], al[4];
    auto afetch_hi = [&](const lds_f* As, int tap, int slot) __attribute__((always_inline)) {
      if (X3W_ABLATE == 3 && tap > 0) return;
      const lds_f* Ah = As + 4 * (h * WNP);
      const int toff = tap / 3 * WHW + tap % 3;
#pragma unroll
      for (int mr = 0; mr < 4; ++mr) ah[slot][mr] = *(const lds_h8*)(Ah + 4 * (pb[mr] + toff));
    };
    auto afetch_lo = [&](const lds_f* As, int tap) __attribute__((always_inline)) {
      if (NPROD == 1 || (X3W_ABLATE == 3 && tap > 0)) return;
      const lds_f* Al = As + 4 * ((2 + h) * WNP);
      const int toff = tap / 3 * WHW + tap % 3;
#pragma unroll
      for (int mr = 0; mr < 4; ++mr) al[mr] = *(const lds_h8*)(Al + 4 * (pb[mr] + toff));
    };
    auto chunk = [&](const lds_f* As, const lds_f* An, int sb, int nxt_ct, int nxt_ch) __attribute__((always_inline)) {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int cur = (sb + tap) & 1;
        const lds_f* Sn = tap + 1 < 9 ? As : An;
        const int tn = tap + 1 < 9 ? tap + 1 : 0;
#pragma unroll
        for (int mr = 0; mr < 4; ++mr) acc[mr] = wmfma(ah[cur][mr], bh[tap], acc[mr]);
        __builtin_amdgcn_sched_barrier(0);
        afetch_hi(Sn, tn, cur ^ 1);
        __builtin_amdgcn_sched_barrier(0);
        if (NPROD == 3) {
#pragma unroll
          for (int mr = 0; mr < 4; ++mr) acc[mr] = wmfma(ah[cur][mr], bl[tap], acc[mr]);
#pragma unroll
          for (int mr = 0; mr < 4; ++mr) acc[mr] = wmfma(al[mr], bh[tap], acc[mr]);
        }
        __builtin_amdgcn_sched_barrier(0);
        afetch_lo(Sn, tn);
        bload(nxt_ct, nxt_ch, tap);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    WUnit t = w_unit(p, lnct, ltx, lty, b, 0);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) bload(t.ct, 0, tap);
    zero();
    WBARRIER();  // chunks 0 and 1 staged
    afetch_hi(A0, 0, 0);
    afetch_lo(A0, 0);
    int sc = 0, sn = 1;  // stages of the current / next chunk
    for (int u = 0; u < nu; ++u) {
      const WUnit tn = u + 1 < nu ? w_unit(p, lnct, ltx, lty, b, u + 1) : t;
      for (int c = 0; c < nch; c += 2) {
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const int cc = c + half;
          if (cc == nch - WPF) prefetch(t);
          const bool last = cc + 1 == nch;
          chunk(A0 + sc * WA, A0 + sn * WA, half, last ? tn.ct : t.ct, last ? 0 : cc + 1);
          sc = sn;
          sn = sn == WST - 1 ? 0 : sn + 1;
          WBARRIER();
        }
      }
      epilogue(t);
      zero();
      t = tn;
    }
    if (IFD_TRACE && p.trace && tid == 0) {
      p.trace[64 * b + 2] = __builtin_amdgcn_s_memtime();
      p.trace[64 * b + 3] = __builtin_amdgcn_s_memrealtime();
    }
    return;
  }

  // ---------------- producers ----------------
  // interval j: prologue + split of chunk j + 2 into stage (j + 2) % 3 (its loads issued two intervals
  // earlier), then the loads of chunk j + 4
  const int pt = tid - NP_T;
  WProducer<XF> P;
  P.init(pt);
  typename WProducer<XF>::Set s0, s1;
  int jl = 0, ul = 0, kl = 0;
  WUnit tl = w_unit(p, lnct, ltx, lty, b, 0);
  int cidx = 0;
  auto issue = [&](typename WProducer<XF>::Set& s) {  // loads of the cursor's chunk, then advance
    if (jl < J) cidx = kl;
    P.enter(p, tl);
    P.load(s, p, cidx);
    if (jl + 1 < J) {
      ++jl;
      if (++kl == nch) {
        kl = 0;
        tl = w_unit(p, lnct, ltx, lty, b, ++ul);
      }
    } else {
      jl += 2;  // past the end: the last chunk re-issued (identical bytes), never read
    }
  };
  issue(s0);  // chunk 0
  issue(s1);  // chunk 1
  P.template store<NPROD>(s0, p.act, A0);
  issue(s0);  // chunk 2
  P.template store<NPROD>(s1, p.act, A0 + WA);
  issue(s1);  // chunk 3
  WBARRIER();
  int sw = 2;  // stage of chunk j + 2
  for (int j = 0; j < J; j += 2) {
    P.template store<NPROD>(s0, p.act, A0 + sw * WA);  // chunk j + 2 (past the end: an unread stage)
    sw = sw == WST - 1 ? 0 : sw + 1;
    issue(s0);  // chunk j + 4
    WBARRIER();
    if (j + 1 >= J) break;
    P.template store<NPROD>(s1, p.act, A0 + sw * WA);  // chunk j + 3
    sw = sw == WST - 1 ? 0 : sw + 1;
    issue(s1);  // chunk j + 5
    WBARRIER();
  }
  if (p.guard && P.gmax >= 65504.0f) atomicOr(p.guard, 1u);
}

template <int XF, int NPROD>
int launch_w_inst(const ConvParams& p, hipStream_t stream) {
  static bool attr_set[kMaxDevices] = {};
  const size_t lds = (size_t)W_LDS_FLOATS * sizeof(float);
  hipError_t e = set_lds_attr_once(attr_set, reinterpret_cast<const void*>(&conv_x3w_kernel<XF, NPROD>), (int)lds);
  if (e != hipSuccess) return (int)e;
  const int ncu = device_cu_count();
  const int grid = p.npix_tiles < ncu ? p.npix_tiles : ncu;  // one workgroup per CU
  hipLaunchKernelGGL((conv_x3w_kernel<XF, NPROD>), dim3(grid), dim3(NT), lds, stream, p);
  return (int)hipGetLastError();
}

}  // namespace

// Geometry of the wide variant: 8 x 16 single-image tiles, 128-channel units, no split-K.
void conv_x3w_geometry(ConvParams& p, int H, int W, int N) {
  p.bm = WTW * WTH;
  p.TW = WTW;
  p.TH = WTH;
  p.IMGS = 1;
  p.tiles_x = W / WTW;
  p.tiles_y = H / WTH;
  p.lg_tw = __builtin_ctz(WTW);
  p.lg_tpi = __builtin_ctz(WTW * WTH);
  p.npix_tiles = N * p.tiles_x * p.tiles_y;
  p.ksplit = 1;
}

bool conv_x3w_eligible(const ConvParams& p, int taps, int xform) {
  const int nct = p.cout / WBN;
  if ((p.cin_pad / 16) % 2) return false;  // chunks run in pairs (A-fragment slot parity)
  return taps == 9 && (xform == XF_NONE || xform == XF_UP) && !p.wskip && p.epi == EPI_NHWC && p.ksplit == 1 &&
         p.TW == WTW && p.TH == WTH && p.IMGS == 1 && p.H % WTH == 0 && p.W % WTW == 0 &&
         (p.tiles_x & (p.tiles_x - 1)) == 0 && (p.tiles_y & (p.tiles_y - 1)) == 0 && p.cout % WBN == 0 &&
         (nct & (nct - 1)) == 0 && p.cout_pad == p.cout && p.c0 % 16 == 0 && p.c1 % 16 == 0 && p.cin_pad >= 16 &&
         (!p.res || p.res_xform == XF_NONE || p.res_xform == XF_UP) && (xform != XF_UP || p.Hin * 2 == p.H);
}

int launch_conv_x3w(const ConvParams& p, int xform, hipStream_t stream) {
  if (p.x3_nprod == 1) return xform == XF_UP ? launch_w_inst<XF_UP, 1>(p, stream) : launch_w_inst<XF_NONE, 1>(p, stream);
  return xform == XF_UP ? launch_w_inst<XF_UP, 3>(p, stream) : launch_w_inst<XF_NONE, 3>(p, stream);
}

}  // namespace ifd
