// Device helpers shared by the conv kernels (conv.hip, conv_stream.hip).
#pragma once
#include "common.h"

// Timing-only ablation builds (never shipped; outputs are garbage):
//   IFD_ABLATE=1  producers skip every load / store (barriers only)
//   IFD_ABLATE=2  consumers skip the fragment ds_reads (MFMAs on stale registers)
#ifndef IFD_ABLATE
#define IFD_ABLATE 0
#endif

namespace ifd {

// Explicit address spaces: without them the LDS / global accesses compile to flat_* ops, which
// count on BOTH vmcnt and lgkmcnt, so an LDS-read wait would also wait for in-flight global loads.
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) float lds_f;
typedef __attribute__((address_space(3))) f32x4 lds_f4;
typedef __attribute__((address_space(1))) const f32x4 glb_f4;
typedef __attribute__((address_space(1))) const float glb_f;

__device__ __forceinline__ f32x4 gld4(const float* p) { return *(glb_f4*)(p); }
__device__ __forceinline__ float gld1(const float* p) { return *(glb_f*)(p); }
__device__ __forceinline__ void gst1(float* p, float v) { *(__attribute__((address_space(1))) float*)(p) = v; }
__device__ __forceinline__ void gst4(float* p, f32x4 v) { *(__attribute__((address_space(1))) f32x4*)(p) = v; }

// SiLU of the GroupNorm-applied value: x * rcp(1 + 2^(-x*log2 e)) on v_exp_f32 / v_rcp_f32
// (relative error < 1e-6 for |x| < 10 against torch's x / (1 + exp(-x)); a whole UNet eval stays
// at ~2e-6 max-abs from the reference). The producer waves bound the pipeline, so the short form.
__device__ __forceinline__ float silu_fast(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }

// Chan-merge statistics (count, mean, M2) for the fused GroupNorm granules.
struct GStat {
  float n, mean, m2;
};
__device__ __forceinline__ GStat gmerge(GStat a, GStat b) {
  const float n = a.n + b.n;
  const float d = b.mean - a.mean;
  const float f = b.n / n;
  return {n, a.mean + d * f, a.m2 + b.m2 + d * d * a.n * f};
}
// two-pass statistics of K quads held in registers
template <int K>
__device__ __forceinline__ GStat gstat_of(const f32x4 (&v)[K]) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < K; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  const float mean = s * (1.0f / (4 * K));
  float m2 = 0.f;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const f32x4 d = v[i] - mean;
    m2 += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
  }
  return {4.0f * K, mean, m2};
}
// merge the statistics of lanes l, l ^ 16, l ^ 32 (butterfly, symmetric: all four lanes end equal)
__device__ __forceinline__ GStat gstat_xlanes16(GStat a) {
#pragma unroll
  for (int off = 16; off <= 32; off <<= 1) {
    GStat b;
    b.n = __shfl_xor(a.n, off);
    b.mean = __shfl_xor(a.mean, off);
    b.m2 = __shfl_xor(a.m2, off);
    const bool lo = (threadIdx.x & off) == 0;
    a = lo ? gmerge(a, b) : gmerge(b, a);
  }
  return a;
}

// Persistent kernels (conv_stream.hip, conv_x3.hip): tile L of a block's strided list -> (image,
// row, column, channel tile), the XCD-aware map of conv.hip (channel tiles of one pixel tile 8 IDs
// apart, so they share an XCD and its L2).
struct STile {
  int n0, y0, x0, ct;
};

__device__ __forceinline__ STile decode_tile(const ConvParams& p, int L, int nct) {
  const int grp = L / (8 * nct), rr = L - grp * 8 * nct;
  STile t;
  t.ct = rr >> 3;
  int bx = grp * 8 + (rr & 7);
  const int tx = bx % p.tiles_x;
  bx /= p.tiles_x;
  const int ty = bx % p.tiles_y;
  t.n0 = bx / p.tiles_y;
  t.y0 = ty * p.TH;
  t.x0 = tx * p.TW;
  return t;
}

// gfx950 executes v_mfma_f32_32x32x2_f32 on the vector ALUs: a producer's VALU instruction
// issues only between MFMAs of the consumer beside it on the SIMD, so every producer VALU cycle
// is a matrix cycle lost (per-interval stamps: interval = MFMA time + producer busy time). The
// producer therefore does its address work once per TILE: loads go through buffer descriptors
// (SGPR base per tile + per-lane 32-bit offset fixed for the tile + scalar chunk offset), so a
// chunk's loads cost no VALU at all; what remains per chunk is the activation math itself.
typedef __amdgpu_buffer_rsrc_t rsrc_t;

__device__ __forceinline__ rsrc_t mkrsrc(const float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, 0x7ffffff0, 0x00020000);
}
__device__ __forceinline__ f32x4 bld4(rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
__device__ __forceinline__ void bst4(rsrc_t r, int voff, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), r, voff,
                                         0, 0);
}

constexpr int NT = 512;    // threads per block
constexpr int NP_T = 256;  // producer threads (waves 4-7)

template <int BM, int BN, int WGM, int WGN>
struct Tile {
  static constexpr int MR = BM / WGM / 32;
  static constexpr int NR = BN / WGN / 32;
  static_assert(MR >= 1 && NR >= 1, "bad wave grid");
  static_assert(WGM * WGN == 4 || WGM * WGN == 8, "4 or 8 consumer waves");
};

template <int BM, int BN, int WGM, int WGN>
using AccArr = f32x16[Tile<BM, BN, WGM, WGN>::MR][Tile<BM, BN, WGM, WGN>::NR];
template <int BM, int BN, int WGM, int WGN>
using PixArr = int[Tile<BM, BN, WGM, WGN>::MR];

// MFMAs over one staged chunk (consumer waves). Fragment reads are software-pipelined one tap
// ahead (two register slots, fully unrolled so the slots are static).
template <int BM, int BN, int WGM, int WGN, int TAPS>
__device__ __forceinline__ void consume(AccArr<BM, BN, WGM, WGN>& acc, const lds_f* As, const lds_f* Ws_, int NP,
                                        int HWd, const PixArr<BM, BN, WGM, WGN>& pb, int wn0) {
  using T = Tile<BM, BN, WGM, WGN>;
  const int lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
  const lds_f* Ab = As + 4 * h * NP;
  const lds_f* Wb = Ws_ + 4 * (h * BN + wn0 + l32);
  f32x4 a[2][T::MR], b[2][T::NR];
  auto fetch = [&](int tap, int slot) {
    if (IFD_ABLATE == 2) {
      asm volatile("" : "+v"(a[slot][0]), "+v"(b[slot][0]));
      return;
    }
    const int toff = (TAPS == 9) ? ((tap / 3) * HWd + (tap % 3)) : 0;
#pragma unroll
    for (int mr = 0; mr < T::MR; ++mr) a[slot][mr] = *(const lds_f4*)(Ab + 4 * (pb[mr] + toff));
#pragma unroll
    for (int nr = 0; nr < T::NR; ++nr) b[slot][nr] = *(const lds_f4*)(Wb + 4 * (tap * 2 * BN + nr * 32));
  };
  fetch(0, 0);
  // One "round" = the MR*NR independent MFMAs of one k-pair; consecutive MFMAs never share an
  // accumulator (a dependent back-to-back v_mfma_f32_32x32x2_f32 stalls the SIMD's issue and
  // starves the producer wave beside it). sched_barrier(0) keeps the rounds in program order and
  // places the next tap's fragment reads after the first round.
  auto round = [&](int cur, int j) {
#pragma unroll
    for (int mr = 0; mr < T::MR; ++mr)
#pragma unroll
      for (int nr = 0; nr < T::NR; ++nr)
        acc[mr][nr] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[cur][mr][j], b[cur][nr][j], acc[mr][nr], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  };
#pragma unroll
  for (int tap = 0; tap < TAPS; ++tap) {
    const int cur = tap & 1;
    round(cur, 0);
    if (tap + 1 < TAPS) fetch(tap + 1, cur ^ 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 1; j < 4; ++j) {
      round(cur, j);
#if defined(IFD_YIELD) && IFD_YIELD == 2
      __builtin_amdgcn_s_sleep(1);
#endif
    }
#if defined(IFD_YIELD) && IFD_YIELD == 1
    __builtin_amdgcn_s_sleep(1);
#endif
  }
}

}  // namespace ifd
