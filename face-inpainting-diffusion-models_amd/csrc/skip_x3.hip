// A ResBlock's 1x1 skip_connection as its own launch in the split-MFMA modes (3xf16 / f16):
//     out[px][co] = bias_s[co] + sum_k W_s[co][k] * x[px][k],   x = cat(s0, s1) along channels
// (code/nn.py:184 builds skip_connection = conv_nd(dims, channels, out_channels, 1); :212 returns
// skip_connection(x) + h). The ResBlock's conv2 then runs as the plain residual instantiation of
// conv_x3 with this output as its residual, which adds it exactly in torch's order, x_res + (conv +
// bias). Before, the 1x1 chunks rode inside conv2's launch with the raw operand split in the MFMA
// waves beside the 3x3 producers: those layers ran at 0.35 of the split rate.
//
// Arithmetic as conv_x3.hip: a = a_hi + a_lo (f16 RNE each), the weights pre-split and pre-scaled
// by 2^11 (unet.hip pack_skip1x1_x3), three f16 MFMAs into one fp32 accumulator at scale 2^11.
//
// Structure: HBM-bound (per pixel K * 4 B in, cout * 4 B out, against K * cout * 6 f16 MACs). One
// persistent 512-thread block per CU holds the split weights of one NTC-channel output tile for the
// whole K in LDS (K * NTC * 4 B <= 128 KiB), loaded once per launch. After that the eight waves run
// independently (no further barrier): wave w walks 32-pixel tiles; per k = 16 step its lane (h, l32)
// loads channels 16 ks + 8 h .. + 7 of tile pixel l32 (two 16-B loads, SK_D steps ahead in a
// register ring that runs on across tiles), splits them in registers, reads the B fragments from
// LDS and issues 3 x NTC / 32 MFMAs. Epilogue: x 2^-11 + bias, quad-transposed dwordx4 stores (8 pixels x
// 128 B per instruction).
#include "conv.h"
#include "conv_dev.h"

namespace ifd {

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) f16x8 lds_h8;
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_u4;

constexpr int SK_NT = 512;  // threads per block (8 independent waves after the weight load)
#ifndef SK_DEPTH
#define SK_DEPTH 4
#endif
constexpr int SK_D = SK_DEPTH;  // k steps of operand in flight per wave
#ifndef SK_LDS_KB
#define SK_LDS_KB 128
#endif
#ifndef SK_WPE
#define SK_WPE 2  // waves per SIMD the registers are budgeted for (blocks per CU = SK_WPE / 2)
#endif
constexpr int SK_LDS_MAX = SK_LDS_KB * 1024;


constexpr float kScale = 2048.0f;  // 2^11

// hi = f16(v) for the pair (one v_cvt_pk_f16_f32), lo = f16(v - hi) (v_fma_mix: v - hi exact in
// fp32, rounded once); the empty asm keeps v an fp32 register value (conv_x3.hip split2).
__device__ __forceinline__ void split_pair(float v0, float v1, unsigned& h, unsigned& l) {
  asm volatile("" : "+v"(v0), "+v"(v1));
  const f16x2 h2 = __builtin_convertvector(f32x2{v0, v1}, f16x2);
  h = __builtin_bit_cast(unsigned, h2);
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%3 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %2, 1.0, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(l)
      : "v"(v0), "v"(v1), "v"(h));
}

__device__ __forceinline__ f32x16 mfma16(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

template <int NTC, int NPROD>
__global__ __launch_bounds__(SK_NT, SK_WPE) void skip_x3_kernel(Skip1x1Params p) {
  constexpr int NR = NTC / 32;
  extern __shared__ __attribute__((aligned(16))) float smem_raw[];
  lds_u4* const W = (lds_u4*)smem_raw;  // [ks][part][h][NTC] x 16 B
  const int K = p.sc0 + p.sc1, KS = K / 16;
  const int nnt = p.cout / NTC;
  const int nt = blockIdx.x % nnt;  // this block's output-channel tile
  const int bi = blockIdx.x / nnt, nb = gridDim.x / nnt;
  const int tid = threadIdx.x;
  {
    // 16-B units of the tile's weights, eight loads in flight per thread
    const int n16 = KS * 4 * NTC;
    const u32x4* src = (const u32x4*)p.wpack + (size_t)nt * n16;
    for (int i0 = 0; i0 < n16; i0 += 8 * SK_NT) {
      u32x4 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = i0 + j * SK_NT + tid;
        if (i < n16) v[j] = *(__attribute__((address_space(1))) const u32x4*)(src + i);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = i0 + j * SK_NT + tid;
        if (i < n16) W[i] = v[j];
      }
    }
  }
  __syncthreads();  // the only barrier: the waves are independent from here on

  const int lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int wave = tid >> 6;
  const int ntiles = p.npix / 32;
  const int GW = nb * (SK_NT / 64);
  const int w0 = bi * (SK_NT / 64) + wave;
  if (w0 >= ntiles) return;

  // load cursor: (tile lt, k step lk); descriptors rebased per tile so every offset is 32-bit
  int lt = w0, lk = 0;
  rsrc_t lr0, lr1;
  auto rebase = [&](int t) {
    lr0 = mkrsrc(p.s0 + (size_t)t * 32 * p.sc0);
    lr1 = p.s1 ? mkrsrc(p.s1 + (size_t)t * 32 * p.sc1) : lr0;
  };
  rebase(lt);
  const int lv0 = (l32 * p.sc0 + 8 * h) * 4, lv1 = (l32 * p.sc1 + 8 * h) * 4;
  auto issue = [&](f32x4(&b)[2]) __attribute__((always_inline)) {
    const int c = 16 * lk;
    if (c < p.sc0) {
      b[0] = bld4(lr0, lv0, c * 4);
      b[1] = bld4(lr0, lv0 + 16, c * 4);
    } else {
      b[0] = bld4(lr1, lv1, (c - p.sc0) * 4);
      b[1] = bld4(lr1, lv1 + 16, (c - p.sc0) * 4);
    }
    if (++lk == KS) {  // next tile of this wave (past the last one: re-load the last tile, unused)
      lk = 0;
      if (lt + GW < ntiles) {
        lt += GW;
        rebase(lt);
      }
    }
  };

  f32x4 ring[SK_D][2];
#pragma unroll
  for (int d = 0; d < SK_D; ++d) issue(ring[d]);

  const lds_u4* Wl = W + h * NTC + l32;
  // the tile's bias, loaded once (a load in the epilogue would make its vmcnt wait drain the ring)
  float bias[NR];
#pragma unroll
  for (int nr = 0; nr < NR; ++nr) bias[nr] = gld1(p.bias + nt * NTC + 32 * nr + l32);
  float gmax = 0.f;
  f32x16 acc[NR], accl[NR];  // hi x hi products; the two correction products (one rounding per output at the end)
  for (int t = w0; t < ntiles; t += GW) {
#pragma unroll
    for (int nr = 0; nr < NR; ++nr)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        acc[nr][r] = 0.f;
        accl[nr][r] = 0.f;
      }
    for (int ks = 0; ks < KS; ks += SK_D) {
#pragma unroll
      for (int d = 0; d < SK_D; ++d) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[i] = ring[d][0][i];
          v[4 + i] = ring[d][1][i];
        }
        // range guard: the skip operand is the raw residual stream (not normalised)
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
            split_pair(v[2 * k], v[2 * k + 1], hw[k], lw[k]);
          }
        }
        const f16x8 ah = __builtin_bit_cast(f16x8, u32x4{hw[0], hw[1], hw[2], hw[3]});
        f16x8 al;
        if (NPROD == 3) al = __builtin_bit_cast(f16x8, u32x4{lw[0], lw[1], lw[2], lw[3]});
        issue(ring[d]);  // the step SK_D ahead into the registers just split
        const int kk = ks + d;
        f16x8 bs[NR], bl[NR];
#pragma unroll
        for (int nr = 0; nr < NR; ++nr) {
          bs[nr] = __builtin_bit_cast(f16x8, Wl[(kk * 4 + 0) * NTC + 32 * nr]);
          if (NPROD == 3) bl[nr] = __builtin_bit_cast(f16x8, Wl[(kk * 4 + 2) * NTC + 32 * nr]);
        }
#pragma unroll
        for (int nr = 0; nr < NR; ++nr) acc[nr] = mfma16(ah, bs[nr], acc[nr]);
        if (NPROD == 3) {
#pragma unroll
          for (int nr = 0; nr < NR; ++nr) accl[nr] = mfma16(ah, bl[nr], accl[nr]);
#pragma unroll
          for (int nr = 0; nr < NR; ++nr) accl[nr] = mfma16(al, bs[nr], accl[nr]);
        }
      }
    }
    // epilogue: register (nr, r) of lane (h, l32) = channel nt NTC + 32 nr + l32 of tile pixel
    // 8 (r >> 2) + 4 h + (r & 3). Per (nr, g) the quad's 4 lanes (channels 4a .. 4a + 3 of the 32-block) x
    // registers 4g .. 4g + 3 (pixels 8 g + 4 h + 0..3) are transposed by two DPP butterflies, so lane 4a + i holds
    // pixel 8 g + 4 h + i's four channels: one dwordx4 store per (nr, g) writes 8 pixels x 128 B. (Round 5: was
    // 64 dword stores per lane and tile; timing ablations put the stores at ~44 % of this memory-bound kernel,
    // and the wide stores take the 256^2 layer 0.675 -> 0.657 ms per eval, profiles/r05i.)
    const rsrc_t ro = mkrsrc(p.out + (size_t)t * 32 * p.cout);
    const int qi = l32 & 3;
    const int vb4 = ((4 * h + qi) * p.cout + nt * NTC + (l32 & ~3)) * 4;
#pragma unroll
    for (int nr = 0; nr < NR; ++nr) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = (acc[nr][4 * g + j] + accl[nr][4 * g + j]) * (1.0f / kScale) + bias[nr];
        // stage 1 (lane ^ 1, registers ^ 1), stage 2 (lane ^ 2, registers ^ 2): v[j] of lane i -> lane j's v[i]
#define SK_QP(x, ctrl) __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), ctrl, 0xf, 0xf, false))
        {
          const float t0 = SK_QP(v[0], 0xB1), t1 = SK_QP(v[1], 0xB1);  // quad_perm [1,0,3,2]
          const float t2 = SK_QP(v[2], 0xB1), t3 = SK_QP(v[3], 0xB1);
          const bool odd = qi & 1;
          v[0] = odd ? t1 : v[0];
          v[1] = odd ? v[1] : t0;
          v[2] = odd ? t3 : v[2];
          v[3] = odd ? v[3] : t2;
        }
        {
          const float t0 = SK_QP(v[0], 0x4E), t1 = SK_QP(v[1], 0x4E);  // quad_perm [2,3,0,1]
          const float t2 = SK_QP(v[2], 0x4E), t3 = SK_QP(v[3], 0x4E);
          const bool hi = qi & 2;
          v[0] = hi ? t2 : v[0];
          v[1] = hi ? t3 : v[1];
          v[2] = hi ? v[2] : t0;
          v[3] = hi ? v[3] : t1;
        }
#undef SK_QP
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, f32x4{v[0], v[1], v[2], v[3]}), ro,
                                               vb4 + nr * 128, 8 * g * p.cout * 4, 0);
      }
    }
  }
  if (p.guard && gmax >= 65504.0f) atomicOr(p.guard, 1u);
}

template <int NTC, int NPROD>
int launch_inst(const Skip1x1Params& p, hipStream_t stream) {
  static bool attr_set[kMaxDevices] = {};
  const int K = p.sc0 + p.sc1;
  const size_t lds = (size_t)K * NTC * 4;
  hipError_t e = set_lds_attr_once(attr_set, reinterpret_cast<const void*>(&skip_x3_kernel<NTC, NPROD>), SK_LDS_MAX);
  if (e != hipSuccess) return (int)e;
  const int nnt = p.cout / NTC;
  const int ncu = device_cu_count();
  const int waves_needed = (p.npix / 32 + (SK_NT / 64) - 1) / (SK_NT / 64);  // blocks per channel tile
  int per = ncu * (SK_WPE / 2) / nnt;
  if (per < 1) per = 1;
  if (per > waves_needed) per = waves_needed;
  hipLaunchKernelGGL((skip_x3_kernel<NTC, NPROD>), dim3(per * nnt), dim3(SK_NT), lds, stream, p);
  return IFD_LAUNCH_STATUS();
}

}  // namespace

int skip_x3_ntc(int K, int cout) {
  for (int ntc = 128; ntc >= 32; ntc >>= 1)
    if (cout % ntc == 0 && (size_t)K * ntc * 4 <= (size_t)SK_LDS_MAX) return ntc;
  return 0;
}

bool skip_x3_eligible(const Skip1x1Params& p) {
  const int K = p.sc0 + p.sc1;
  return p.s0 && p.sc0 % 16 == 0 && p.sc1 % 16 == 0 && (p.sc1 == 0 || p.s1) && K > 0 && (K / 16) % SK_D == 0 &&
         p.npix % 32 == 0 && p.ntc == skip_x3_ntc(K, p.cout) && p.ntc > 0 && p.cout % p.ntc == 0 &&
         (p.nprod == 1 || p.nprod == 3);
}

int launch_skip_x3(const Skip1x1Params& p, hipStream_t stream) {
  if (!skip_x3_eligible(p)) return (int)hipErrorInvalidValue;
  if (p.nprod == 1) {
    if (p.ntc == 128) return launch_inst<128, 1>(p, stream);
    if (p.ntc == 64) return launch_inst<64, 1>(p, stream);
    return launch_inst<32, 1>(p, stream);
  }
  if (p.ntc == 128) return launch_inst<128, 3>(p, stream);
  if (p.ntc == 64) return launch_inst<64, 3>(p, stream);
  return launch_inst<32, 3>(p, stream);
}

}  // namespace ifd
