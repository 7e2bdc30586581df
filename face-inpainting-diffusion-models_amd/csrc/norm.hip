// GroupNorm(32, C) statistics for NHWC activations, fused into per-(n, c) affine coefficients.
//
// code/nn.py:46-48 (normalization = GroupNorm(32, C), eps 1e-5, biased variance) and the
// scale-shift of code/nn.py:203-206 (`GN(h) * (1 + scale) + shift`) reduce, per image n and
// channel c, to   y = A[n,c] * x + B[n,c]   with
//   A = rstd * gamma[c] * (1 + scale[n,c]),
//   B = (beta[c] - mean * rstd * gamma[c]) * (1 + scale[n,c]) + shift[n,c].
// The conv prologue (conv.hip) applies A, B (+ SiLU) while staging its input halo, so the
// normalised tensor never goes to HBM.
//
// Pass 1 (gn_partial): one block per (n, slice of pixels) streams its slice ONCE from HBM
// (16-byte loads, coalesced along channels). Each thread keeps shifted sums per channel quad,
// S1 = sum(x - K), S2 = sum((x - K)^2) with K its first sample (no cancellation: |x - K| is on the
// scale of the group's spread), converts them to (count, mean, M2), and the block merges threads,
// then channels of a group, with Chan's pairwise formula in a fixed order (deterministic).
// Pass 2 (gn_finalize): one block per image; each group's slice partials are merged in float64
// by a 32-lane tree per group, then A/B are written.
#include "common.h"

namespace ifd {

constexpr int GN_NT = 256;
constexpr int GN_G = 32;

struct GnPartialParams {
  const float* p0; int c0;
  const float* p1; int c1;
  int HW;         // pixels per image
  int slice;      // pixels per block
  int nslices;
  float* part;    // [N][nslices][G][3]: count, mean, M2
};

struct Stat {
  float n, mean, m2;
};

__device__ __forceinline__ Stat merge(Stat a, Stat b) {
  const float n = a.n + b.n;
  if (n == 0.f) return a;
  const float d = b.mean - a.mean;
  const float f = b.n / n;
  return {n, a.mean + d * f, a.m2 + b.m2 + d * d * a.n * f};
}

__global__ __launch_bounds__(GN_NT) void gn_partial_kernel(GnPartialParams p) {
  __shared__ Stat red[GN_NT * 4];  // [pixel lane][channel]
  __shared__ Stat chs[1024];
  const int C = p.c0 + p.c1;
  const int QPT = C >> 2;                 // channel quads
  const int PL = GN_NT / QPT;             // pixel lanes (>= 1, C <= 1024)
  const int tid = threadIdx.x;
  const int q = tid % QPT, pl = tid / QPT;
  const int n = blockIdx.y, s = blockIdx.x;
  const int px0 = s * p.slice;
  const int px1 = min(px0 + p.slice, p.HW);
  const int c = 4 * q;
  const float* src;
  int cs, co;
  if (c < p.c0) { src = p.p0; cs = p.c0; co = c; }
  else { src = p.p1; cs = p.c1; co = c - p.c0; }
  const int Cg = C / GN_G;
  const bool active = pl < PL;

  f32x4 K = {0.f, 0.f, 0.f, 0.f}, s1 = K, s2 = K;
  float cnt = 0.f;
  if (active) {
    const float* base = src + (size_t)n * p.HW * cs + co;
    int px = px0 + pl;
    if (px < px1) K = *reinterpret_cast<const f32x4*>(base + (size_t)px * cs);
#pragma unroll 4
    for (; px < px1; px += PL) {
      const f32x4 d = *reinterpret_cast<const f32x4*>(base + (size_t)px * cs) - K;
      s1 += d;
      s2 += d * d;
      cnt += 1.f;
    }
    for (int j = 0; j < 4; ++j) {
      Stat st;
      st.n = cnt;
      st.mean = cnt > 0.f ? K[j] + s1[j] / cnt : 0.f;
      st.m2 = cnt > 0.f ? fmaxf(s2[j] - s1[j] * (s1[j] / cnt), 0.f) : 0.f;
      red[pl * C + c + j] = st;
    }
  }
  __syncthreads();
  for (int ch = tid; ch < C; ch += GN_NT) {
    Stat a = red[ch];
    for (int l = 1; l < PL; ++l) a = merge(a, red[l * C + ch]);
    chs[ch] = a;
  }
  __syncthreads();
  if (tid < GN_G) {
    Stat a = chs[tid * Cg];
    for (int j = 1; j < Cg; ++j) a = merge(a, chs[tid * Cg + j]);
    float* o = p.part + (((size_t)n * p.nslices + s) * GN_G + tid) * 3;
    o[0] = a.n;
    o[1] = a.mean;
    o[2] = a.m2;
  }
}

struct GnFinalizeParams {
  const float* part;
  int nslices, C;
  const float* gamma; const float* beta;
  const float* emb;   // optional [N][emb_stride] scale at emb_off, shift at emb_off + C
  int emb_stride, emb_off;
  float eps;
  float* A; float* B;  // [N][C]
};

// 256 threads = 8 groups x 32 lanes per pass; each lane merges a strided subset of the slices in
// float64, then a fixed 5-level butterfly merges the 32 lanes (deterministic).
__global__ __launch_bounds__(GN_NT) void gn_finalize_kernel(GnFinalizeParams p) {
  __shared__ float smean[GN_G], srstd[GN_G];
  const int n = blockIdx.x, tid = threadIdx.x;
  const int lane = tid & 31, gsub = tid >> 5;
  for (int g = gsub; g < GN_G; g += GN_NT / 32) {
    double cnt = 0.0, mean = 0.0, m2 = 0.0;
    for (int s = lane; s < p.nslices; s += 32) {
      const float* o = p.part + (((size_t)n * p.nslices + s) * GN_G + g) * 3;
      const double nb = o[0], mb = o[1], m2b = o[2];
      if (nb <= 0) continue;
      const double tot = cnt + nb, d = mb - mean;
      mean += d * (nb / tot);
      m2 += m2b + d * d * (cnt * nb / tot);
      cnt = tot;
    }
    for (int off = 16; off > 0; off >>= 1) {
      const double nb = __shfl_xor(cnt, off, 32), mb = __shfl_xor(mean, off, 32), m2b = __shfl_xor(m2, off, 32);
      const double tot = cnt + nb;
      if (tot > 0) {
        // symmetric form so both lanes of a pair compute the same value
        const double lo_n = (lane & off) ? nb : cnt, lo_m = (lane & off) ? mb : mean, lo_2 = (lane & off) ? m2b : m2;
        const double hi_n = (lane & off) ? cnt : nb, hi_m = (lane & off) ? mean : mb, hi_2 = (lane & off) ? m2 : m2b;
        const double d = hi_m - lo_m;
        mean = lo_m + d * (hi_n / tot);
        m2 = lo_2 + hi_2 + d * d * (lo_n * hi_n / tot);
        cnt = tot;
      }
    }
    if (lane == 0) {
      smean[g] = (float)mean;
      srstd[g] = (float)(1.0 / sqrt(m2 / cnt + (double)p.eps));
    }
  }
  __syncthreads();
  const int Cg = p.C / GN_G;
  for (int c = tid; c < p.C; c += GN_NT) {
    const int g = c / Cg;
    const float a = srstd[g] * p.gamma[c];
    const float b = p.beta[c] - smean[g] * a;
    float A = a, B = b;
    if (p.emb) {
      const float sc = 1.0f + p.emb[(size_t)n * p.emb_stride + p.emb_off + c];
      const float sh = p.emb[(size_t)n * p.emb_stride + p.emb_off + p.C + c];
      A = a * sc;
      B = b * sc + sh;
    }
    p.A[(size_t)n * p.C + c] = A;
    p.B[(size_t)n * p.C + c] = B;
  }
}

// Pixels per partial block: large enough to stream (>= 1024 pixels where possible), small enough
// that B x slices fills the chip.
int gn_slices(int HW, int* slice) {
  int s = HW < 1024 ? HW : 1024;
  *slice = s;
  return (HW + s - 1) / s;
}

int launch_gn(const float* p0, int c0, const float* p1, int c1, int N, int HW, const float* gamma, const float* beta,
              const float* emb, int emb_stride, int emb_off, float* part, float* A, float* B, hipStream_t stream) {
  GnPartialParams pp;
  pp.p0 = p0; pp.c0 = c0; pp.p1 = p1; pp.c1 = c1;
  pp.HW = HW;
  pp.nslices = gn_slices(HW, &pp.slice);
  pp.part = part;
  hipLaunchKernelGGL(gn_partial_kernel, dim3(pp.nslices, N), dim3(GN_NT), 0, stream, pp);
  GnFinalizeParams fp;
  fp.part = part; fp.nslices = pp.nslices; fp.C = c0 + c1;
  fp.gamma = gamma; fp.beta = beta;
  fp.emb = emb; fp.emb_stride = emb_stride; fp.emb_off = emb_off;
  fp.eps = 1e-5f;
  fp.A = A; fp.B = B;
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(N), dim3(GN_NT), 0, stream, fp);
  return IFD_LAUNCH_STATUS();
}

// ---------------------------------------------------------------------------------------------
// Granule statistics. Every activation tensor can carry per-(image, entry, channel quad)
// partial statistics P[n][c/4][e] = (mean, M2) over `cnt` values (an entry = a fixed set of
// pixels, the same for all granules). The convs that PRODUCE a tensor write them from their
// epilogue (conv.hip / conv_stream.hip, ConvParams::gstat), so the GroupNorm of the next layer
// needs no pass over the tensor; tensors without them get gn_granules_kernel (one streaming pass).
// gn_finalize2 combines the entries of each granule and the granules of each group — across the
// two concat sources when the GroupNorm input is cat(h, skip) — in float64, in a fixed order.

struct GnGranuleParams {
  const float* x; int C;
  int HW;         // pixels per image
  int slice;      // pixels per entry (block)
  int E;          // entries per image
  float* part;    // [N][C/4][E][2]
};

// one block per (entry, n): thread layout as gn_partial_kernel (channel quad x pixel lane),
// shifted sums per thread, Chan merges over pixel lanes in a fixed order
__global__ __launch_bounds__(GN_NT) void gn_granules_kernel(GnGranuleParams p) {
  __shared__ float red[GN_NT * 3 * 4];
  const int QPT = p.C >> 2;
  const int PL = GN_NT / QPT;
  const int tid = threadIdx.x;
  const int q = tid % QPT, pl = tid / QPT;
  const int n = blockIdx.y, s = blockIdx.x;
  const int px0 = s * p.slice, px1 = min(px0 + p.slice, p.HW);
  const bool active = pl < PL;
  f32x4 K = {0.f, 0.f, 0.f, 0.f}, s1 = K, s2 = K;
  float cnt = 0.f;
  if (active) {
    const float* base = p.x + (size_t)n * p.HW * p.C + 4 * q;
    int px = px0 + pl;
    if (px < px1) K = *reinterpret_cast<const f32x4*>(base + (size_t)px * p.C);
#pragma unroll 4
    for (; px < px1; px += PL) {
      const f32x4 d = *reinterpret_cast<const f32x4*>(base + (size_t)px * p.C) - K;
      s1 += d;
      s2 += d * d;
      cnt += 1.f;
    }
    // the quad's 4 channels as 4 stats, merged into one granule stat
    Stat g = {0.f, 0.f, 0.f};
    for (int j = 0; j < 4; ++j) {
      Stat st;
      st.n = cnt;
      st.mean = cnt > 0.f ? K[j] + s1[j] / cnt : 0.f;
      st.m2 = cnt > 0.f ? fmaxf(s2[j] - s1[j] * (s1[j] / cnt), 0.f) : 0.f;
      g = j == 0 ? st : merge(g, st);
    }
    red[(pl * QPT + q) * 3 + 0] = g.n;
    red[(pl * QPT + q) * 3 + 1] = g.mean;
    red[(pl * QPT + q) * 3 + 2] = g.m2;
  }
  __syncthreads();
  for (int qq = tid; qq < QPT; qq += GN_NT) {
    Stat a = {red[qq * 3], red[qq * 3 + 1], red[qq * 3 + 2]};
    for (int l = 1; l < PL; ++l) {
      const int o = (l * QPT + qq) * 3;
      a = merge(a, Stat{red[o], red[o + 1], red[o + 2]});
    }
    float* o = p.part + (((size_t)n * QPT + qq) * p.E + s) * 2;
    o[0] = a.mean;
    o[1] = a.m2;
  }
}

struct GnSrc {
  const float* part;  // [N][C/4][E][2]
  int E, C;
  float cnt;          // values per (entry, granule)
};

struct GnFinalize2Params {
  GnSrc s0, s1;       // s1.C == 0: single source
  const float* gamma; const float* beta;
  const float* emb;   // optional [N][emb_stride] scale at emb_off, shift at emb_off + C
  int emb_stride, emb_off;
  float eps;
  float* A; float* B;  // [N][C]
};

// Block-wide fp64 sum in a fixed order (wave xor-tree, then the 4 wave sums in order): deterministic.
__device__ __forceinline__ double block_sum64(double v, double* sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  __syncthreads();  // sh reuse across calls
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  double s = sh[0];
  for (int i = 1; i < GN_NT / 64; ++i) s += sh[i];
  return s;
}

// one block per (group g, image n). Every entry of a source holds `cnt` values (mean, M2). One fp64
// pass over the group's entries (all granules, both concat sources) collects n = sum(cnt),
// S1 = sum(cnt * mean_e) and S2 = sum(M2_e + cnt * mean_e^2); then mean = S1 / n and
// M2 = S2 - n * mean^2 (fp64 keeps the cancellation far below fp32 resolution for GroupNorm inputs).
// One block reduction of the three sums (was: two passes and three reductions).
__device__ __forceinline__ void block_sum64x3(double& a, double& b, double& c, double* sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o);
    b += __shfl_xor(b, o);
    c += __shfl_xor(c, o);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[3 * w] = a;
    sh[3 * w + 1] = b;
    sh[3 * w + 2] = c;
  }
  __syncthreads();
  a = sh[0];
  b = sh[1];
  c = sh[2];
  for (int i = 1; i < GN_NT / 64; ++i) {
    a += sh[3 * i];
    b += sh[3 * i + 1];
    c += sh[3 * i + 2];
  }
}

__global__ __launch_bounds__(GN_NT) void gn_finalize2_kernel(GnFinalize2Params p) {
  __shared__ double sh[3 * (GN_NT / 64)];
  const int g = blockIdx.x, n = blockIdx.y, tid = threadIdx.x;
  const int C = p.s0.C + p.s1.C;
  const int Cg = C / GN_G;
  const int ng = Cg / 4;  // granules of the group
  // the per-channel parameters are loaded before the reduction so their latency overlaps it
  // (Cg <= GN_NT: one channel per thread)
  const int cc = g * Cg + tid;
  const bool has_c = tid < Cg;
  float gam = 0.f, bet = 0.f, esc = 0.f, esh = 0.f;
  if (has_c) {
    gam = p.gamma[cc];
    bet = p.beta[cc];
    if (p.emb) {
      esc = p.emb[(size_t)n * p.emb_stride + p.emb_off + cc];
      esh = p.emb[(size_t)n * p.emb_stride + p.emb_off + C + cc];
    }
  }
  double sn = 0.0, sm = 0.0, sq = 0.0;
  for (int k = 0; k < ng; ++k) {
    const int c = g * Cg + 4 * k;
    const bool first = c < p.s0.C;
    const GnSrc& S = first ? p.s0 : p.s1;
    const int gr = (first ? c : c - p.s0.C) >> 2;
    const int QP = S.C >> 2;
    const float* base = S.part + ((size_t)n * QP + gr) * S.E * 2;  // the granule's entries, contiguous
    const double cnt = (double)S.cnt;
    for (int e = tid; e < S.E; e += GN_NT) {
      const float2 o = *reinterpret_cast<const float2*>(base + (size_t)e * 2);
      const double m = (double)o.x;
      sn += cnt;
      sm += cnt * m;
      sq += (double)o.y + cnt * m * m;
    }
  }
  block_sum64x3(sn, sm, sq, sh);
  const double ntot = sn;
  const double mean = sm / ntot;
  // one-pass M2 in fp64 can cancel below zero for a group whose mean dwarfs its spread: clamp (as the
  // training merge gn_granule_final_kernel does) so rstd stays finite
  const double m2 = fmax(sq - ntot * mean * mean, 0.0);
  const float meanf = (float)mean;
  const float rstd = (float)(1.0 / sqrt(m2 / ntot + (double)p.eps));
  if (has_c) {
    const float a = rstd * gam;
    const float b = bet - meanf * a;
    float A = a, B = b;
    if (p.emb) {
      const float sc = 1.0f + esc;
      A = a * sc;
      B = b * sc + esh;
    }
    p.A[(size_t)n * C + cc] = A;
    p.B[(size_t)n * C + cc] = B;
  }
}

int launch_gn_granules(const float* x, int C, int N, int HW, float* part, int* E, float* cnt, hipStream_t stream) {
  GnGranuleParams gp;
  gp.x = x; gp.C = C; gp.HW = HW;
  gp.E = gn_slices(HW, &gp.slice);
  gp.part = part;
  IFD_REQUIRE(HW % gp.slice == 0, "granule entries must be equal-sized");
  hipLaunchKernelGGL(gn_granules_kernel, dim3(gp.E, N), dim3(GN_NT), 0, stream, gp);
  *E = gp.E;
  *cnt = 4.0f * gp.slice;
  return IFD_LAUNCH_STATUS();
}

int launch_gn_finalize2(const float* part0, int E0, float cnt0, int C0, const float* part1, int E1, float cnt1,
                        int C1, int N, const float* gamma, const float* beta, const float* emb, int emb_stride,
                        int emb_off, float* A, float* B, hipStream_t stream) {
  GnFinalize2Params fp;
  fp.s0 = GnSrc{part0, E0, C0, cnt0};
  fp.s1 = GnSrc{part1, E1, C1, cnt1};
  fp.gamma = gamma; fp.beta = beta;
  fp.emb = emb; fp.emb_stride = emb_stride; fp.emb_off = emb_off;
  fp.eps = 1e-5f;
  fp.A = A; fp.B = B;
  IFD_REQUIRE((C0 + C1) % GN_G == 0 && (C0 + C1) / GN_G <= GN_NT, "GroupNorm group width");
  hipLaunchKernelGGL(gn_finalize2_kernel, dim3(GN_G, N), dim3(GN_NT), 0, stream, fp);
  return IFD_LAUNCH_STATUS();
}

}  // namespace ifd
