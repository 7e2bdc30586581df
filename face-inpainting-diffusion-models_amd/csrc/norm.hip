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
// Pass 1 (gn_partial): one block per (n, slice of pixels) reads its slice once from HBM and
// computes per group (count, mean, M2) with a two-pass (mean, then centred squares) reduction
// over the L1/L2-resident slice — deterministic (fixed reduction tree, no atomics).
// Pass 2 (gn_finalize): per (n, group), Chan's parallel combination in float64, then A/B.
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

__global__ __launch_bounds__(GN_NT) void gn_partial_kernel(GnPartialParams p) {
  __shared__ float red[GN_NT * 4];
  __shared__ float chs[1024];
  __shared__ float gmean[GN_G];
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

  // pass 1: per-channel sums over this thread's pixels
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (active)
    for (int px = px0 + pl; px < px1; px += PL) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(src + ((size_t)n * p.HW + px) * cs + co);
      acc += v;
    }
  if (active) *reinterpret_cast<f32x4*>(red + 4 * (pl * QPT + q)) = acc;
  __syncthreads();
  for (int ch = tid; ch < C; ch += GN_NT) {
    float t = 0.f;
    for (int l = 0; l < PL; ++l) t += red[l * C + ch];
    chs[ch] = t;
  }
  __syncthreads();
  const float cnt = (float)(px1 - px0) * Cg;
  if (tid < GN_G) {
    float t = 0.f;
    for (int j = 0; j < Cg; ++j) t += chs[tid * Cg + j];
    gmean[tid] = t / cnt;
  }
  __syncthreads();
  // pass 2: centred squares against the slice mean (re-read hits L1/L2)
  f32x4 m2 = {0.f, 0.f, 0.f, 0.f};
  if (active) {
    f32x4 mu;
    for (int j = 0; j < 4; ++j) mu[j] = gmean[(c + j) / Cg];
    for (int px = px0 + pl; px < px1; px += PL) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(src + ((size_t)n * p.HW + px) * cs + co) - mu;
      m2 += v * v;
    }
  }
  __syncthreads();
  if (active) *reinterpret_cast<f32x4*>(red + 4 * (pl * QPT + q)) = m2;
  __syncthreads();
  for (int ch = tid; ch < C; ch += GN_NT) {
    float t = 0.f;
    for (int l = 0; l < PL; ++l) t += red[l * C + ch];
    chs[ch] = t;
  }
  __syncthreads();
  if (tid < GN_G) {
    float t = 0.f;
    for (int j = 0; j < Cg; ++j) t += chs[tid * Cg + j];
    float* o = p.part + (((size_t)n * p.nslices + s) * GN_G + tid) * 3;
    o[0] = cnt;
    o[1] = gmean[tid];
    o[2] = t;
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

__global__ __launch_bounds__(GN_NT) void gn_finalize_kernel(GnFinalizeParams p) {
  __shared__ float smean[GN_G], srstd[GN_G];
  const int n = blockIdx.x, tid = threadIdx.x;
  if (tid < GN_G) {
    double cnt = 0.0, mean = 0.0, m2 = 0.0;
    for (int s = 0; s < p.nslices; ++s) {
      const float* o = p.part + (((size_t)n * p.nslices + s) * GN_G + tid) * 3;
      const double nb = o[0], mb = o[1], m2b = o[2];
      if (nb <= 0) continue;
      const double tot = cnt + nb;
      const double d = mb - mean;
      mean += d * (nb / tot);
      m2 += m2b + d * d * (cnt * nb / tot);
      cnt = tot;
    }
    const double var = m2 / cnt;
    smean[tid] = (float)mean;
    srstd[tid] = (float)(1.0 / sqrt(var + (double)p.eps));
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

int gn_slices(int HW, int* slice) {
  int s = HW < 256 ? HW : 256;
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
  return (int)hipGetLastError();
}

}  // namespace ifd
