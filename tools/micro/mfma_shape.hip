// Development microbenchmark: chip-wide f16 MFMA throughput (power-limited regime) of
// v_mfma_f32_32x32x16_f16 vs v_mfma_f32_16x16x32_f16 with random operands, operands either held in
// registers or re-read from LDS by ds_read_b128 before every MFMA group (the conv kernels' pattern).
//   hipcc --offload-arch=gfx950 -O3 tools/micro/mfma_shape.hip -o tools/micro/mfma_shape
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) f16x8 lds_h8;

__device__ __forceinline__ void fill(f16x8 (&a)[4], f16x8 (&b)[4]) {
  unsigned sd = 2654435761u * (threadIdx.x + 1) + blockIdx.x;
  for (int q = 0; q < 4; ++q)
    for (int i = 0; i < 8; ++i) {
      sd = sd * 1664525u + 1013904223u;
      a[q][i] = (_Float16)((float)(sd >> 8) * (1.0f / 16777216.0f) - 0.5f);
      sd = sd * 1664525u + 1013904223u;
      b[q][i] = (_Float16)((float)(sd >> 8) * (1.0f / 16777216.0f) - 0.5f);
    }
}

// SHAPE 0: 32x32x16 (4 accumulators: the conv kernels' 2 x 2 blocks); SHAPE 1: 16x16x32 (16 accumulators
// of f32x4: the same 64 x 64 output per wave). LDS: operands re-read from LDS every group.
template <int SHAPE, bool LDS>
__global__ __launch_bounds__(256) void loop(int iters, float* sink) {
  __shared__ __attribute__((aligned(16))) _Float16 sm[4 * 64 * 8 * 8];
  f16x8 a[4], b[4];
  fill(a, b);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  lds_h8* L = (lds_h8*)sm;
  for (int q = 0; q < 4; ++q) {
    L[(w * 8 + q) * 64 + lane] = a[q];
    L[(w * 8 + 4 + q) * 64 + lane] = b[q];
  }
  __syncthreads();
  float s = 0.f;
  if (SHAPE == 0) {
    f32x16 c[2][2] = {};
    for (int i = 0; i < iters; ++i) {
      if (LDS) {
        for (int q = 0; q < 2; ++q) {
          a[q] = L[(w * 8 + ((i + q) & 3)) * 64 + lane];
          b[q] = L[(w * 8 + 4 + ((i + q) & 3)) * 64 + lane];
        }
      }
      for (int r = 0; r < 3; ++r)  // 3 products per group, as a tap of the split kernel
        for (int m = 0; m < 2; ++m)
          for (int n = 0; n < 2; ++n) c[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[m ^ (r & 1)], b[n], c[m][n], 0, 0, 0);
    }
    for (int m = 0; m < 2; ++m)
      for (int n = 0; n < 2; ++n)
        for (int r = 0; r < 16; ++r) s += c[m][n][r];
  } else {
    f32x4 c[4][4] = {};
    for (int i = 0; i < iters; ++i) {
      if (LDS) {
        for (int q = 0; q < 4; ++q) {
          a[q] = L[(w * 8 + ((i + q) & 3)) * 64 + lane];
          b[q] = L[(w * 8 + 4 + ((i + q) & 3)) * 64 + lane];
        }
      }
      // 1.5 groups of 16 MFMAs x K32 = the FLOPs of 3 x 4 MFMAs 32x32x16 above (same work per iteration)
      for (int m = 0; m < 4; ++m)
        for (int n = 0; n < 4; ++n) c[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[m], b[n], c[m][n], 0, 0, 0);
      for (int m = 0; m < 2; ++m)
        for (int n = 0; n < 4; ++n) c[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[m + 2], b[n], c[m][n], 0, 0, 0);
    }
    for (int m = 0; m < 4; ++m)
      for (int n = 0; n < 4; ++n)
        for (int r = 0; r < 4; ++r) s += c[m][n][r];
  }
  if (s == 12345.f) sink[threadIdx.x] = s;
}

int main() {
  const int iters = 4000;
  float* sink;
  hipMalloc(&sink, 1024 * sizeof(float));
  const double flop_iter = 12.0 * 32 * 32 * 16 * 2;  // per wave per iteration, both shapes
  auto run = [&](const char* name, auto kern) {
    for (int grid : {256, 1024}) {
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {
        hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
        hipEventRecord(e0);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, iters, sink);
        hipEventRecord(e1);
        hipDeviceSynchronize();
        float ms; hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      printf("%-28s grid %5d: %.3f ms  %.0f TF/s f16\n", name, grid, best,
             (double)grid * 4 * iters * flop_iter / (best * 1e-3) / 1e12);
    }
  };
  run("32x32x16 regs", loop<0, false>);
  run("16x16x32 regs", loop<1, false>);
  run("32x32x16 lds", loop<0, true>);
  run("16x16x32 lds", loop<1, true>);
  return 0;
}
