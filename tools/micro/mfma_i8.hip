// Development microbenchmark: chip-wide sustained rate of v_mfma_i32_32x32x32_i8 vs v_mfma_f32_32x32x16_f16
// with random operands held in registers (the power-limited regime of the split conv kernels). Question it
// answers: would exact 8-bit limb arithmetic (6 i8 limb products per fp32-accurate MAC, against 3 f16
// products for 3xf16) run faster under the MI355X power cap? Only if one i8 MAC costs less than half the
// time of one f16 MAC at the cap.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/mfma_i8.hip -o tools/micro/mfma_i8 && tools/micro/mfma_i8
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned lcg(unsigned& s) {
  s = s * 1664525u + 1013904223u;
  return s;
}

// 4 accumulators (2 x 2 blocks, as the conv kernels), 4 operand registers per side rotating
template <bool I8>
__global__ __launch_bounds__(256) void loop(int iters, float* sink) {
  unsigned sd = 2654435761u * (threadIdx.x + 1) + 7919u * blockIdx.x;
  float s = 0.f;
  if (I8) {
    i32x4 a[4], b[4];
    for (int q = 0; q < 4; ++q)
      for (int i = 0; i < 4; ++i) {
        a[q][i] = (int)lcg(sd);
        b[q][i] = (int)lcg(sd);
      }
    i32x16 c[2][2] = {};
    for (int it0 = 0; it0 < iters; it0 += 4)
#pragma unroll
      for (int it = 0; it < 4; ++it)  // (static operand indices: a runtime index would go through scratch)
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
          for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int n = 0; n < 2; ++n)
              c[m][n] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[(m + r + it) & 3], b[(n + 2 * r + it) & 3], c[m][n], 0, 0, 0);
    for (int m = 0; m < 2; ++m)
      for (int n = 0; n < 2; ++n)
        for (int i = 0; i < 16; ++i) s += (float)c[m][n][i];
  } else {
    f16x8 a[4], b[4];
    for (int q = 0; q < 4; ++q)
      for (int i = 0; i < 8; ++i) {
        a[q][i] = (_Float16)((float)(lcg(sd) >> 8) * (1.0f / 16777216.0f) - 0.5f);
        b[q][i] = (_Float16)((float)(lcg(sd) >> 8) * (1.0f / 16777216.0f) - 0.5f);
      }
    f32x16 c[2][2] = {};
    for (int it0 = 0; it0 < iters; it0 += 4)
#pragma unroll
      for (int it = 0; it < 4; ++it)
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
          for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int n = 0; n < 2; ++n)
              c[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[(m + r + it) & 3], b[(n + 2 * r + it) & 3], c[m][n], 0, 0, 0);
    for (int m = 0; m < 2; ++m)
      for (int n = 0; n < 2; ++n)
        for (int i = 0; i < 16; ++i) s += c[m][n][i];
  }
  if (s == 1234.5f) sink[blockIdx.x] = s;  // keep the work
}

int main() {
  int dev = 0, ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  float* sink;
  (void)hipMalloc(&sink, 4096 * sizeof(float));
  const int blocks = ncu * 2, iters = 20000;  // 8 waves per CU (2 per SIMD)
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    for (int i8 = 0; i8 < 2; ++i8) {
      // warm-up then timed
      if (i8) hipLaunchKernelGGL(loop<true>, dim3(blocks), dim3(256), 0, 0, iters / 10, sink);
      else hipLaunchKernelGGL(loop<false>, dim3(blocks), dim3(256), 0, 0, iters / 10, sink);
      hipEventRecord(e0);
      if (i8) hipLaunchKernelGGL(loop<true>, dim3(blocks), dim3(256), 0, 0, iters, sink);
      else hipLaunchKernelGGL(loop<false>, dim3(blocks), dim3(256), 0, 0, iters, sink);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      const double macs_per_mfma = i8 ? 32.0 * 32 * 32 : 32.0 * 32 * 16;
      const double ops = 2.0 * macs_per_mfma * 12 * iters * (double)blocks * 4;  // 4 waves per block
      printf("%s  %.2f ms  %.1f T%s/s\n", i8 ? "i8  32x32x32" : "f16 32x32x16", ms, ops / (ms * 1e-3) / 1e12,
             i8 ? "OP" : "FLOP");
    }
  }
  return 0;
}
