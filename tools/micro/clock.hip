// Development microbenchmark: s_memtime vs s_memrealtime (100 MHz) over an f16 MFMA loop, one
// workgroup vs a full grid -> the shader clock under light and under full MFMA load.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
template <bool RND>
__global__ __launch_bounds__(256) void mfma_loop(int iters, unsigned long long* out, float* sink) {
  // RND: 4 distinct pseudo-random operand pairs per lane (high toggling, like real data)
  f16x8 a[4], b[4];
  unsigned sd = 2654435761u * (threadIdx.x + 1) + blockIdx.x;
  for (int q = 0; q < 4; ++q)
    for (int i = 0; i < 8; ++i) {
      sd = sd * 1664525u + 1013904223u;
      const float ra = (float)(sd >> 8) * (1.0f / 16777216.0f) - 0.5f;
      sd = sd * 1664525u + 1013904223u;
      const float rb = (float)(sd >> 8) * (1.0f / 16777216.0f) - 0.5f;
      a[q][i] = RND ? (_Float16)ra : (_Float16)(threadIdx.x * 0.001f + i);
      b[q][i] = RND ? (_Float16)rb : (_Float16)0.5f;
    }
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0], b[0], c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1], b[1], c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2], b[2], c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[3], b[3], c3, 0, 0, 0);
  }
  float s = 0;
  for (int i = 0; i < 16; ++i) s += c0[i] + c1[i] + c2[i] + c3[i];
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = t1 - t0;
    out[2 * blockIdx.x + 1] = r1 - r0;
  }
  if (s == 12345.f) sink[threadIdx.x] = s;
}
int main() {
  const int iters = 20000;
  unsigned long long* d; float* sink;
  hipMalloc(&d, 2 * 4096 * sizeof(unsigned long long));
  hipMalloc(&sink, 1024 * sizeof(float));
  for (int rnd = 0; rnd < 2; ++rnd)
  for (int grid : {1, 256, 1024}) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
      hipEventRecord(e0);
      if (rnd) mfma_loop<true><<<grid, 256>>>(iters, d, sink);
      else mfma_loop<false><<<grid, 256>>>(iters, d, sink);
      hipEventRecord(e1);
      hipDeviceSynchronize();
      float ms; hipEventElapsedTime(&ms, e0, e1);
      unsigned long long h[2];
      hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
      const double mf = 4.0 * iters;
      const double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;
      const double tflops = (double)grid * 4 * mf * 32 * 32 * 16 * 2 / (ms * 1e-3) / 1e12;
      printf("%s grid %5d: memtime/MFMA %.2f  realtime %.1f us  memtime-rate %.3f GHz  kernel %.3f ms  %.0f TF/s f16\n",
             rnd ? "random" : "const ", grid, h[0] / mf, h[1] / 100.0, ghz, ms, tflops);
    }
  }
  return 0;
}
