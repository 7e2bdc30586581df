// Development microbenchmark: back-to-back dispatch cost of short kernels on one stream, plain
// launches vs the same sequence captured into a hipGraph; LDS-heavy 512-thread blocks as the
// conv kernels use, and small 256-thread blocks as the GroupNorm kernels.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
__global__ __launch_bounds__(256) void small_k(float* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * 1.0001f + 1.0f;
}
__global__ __launch_bounds__(512) void big_k(float* p, int n) {
  extern __shared__ float sm[];
  sm[threadIdx.x] = (float)threadIdx.x;
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] + sm[(threadIdx.x + 1) & 511];
}
int main() {
  float* d;
  const int n = 1 << 20;
  hipMalloc(&d, n * sizeof(float));
  hipMemset(d, 0, n * sizeof(float));
  hipFuncSetAttribute((const void*)big_k, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
  hipStream_t s;
  hipStreamCreate(&s);
  const int K = 400;
  auto seq = [&](int mode) {
    for (int k = 0; k < K; ++k) {
      if (mode == 0 || (mode == 2 && (k & 1))) hipLaunchKernelGGL(small_k, dim3(512), dim3(256), 0, s, d, n);
      else hipLaunchKernelGGL(big_k, dim3(256), dim3(512), 150 * 1024, s, d, n);
    }
  };
  for (int mode = 0; mode < 3; ++mode) {
    const char* nm = mode == 0 ? "small" : (mode == 1 ? "big(150KB LDS)" : "alternating");
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
      seq(mode); hipStreamSynchronize(s);
      hipEventRecord(e0, s);
      seq(mode);
      hipEventRecord(e1, s);
      hipStreamSynchronize(s);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      // graph
      hipGraph_t g; hipGraphExec_t ge;
      hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
      seq(mode);
      hipStreamEndCapture(s, &g);
      hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
      hipGraphLaunch(ge, s); hipStreamSynchronize(s);
      hipEventRecord(e0, s);
      hipGraphLaunch(ge, s);
      hipEventRecord(e1, s);
      hipStreamSynchronize(s);
      float msg; hipEventElapsedTime(&msg, e0, e1);
      printf("%-16s stream %.2f us/kernel   graph %.2f us/kernel\n", nm, 1000 * ms / K, 1000 * msg / K);
      hipGraphExecDestroy(ge); hipGraphDestroy(g);
    }
  }
  return 0;
}
