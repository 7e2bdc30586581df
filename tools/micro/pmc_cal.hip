// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the conv
// kernels use (MI355X_MICROARCH.md §HBM: only 16-B streaming reads/writes are calibrated there).
// Each kernel moves a known byte count over a 512 MiB buffer (> the 256 MiB Infinity Cache):
//   w_dword      4 B per lane, a wave = 256 contiguous bytes
//   w_dwordx4    16 B per lane
//   w_epi        the conv epilogues' pattern: 4 B per lane, lanes 0-31 and 32-63 on two rows
//                (two 128-B segments per wave-instruction)
//   r_dword      4 B per lane loads (the residual prefetch), summed into a tiny output
//   r_dwordx4    16 B per lane loads
// Printed: kernel name and true bytes; compare with the counter value (KiB) per dispatch.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr size_t kBytes = 512ull << 20;
constexpr size_t kN = kBytes / 4;

__global__ void w_dword(float* p) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (size_t k = i; k < kN; k += (size_t)gridDim.x * blockDim.x) p[k] = (float)k;
}
__global__ void w_dwordx4(float4* p) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (size_t k = i; k < kN / 4; k += (size_t)gridDim.x * blockDim.x) p[k] = make_float4(k, k, k, k);
}
// rows of 256 floats; wave w of the grid writes, per step, row pair (2r, 2r+1) columns [32 s, 32 s + 32)
__global__ void w_epi(float* p) {
  const int lane = threadIdx.x & 63;
  const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const size_t nwave = ((size_t)gridDim.x * blockDim.x) >> 6;
  const size_t segs = kN / 64;  // one wave-instruction = 64 floats in two 32-float row pieces
  for (size_t s = wave; s < segs; s += nwave) {
    const size_t rowpair = s / 8, col = (s % 8) * 32;
    p[(2 * rowpair + (lane >> 5)) * 256 + col + (lane & 31)] = (float)s;
  }
}
__global__ void r_dword(const float* p, float* out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  float acc = 0.f;
  for (size_t k = i; k < kN; k += (size_t)gridDim.x * blockDim.x) acc += p[k];
  if (acc == 12345.f) out[0] = acc;
}
__global__ void r_dwordx4(const float4* p, float* out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  float acc = 0.f;
  for (size_t k = i; k < kN / 4; k += (size_t)gridDim.x * blockDim.x) {
    const float4 v = p[k];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.f) out[0] = acc;
}

int main() {
  float *a, *o;
  if (hipMalloc(&a, kBytes) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) return 1;
  hipMemset(a, 0, kBytes);
  const dim3 g(4096), b(256);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(w_dword, g, b, 0, 0, a);
    hipLaunchKernelGGL(w_dwordx4, g, b, 0, 0, (float4*)a);
    hipLaunchKernelGGL(w_epi, g, b, 0, 0, a);
    hipLaunchKernelGGL(r_dword, g, b, 0, 0, a, o);
    hipLaunchKernelGGL(r_dwordx4, g, b, 0, 0, (const float4*)a, o);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("{\"true_bytes_per_dispatch\": %zu, \"true_kib\": %zu}\n", kBytes, kBytes >> 10);
  return 0;
}
