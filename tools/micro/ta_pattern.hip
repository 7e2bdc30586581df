// Vector-memory cost by access shape (development micro-benchmark for conv_x3's operand loads).
// Every wave issues dwordx4 buffer loads, 8 in flight, over lines of 128 B spaced `stride` bytes
// apart (512 B = one pixel of a 128-channel fp32 NHWC tensor). G = lanes per line per instruction:
//   G = 2: 32 lines x 32 B per instruction (the halo / skip operand loads of conv_x3: two lanes
//          per pixel), 4 instructions cover the 32 lines' 128 B
//   G = 4: 16 lines x 64 B, 2 instructions per 16 lines
//   G = 8:  8 lines x 128 B, 1 instruction
// Every shape moves the same bytes (whole lines), so a difference in time is the per-request cost.
// Region: 2 MiB (L2-resident after the first pass) or 1 GiB (HBM). Prints ns per wave-instruction
// per CU and GB/s.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/micro/ta_pattern tools/micro/ta_pattern.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

template <int G>
__global__ void ld(const float* base, unsigned lines, unsigned stride, int iters, float* out) {
  const rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7ffffff0, 0x00020000);
  const int lane = threadIdx.x & 63;
  const unsigned wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  constexpr int LPI = 64 / G;  // lines per instruction
  constexpr int T = 8 / G;     // instructions per group of LPI lines
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  unsigned grp = wave * 977u;  // group cursor (groups of LPI lines)
  const unsigned ngrp = lines / LPI;
  for (int it = 0; it < iters; ++it) {
    f32x4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int t = k % T;
      const unsigned g = (grp + k / T) % ngrp;
      const unsigned line = g * LPI + lane / G;
      const unsigned off = line * stride + ((lane % G) + G * t) * 16;
      v[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += v[k];
    grp += 8 / T * 131u;
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] == 1234.5f) out[0] = acc[0];
}

template <int G>
static void run(const float* buf, size_t bytes, unsigned stride, int wpc, float* out, const char* tag, int blocks = 256) {
  const unsigned lines = (unsigned)(bytes / stride);
  const int iters = 2000;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  ld<G><<<blocks, 64 * wpc>>>(buf, lines, stride, iters, out);  // warm-up
  hipEventRecord(a);
  ld<G><<<blocks, 64 * wpc>>>(buf, lines, stride, iters, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  const double instr = (double)blocks * wpc * iters * 8;  // wave-instructions
  const double ns_per = ms * 1e6 / (instr / blocks);      // per CU (one block per CU)
  printf("%-4s G=%d stride=%4u waves/CU=%d CUs=%d: %.2f ms, %.1f ns per wave-instruction per CU, %.0f GB/s\n", tag, G,
         stride, wpc, blocks, ms, ns_per, instr * 1024 / (ms * 1e-3) / 1e9);
}

int main() {
  const size_t big = 1ull << 30, small = 2ull << 20;
  float *buf, *out;
  hipMalloc(&buf, big);
  hipMalloc(&out, 64);
  hipMemset(buf, 0, big);
  // per-CU limits: few CUs, so the chip's HBM bandwidth is not the bound
  for (int nb : {32, 64})
    for (int wpc : {4, 8}) {
      run<2>(buf, big, 512, wpc, out, "HBM", nb);
      run<4>(buf, big, 512, wpc, out, "HBM", nb);
      run<8>(buf, big, 512, wpc, out, "HBM", nb);
    }
  for (int wpc : {4, 8})
    for (unsigned stride : {512u}) {
      run<2>(buf, small, stride, wpc, out, "L2");
      run<4>(buf, small, stride, wpc, out, "L2");
      run<8>(buf, small, stride, wpc, out, "L2");
      run<2>(buf, big, stride, wpc, out, "HBM");
      run<4>(buf, big, stride, wpc, out, "HBM");
      run<8>(buf, big, stride, wpc, out, "HBM");
    }
  hipFree(buf);
  hipFree(out);
  return 0;
}
