// Rounding of v_mfma_f32_32x32x16_f16's fp32 accumulation (development probe for the C1 parity study):
// one wave, A = 32x16, B = 16x32 chosen so that output (0, 0) receives chosen products on top of C.
// Cases print C_out(0,0) as hex next to the round-to-nearest-even result of the exact sum.
//   hipcc --offload-arch=gfx950 -O2 tools/micro/mfma_round.hip -o tools/micro/mfma_round
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// a[k], b[k] (16 products for output (0,0)), c = C(0,0); every other entry 0
__global__ void probe(const _Float16* a, const _Float16* b, float c, float* out) {
  const int lane = threadIdx.x;
  f16x8 av, bv;
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * (lane >> 5) + j;
    av[j] = (lane & 31) == 0 ? a[k] : (_Float16)0.f;  // A[row = lane%32][k]
    bv[j] = (lane & 31) == 0 ? b[k] : (_Float16)0.f;  // B[k][col = lane%32]
  }
  f32x16 acc;
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  if (lane == 0) acc[0] = c;  // C[0][0]: lane 0, register 0
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bv, acc, 0, 0, 0);
  if (lane == 0) out[0] = acc[0];
}

// v_mfma_f32_32x32x2_f32: output (0,0) = C + a0 b0 + a1 b1 (K = 2; lane 0 holds k = 0, lane 32 k = 1)
__global__ void probe32(float a0, float b0, float a1, float b1, float c, float* out) {
  const int lane = threadIdx.x;
  const float av = (lane & 31) == 0 ? (lane < 32 ? a0 : a1) : 0.f;
  const float bv = (lane & 31) == 0 ? (lane < 32 ? b0 : b1) : 0.f;
  f32x16 acc;
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  if (lane == 0) acc[0] = c;
  acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
  if (lane == 0) out[0] = acc[0];
}
static void f32_probe();
static unsigned bits(float f) { unsigned u; memcpy(&u, &f, 4); return u; }

static void run(const char* name, float c, const double* pa, const double* pb, int n) {
  _Float16 ha[16] = {}, hb[16] = {};
  double exact = c;
  for (int i = 0; i < n; ++i) {
    ha[i] = (_Float16)pa[i];
    hb[i] = (_Float16)pb[i];
    exact += (double)(float)ha[i] * (double)(float)hb[i];
  }
  _Float16 *da, *db; float* dout;
  hipMalloc(&da, 32); hipMalloc(&db, 32); hipMalloc(&dout, 4);
  hipMemcpy(da, ha, 32, hipMemcpyHostToDevice);
  hipMemcpy(db, hb, 32, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, da, db, c, dout);
  float r = 0.f;
  hipMemcpy(&r, dout, 4, hipMemcpyDeviceToHost);
  const float rne = (float)exact;
  printf("%-44s mfma %.9g (%08x)  rne(exact) %.9g (%08x)  %s\n", name, r, bits(r), rne, bits(rne),
         r == rne ? "same" : (std::fabs((double)r - exact) < std::fabs((double)rne - exact) ? "closer" : "DIFFERS"));
  hipFree(da); hipFree(db); hipFree(dout);
}

int main() {
  const double e = std::ldexp(1.0, -12);
  {  // 1 + 0.625 ulp: RNE rounds up, truncation keeps 1
    double a[1] = {e}, b[1] = {1.25 * e};
    run("1 + 0.625 ulp", 1.0f, a, b, 1);
  }
  {  // 1 + 0.5 ulp exactly: RNE ties to even (1.0)
    double a[1] = {e}, b[1] = {e};
    run("1 + 0.5 ulp (tie)", 1.0f, a, b, 1);
  }
  {  // 1 + 0.75 ulp
    double a[1] = {e}, b[1] = {1.5 * e};
    run("1 + 0.75 ulp", 1.0f, a, b, 1);
  }
  {  // 1 - 0.625 ulp(below 1 = 2^-24)
    double a[1] = {e}, b[1] = {-0.625 * e};
    run("1 - 0.625 ulp_below", 1.0f, a, b, 1);
  }
  {  // two 0.375 ulp products: exact sum 0.75 ulp rounds up; per-product rounding keeps 1
    double a[2] = {e, e}, b[2] = {0.75 * e, 0.75 * e};
    run("1 + 2 x 0.375 ulp", 1.0f, a, b, 2);
  }
  {  // sixteen 0.0625 ulp products: exact sum 1 ulp
    double a[16], b[16];
    for (int i = 0; i < 16; ++i) { a[i] = e; b[i] = 0.125 * e; }
    run("1 + 16 x 0.0625 ulp", 1.0f, a, b, 16);
  }
  {  // sixteen -0.0625 ulp products on 1 (truncation toward zero keeps 1.0; toward -inf lowers it)
    double a[16], b[16];
    for (int i = 0; i < 16; ++i) { a[i] = e; b[i] = -0.125 * e; }
    run("1 - 16 x 0.0625 ulp", 1.0f, a, b, 16);
  }
  {  // sixteen 0.0625 ulp products on -1
    double a[16], b[16];
    for (int i = 0; i < 16; ++i) { a[i] = e; b[i] = -0.125 * e; }
    run("-1 - 16 x 0.0625 ulp", -1.0f, a, b, 16);
  }
  {  // eight 0.1875 ulp products on 1: 3 bits below the ulp
    double a[8], b[8];
    for (int i = 0; i < 8; ++i) { a[i] = e; b[i] = 0.375 * e; }
    run("1 + 8 x 0.1875 ulp", 1.0f, a, b, 8);
  }
  {  // the products alone (C = 0): 1.0 and sixteen 2^-27 products
    double a[16], b[16];
    a[0] = 1.0; b[0] = 1.0;
    for (int i = 1; i < 16; ++i) { a[i] = e; b[i] = 0.125 * e; }
    run("0 + 1 + 15 x 2^-27", 0.0f, a, b, 16);
  }
  {  // -1 - 0.625 ulp (sign symmetry of the rounding)
    double a[1] = {e}, b[1] = {-1.25 * e};
    run("-1 - 0.625 ulp", -1.0f, a, b, 1);
  }
  {  // cancellation: 1 + big - big + small
    double a[3] = {1.0, 1.0, e}, b[3] = {1024.0, -1024.0, 1.25 * e};
    run("1 + 1024 - 1024 + 0.625 ulp", 1.0f, a, b, 3);
  }
  f32_probe();
  return 0;
}

static void f32_probe() {
  float* d;
  hipMalloc(&d, 4);
  const double u = std::ldexp(1.0, -23);
  struct Case { const char* n; double a0, b0, a1, b1, c; } cs[] = {
      {"f32: 1 + 0.625 ulp", 1.0, 0.625 * u, 0, 0, 1.0},
      {"f32: 1 + 0.3 ulp + 0.3 ulp", 1.0, 0.3 * u, 1.0, 0.3 * u, 1.0},
      {"f32: 1 + (1 + 2^-23)(1 + 2^-23) - 1", 1.0 + u, 1.0 + u, -1.0, 1.0, 1.0},
      {"f32: 0 + (1 + 2^-23)^2 (product rounding)", 1.0 + u, 1.0 + u, 0, 0, 0.0},
      {"f32: 1 + 2^-26 + 2^-26 (two small)", 1.0, 0.125 * u, 1.0, 0.125 * u, 1.0},
      {"f32: 1 - 2^-26 - 2^-26", 1.0, -0.125 * u, 1.0, -0.125 * u, 1.0},
  };
  for (auto& c : cs) {
    hipLaunchKernelGGL(probe32, dim3(1), dim3(64), 0, 0, (float)c.a0, (float)c.b0, (float)c.a1, (float)c.b1, (float)c.c, d);
    float r = 0.f;
    hipMemcpy(&r, d, 4, hipMemcpyDeviceToHost);
    const double exact = (double)(float)c.c + (double)(float)c.a0 * (double)(float)c.b0 + (double)(float)c.a1 * (double)(float)c.b1;
    const float rne = (float)exact;
    printf("%-44s mfma %.9g (%08x)  rne(exact) %.9g (%08x)  %s\n", c.n, r, bits(r), rne, bits(rne), r == rne ? "same" : "DIFFERS");
  }
  hipFree(d);
}
