// Development check of the cross-lane builtins the split kernel's epilogue uses (gfx950):
// v_permlane32_swap and DPP quad_perm. Prints, for lanes 0..7 and 32..39, what each returns for x = lane.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* out) {
  const int l = threadIdx.x;
  const auto r = __builtin_amdgcn_permlane32_swap((unsigned)l, (unsigned)l, false, false);
  out[l * 4 + 0] = (int)r[0];
  out[l * 4 + 1] = (int)r[1];
  out[l * 4 + 2] = __builtin_amdgcn_mov_dpp(l, 0xA0, 0xf, 0xf, false);
  out[l * 4 + 3] = __builtin_amdgcn_mov_dpp(l, 0xEE, 0xf, 0xf, false);
}
int main() {
  int* d; hipMalloc(&d, 64 * 4 * sizeof(int));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  int h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l : {0, 1, 2, 3, 4, 5, 31, 32, 33, 63})
    printf("lane %2d: swap[0]=%2d swap[1]=%2d dpp(A0)=%2d dpp(EE)=%2d\n", l, h[l * 4], h[l * 4 + 1], h[l * 4 + 2], h[l * 4 + 3]);
  return 0;
}
