#include <hip/hip_runtime.h>
#include <cstdint>
__global__ void addk(const float* a, float* b, int n){int i=blockIdx.x*blockDim.x+threadIdx.x; if(i<n) b[i]=a[i]*2.f+1.f;}
__global__ void mfmak(const float* a, const float* b, float* c){
  typedef float f16v __attribute__((ext_vector_type(16)));
  int l=threadIdx.x; f16v acc={0};
  acc=__builtin_amdgcn_mfma_f32_32x32x2f32(a[l], b[l], acc, 0,0,0);
  for(int r=0;r<16;r++) c[l*16+r]=acc[r];
}
extern "C" int run_add(const float* a, float* b, int n, void* stream){
  hipLaunchKernelGGL(addk, dim3((n+255)/256), dim3(256), 0, (hipStream_t)stream, a,b,n);
  return (int)hipGetLastError();
}
extern "C" int run_mfma(const float* a, const float* b, float* c, void* stream){
  hipLaunchKernelGGL(mfmak, dim3(1), dim3(64), 0, (hipStream_t)stream, a,b,c);
  return (int)hipGetLastError();
}
