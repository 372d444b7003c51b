#include <hip/hip_runtime.h>
__device__ float x16(float v) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(((threadIdx.x >> 4) & 1) ? p[0] : p[1]);
}
__device__ float x32(float v) {
  auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float((threadIdx.x & 32) ? p[0] : p[1]);
}
__global__ void k(float* o) { float v = o[threadIdx.x]; o[64 + threadIdx.x] = x16(v); o[128 + threadIdx.x] = x32(v); }
int main() {
  float h[192]; for (int i = 0; i < 64; ++i) h[i] = i; float* d; (void)hipMalloc(&d, sizeof(h));
  (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice); hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0; for (int i = 0; i < 64; ++i) { bad += h[64 + i] != (float)(i ^ 16); bad += h[128 + i] != (float)(i ^ 32); }
  printf("permlane xor16/xor32 mismatches: %d  (x16[0..3]=%g %g %g %g x32[0]=%g)\n", bad, h[64], h[65], h[80], h[81], h[128]);
  return 0;
}
