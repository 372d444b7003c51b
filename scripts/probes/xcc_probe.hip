// Probe: HW_REG_XCC_ID (hwreg 20) per workgroup, to confirm round-robin XCD placement.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void probe(unsigned* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);
}
int main() {
  unsigned* d;
  (void)hipMalloc(&d, 256 * 4);
  unsigned h[256];
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(probe, dim3(64), dim3(512), 0, 0, d);
    (void)hipMemcpy(h, d, 64 * 4, hipMemcpyDeviceToHost);
    printf("rep %d:", rep);
    for (int b = 0; b < 64; ++b) printf(" %x", h[b]);
    printf("\n");
  }
  return 0;
}
