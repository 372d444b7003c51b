// Probe: lane mapping of ds_read_b64_tr_b8 on gfx950 (not documented in the guides here).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v2i __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) v2i lds_v2i;

__global__ void probe(unsigned* out, int mode) {
  __shared__ __attribute__((aligned(16))) unsigned char img[16 * 16];
  const int l = threadIdx.x;
  for (int k = l; k < 256; k += 64) img[k] = (unsigned char)k;  // byte (row, col) = row*16 + col
  __syncthreads();
  const int i = l & 15;
  int addr;
  if (mode == 0) addr = (i >> 1) * 16 + 8 * (i & 1);   // H1: lane 2q+p -> row q, cols 8p..8p+7
  else addr = i * 16;                                 // every lane its own row, col 0
  v2i v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)(img + addr));
  out[2 * l] = (unsigned)v.x;
  out[2 * l + 1] = (unsigned)v.y;
}

int main() {
  unsigned* d;
  hipMalloc(&d, 128 * 4);
  unsigned h[128];
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, mode);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("mode %d\n", mode);
    for (int l = 0; l < 20; ++l) {
      printf("lane %2d:", l);
      for (int b = 0; b < 8; ++b) {
        unsigned byte = (h[2 * l + b / 4] >> (8 * (b % 4))) & 255;
        printf(" r%02d.c%02d", byte >> 4, byte & 15);
      }
      printf("\n");
    }
  }
  return 0;
}
