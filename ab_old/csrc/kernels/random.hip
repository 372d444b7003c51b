// Reached by: ops.philox_normal_ (sharded tables, compat random_normal init); tests/test_ops_gpu.py
// Counter-based normal initialisation: tf.random_normal for device-resident
// tables (reference: W = tf.Variable(tf.random_normal([F, 1])), lr2.py:384;
// example.py:84-85).
//
// Philox4x32-10 (the generator behind TF's random ops) keyed by the seed, with
// the element's *global* index as the counter: element e = grow * dim + col
// uses counter q = e / 4 and output word pair (e % 4) / 2 -> Box-Muller as in
// TF's BoxMullerFloat (u1 from the top 23 bits, clamped to 1e-7; v1 = 2 pi u2;
// n0 = sin(v1) r, n1 = cos(v1) r).  A row therefore gets the same values on
// whichever rank owns it (rows are dealt r -> rank r % W at local r / W), so a
// sharded table is bit-identical for any world size.  One thread per output
// element; ~60 integer/float ops per element keep a 1e9-row init HBM-bound.
#include "common.h"

namespace dtfk {
namespace rnd {

__device__ __forceinline__ void philox_round(uint32_t c[4], uint32_t k0, uint32_t k1) {
  const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
  const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
  const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
  const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
  const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
  c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
}

__device__ __forceinline__ void philox10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(c, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

__device__ __forceinline__ float u32_to_unit(uint32_t x) {   // [0, 1) from 23 mantissa bits
  return __uint_as_float((x & 0x7FFFFFu) | 0x3F800000u) - 1.0f;
}

__global__ __launch_bounds__(256) void philox_normal(float* __restrict__ out, long long n, int dim, long long row_mul,
                                                     long long row_add, uint32_t k0, uint32_t k1, float mean,
                                                     float stddev) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const long long lrow = i / dim, col = i - lrow * dim;
    const unsigned long long e = (unsigned long long)(lrow * row_mul + row_add) * dim + col;
    const unsigned long long q = e >> 2;
    uint32_t c[4] = {(uint32_t)q, (uint32_t)(q >> 32), 0u, 0u};
    philox10(c, k0, k1);
    const int w = (int)(e & 3);
    const uint32_t x0 = (w < 2) ? c[0] : c[2];
    const uint32_t x1 = (w < 2) ? c[1] : c[3];
    const float u1 = fmaxf(u32_to_unit(x0), 1.0e-7f);
    const float v1 = 6.2831853071795864769f * u32_to_unit(x1);
    const float r = sqrtf(-2.0f * logf(u1));
    float s, co;
    sincosf(v1, &s, &co);
    out[i] = mean + stddev * ((w & 1) ? co * r : s * r);
  }
}

}  // namespace rnd
}  // namespace dtfk

// out[lrow, col] = N(mean, std) of global element (lrow * row_mul + row_add) * dim + col
extern "C" hipError_t dtfk_philox_normal(float* out, long long rows, int dim, long long row_mul, long long row_add,
                                         unsigned long long seed, float mean, float stddev, hipStream_t stream) {
  const long long n = rows * (long long)dim;
  if (n <= 0) return hipSuccess;
  long long blocks = (n + 255) / 256;
  if (blocks > 256LL * 64) blocks = 256LL * 64;   // grid-stride beyond 64 waves/CU worth of blocks
  hipLaunchKernelGGL(dtfk::rnd::philox_normal, dim3((unsigned)blocks), dim3(256), 0, stream, out, n, dim, row_mul,
                     row_add, (uint32_t)seed, (uint32_t)(seed >> 32), mean, stddev);
  return hipGetLastError();
}
