// Reached by: ops/pool.py (ResNet-50 stem max pool); tests/test_vision_ops_gpu.py
// Max pooling on NHWC bf16 activations (ResNet-50's 3x3 / stride-2 stem pool).
//
// torch's NHWC max-pool ran 125 us forward + 308 us backward per ResNet-50 step
// at B = 128 (int64 argmax indices, scatter-style backward).  Here one thread
// owns 8 channels of one output (forward) or one input (backward) position:
//   forward   9 x 16-byte loads, max + first-argmax per channel, a 16-byte
//             store of y and an 8-byte store of the window position (uint8);
//   backward  a gather, no atomics: an input pixel sums dy over the <= 4
//             windows that cover it whose argmax is this pixel (fp32 sum,
//             one bf16 rounding), 16-byte store of dx.
// NaN propagates like torch (a NaN wins the window); ties keep the first
// maximum in (kh, kw) scan order, as torch does.
#include "common.h"

namespace dtfk {
namespace pool {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float lo16(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi16(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

__global__ __launch_bounds__(256) void maxpool_fwd(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                   uint8_t* __restrict__ idx, int N, int H, int W, int C, int Ho,
                                                   int Wo, int k, int s, int p) {
  const int C8 = C >> 3;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)N * Ho * Wo * C8) return;
  const int c8 = (int)(i % C8);
  long long r = i / C8;
  const int wo = (int)(r % Wo);
  r /= Wo;
  const int ho = (int)(r % Ho);
  const int n = (int)(r / Ho);
  float m[8];
  int am[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { m[j] = -INFINITY; am[j] = 0; }
  bool any = false;
  for (int kh = 0; kh < k; ++kh) {
    const int h = ho * s - p + kh;
    if (h < 0 || h >= H) continue;
    for (int kw = 0; kw < k; ++kw) {
      const int w = wo * s - p + kw;
      if (w < 0 || w >= W) continue;
      const u32x4 v = *reinterpret_cast<const u32x4*>(x + (((size_t)n * H + h) * W + w) * C + 8 * c8);
      const int pos = kh * k + kw;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float f = (j & 1) ? hi16(v[j >> 1]) : lo16(v[j >> 1]);
        if (!any || f > m[j] || (f != f && m[j] == m[j])) { m[j] = f; am[j] = pos; }
      }
      any = true;
    }
  }
  u32x4 o;
  u32x2 ix;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    // the max of bf16 values is one of them: exact in bf16 (truncation is lossless)
    o[q] = (__float_as_uint(m[2 * q]) >> 16) | (__float_as_uint(m[2 * q + 1]) & 0xffff0000u);
  }
  ix[0] = (uint32_t)am[0] | ((uint32_t)am[1] << 8) | ((uint32_t)am[2] << 16) | ((uint32_t)am[3] << 24);
  ix[1] = (uint32_t)am[4] | ((uint32_t)am[5] << 8) | ((uint32_t)am[6] << 16) | ((uint32_t)am[7] << 24);
  const size_t oo = (((size_t)n * Ho + ho) * Wo + wo) * C + 8 * c8;
  *reinterpret_cast<u32x4*>(y + oo) = o;
  *reinterpret_cast<u32x2*>(idx + oo) = ix;
}

__global__ __launch_bounds__(256) void maxpool_bwd(const uint16_t* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                   uint16_t* __restrict__ dx, int N, int H, int W, int C, int Ho,
                                                   int Wo, int k, int s, int p) {
  const int C8 = C >> 3;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)N * H * W * C8) return;
  const int c8 = (int)(i % C8);
  long long r = i / C8;
  const int w = (int)(r % W);
  r /= W;
  const int h = (int)(r % H);
  const int n = (int)(r / H);
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  // windows covering (h, w): ho*s - p <= h <= ho*s - p + k - 1
  const int ho0 = max(0, (h + p - k + s) / s), ho1 = min(Ho - 1, (h + p) / s);
  const int wo0 = max(0, (w + p - k + s) / s), wo1 = min(Wo - 1, (w + p) / s);
  for (int ho = ho0; ho <= ho1; ++ho) {
    const int kh = h + p - ho * s;
    if (kh < 0 || kh >= k) continue;
    for (int wo = wo0; wo <= wo1; ++wo) {
      const int kw = w + p - wo * s;
      if (kw < 0 || kw >= k) continue;
      const size_t oo = (((size_t)n * Ho + ho) * Wo + wo) * C + 8 * c8;
      const u32x2 ix = *reinterpret_cast<const u32x2*>(idx + oo);
      const u32x4 g = *reinterpret_cast<const u32x4*>(dy + oo);
      const uint32_t pos = (uint32_t)(kh * k + kw);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t a = (ix[j >> 2] >> (8 * (j & 3))) & 255u;
        const float f = (j & 1) ? hi16(g[j >> 1]) : lo16(g[j >> 1]);
        if (a == pos) acc[j] += f;
      }
    }
  }
  u32x4 o;
#pragma unroll
  for (int q = 0; q < 4; ++q) o[q] = (uint32_t)f2bf(acc[2 * q]) | ((uint32_t)f2bf(acc[2 * q + 1]) << 16);
  *reinterpret_cast<u32x4*>(dx + (((size_t)n * H + h) * W + w) * C + 8 * c8) = o;
}

// The 3x3 / stride-2 window (ResNet's stem pool) with 32-bit index math and
// every load of a thread issued before the first is used: the generic loops
// above branch around each load (the compiler then waits for each in turn)
// and divide in 64 bits -- 108 / 114 us per ResNet-50 step at ~2.5 TB/s.
// Same results: the scan order, NaN and first-maximum rules, and the backward's
// fp32 summation order are the generic kernels'.
__global__ __launch_bounds__(256) void maxpool3s2_fwd(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                      uint8_t* __restrict__ idx, int N, int H, int W, int C, int Ho,
                                                      int Wo, int p) {
  const unsigned C8 = (unsigned)C >> 3;
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (unsigned)N * Ho * Wo * C8) return;
  const unsigned c8 = i % C8;
  unsigned r = i / C8;
  const int wo = (int)(r % (unsigned)Wo);
  r /= (unsigned)Wo;
  const int ho = (int)(r % (unsigned)Ho);
  const int n = (int)(r / (unsigned)Ho);
  const int h0 = ho * 2 - p, w0 = wo * 2 - p;
  u32x4 v[9];
  bool ok[9];
#pragma unroll
  for (int kh = 0; kh < 3; ++kh)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int h = h0 + kh, w = w0 + kw;
      const bool val = h >= 0 && h < H && w >= 0 && w < W;
      ok[kh * 3 + kw] = val;
      const int hh = val ? h : 0, ww = val ? w : 0;
      v[kh * 3 + kw] = *reinterpret_cast<const u32x4*>(x + (((size_t)n * H + hh) * W + ww) * C + 8 * c8);
    }
  float m[8];
  int am[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { m[j] = -INFINITY; am[j] = 0; }
  bool any = false;
#pragma unroll
  for (int pos = 0; pos < 9; ++pos) {
    if (!ok[pos]) continue;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float f = (j & 1) ? hi16(v[pos][j >> 1]) : lo16(v[pos][j >> 1]);
      if (!any || f > m[j] || (f != f && m[j] == m[j])) { m[j] = f; am[j] = pos; }
    }
    any = true;
  }
  u32x4 o;
  u32x2 ix;
#pragma unroll
  for (int q = 0; q < 4; ++q) o[q] = (__float_as_uint(m[2 * q]) >> 16) | (__float_as_uint(m[2 * q + 1]) & 0xffff0000u);
  ix[0] = (uint32_t)am[0] | ((uint32_t)am[1] << 8) | ((uint32_t)am[2] << 16) | ((uint32_t)am[3] << 24);
  ix[1] = (uint32_t)am[4] | ((uint32_t)am[5] << 8) | ((uint32_t)am[6] << 16) | ((uint32_t)am[7] << 24);
  const size_t oo = (((size_t)n * Ho + ho) * Wo + wo) * C + 8 * c8;
  *reinterpret_cast<u32x4*>(y + oo) = o;
  *reinterpret_cast<u32x2*>(idx + oo) = ix;
}

__global__ __launch_bounds__(256) void maxpool3s2_bwd(const uint16_t* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                      uint16_t* __restrict__ dx, int N, int H, int W, int C, int Ho,
                                                      int Wo, int p) {
  const unsigned C8 = (unsigned)C >> 3;
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (unsigned)N * H * W * C8) return;
  const unsigned c8 = i % C8;
  unsigned r = i / C8;
  const int w = (int)(r % (unsigned)W);
  r /= (unsigned)W;
  const int h = (int)(r % (unsigned)H);
  const int n = (int)(r / (unsigned)H);
  // windows covering h: ho in {hh - 1, hh} with hh = floor((h + p) / 2), kh = h + p - 2 ho in [0, 2]
  const int hh = (h + p) >> 1, wh = (w + p) >> 1;
  u32x2 ix[4];
  u32x4 g[4];
  bool ok[4];
  uint32_t pos[4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int ho = hh - 1 + a, wo = wh - 1 + b, t = 2 * a + b;
      const int kh = h + p - 2 * ho, kw = w + p - 2 * wo;
      const bool val = ho >= 0 && ho < Ho && wo >= 0 && wo < Wo && kh <= 2 && kw <= 2;
      ok[t] = val;
      pos[t] = (uint32_t)(kh * 3 + kw);
      const size_t oo = (((size_t)n * Ho + (val ? ho : 0)) * Wo + (val ? wo : 0)) * C + 8 * c8;
      ix[t] = *reinterpret_cast<const u32x2*>(idx + oo);
      g[t] = *reinterpret_cast<const u32x4*>(dy + oo);
    }
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (!ok[t]) continue;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t a = (ix[t][j >> 2] >> (8 * (j & 3))) & 255u;
      const float f = (j & 1) ? hi16(g[t][j >> 1]) : lo16(g[t][j >> 1]);
      if (a == pos[t]) acc[j] += f;
    }
  }
  u32x4 o;
#pragma unroll
  for (int q = 0; q < 4; ++q) o[q] = (uint32_t)f2bf(acc[2 * q]) | ((uint32_t)f2bf(acc[2 * q + 1]) << 16);
  *reinterpret_cast<u32x4*>(dx + (((size_t)n * H + h) * W + w) * C + 8 * c8) = o;
}

// full[n, s*i, s*j, :] += comp[n, i, j, :] (NHWC bf16, fp32 add, one rounding):
// the input gradient of a 1x1 / stride-s / unpadded convolution (a GEMM over
// the strided pixels) folded into the other branch's full-size gradient of the
// same input, instead of a zero-filled full-size dx and an add pass over it.
__global__ __launch_bounds__(256) void strided_add(uint16_t* __restrict__ full, const uint16_t* __restrict__ comp,
                                                   int N, int H, int W, int C, int Ho, int Wo, int s) {
  const int C8 = C >> 3;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)N * Ho * Wo * C8) return;
  const int c8 = (int)(i % C8);
  long long r = i / C8;
  const int wo = (int)(r % Wo);
  r /= Wo;
  const int ho = (int)(r % Ho);
  const int n = (int)(r / Ho);
  uint16_t* f = full + (((size_t)n * H + (size_t)ho * s) * W + (size_t)wo * s) * C + 8 * c8;
  const u32x4 a = *reinterpret_cast<const u32x4*>(f);
  const u32x4 b = *reinterpret_cast<const u32x4*>(comp + (size_t)i * 8);
  u32x4 o;
#pragma unroll
  for (int q = 0; q < 4; ++q) o[q] = pack2bf(lo16(a[q]) + lo16(b[q]), hi16(a[q]) + hi16(b[q]));
  *reinterpret_cast<u32x4*>(f) = o;
}

}  // namespace pool
}  // namespace dtfk

extern "C" hipError_t dtfk_maxpool_fwd(const void* x, void* y, void* idx, int N, int H, int W, int C, int Ho, int Wo,
                                       int k, int s, int p, hipStream_t st) {
  const long long n = (long long)N * Ho * Wo * (C / 8);
  if (n == 0) return hipSuccess;
  if (k == 3 && s == 2 && p >= 0 && p <= 1 && (long long)N * H * W * (C / 8) < 0x7fffffffLL) {
    hipLaunchKernelGGL(dtfk::pool::maxpool3s2_fwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       (const uint16_t*)x, (uint16_t*)y, (uint8_t*)idx, N, H, W, C, Ho, Wo, p);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(dtfk::pool::maxpool_fwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     (const uint16_t*)x, (uint16_t*)y, (uint8_t*)idx, N, H, W, C, Ho, Wo, k, s, p);
  return hipGetLastError();
}

extern "C" hipError_t dtfk_maxpool_bwd(const void* dy, const void* idx, void* dx, int N, int H, int W, int C, int Ho,
                                       int Wo, int k, int s, int p, hipStream_t st) {
  const long long n = (long long)N * H * W * (C / 8);
  if (n == 0) return hipSuccess;
  if (k == 3 && s == 2 && p >= 0 && p <= 1 && n < 0x7fffffffLL) {
    hipLaunchKernelGGL(dtfk::pool::maxpool3s2_bwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       (const uint16_t*)dy, (const uint8_t*)idx, (uint16_t*)dx, N, H, W, C, Ho, Wo, p);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(dtfk::pool::maxpool_bwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     (const uint16_t*)dy, (const uint8_t*)idx, (uint16_t*)dx, N, H, W, C, Ho, Wo, k, s, p);
  return hipGetLastError();
}

extern "C" hipError_t dtfk_strided_add(void* full, const void* comp, int N, int H, int W, int C, int Ho, int Wo, int s,
                                       hipStream_t st) {
  if (C % 8 || s < 1 || (long long)(Ho - 1) * s >= H || (long long)(Wo - 1) * s >= W) return hipErrorInvalidValue;
  const long long n = (long long)N * Ho * Wo * (C / 8);
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(dtfk::pool::strided_add, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, (uint16_t*)full,
                     (const uint16_t*)comp, N, H, W, C, Ho, Wo, s);
  return hipGetLastError();
}
