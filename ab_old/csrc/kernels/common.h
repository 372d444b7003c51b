// Shared CDNA4 (gfx950) device helpers: bf16 packing, MFMA wrappers, wave64
// reductions.  Every kernel in csrc/kernels includes this header; nothing here
// is CUDA-derived -- wave width is hard-coded to 64 and MFMA shapes are the
// gfx950 16x16x32 / 32x32x16 bf16 forms.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

namespace dtfk {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int kWave = 64;

// D = A(16x32) * B(32x16) + C, fp32 accumulate.
// Lane l holds A[l&15][8*(l>>4)+j], B[8*(l>>4)+j][l&15] (j = 0..7) and
// C/D[4*(l>>4)+i][l&15] (i = 0..3).
__device__ __forceinline__ f32x4 mfma16x16x32(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// D = A(32x16) * B(16x32) + C. Lane l holds A[l&31][8*(l>>5)+j],
// B[8*(l>>5)+j][l&31]; C/D[(r&3)+8*(r>>2)+4*(l>>5)][l&31] (r = 0..15).
__device__ __forceinline__ f32x16 mfma32x32x16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// Zero an [M, N] fp32 block of row stride ldc (the output of a split-K /
// atomically accumulated product).  A kernel, not hipMemset2DAsync /
// hipMemsetAsync: those memsets do not take effect when replayed from a
// captured hipGraph on this stack (measured: a [256, 1] 2-D memset and a
// 40-byte 1-D memset both left the previous replay's sums in place), so
// Wide&Deep's graphed step accumulated its tower gradients across replays and
// diverged (tests/test_graph_replay_gpu.py; DTF_ZERO_MEMSET2D=1 restores the
// old path for that A/B).
__global__ static __launch_bounds__(256) void zero2d_f32_kernel(float* __restrict__ C, int ldc, int M, int N) {
  const long long n = (long long)M * N;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    C[(i / N) * ldc + i % N] = 0.f;
}
static inline hipError_t zero2d_f32(float* C, int ldc, int M, int N, hipStream_t s) {
  const long long n = (long long)M * N;
  if (n <= 0) return hipSuccess;
  static const bool memset2d = getenv("DTF_ZERO_MEMSET2D") != nullptr;   // A/B probe of the old path
  if (memset2d) return hipMemset2DAsync(C, (size_t)ldc * sizeof(float), 0, (size_t)N * sizeof(float), M, s);
  const unsigned blocks = (unsigned)((n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048);
  hipLaunchKernelGGL(zero2d_f32_kernel, dim3(blocks), dim3(256), 0, s, C, ldc, M, N);
  return hipGetLastError();
}

// fp32 -> bf16 bits, round-to-nearest-even (hardware cvt on gfx950).
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 h = static_cast<__bf16>(f);
  return __builtin_bit_cast(uint16_t, h);
}
__device__ __forceinline__ float bf2f(uint16_t b) {
  return __uint_as_float(static_cast<uint32_t>(b) << 16);
}
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  return static_cast<uint32_t>(f2bf(lo)) | (static_cast<uint32_t>(f2bf(hi)) << 16);
}

// Counter-based dropout hash: keep(i) = hash32(seed, i) >= p * 2^32.  Shared by
// every kernel that regenerates a mask in backward.  Seeds with bit 63 set (what
// ops/transformer.py hands out by default) take a 32-bit lowbias32 finaliser of
// the element index xor a mixed seed -- ~8 VALU ops, all 32-bit; the others the
// splitmix64 finaliser (~30 ops incl. 64-bit multiplies: ~25 us of a BERT-base
// attention forward at B = 128, S = 128, scripts/probes/attn_dropout_cost.py).
// The branch is wave-uniform (the seed is a kernel argument).
__device__ __forceinline__ uint32_t hash32(uint64_t seed, uint64_t i) {
  if (seed >> 63) {
    const uint32_t k = (uint32_t)seed ^ ((uint32_t)(seed >> 32) * 0x85EBCA6Bu);
    uint32_t x = ((uint32_t)i ^ k) + (uint32_t)(i >> 32) * 0x9E3779B9u;
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
  }
  uint64_t x = seed ^ (i * 0x9E3779B97F4A7C15ull);
  x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27; x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return static_cast<uint32_t>(x);
}

__device__ __forceinline__ bf16x8 ld_bf16x8(const uint16_t* p) {
  return *reinterpret_cast<const bf16x8*>(p);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}
// Reductions over aligned groups of 16 lanes (one MFMA 16x16 output row group).
__device__ __forceinline__ float group16_sum(float v) {
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) v += __shfl_xor(v, off, 16);
  return v;
}
__device__ __forceinline__ float group16_max(float v) {
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 16));
  return v;
}

// Block-wide sum for blockDim.x a multiple of 64 (<= 1024). `scratch` needs
// blockDim.x/64 floats of LDS. Result valid in every thread.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += scratch[i];
  return t;
}

// DPP row (16-lane) all-reduce: rotate-right by 8, 4, 2, 1 within each row of 16
// lanes; every lane of the row ends with the result.  A few VALU cycles per
// step instead of an LDS-latency ds_bpermute per __shfl.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                              0xF, 0xF, false));
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp_f<0x128>(v));
  v = fmaxf(v, dpp_f<0x124>(v));
  v = fmaxf(v, dpp_f<0x122>(v));
  v = fmaxf(v, dpp_f<0x121>(v));
  return v;
}
__device__ __forceinline__ float row16_min(float v) {
  v = fminf(v, dpp_f<0x128>(v));
  v = fminf(v, dpp_f<0x124>(v));
  v = fminf(v, dpp_f<0x122>(v));
  v = fminf(v, dpp_f<0x121>(v));
  return v;
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<0x128>(v);
  v += dpp_f<0x124>(v);
  v += dpp_f<0x122>(v);
  v += dpp_f<0x121>(v);
  return v;
}

__device__ __forceinline__ float sigmoidf_(float z) { return 1.f / (1.f + __expf(-z)); }

// Peer (IPC-mapped) exchange data is read with system-scope loads (sc0 sc1):
// never served from a cache line of this XCD or device, whatever memory type
// the importing process's mapping of the peer buffer got.  (Non-temporal loads
// are L2-served: a stale line there breaks bit-identical replicas.)
__device__ __forceinline__ unsigned long long ld_sys_u64(const void* p) {
  return __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t ld_sys_u32(const void* p) {
  return __hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint16_t ld_sys_u16(const void* p) {
  return __hip_atomic_load(reinterpret_cast<const uint16_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ float ld_sys_f32(const void* p) { return __uint_as_float(ld_sys_u32(p)); }
__device__ __forceinline__ f32x4 ld_sys_f32x4(const void* p) {
  const unsigned long long a = ld_sys_u64(p), b = ld_sys_u64(static_cast<const char*>(p) + 8);
  return f32x4{__uint_as_float((uint32_t)a), __uint_as_float((uint32_t)(a >> 32)), __uint_as_float((uint32_t)b),
               __uint_as_float((uint32_t)(b >> 32))};
}

// GELU (erf form) cdf and pdf with the A&S 7.1.26 erfc polynomial: libm erff
// made the [tokens, 3072] GELU passes VALU-bound (shared by transformer.hip's
// elementwise kernels and gemm_big.hip's fused GELU-backward epilogue).
__device__ __forceinline__ void gelu_cdf_pdf(float z, float& cdf, float& pdf) {
  const float x = fabsf(z) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, x, 1.f));
  const float poly = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f),
                                      -0.284496736f), 0.254829592f);
  const float e = __expf(-0.5f * z * z);
  const float tail = 0.5f * poly * e;           // 0.5 * (1 - erf(|z| / sqrt2))
  cdf = z >= 0.f ? 1.f - tail : tail;
  pdf = 0.3989422804014327f * e;
}
}  // namespace dtfk

#define DTFK_CHECK_LAUNCH() (hipGetLastError())
