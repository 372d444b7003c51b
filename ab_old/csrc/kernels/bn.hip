// Reached by: ops/bn.py FusedBatchNorm2d (ResNet-50: bench_models.py --model resnet50); tests/test_bn_gpu.py
// Fused BatchNorm(+residual)(+ReLU) for NHWC (channels_last) bf16 activations
// -- the ResNet-50 path (BASELINE config #3).  MIOpen's BN needs three
// kernels forward/backward plus separate add / ReLU / ReLU-backward passes;
// here the normalise, affine, residual add and ReLU are one read+write pass,
// and the backward recomputes x_hat and the ReLU mask from x instead of
// storing them.
//
//   bn_partials    per-block channel sums of x and x^2        (fwd stats)
//   bn_finalize    mean / inv-std (+ running-stat update), scale/shift
//   bn_apply       y = relu(x * scale + shift [+ res])
//   bn_bwd_partials per-block channel sums of g and g * x_hat, g = dy * relu'
//   bn_bwd_finalize dgamma, dbeta, coefficients
//   bn_bwd_apply   dx = a*g + b*x + c  (per channel), d_res = g
//
// Layout: x is [M, C] with M = N*H*W rows, 8 channels per thread (16-byte
// bf16x8 accesses), C % 8 == 0.  Partial buffers are [P, C] fp32 and are
// reduced in a fixed order (deterministic).
#include "common.h"
#include <cstdlib>

namespace dtfk {
namespace bn {

__device__ __forceinline__ void ld8(const uint16_t* p, float* f) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) { f[2 * j] = bf2f(w[j] & 0xffff); f[2 * j + 1] = bf2f(w[j] >> 16); }
}
__device__ __forceinline__ void st8(uint16_t* p, const float* f) {
  uint4 u;
  u.x = pack2bf(f[0], f[1]); u.y = pack2bf(f[2], f[3]); u.z = pack2bf(f[4], f[5]); u.w = pack2bf(f[6], f[7]);
  *reinterpret_cast<uint4*>(p) = u;
}

// Partial-sum blocks: 256 threads = 8 channel threads (a 64-channel tile, 8
// channels each, 128 contiguous bytes per row) x 32 row lanes.  Grid is
// (channel tiles, P); block (t, p) covers rows p*32 + lane, stepping 32*P, four
// rows in flight per thread.  The 32 row lanes are combined in LDS and written
// as part[pass][p][c] (pass 0 / 1 = the two sums), so P stays small enough for
// the finalize to read the partials in a few microseconds.
//
// f is called as f(NR, rows) with NR = 4 (four valid rows, the main loop) or
// NR = 1 (the tail): both forms load unconditionally.  With a validity test
// around each row's load (the first version) the compiler waited for every
// load inside its branch, i.e. four serialized memory latencies per iteration.
template <int NR>
struct Rows {
  static constexpr int n = NR;
  int r[4];
};
template <typename F>
__device__ __forceinline__ void bn_tile_rows(int M, int P, F&& f) {
  const int tr = threadIdx.x >> 3;
  const int stride = 32 * P;
  int r = blockIdx.y * 32 + tr;
  for (; r + 3 * stride < M; r += 4 * stride) f(Rows<4>{{r, r + stride, r + 2 * stride, r + 3 * stride}});
  for (; r < M; r += stride) f(Rows<1>{{r, r, r, r}});
}

__device__ __forceinline__ void bn_tile_store(const float* s, const float* q, float* __restrict__ part, int P, int C,
                                              int c0) {
  __shared__ float red[2][32][65];
  const int tc = threadIdx.x & 7, tr = threadIdx.x >> 3;
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[0][tr][tc * 8 + j] = s[j]; red[1][tr][tc * 8 + j] = q[j]; }
  __syncthreads();
  if (threadIdx.x < 128) {
    const int pass = threadIdx.x >> 6, c = threadIdx.x & 63;
    float t = 0.f;
#pragma unroll 8
    for (int i = 0; i < 32; ++i) t += red[pass][i][c];
    if (c0 + c < C) part[((size_t)pass * P + blockIdx.y) * C + c0 + c] = t;
  }
}

__global__ __launch_bounds__(256) void bn_partials(const uint16_t* __restrict__ x, float* __restrict__ part, int M,
                                                   int C) {
  const int P = gridDim.y;
  const int c0 = blockIdx.x * 64;
  const int cc = c0 + (threadIdx.x & 7) * 8;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (cc < C)
    bn_tile_rows(M, P, [&](auto rows) {
      constexpr int NR = decltype(rows)::n;
      float v[4][8];
#pragma unroll
      for (int k = 0; k < NR; ++k) ld8(x + (size_t)rows.r[k] * C + cc, v[k]);
#pragma unroll
      for (int k = 0; k < NR; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) { s[j] += v[k][j]; q[j] += v[k][j] * v[k][j]; }
    });
  bn_tile_store(s, q, part, P, C, c0);
}

// Column sums of the [2P, C] partials: 1024 threads = FC channels x (1024 / FC)
// row groups, then an LDS tree over the groups (fixed order, deterministic).
// The finalize kernels are latency-bound chains of partial-row loads: FC = 4
// for narrow layers (C < 512: 4x the blocks and a quarter of the rows per thread
// of FC = 16 -- a 64-channel 3x3 conv at 56x56 hands over P = 3136 partial rows),
// 8 / 16 for wide ones.  Returns (sum of pass 0, sum of pass 1) to the g == 0 threads.
template <int FC>
__device__ __forceinline__ void sum_partials(const float* __restrict__ part, int P, int C, int c, int lane, int g,
                                             double& s0, double& s1) {
  constexpr int FG = 1024 / FC;
  static_assert(FC <= 64 && 64 % FC == 0, "channels per block divide a wave");
  __shared__ double red[2][16][FC];
  double a = 0.0, b = 0.0;
  if (c < C) {
    // four rows per trip, all eight loads issued unconditionally (rows past P
    // re-read row p and are masked out): one round of loads per four rows
    for (int p = g; p < P; p += 4 * FG) {
      float xv[4], yv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = p + j * FG < P ? p + j * FG : p;
        xv[j] = part[(size_t)q * C + c];
        yv[j] = part[((size_t)P + q) * C + c];
      }
#pragma unroll
      for (int j = 1; j < 4; ++j) {
        if (p + j * FG >= P) xv[j] = yv[j] = 0.f;
      }
      a += ((double)xv[0] + xv[1]) + ((double)xv[2] + xv[3]);
      b += ((double)yv[0] + yv[1]) + ((double)yv[2] + yv[3]);
    }
  }
  // row groups of a wave combined with xor shuffles (fixed pairing), then the
  // 16 waves' sums in wave order through LDS: one barrier instead of a
  // log2(FG)-level LDS tree (deterministic either way)
#pragma unroll
  for (int m = FC; m < 64; m <<= 1) {
    a += __shfl_xor(a, m);
    b += __shfl_xor(b, m);
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) < FC) {
    red[0][wave][lane] = a;
    red[1][wave][lane] = b;
  }
  __syncthreads();
  double x = 0.0, y = 0.0;
  if (g == 0) {
#pragma unroll
    for (int w = 0; w < 16; ++w) {
      x += red[0][w][lane];
      y += red[1][w][lane];
    }
  }
  s0 = x;
  s1 = y;
}

// mean/var (double), running stats, scale = gamma*invstd, shift = beta - mean*scale.
template <int FC>
__global__ __launch_bounds__(1024) void bn_finalize(const float* __restrict__ part, int P, int M, int C,
                                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                                    float* __restrict__ mean, float* __restrict__ invstd,
                                                    float* __restrict__ scale, float* __restrict__ shift,
                                                    float* __restrict__ run_mean, float* __restrict__ run_var,
                                                    float momentum, float eps) {
  const int lane = threadIdx.x % FC, g = threadIdx.x / FC;
  const int c = blockIdx.x * FC + lane;
  double s, q;
  sum_partials<FC>(part, P, C, c, lane, g, s, q);
  if (g != 0 || c >= C) return;
  const double mu = s / M;
  double var = q / M - mu * mu;
  if (var < 0.0) var = 0.0;
  const float is = (float)(1.0 / sqrt(var + (double)eps));
  mean[c] = (float)mu;
  invstd[c] = is;
  const float sc = gamma[c] * is;
  scale[c] = sc;
  shift[c] = beta[c] - (float)mu * sc;
  if (run_mean) {
    const double unbiased = M > 1 ? var * M / (M - 1) : var;
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (float)mu;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)unbiased;
  }
}

template <bool RES, bool RELU>
__global__ __launch_bounds__(256) void bn_apply(const uint16_t* __restrict__ x, const uint16_t* __restrict__ res,
                                                const float* __restrict__ scale, const float* __restrict__ shift,
                                                uint16_t* __restrict__ y, int64_t n8, int C) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)((i * 8) % C);
    float v[8], sc[8], sh[8];
    ld8(x + i * 8, v);
    *reinterpret_cast<float4*>(sc) = *reinterpret_cast<const float4*>(scale + c0);
    *reinterpret_cast<float4*>(sc + 4) = *reinterpret_cast<const float4*>(scale + c0 + 4);
    *reinterpret_cast<float4*>(sh) = *reinterpret_cast<const float4*>(shift + c0);
    *reinterpret_cast<float4*>(sh + 4) = *reinterpret_cast<const float4*>(shift + c0 + 4);
    float r[8];
    if constexpr (RES) ld8(res + i * 8, r);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float o = v[j] * sc[j] + sh[j];
      if constexpr (RES) o += r[j];
      if constexpr (RELU) o = fmaxf(o, 0.f);
      v[j] = o;
    }
    st8(y + i * 8, v);
  }
}

// g = dy * relu'(y) with y recomputed from x (and res); partial sums of g and g*x_hat.
// WG (residual + ReLU blocks): g is also stored (it IS the residual branch's
// gradient, exact in bf16: dy or 0), and the apply pass then reads g and x
// only -- 7 tensor passes instead of 8 (dy, x, res read twice; dx, dres written).
template <bool RES, bool RELU, bool WG = false>
__global__ __launch_bounds__(256) void bn_bwd_partials(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
                                                       const uint16_t* __restrict__ res,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ invstd,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift, float* __restrict__ part,
                                                       int M, int C, uint16_t* __restrict__ gout = nullptr) {
  static_assert(!WG || (RES && RELU), "g is only worth storing for residual + ReLU blocks");
  const int P = gridDim.y;
  const int c0 = blockIdx.x * 64;
  const int cc = c0 + (threadIdx.x & 7) * 8;
  float sg[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sgx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (cc < C) {
    float mu[8], is[8], sc[8], sh[8];
    *reinterpret_cast<float4*>(mu) = *reinterpret_cast<const float4*>(mean + cc);
    *reinterpret_cast<float4*>(mu + 4) = *reinterpret_cast<const float4*>(mean + cc + 4);
    *reinterpret_cast<float4*>(is) = *reinterpret_cast<const float4*>(invstd + cc);
    *reinterpret_cast<float4*>(is + 4) = *reinterpret_cast<const float4*>(invstd + cc + 4);
    *reinterpret_cast<float4*>(sc) = *reinterpret_cast<const float4*>(scale + cc);
    *reinterpret_cast<float4*>(sc + 4) = *reinterpret_cast<const float4*>(scale + cc + 4);
    *reinterpret_cast<float4*>(sh) = *reinterpret_cast<const float4*>(shift + cc);
    *reinterpret_cast<float4*>(sh + 4) = *reinterpret_cast<const float4*>(shift + cc + 4);
    bn_tile_rows(M, P, [&](auto rows) {
      constexpr int NR = decltype(rows)::n;
      float d[4][8], v[4][8], rr[4][8];
#pragma unroll
      for (int k = 0; k < NR; ++k) {
        const size_t e = (size_t)rows.r[k] * C + cc;
        ld8(dy + e, d[k]);
        ld8(x + e, v[k]);
        if constexpr (RES) ld8(res + e, rr[k]);
      }
#pragma unroll
      for (int k = 0; k < NR; ++k) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float g = d[k][j];
            if constexpr (RELU) {
              float o = v[k][j] * sc[j] + sh[j];
              if constexpr (RES) o += rr[k][j];
              g = o > 0.f ? g : 0.f;
            }
            d[k][j] = g;
            sg[j] += g;
            sgx[j] += g * (v[k][j] - mu[j]) * is[j];
          }
        if constexpr (WG) st8(gout + (size_t)rows.r[k] * C + cc, d[k]);
      }
    });
  }
  bn_tile_store(sg, sgx, part, P, C, c0);
}

// dbeta = sum g, dgamma = sum g*x_hat; dx = gamma*is*(g - dbeta/M - x_hat*dgamma/M)
//   = A*g + B*x + Cc with A = gamma*is, B = -gamma*is^2*dgamma/M, Cc = -A*dbeta/M - B*mean
template <int FC>
__global__ __launch_bounds__(1024) void bn_bwd_finalize(const float* __restrict__ part, int P, int M, int C,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ invstd, float* __restrict__ dgamma,
                                                        float* __restrict__ dbeta, float* __restrict__ coef,
                                                        int accum) {
  const int lane = threadIdx.x % FC, g = threadIdx.x / FC;
  const int c = blockIdx.x * FC + lane;
  double sgd, sgxd;
  sum_partials<FC>(part, P, C, c, lane, g, sgd, sgxd);
  if (g != 0 || c >= C) return;
  const float sg = (float)sgd, sgx = (float)sgxd;
  // accum: dgamma/dbeta are the parameters' .grad (e.g. DDP bucket views) and
  // are accumulated into, as autograd would
  dbeta[c] = accum ? dbeta[c] + sg : sg;
  dgamma[c] = accum ? dgamma[c] + sgx : sgx;
  const float is = invstd[c];
  const float A = gamma[c] * is;
  const float Bc = -A * is * sgx / M;
  coef[c] = A;
  coef[C + c] = Bc;
  coef[2 * C + c] = -A * sg / M - Bc * mean[c];
}

__device__ __forceinline__ void ld8f(const float* p, float* f) {
  *reinterpret_cast<float4*>(f) = *reinterpret_cast<const float4*>(p);
  *reinterpret_cast<float4*>(f + 4) = *reinterpret_cast<const float4*>(p + 4);
}

template <bool RES, bool RELU>
__global__ __launch_bounds__(256) void bn_bwd_apply(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
                                                    const uint16_t* __restrict__ res,
                                                    const float* __restrict__ scale, const float* __restrict__ shift,
                                                    const float* __restrict__ coef, uint16_t* __restrict__ dx,
                                                    uint16_t* __restrict__ dres, int64_t n8, int C) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)((i * 8) % C);
    float d[8], v[8], rr[8], o[8], g[8], A[8], Bv[8], Cv[8], sc[8], sh[8];
    ld8(dy + i * 8, d);
    ld8(x + i * 8, v);
    if constexpr (RES) ld8(res + i * 8, rr);
    ld8f(coef + c0, A);
    ld8f(coef + C + c0, Bv);
    ld8f(coef + 2 * C + c0, Cv);
    if constexpr (RELU) {
      ld8f(scale + c0, sc);
      ld8f(shift + c0, sh);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float gj = d[j];
      if constexpr (RELU) {
        float y = v[j] * sc[j] + sh[j];
        if constexpr (RES) y += rr[j];
        gj = y > 0.f ? gj : 0.f;
      }
      g[j] = gj;
      o[j] = A[j] * gj + Bv[j] * v[j] + Cv[j];
    }
    st8(dx + i * 8, o);
    if constexpr (RES) st8(dres + i * 8, g);
  }
}

}  // namespace bn
}  // namespace dtfk

using namespace dtfk::bn;

// partial rows P: >= 8 rows per thread, ~2048 blocks in total, at most 512
static int bn_grid(int M, int C) {
  const int ct = (C + 63) / 64;
  int g = (M + 32 * 8 - 1) / (32 * 8);
  const int cap = (2048 + ct - 1) / ct;
  if (g > cap) g = cap;
  if (g > 512) g = 512;
  return g < 1 ? 1 : g;
}
// the finalize kernels' channels per block (sum_partials): 16 for C >= 1024,
// 8 for >= 512, else 4.  Fewer channels per block for the long (P = 3136)
// partials of the 56x56 convolutions measured slower: FC = 1 took 11-13 us
// against 6-8 us (1024-deep LDS tree, one float per row per lane;
// profiles/resnet50_b128_steps_r5_fc1.txt)
static int finalize_fc(int /*P*/, int C) { return C >= 1024 ? 16 : (C >= 512 ? 8 : 4); }
static void launch_finalize(const float* part, int P, int M, int C, const float* gamma, const float* beta, float* mean,
                            float* invstd, float* scale, float* shift, float* run_mean, float* run_var, float momentum,
                            float eps, hipStream_t st) {
#define DTFK_FIN(FC)                                                                                                \
  hipLaunchKernelGGL((bn_finalize<FC>), dim3((C + FC - 1) / FC), dim3(1024), 0, st, part, P, M, C, gamma, beta, mean, \
                     invstd, scale, shift, run_mean, run_var, momentum, eps)
  switch (finalize_fc(P, C)) {
    case 16: DTFK_FIN(16); break;
    case 8: DTFK_FIN(8); break;
    case 4: DTFK_FIN(4); break;
    case 2: DTFK_FIN(2); break;
    default: DTFK_FIN(1);
  }
#undef DTFK_FIN
}
static void launch_bwd_finalize(const float* part, int P, int M, int C, const float* gamma, const float* mean,
                                const float* invstd, float* dgamma, float* dbeta, float* coef, int accum, hipStream_t st) {
#define DTFK_FIN(FC)                                                                                                   \
  hipLaunchKernelGGL((bn_bwd_finalize<FC>), dim3((C + FC - 1) / FC), dim3(1024), 0, st, part, P, M, C, gamma, mean, \
                     invstd, dgamma, dbeta, coef, accum)
  switch (finalize_fc(P, C)) {
    case 16: DTFK_FIN(16); break;
    case 8: DTFK_FIN(8); break;
    case 4: DTFK_FIN(4); break;
    case 2: DTFK_FIN(2); break;
    default: DTFK_FIN(1);
  }
#undef DTFK_FIN
}
// grid of the elementwise passes: one 8-channel chunk per thread, capped at
// DTF_BN_EW_CAP blocks (default 16384; beyond it the threads grid-stride)
static unsigned ew_grid(long long n8) {
  static const long long cap = [] {
    const char* e = getenv("DTF_BN_EW_CAP");
    return e ? atoll(e) : 16384LL;
  }();
  long long g = (n8 + 255) / 256;
  return (unsigned)(g > cap ? cap : (g < 1 ? 1 : g));
}

extern "C" {

int dtfk_bn_partial_rows(int M, int C) { return bn_grid(M, C); }

// forward: stats + finalize + apply.  part: [2 * P, C] fp32, stats: mean, invstd, scale, shift [C]
hipError_t dtfk_bn_fwd(const void* x, const void* res, const float* gamma, const float* beta, void* y, float* part,
                       float* mean, float* invstd, float* scale, float* shift, float* run_mean, float* run_var,
                       int M, int C, float momentum, float eps, int relu, hipStream_t st) {
  if (C % 8) return hipErrorInvalidValue;
  const int P = bn_grid(M, C);
  hipLaunchKernelGGL(bn_partials, dim3((C + 63) / 64, P), dim3(256), 0, st, (const uint16_t*)x, part, M, C);
  launch_finalize(part, P, M, C, gamma, beta, mean, invstd, scale, shift, run_mean, run_var, momentum, eps, st);
  const long long n8 = (long long)M * C / 8;
  const uint16_t* xp = (const uint16_t*)x;
  const uint16_t* rp = (const uint16_t*)res;
  uint16_t* yp = (uint16_t*)y;
  if (res && relu) hipLaunchKernelGGL((bn_apply<true, true>), dim3(ew_grid(n8)), dim3(256), 0, st, xp, rp, scale, shift, yp, n8, C);
  else if (res) hipLaunchKernelGGL((bn_apply<true, false>), dim3(ew_grid(n8)), dim3(256), 0, st, xp, rp, scale, shift, yp, n8, C);
  else if (relu) hipLaunchKernelGGL((bn_apply<false, true>), dim3(ew_grid(n8)), dim3(256), 0, st, xp, rp, scale, shift, yp, n8, C);
  else hipLaunchKernelGGL((bn_apply<false, false>), dim3(ew_grid(n8)), dim3(256), 0, st, xp, rp, scale, shift, yp, n8, C);
  return hipGetLastError();
}

// the statistics pass alone: part [2, P, C] (P = dtfk_bn_partial_rows) -- the
// cost a convolution without a statistics epilogue leaves to its BatchNorm
hipError_t dtfk_bn_stat_partials(const void* x, float* part, int M, int C, hipStream_t st) {
  if (C % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bn_partials, dim3((C + 63) / 64, bn_grid(M, C)), dim3(256), 0, st, (const uint16_t*)x, part, M, C);
  return hipGetLastError();
}

// the same forward when the per-channel sums of x and x^2 already exist as [2, P, C]
// partials (written by the producing convolution's epilogue, csrc/kernels/conv_igemm.hip):
// finalize + apply, no statistics pass over x
hipError_t dtfk_bn_fwd_parts(const void* x, const void* res, const float* gamma, const float* beta, void* y,
                             const float* part, int P, float* mean, float* invstd, float* scale, float* shift,
                             float* run_mean, float* run_var, int M, int C, float momentum, float eps, int relu,
                             hipStream_t st) {
  if (C % 8 || P < 1) return hipErrorInvalidValue;
  launch_finalize(part, P, M, C, gamma, beta, mean, invstd, scale, shift, run_mean, run_var, momentum, eps, st);
  const long long n8 = (long long)M * C / 8;
  const uint16_t* xp = (const uint16_t*)x;
  const uint16_t* rp = (const uint16_t*)res;
  uint16_t* yp = (uint16_t*)y;
  if (res && relu) hipLaunchKernelGGL((bn_apply<true, true>), dim3(ew_grid(n8)), dim3(256), 0, st, xp, rp, scale, shift, yp, n8, C);
  else if (res) hipLaunchKernelGGL((bn_apply<true, false>), dim3(ew_grid(n8)), dim3(256), 0, st, xp, rp, scale, shift, yp, n8, C);
  else if (relu) hipLaunchKernelGGL((bn_apply<false, true>), dim3(ew_grid(n8)), dim3(256), 0, st, xp, rp, scale, shift, yp, n8, C);
  else hipLaunchKernelGGL((bn_apply<false, false>), dim3(ew_grid(n8)), dim3(256), 0, st, xp, rp, scale, shift, yp, n8, C);
  return hipGetLastError();
}

// eval-mode / inference apply with given scale/shift
hipError_t dtfk_bn_apply(const void* x, const void* res, const float* scale, const float* shift, void* y, int M, int C,
                         int relu, hipStream_t st) {
  if (C % 8) return hipErrorInvalidValue;
  const long long n8 = (long long)M * C / 8;
  const uint16_t* xp = (const uint16_t*)x;
  const uint16_t* rp = (const uint16_t*)res;
  uint16_t* yp = (uint16_t*)y;
  if (res && relu) hipLaunchKernelGGL((bn_apply<true, true>), dim3(ew_grid(n8)), dim3(256), 0, st, xp, rp, scale, shift, yp, n8, C);
  else if (res) hipLaunchKernelGGL((bn_apply<true, false>), dim3(ew_grid(n8)), dim3(256), 0, st, xp, rp, scale, shift, yp, n8, C);
  else if (relu) hipLaunchKernelGGL((bn_apply<false, true>), dim3(ew_grid(n8)), dim3(256), 0, st, xp, rp, scale, shift, yp, n8, C);
  else hipLaunchKernelGGL((bn_apply<false, false>), dim3(ew_grid(n8)), dim3(256), 0, st, xp, rp, scale, shift, yp, n8, C);
  return hipGetLastError();
}

// backward with the partials (sum g, sum g x_hat) [2, P, C] and the ReLU-masked
// output gradient g supplied by its producer (conv_igemm.hip conv_fwd EPI 2):
// finalize + apply, no partials pass over dy / x
hipError_t dtfk_bn_bwd_parts(const void* g, const void* x, const float* gamma, const float* mean, const float* invstd,
                             const float* part, int P, float* coef, void* dx, float* dgamma, float* dbeta, int M, int C,
                             int accum, hipStream_t st) {
  if (C % 8 || P < 1) return hipErrorInvalidValue;
  launch_bwd_finalize(part, P, M, C, gamma, mean, invstd, dgamma, dbeta, coef, accum, st);
  const long long n8 = (long long)M * C / 8;
  hipLaunchKernelGGL((bn_bwd_apply<false, false>), dim3(ew_grid(n8)), dim3(256), 0, st, (const uint16_t*)g,
                     (const uint16_t*)x, nullptr, nullptr, nullptr, coef, (uint16_t*)dx, nullptr, n8, C);
  return hipGetLastError();
}

// backward.  coef: [3, C] scratch; part: [2 * P, C]
// write_g (residual + ReLU only): the partials pass stores g into dres and the
// apply pass reads (g, x) instead of (dy, x, res).
hipError_t dtfk_bn_bwd(const void* dy, const void* x, const void* res, const float* gamma, const float* mean,
                       const float* invstd, const float* scale, const float* shift, float* part, float* coef,
                       void* dx, void* dres, float* dgamma, float* dbeta, int M, int C, int relu, int accum,
                       int write_g, hipStream_t st) {
  if (C % 8) return hipErrorInvalidValue;
  const int P = bn_grid(M, C);
  const uint16_t* dyp = (const uint16_t*)dy;
  const uint16_t* xp = (const uint16_t*)x;
  const uint16_t* rp = (const uint16_t*)res;
  const long long n8 = (long long)M * C / 8;
  if (res && relu && write_g && dres) {
    hipLaunchKernelGGL((bn_bwd_partials<true, true, true>), dim3((C + 63) / 64, P), dim3(256), 0, st, dyp, xp, rp,
                       mean, invstd, scale, shift, part, M, C, (uint16_t*)dres);
    launch_bwd_finalize(part, P, M, C, gamma, mean, invstd, dgamma, dbeta, coef, accum, st);
    hipLaunchKernelGGL((bn_bwd_apply<false, false>), dim3(ew_grid(n8)), dim3(256), 0, st, (const uint16_t*)dres, xp,
                       nullptr, scale, shift, coef, (uint16_t*)dx, nullptr, n8, C);
    return hipGetLastError();
  }
#define DTFK_BNP(R, L) hipLaunchKernelGGL((bn_bwd_partials<R, L>), dim3((C + 63) / 64, P), dim3(256), 0, st, dyp, xp, rp, mean, invstd, scale, shift, part, M, C, nullptr)
  if (res && relu) DTFK_BNP(true, true); else if (res) DTFK_BNP(true, false);
  else if (relu) DTFK_BNP(false, true); else DTFK_BNP(false, false);
#undef DTFK_BNP
  launch_bwd_finalize(part, P, M, C, gamma, mean, invstd, dgamma, dbeta, coef, accum, st);
#define DTFK_BNA(R, L) hipLaunchKernelGGL((bn_bwd_apply<R, L>), dim3(ew_grid(n8)), dim3(256), 0, st, dyp, xp, rp, scale, shift, coef, (uint16_t*)dx, (uint16_t*)dres, n8, C)
  if (res && relu) DTFK_BNA(true, true); else if (res) DTFK_BNA(true, false);
  else if (relu) DTFK_BNA(false, true); else DTFK_BNA(false, false);
#undef DTFK_BNA
  return hipGetLastError();
}

}  // extern "C"
