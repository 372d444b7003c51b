// Reached by: models/bert.py (BERT-base: bench_models.py --model bert_base); tests/test_transformer_gpu.py
// Fused multi-head self-attention for BERT-shaped layers (head dim 64,
// S <= 256, S % 32 == 0) on CDNA4 MFMA -- forward and backward.
//
// The unfused path is QK^T (batched GEMM) -> masked softmax + dropout ->
// PV (batched GEMM), plus permute copies of q/k/v/ctx in both directions,
// slice-backward fills and the qkv bias add: ~0.5 ms per BERT-base layer at
// B=128, S=128 on MI355X.  Here one workgroup owns (batch, head, 128 rows):
//
//   attn_fwd      reads q/k/v straight out of the packed [B, S, 3, NH, 64]
//                 projection (+ bias, fused), keeps the whole score row in
//                 registers (S <= 256), writes ctx as [B, S, NH*64] and the
//                 row log-sum-exp for the backward.
//   attn_bwd_dq   recomputes P from lse, dP = dO V^T, dS, writes dQ and
//                 D = rowsum(dO * O).
//   attn_bwd_dkv  per 16-key slab, loops over all queries: dV += Pd^T dO,
//                 dK += dS^T Q.
//
// MFMA orientation (16x16x32 bf16; lane l, g = l >> 4, c = l & 15):
// the score tile is computed transposed, S^T = K Q^T, so a lane holds keys
// 4g+i of a 16-key tile for ONE query c.  The next product (O^T = V^T P^T)
// sums over keys, i.e. over the accumulator's row index, so P^T feeds the
// B operand straight from registers: the k-slot (g, j) of a 32-key block is
// key 4g+j (j < 4) or 16+4g+(j-4) (j >= 4), and the A operand (V^T) is read
// from the row-major LDS image of V with the same key permutation by two
// transposed LDS reads (ds_read_b64_tr_b16, ld_tr_pair).  The backward products
// follow the same rule (dQ^T = K^T dS^T; dV = Pd^T dO, dK = dS^T Q in the
// key-major kernel), reading the row images of K, Q and dO transposed -- no
// second, transposed image is written.
//
// Dropout keep(i) = hash32(seed, i) >= p * 2^32 with i the element index of
// the [B, NH, S, S] probability tensor -- the same convention as the unfused
// softmax kernel (transformer.hip), so both paths drop the same elements.
#include "common.h"

#include <cstdlib>
#include <string>

namespace dtfk {
namespace attn {

constexpr int D = 64;
constexpr int KP = 72;     // padded row of a [S][64] LDS image (144 B: rows spread over banks)

__device__ __forceinline__ uint4 add_bias8(uint4 u, const float* __restrict__ bias) {
  if (!bias) return u;
  const float4 b0 = *reinterpret_cast<const float4*>(bias);
  const float4 b1 = *reinterpret_cast<const float4*>(bias + 4);
  const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
  uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 4; ++j)
    w[j] = pack2bf(bf2f(w[j] & 0xffff) + bb[2 * j], bf2f(w[j] >> 16) + bb[2 * j + 1]);
  return uint4{w[0], w[1], w[2], w[3]};
}

__device__ __forceinline__ uint4 ld16(const uint16_t* p) { return *reinterpret_cast<const uint4*>(p); }

__device__ __forceinline__ bf16x8 as_frag(uint4 u) { return __builtin_bit_cast(bf16x8, u); }

// The permuted 32-key fragment of a TRANSPOSED operand straight from a
// row-major [S][KP] image with the gfx950 transposed LDS read
// (ds_read_b64_tr_b16: per 16-lane group, lane 4q+p addresses row q, columns
// 4p..4p+3 of a 4 x 16 block; lane i receives column i): lane (g, c) gets
// column col0 + c of rows row0 + 4g + 0..3 (elements 0..3) and row0 + 16 + 4g +
// 0..3 (elements 4..7) -- the k-slot order of the score accumulators.  Replaces
// a second, transposed LDS image written with 2-byte scatter stores.  EXEC must
// be full (wave-uniform control flow only).
typedef __attribute__((ext_vector_type(4))) short v4s_t;
typedef __attribute__((address_space(3))) v4s_t lds_v4s_t;
__device__ __forceinline__ bf16x8 ld_tr_pair(const uint16_t* img, int row0, int col0, int l) {
  const int g = l >> 4, q = (l >> 2) & 3, p = l & 3;
  const uint16_t* a = img + (row0 + 4 * g + q) * KP + col0 + 4 * p;
  const v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)(a));
  const v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t*)(a + 16 * KP));
  typedef __attribute__((ext_vector_type(8))) short v8s_t;
  const v8s_t v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ bf16x8 pack8(const float* f) {
  return as_frag(uint4{pack2bf(f[0], f[1]), pack2bf(f[2], f[3]), pack2bf(f[4], f[5]), pack2bf(f[6], f[7])});
}

__device__ __forceinline__ float keepf(uint64_t seed, uint64_t i, uint32_t thresh, float inv_keep) {
  return (thresh == 0u) ? 1.f : (hash32(seed, i) >= thresh ? inv_keep : 0.f);
}

// stage a [S][64] tile (rows of the packed projection, or of a [B,S,NH*64]
// tensor) into a row image rows[S][KP] (the products that need it transposed
// read it with ld_tr_pair).  Two halves so a kernel issues every global load of all its
// stages (and its per-wave fragments) before the first LDS store: a
// load -> store loop per stage costs one memory round trip per iteration.  With
// 512 threads a thread's 16-byte column part (ch & 7) is the same in every
// iteration, so its 8 bias values are loaded once.
template <int S>
struct StageRegs {
  static constexpr int N = (S * 8 + 511) / 512;   // 16-byte chunks per thread
  uint4 v[N];
  float4 b0, b1;
};
template <int S>
__device__ __forceinline__ void stage_load(const uint16_t* __restrict__ src, long long row_stride,
                                           const float* __restrict__ bias, StageRegs<S>& R) {
  const int part = threadIdx.x & 7;
#pragma unroll
  for (int it = 0; it < StageRegs<S>::N; ++it) {
    const int ch = threadIdx.x + 512 * it;
    if (ch < S * 8) R.v[it] = ld16(src + (ch >> 3) * row_stride + part * 8);
  }
  if (bias) {
    R.b0 = *reinterpret_cast<const float4*>(bias + part * 8);
    R.b1 = *reinterpret_cast<const float4*>(bias + part * 8 + 4);
  }
}
template <int S>
__device__ __forceinline__ void stage_store(const StageRegs<S>& R, bool has_bias, uint16_t* rows) {
  const int part = threadIdx.x & 7;
  const float bb[8] = {R.b0.x, R.b0.y, R.b0.z, R.b0.w, R.b1.x, R.b1.y, R.b1.z, R.b1.w};
#pragma unroll
  for (int it = 0; it < StageRegs<S>::N; ++it) {
    const int ch = threadIdx.x + 512 * it;
    if (ch >= S * 8) break;
    const int r = ch >> 3;
    uint4 v = R.v[it];
    if (has_bias) {
      uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        w[j] = pack2bf(bf2f(w[j] & 0xffff) + bb[2 * j], bf2f(w[j] >> 16) + bb[2 * j + 1]);
      v = uint4{w[0], w[1], w[2], w[3]};
    }
    *reinterpret_cast<uint4*>(rows + r * KP + part * 8) = v;
  }
}

template <int NKB>
__global__ __launch_bounds__(512) void attn_fwd(const uint16_t* __restrict__ qkv, const float* __restrict__ bias,
                                                const float* __restrict__ mask, uint16_t* __restrict__ ctx,
                                                float* __restrict__ lse, int NH, float scale, uint32_t thresh,
                                                float inv_keep, uint64_t seed) {
  constexpr int S = 32 * NKB;
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  uint16_t* Ks = lds;                 // [S][KP]
  uint16_t* Vs = lds + S * KP;        // [S][KP] (read transposed: ld_tr_pair)
  const int b = blockIdx.z, h = blockIdx.y;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, c = l & 15;
  const long long RS = 3LL * NH * D;
  const uint16_t* base = qkv + (long long)b * S * RS + h * D;
  const float* bq = bias ? bias + h * D : nullptr;
  const float* bk = bias ? bias + (NH + h) * D : nullptr;
  const float* bv = bias ? bias + (2 * NH + h) * D : nullptr;
  StageRegs<S> rk, rv;
  stage_load<S>(base + NH * D, RS, bk, rk);
  stage_load<S>(base + 2 * NH * D, RS, bv, rv);
  const int q = blockIdx.x * 128 + w * 16 + c;
  const bool active = blockIdx.x * 128 + w * 16 < S;   // wave-uniform
  uint4 qraw[2];   // this wave's query fragments, in flight with the stages
#pragma unroll
  for (int s = 0; s < 2; ++s) qraw[s] = ld16(base + (long long)min(q, S - 1) * RS + 32 * s + 8 * g);
  stage_store<S>(rk, bk != nullptr, Ks);
  stage_store<S>(rv, bv != nullptr, Vs);
  __syncthreads();
  if (!active) return;                                 // no barrier follows

  bf16x8 bqf[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) bqf[s] = as_frag(add_bias8(qraw[s], bq ? bq + 32 * s + 8 * g : nullptr));
  f32x4 sc[2 * NKB];
#pragma unroll
  for (int t = 0; t < 2 * NKB; ++t) {
    sc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 2; ++s) sc[t] = mfma16x16x32(ld_bf16x8(Ks + (16 * t + c) * KP + 32 * s + 8 * g), bqf[s], sc[t]);
  }
  float mx = -3.0e38f;
#pragma unroll
  for (int t = 0; t < 2 * NKB; ++t) {
    float4 mk = mask ? *reinterpret_cast<const float4*>(mask + (long long)b * S + 16 * t + 4 * g)
                     : float4{0.f, 0.f, 0.f, 0.f};
    const float m4[4] = {mk.x, mk.y, mk.z, mk.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      sc[t][i] = sc[t][i] * scale + m4[i];
      mx = fmaxf(mx, sc[t][i]);
    }
  }
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int t = 0; t < 2 * NKB; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      sc[t][i] = __expf(sc[t][i] - mx);
      sum += sc[t][i];
    }
  sum += __shfl_xor(sum, 16, 64);
  sum += __shfl_xor(sum, 32, 64);
  const float inv = 1.f / sum;
  const long long row = ((long long)b * NH + h) * S + q;
  if (g == 0) lse[row] = mx + __logf(sum);
  const uint64_t ebase = (uint64_t)row * S;
  bf16x8 pb[NKB];
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) {
    float f[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k0 = 32 * kb + 4 * g + j;
      f[j] = sc[2 * kb][j] * inv * keepf(seed, ebase + k0, thresh, inv_keep);
      f[4 + j] = sc[2 * kb + 1][j] * inv * keepf(seed, ebase + k0 + 16, thresh, inv_keep);
    }
    pb[kb] = pack8(f);
  }
  uint16_t* out = ctx + ((long long)b * S + q) * NH * D + h * D;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) o = mfma16x16x32(ld_tr_pair(Vs, 32 * kb, 16 * u, l), pb[kb], o);
    *reinterpret_cast<uint2*>(out + 16 * u + 4 * g) = uint2{pack2bf(o[0], o[1]), pack2bf(o[2], o[3])};
  }
}

template <int NKB>
__global__ __launch_bounds__(512) void attn_bwd_dq(const uint16_t* __restrict__ qkv, const float* __restrict__ bias,
                                                   const float* __restrict__ mask, const uint16_t* __restrict__ ctx,
                                                   const uint16_t* __restrict__ dctx, const float* __restrict__ lse,
                                                   float* __restrict__ Dbuf, uint16_t* __restrict__ dqkv, int NH,
                                                   float scale, uint32_t thresh, float inv_keep, uint64_t seed,
                                                   float* __restrict__ bpart) {
  constexpr int S = 32 * NKB;
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  uint16_t* Ks = lds;                    // [S][KP] (also read transposed: ld_tr_pair)
  uint16_t* Vs = lds + S * KP;           // [S][KP]
  const int b = blockIdx.z, h = blockIdx.y;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, c = l & 15;
  const long long RS = 3LL * NH * D, HS = (long long)NH * D;
  const uint16_t* base = qkv + (long long)b * S * RS + h * D;
  const float* bq = bias ? bias + h * D : nullptr;
  StageRegs<S> rk, rv;
  const float* bkp = bias ? bias + (NH + h) * D : nullptr;
  const float* bvp = bias ? bias + (2 * NH + h) * D : nullptr;
  stage_load<S>(base + NH * D, RS, bkp, rk);
  stage_load<S>(base + 2 * NH * D, RS, bvp, rv);
  const bool active = blockIdx.x * 128 + w * 16 < S;   // wave-uniform
  const int q = min(blockIdx.x * 128 + w * 16 + c, S - 1);
  const uint16_t* dor = dctx + ((long long)b * S + q) * HS + h * D;
  uint4 qraw[2], doraw[2];   // this wave's fragments, in flight with the stages
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    qraw[s] = ld16(base + (long long)q * RS + 32 * s + 8 * g);
    doraw[s] = ld16(dor + 32 * s + 8 * g);
  }
  stage_store<S>(rk, bkp != nullptr, Ks);
  stage_store<S>(rv, bvp != nullptr, Vs);
  __syncthreads();
  if (!active) return;

  bf16x8 bqf[2], bdo[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    bqf[s] = as_frag(add_bias8(qraw[s], bq ? bq + 32 * s + 8 * g : nullptr));
    bdo[s] = as_frag(doraw[s]);
  }
  // D = rowsum(dO * O): lane group g covers d = 16g .. 16g+15
  const uint16_t* orow = ctx + ((long long)b * S + q) * HS + h * D + 16 * g;
  float dsum = 0.f;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const uint4 ov = ld16(orow + 8 * half), dv = ld16(dor + 16 * g + 8 * half);
    const uint32_t a[4] = {ov.x, ov.y, ov.z, ov.w}, d4[4] = {dv.x, dv.y, dv.z, dv.w};
#pragma unroll
    for (int j = 0; j < 4; ++j)
      dsum += bf2f(a[j] & 0xffff) * bf2f(d4[j] & 0xffff) + bf2f(a[j] >> 16) * bf2f(d4[j] >> 16);
  }
  dsum += __shfl_xor(dsum, 16, 64);
  dsum += __shfl_xor(dsum, 32, 64);
  const long long row = ((long long)b * NH + h) * S + q;
  if (g == 0) Dbuf[row] = dsum;
  const float L = lse[row];
  const uint64_t ebase = (uint64_t)row * S;
  // dQ^T accumulates key block by key block as each block's dS is formed (no
  // [NKB] dS array: with every block's operand loads hoisted the fully unrolled
  // form held 152 VGPRs = one workgroup per CU); same MFMA order per output
  f32x4 acc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
  for (int kb = 0; kb < NKB; ++kb) {
    float f[8];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int t = 2 * kb + tt;
      f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        sv = mfma16x16x32(ld_bf16x8(Ks + (16 * t + c) * KP + 32 * s + 8 * g), bqf[s], sv);
        dp = mfma16x16x32(ld_bf16x8(Vs + (16 * t + c) * KP + 32 * s + 8 * g), bdo[s], dp);
      }
      float4 mk = mask ? *reinterpret_cast<const float4*>(mask + (long long)b * S + 16 * t + 4 * g)
                       : float4{0.f, 0.f, 0.f, 0.f};
      const float m4[4] = {mk.x, mk.y, mk.z, mk.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = 16 * t + 4 * g + i;
        const float P = __expf(sv[i] * scale + m4[i] - L);
        const float dpd = dp[i] * keepf(seed, ebase + key, thresh, inv_keep);
        f[4 * tt + i] = P * (dpd - dsum);
      }
    }
    const bf16x8 dsb = pack8(f);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = mfma16x16x32(ld_tr_pair(Ks, 32 * kb, 16 * u, l), dsb, acc[u]);
  }
  uint16_t* dq = dqkv + ((long long)b * S + q) * RS + h * D;
#pragma unroll
  for (int u = 0; u < 4; ++u)
    *reinterpret_cast<uint2*>(dq + 16 * u + 4 * g) =
        uint2{pack2bf(acc[u][0] * scale, acc[u][1] * scale), pack2bf(acc[u][2] * scale, acc[u][3] * scale)};
  if (bpart != nullptr) {
    // q-bias gradient partials: this wave's 16 queries summed per dimension
    // (lanes c = 0..15 of a group hold the 16 queries) -> bpart[b * S/16 + wave row][h * 64 + d]
    float cs[16];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v = acc[u][j] * scale;
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        v += __shfl_xor(v, 4, 64);
        v += __shfl_xor(v, 8, 64);
        cs[4 * u + j] = v;
      }
    if (c == 0) {
      float* pr = bpart + ((long long)b * (S / 16) + blockIdx.x * 8 + w) * RS + h * D;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        *reinterpret_cast<float4*>(pr + 16 * u + 4 * g) = float4{cs[4 * u], cs[4 * u + 1], cs[4 * u + 2], cs[4 * u + 3]};
    }
  }
}

template <int NKB>
__global__ __launch_bounds__(512) void attn_bwd_dkv(const uint16_t* __restrict__ qkv, const float* __restrict__ bias,
                                                    const float* __restrict__ mask, const uint16_t* __restrict__ dctx,
                                                    const float* __restrict__ lse, const float* __restrict__ Dbuf,
                                                    uint16_t* __restrict__ dqkv, int NH, float scale, uint32_t thresh,
                                                    float inv_keep, uint64_t seed, float* __restrict__ bpart) {
  constexpr int S = 32 * NKB;
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  uint16_t* Qs = lds;                          // [S][KP] (also read transposed: ld_tr_pair)
  uint16_t* dOs = lds + S * KP;                // [S][KP] (likewise)
  float* Ls = reinterpret_cast<float*>(lds + 2 * S * KP);   // [S] lse of every query row
  float* Dl = Ls + S;                                                     // [S] rowsum(dO * O)
  const int b = blockIdx.z, h = blockIdx.y;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, c = l & 15;
  const long long RS = 3LL * NH * D, HS = (long long)NH * D;
  const uint16_t* base = qkv + (long long)b * S * RS + h * D;
  StageRegs<S> rq, rd;
  const float* bqp = bias ? bias + h * D : nullptr;
  stage_load<S>(base, RS, bqp, rq);
  stage_load<S>(dctx + (long long)b * S * HS + h * D, HS, nullptr, rd);
  const int k0 = blockIdx.x * 128 + w * 16;
  const bool active = k0 < S;   // wave-uniform
  const int key = min(k0 + c, S - 1);
  uint4 kraw[2], vraw[2];   // this wave's key / value fragments, in flight with the stages
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    kraw[s] = ld16(base + (long long)key * RS + NH * D + 32 * s + 8 * g);
    vraw[s] = ld16(base + (long long)key * RS + 2 * NH * D + 32 * s + 8 * g);
  }
  const long long rbase = ((long long)b * NH + h) * S;
  // the per-query lse / D rows go to LDS with the stages (global float4 loads in
  // the query loop exposed their latency every iteration)
  float lsv = 0.f, dlv = 0.f;
  if (threadIdx.x < S) {
    lsv = lse[rbase + threadIdx.x];
    dlv = Dbuf[rbase + threadIdx.x];
  }
  stage_store<S>(rq, bqp != nullptr, Qs);
  stage_store<S>(rd, false, dOs);
  if (threadIdx.x < S) {
    Ls[threadIdx.x] = lsv;
    Dl[threadIdx.x] = dlv;
  }
  __syncthreads();
  if (!active) return;

  const float* bk = bias ? bias + (NH + h) * D : nullptr;
  const float* bv = bias ? bias + (2 * NH + h) * D : nullptr;
  bf16x8 kf[2], vf[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    kf[s] = as_frag(add_bias8(kraw[s], bk ? bk + 32 * s + 8 * g : nullptr));
    vf[s] = as_frag(add_bias8(vraw[s], bv ? bv + 32 * s + 8 * g : nullptr));
  }
  const float mk = mask ? mask[(long long)b * S + key] : 0.f;
  f32x4 dv[4], dk[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    dv[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    dk[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  for (int qb = 0; qb < NKB; ++qb) {
    float pd[8], ds[8];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int t = 2 * qb + tt;
      f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        sv = mfma16x16x32(ld_bf16x8(Qs + (16 * t + c) * KP + 32 * s + 8 * g), kf[s], sv);
        dp = mfma16x16x32(ld_bf16x8(dOs + (16 * t + c) * KP + 32 * s + 8 * g), vf[s], dp);
      }
      const float4 L4 = *reinterpret_cast<const float4*>(Ls + 16 * t + 4 * g);
      const float4 D4 = *reinterpret_cast<const float4*>(Dl + 16 * t + 4 * g);
      const float Lq[4] = {L4.x, L4.y, L4.z, L4.w}, Ds[4] = {D4.x, D4.y, D4.z, D4.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = 16 * t + 4 * g + i;
        const float P = __expf(sv[i] * scale + mk - Lq[i]);
        const float kp = keepf(seed, (uint64_t)(rbase + q) * S + key, thresh, inv_keep);
        pd[4 * tt + i] = P * kp;
        ds[4 * tt + i] = P * (dp[i] * kp - Ds[i]);
      }
    }
    const bf16x8 ap = pack8(pd), as = pack8(ds);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      dv[u] = mfma16x16x32(ap, ld_tr_pair(dOs, 32 * qb, 16 * u, l), dv[u]);
      dk[u] = mfma16x16x32(as, ld_tr_pair(Qs, 32 * qb, 16 * u, l), dk[u]);
    }
  }
  // lane holds dV/dK[key k0 + 4g + i][d 16u + c]
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint16_t* rowp = dqkv + ((long long)b * S + k0 + 4 * g + i) * RS + h * D + c;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      rowp[NH * D + 16 * u] = f2bf(dk[u][i] * scale);
      rowp[2 * NH * D + 16 * u] = f2bf(dv[u][i]);
    }
  }
  if (bpart != nullptr) {
    // k / v-bias gradient partials: this wave's 16 keys (4 per lane x the 4 lane
    // groups g) summed per dimension d = 16u + c
    float* pr = bpart + ((long long)b * (S / 16) + k0 / 16) * RS + h * D + c;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float sk = (dk[u][0] + dk[u][1]) + (dk[u][2] + dk[u][3]);
      float sv = (dv[u][0] + dv[u][1]) + (dv[u][2] + dv[u][3]);
      sk += __shfl_xor(sk, 16, 64);
      sk += __shfl_xor(sk, 32, 64);
      sv += __shfl_xor(sv, 16, 64);
      sv += __shfl_xor(sv, 32, 64);
      if (g == 0) {
        pr[NH * D + 16 * u] = sk * scale;
        pr[2 * NH * D + 16 * u] = sv;
      }
    }
  }
}

// S <= 128: the whole backward of one (batch, head) in ONE workgroup -- phase 1
// is attn_bwd_dq's work (wave w: queries 16w..16w+15; D and lse of every query
// go to LDS instead of a global round trip), phase 2 attn_bwd_dkv's (wave w:
// keys 16w..16w+15) on the Q / dO / K / V images phase 1 already staged: one
// staging pass and one launch instead of two of each.  Same MFMA order per
// output as the two-kernel path.
template <int NKB>
__global__ __launch_bounds__(512) void attn_bwd_fused(const uint16_t* __restrict__ qkv, const float* __restrict__ bias,
                                                      const float* __restrict__ mask, const uint16_t* __restrict__ ctx,
                                                      const uint16_t* __restrict__ dctx, const float* __restrict__ lse,
                                                      uint16_t* __restrict__ dqkv, int NH, float scale, uint32_t thresh,
                                                      float inv_keep, uint64_t seed, float* __restrict__ bpart) {
  constexpr int S = 32 * NKB;
  static_assert(S <= 128, "one workgroup per (batch, head)");
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  uint16_t* Ks = lds;                    // [S][KP] each; all four also read transposed (ld_tr_pair)
  uint16_t* Vs = lds + S * KP;
  uint16_t* Qs = lds + 2 * S * KP;
  uint16_t* dOs = lds + 3 * S * KP;
  float* Ls = reinterpret_cast<float*>(lds + 4 * S * KP);   // [S] lse of every query row
  float* Dl = Ls + S;                                        // [S] rowsum(dO * O)
  const int b = blockIdx.z, h = blockIdx.y;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, c = l & 15;
  const long long RS = 3LL * NH * D, HS = (long long)NH * D;
  const uint16_t* base = qkv + (long long)b * S * RS + h * D;
  const float* bq = bias ? bias + h * D : nullptr;
  const float* bkp = bias ? bias + (NH + h) * D : nullptr;
  const float* bvp = bias ? bias + (2 * NH + h) * D : nullptr;
  StageRegs<S> rk, rv, rq, rd;
  stage_load<S>(base + NH * D, RS, bkp, rk);
  stage_load<S>(base + 2 * NH * D, RS, bvp, rv);
  stage_load<S>(base, RS, bq, rq);
  stage_load<S>(dctx + (long long)b * S * HS + h * D, HS, nullptr, rd);
  const bool active = w * 16 < S;   // wave-uniform
  const int q = min(w * 16 + c, S - 1);
  const long long rbase = ((long long)b * NH + h) * S;
  // O rows for D = rowsum(dO * O), lse: in flight with the stages
  const uint16_t* orow = ctx + ((long long)b * S + q) * HS + h * D + 16 * g;
  const uint4 ov0 = ld16(orow), ov1 = ld16(orow + 8);
  const float L = lse[rbase + q];
  stage_store<S>(rk, bkp != nullptr, Ks);
  stage_store<S>(rv, bvp != nullptr, Vs);
  stage_store<S>(rq, bq != nullptr, Qs);
  stage_store<S>(rd, false, dOs);
  __syncthreads();

  // ---- phase 1: dQ of this wave's 16 queries, D and lse to LDS
  if (active) {
    bf16x8 bqf[2], bdo[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bqf[s] = ld_bf16x8(Qs + q * KP + 32 * s + 8 * g);
      bdo[s] = ld_bf16x8(dOs + q * KP + 32 * s + 8 * g);
    }
    float dsum = 0.f;
    {
      const uint4 dv0 = *reinterpret_cast<const uint4*>(dOs + q * KP + 16 * g);
      const uint4 dv1 = *reinterpret_cast<const uint4*>(dOs + q * KP + 16 * g + 8);
      const uint32_t a[8] = {ov0.x, ov0.y, ov0.z, ov0.w, ov1.x, ov1.y, ov1.z, ov1.w};
      const uint32_t d8[8] = {dv0.x, dv0.y, dv0.z, dv0.w, dv1.x, dv1.y, dv1.z, dv1.w};
#pragma unroll
      for (int j = 0; j < 8; ++j)
        dsum += bf2f(a[j] & 0xffff) * bf2f(d8[j] & 0xffff) + bf2f(a[j] >> 16) * bf2f(d8[j] >> 16);
    }
    dsum += __shfl_xor(dsum, 16, 64);
    dsum += __shfl_xor(dsum, 32, 64);
    if (g == 0) {
      Dl[q] = dsum;
      Ls[q] = L;
    }
    const uint64_t ebase = (uint64_t)(rbase + q) * S;
    f32x4 acc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
    for (int kb = 0; kb < NKB; ++kb) {
      float f[8];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const int t = 2 * kb + tt;
        f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          sv = mfma16x16x32(ld_bf16x8(Ks + (16 * t + c) * KP + 32 * s + 8 * g), bqf[s], sv);
          dp = mfma16x16x32(ld_bf16x8(Vs + (16 * t + c) * KP + 32 * s + 8 * g), bdo[s], dp);
        }
        float4 mk = mask ? *reinterpret_cast<const float4*>(mask + (long long)b * S + 16 * t + 4 * g)
                         : float4{0.f, 0.f, 0.f, 0.f};
        const float m4[4] = {mk.x, mk.y, mk.z, mk.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key = 16 * t + 4 * g + i;
          const float P = __expf(sv[i] * scale + m4[i] - L);
          const float dpd = dp[i] * keepf(seed, ebase + key, thresh, inv_keep);
          f[4 * tt + i] = P * (dpd - dsum);
        }
      }
      const bf16x8 dsb = pack8(f);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] = mfma16x16x32(ld_tr_pair(Ks, 32 * kb, 16 * u, l), dsb, acc[u]);
    }
    uint16_t* dq = dqkv + ((long long)b * S + q) * RS + h * D;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      *reinterpret_cast<uint2*>(dq + 16 * u + 4 * g) =
          uint2{pack2bf(acc[u][0] * scale, acc[u][1] * scale), pack2bf(acc[u][2] * scale, acc[u][3] * scale)};
    if (bpart != nullptr) {
      float cs[16];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float v = acc[u][j] * scale;
          v += __shfl_xor(v, 1, 64);
          v += __shfl_xor(v, 2, 64);
          v += __shfl_xor(v, 4, 64);
          v += __shfl_xor(v, 8, 64);
          cs[4 * u + j] = v;
        }
      if (c == 0) {
        float* pr = bpart + ((long long)b * (S / 16) + w) * RS + h * D;
#pragma unroll
        for (int u = 0; u < 4; ++u)
          *reinterpret_cast<float4*>(pr + 16 * u + 4 * g) = float4{cs[4 * u], cs[4 * u + 1], cs[4 * u + 2], cs[4 * u + 3]};
      }
    }
  }
  __syncthreads();

  // ---- phase 2: dK, dV of this wave's 16 keys over every query
  if (!active) return;
  const int k0 = w * 16;
  const int key = k0 + c;
  bf16x8 kf[2], vf[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    kf[s] = ld_bf16x8(Ks + key * KP + 32 * s + 8 * g);
    vf[s] = ld_bf16x8(Vs + key * KP + 32 * s + 8 * g);
  }
  const float mk = mask ? mask[(long long)b * S + key] : 0.f;
  f32x4 dv[4], dk[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    dv[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    dk[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  for (int qb = 0; qb < NKB; ++qb) {
    float pd[8], ds[8];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int t = 2 * qb + tt;
      f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        sv = mfma16x16x32(ld_bf16x8(Qs + (16 * t + c) * KP + 32 * s + 8 * g), kf[s], sv);
        dp = mfma16x16x32(ld_bf16x8(dOs + (16 * t + c) * KP + 32 * s + 8 * g), vf[s], dp);
      }
      const float4 L4 = *reinterpret_cast<const float4*>(Ls + 16 * t + 4 * g);
      const float4 D4 = *reinterpret_cast<const float4*>(Dl + 16 * t + 4 * g);
      const float Lq[4] = {L4.x, L4.y, L4.z, L4.w}, Ds[4] = {D4.x, D4.y, D4.z, D4.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int qq = 16 * t + 4 * g + i;
        const float P = __expf(sv[i] * scale + mk - Lq[i]);
        const float kp = keepf(seed, (uint64_t)(rbase + qq) * S + key, thresh, inv_keep);
        pd[4 * tt + i] = P * kp;
        ds[4 * tt + i] = P * (dp[i] * kp - Ds[i]);
      }
    }
    const bf16x8 ap = pack8(pd), as = pack8(ds);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      dv[u] = mfma16x16x32(ap, ld_tr_pair(dOs, 32 * qb, 16 * u, l), dv[u]);
      dk[u] = mfma16x16x32(as, ld_tr_pair(Qs, 32 * qb, 16 * u, l), dk[u]);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint16_t* rowp = dqkv + ((long long)b * S + k0 + 4 * g + i) * RS + h * D + c;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      rowp[NH * D + 16 * u] = f2bf(dk[u][i] * scale);
      rowp[2 * NH * D + 16 * u] = f2bf(dv[u][i]);
    }
  }
  if (bpart != nullptr) {
    float* pr = bpart + ((long long)b * (S / 16) + k0 / 16) * RS + h * D + c;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float sk = (dk[u][0] + dk[u][1]) + (dk[u][2] + dk[u][3]);
      float sv = (dv[u][0] + dv[u][1]) + (dv[u][2] + dv[u][3]);
      sk += __shfl_xor(sk, 16, 64);
      sk += __shfl_xor(sk, 32, 64);
      sv += __shfl_xor(sv, 16, 64);
      sv += __shfl_xor(sv, 32, 64);
      if (g == 0) {
        pr[NH * D + 16 * u] = sk * scale;
        pr[2 * NH * D + 16 * u] = sv;
      }
    }
  }
}

}  // namespace attn
}  // namespace dtfk

using namespace dtfk::attn;

static inline uint32_t attn_thresh(float p) {
  if (p <= 0.f) return 0u;
  double t = (double)p * 4294967296.0;
  return t >= 4294967295.0 ? 4294967295u : (uint32_t)t;
}

// >64 KB dynamic LDS must be opted into once per kernel instantiation
template <typename K>
static hipError_t allow_lds(K kern, size_t lds) {
  return hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)lds);
}

extern "C" {

int dtfk_attn_supported(int S, int d) {
  const int n = S / 32;
  return d == D && S % 32 == 0 && (n == 1 || n == 2 || n == 4 || n == 6 || n == 8);
}

#define DTFK_ATTN_DISPATCH(S, MACRO) \
  switch ((S) / 32) {                \
    case 1: MACRO(1); break;         \
    case 2: MACRO(2); break;         \
    case 4: MACRO(4); break;         \
    case 6: MACRO(6); break;         \
    case 8: MACRO(8); break;         \
    default: return hipErrorInvalidValue; \
  }

hipError_t dtfk_attn_fwd(const void* qkv, const float* bias, const float* mask, void* ctx, float* lse, int B, int S,
                         int NH, float scale, float p, unsigned long long seed, hipStream_t st) {
  if (!dtfk_attn_supported(S, D)) return hipErrorInvalidValue;
  const dim3 grid((S + 127) / 128, NH, B);
  const float ik = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const size_t lds = (size_t)(2 * S * KP) * 2;
#define L_FWD(N)                                                                                                \
  {                                                                                                             \
    static hipError_t e = allow_lds(attn_fwd<N>, lds);                                                          \
    if (e != hipSuccess) return e;                                                                              \
    hipLaunchKernelGGL(attn_fwd<N>, grid, dim3(512), lds, st, (const uint16_t*)qkv, bias, mask, (uint16_t*)ctx, \
                       lse, NH, scale, attn_thresh(p), ik, (uint64_t)seed);                                     \
  }
  DTFK_ATTN_DISPATCH(S, L_FWD)
#undef L_FWD
  return hipGetLastError();
}

// dqkv [B, S, 3, NH, 64] is fully written; Dbuf [B, NH, S] fp32 scratch
hipError_t dtfk_attn_bwd(const void* qkv, const float* bias, const float* mask, const void* ctx, const void* dctx,
                         const float* lse, float* Dbuf, void* dqkv, int B, int S, int NH, float scale, float p,
                         unsigned long long seed, float* bpart, hipStream_t st) {
  // bpart (optional): [B * S / 16, 3 * NH * 64] fp32 partial column sums of dqkv
  // (the qkv bias gradient before its colsum_partials reduction)
  if (!dtfk_attn_supported(S, D)) return hipErrorInvalidValue;
  const dim3 grid((S + 127) / 128, NH, B);
  const float ik = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const uint32_t th = attn_thresh(p);
  const size_t lds_q = (size_t)(2 * S * KP) * 2;
  const size_t lds_kv = (size_t)(2 * S * KP) * 2 + 2 * S * sizeof(float);
  static const bool fused_ok = [] {
    const char* e = std::getenv("DTF_ATTN_BWD_FUSED");
    return e == nullptr || std::string(e) != "0";
  }();
  if (fused_ok && S <= 128) {
    const size_t lds_f = (size_t)(4 * S * KP) * 2 + 2 * S * sizeof(float);
    const dim3 gridf(1, NH, B);
#define L_BWDF(N)                                                                                                  \
  {                                                                                                                \
    static hipError_t e = allow_lds(attn_bwd_fused<N>, lds_f);                                                     \
    if (e != hipSuccess) return e;                                                                                 \
    hipLaunchKernelGGL(attn_bwd_fused<N>, gridf, dim3(512), lds_f, st, (const uint16_t*)qkv, bias, mask,           \
                       (const uint16_t*)ctx, (const uint16_t*)dctx, lse, (uint16_t*)dqkv, NH, scale, th, ik,       \
                       (uint64_t)seed, bpart);                                                                     \
  }
    switch (S / 32) {
      case 1: L_BWDF(1); break;
      case 2: L_BWDF(2); break;
      case 4: L_BWDF(4); break;
      default: return hipErrorInvalidValue;
    }
#undef L_BWDF
    return hipGetLastError();
  }
#define L_BWD(N)                                                                                                   \
  {                                                                                                                \
    static hipError_t e1 = allow_lds(attn_bwd_dq<N>, lds_q);                                                       \
    static hipError_t e2 = allow_lds(attn_bwd_dkv<N>, lds_kv);                                                     \
    if (e1 != hipSuccess) return e1;                                                                               \
    if (e2 != hipSuccess) return e2;                                                                               \
    hipLaunchKernelGGL(attn_bwd_dq<N>, grid, dim3(512), lds_q, st, (const uint16_t*)qkv, bias, mask,               \
                       (const uint16_t*)ctx, (const uint16_t*)dctx, lse, Dbuf, (uint16_t*)dqkv, NH, scale, th, ik, \
                       (uint64_t)seed, bpart);                                                                     \
    hipLaunchKernelGGL(attn_bwd_dkv<N>, grid, dim3(512), lds_kv, st, (const uint16_t*)qkv, bias, mask,             \
                       (const uint16_t*)dctx, lse, Dbuf, (uint16_t*)dqkv, NH, scale, th, ik, (uint64_t)seed, bpart); \
  }
  DTFK_ATTN_DISPATCH(S, L_BWD)
#undef L_BWD
  return hipGetLastError();
}

}  // extern "C"
