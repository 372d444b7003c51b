// Reached by: ops.linear_act / ops.matmul (Wide&Deep tower, compat MatMul); tests/test_ops_gpu.py
// Generic MFMA GEMM with a fused epilogue: C = act(alpha * op(A) op(B) + bias).
// bf16 (or mixed) operands: 16x16x32 bf16 MFMA below; fp32 x fp32 with an fp32
// output: the exact-f32 MFMA kernel at the end (no silent bf16 rounding).
//
// Backs `ops.linear_act` (forward: bias + {none, relu, sigmoid, tanh, gelu}),
// its backward GEMMs (dX = dZ W^T with transB, dW = X^T dZ with transA) and the
// dense layers of the Wide&Deep / BERT / ResNet heads.  The reference graph's
// matmul + bias + sigmoid (example.py:95-97) is exactly this op.
//
// Tiling for CDNA4: 256-thread workgroup = 4 waves (2x2), 64x64 output tile,
// each wave 32x32 = 2x2 MFMA 16x16x32 bf16 tiles, K-step 32.  Operands are
// read in any of fp32 / bf16 with any transpose, converted to bf16 and staged
// in LDS as [row][k] (A) and [col][k] (B) with a +8 element pad so every MFMA
// fragment is one conflict-free 16-byte ds_read (bf16 path).  Interior runs of 8 elements
// are one (bf16) or two (fp32) 16-byte loads; edge runs fall back to clamped,
// masked scalar loads with no per-element branch (see mlp_step.hip for why),
// and the next K-tile is prefetched into registers while the current one is
// multiplied.  Block ids
// are remapped so consecutive tiles of one output row band land on one XCD
// (shared A panel in that XCD's L2).
#include "common.h"

#include <algorithm>

namespace dtfk {
namespace gemm {

constexpr int BM = 64, BN = 64, BK = 32, LDK = BK + 8;

enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_SIGMOID = 2, ACT_TANH = 3, ACT_GELU = 4 };

__device__ __forceinline__ float apply_act(float z, int act) {
  switch (act) {
    case ACT_RELU: return fmaxf(z, 0.f);
    case ACT_SIGMOID: return 1.f / (1.f + __expf(-z));
    case ACT_TANH: return tanhf(z);
    case ACT_GELU: return 0.5f * z * (1.f + erff(z * 0.70710678118654752f));
    default: return z;
  }
}

template <bool BF16>
__device__ __forceinline__ float ld_elem(const void* p, size_t i) {
  if constexpr (BF16) return bf2f(reinterpret_cast<const uint16_t*>(p)[i]);
  else return reinterpret_cast<const float*>(p)[i];
}

// Loads this thread's share of a 64 x 32 operand tile into registers.
// Tile element (r, k) lives at  base[(r0 + r) * ld + k0 + k]  when K is the
// contiguous dimension (KCONT), else at base[(k0 + k) * ld + r0 + r].
// 256 threads x 8 elements = 2048 = 64 x 32.
template <bool BF16, bool KCONT>
__device__ __forceinline__ void load_tile(const void* base, int ld, int R, int K, int r0, int k0,
                                          float v[8]) {
  const int t = threadIdx.x;
  {
    // interior fast path: the thread's 8 elements are contiguous in memory
    // (along k when KCONT, along r otherwise) -> one 16-byte (bf16) or two
    // 16-byte (fp32) loads instead of 8 clamped scalar loads
    int outer, inner;
    bool full;
    if constexpr (KCONT) {
      outer = r0 + (t >> 2); inner = k0 + (t & 3) * 8;
      full = outer < R && inner + 8 <= K;
    } else {
      outer = k0 + (t >> 3); inner = r0 + (t & 7) * 8;
      full = outer < K && inner + 8 <= R;
    }
    const size_t off = (size_t)outer * ld + inner;
    if (full && ((reinterpret_cast<uintptr_t>(base) + off * (BF16 ? 2 : 4)) & 15) == 0) {
      if constexpr (BF16) {
        const uint4 u = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(base) + off);
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) { v[2 * j] = bf2f(w[j] & 0xFFFF); v[2 * j + 1] = bf2f(w[j] >> 16); }
      } else {
        const float4 a = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(base) + off);
        const float4 b = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(base) + off + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
      }
      return;
    }
  }
  if constexpr (KCONT) {
    const int r = t >> 2, kk = (t & 3) * 8;  // 8 consecutive k of row r
    const int rr = min(r0 + r, R - 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = min(k0 + kk + j, K - 1);
      const float x = ld_elem<BF16>(base, (size_t)rr * ld + k);
      v[j] = (r0 + r < R && k0 + kk + j < K) ? x : 0.f;
    }
  } else {
    const int k = t >> 3, rr8 = (t & 7) * 8;  // 8 consecutive r of k-row k
    const int kc = min(k0 + k, K - 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = min(r0 + rr8 + j, R - 1);
      const float x = ld_elem<BF16>(base, (size_t)kc * ld + r);
      v[j] = (r0 + rr8 + j < R && k0 + k < K) ? x : 0.f;
    }
  }
}

template <bool KCONT>
__device__ __forceinline__ void store_tile(uint16_t* s, const float v[8]) {
  const int t = threadIdx.x;
  if constexpr (KCONT) {
    const int r = t >> 2, kk = (t & 3) * 8;
    *reinterpret_cast<uint4*>(&s[r * LDK + kk]) =
        make_uint4(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7]));
  } else {
    const int k = t >> 3, rr8 = (t & 7) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) s[(rr8 + j) * LDK + k] = f2bf(v[j]);
  }
}

// C[M,N] = act(alpha * A'[M,K] B'[K,N] + bias[N]) (+ beta * C_in when accumulate)
// A' = A (row-major [M,K], lda) or A^T (A is [K,M]);  B' = B ([K,N]) or B^T ([N,K]).
template <bool ABF, bool BBF, bool TA, bool TB, bool OBF>
__global__ __launch_bounds__(256) void gemm_bias_act(
    const void* __restrict__ A, int lda, const void* __restrict__ Bm, int ldb,
    void* __restrict__ C, int ldc, float* __restrict__ Zout, const float* __restrict__ bias,
    int M, int N, int K, float alpha, float beta, int act, int kchunk) {
  __shared__ __attribute__((aligned(16))) uint16_t As[BM * LDK];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[BN * LDK];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lh = lane >> 4;
  const int wr = wave >> 1, wc = wave & 1;

  // XCD-aware remap: hardware deals block ids round-robin over 8 XCDs; give
  // each XCD a contiguous run of tiles (bijective for any grid size).
  const int nt_n = (N + BN - 1) / BN;
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig % 8, q = nwg / 8, rem = nwg % 8;
  const int wg = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + orig / 8;
  const int m0 = (wg / nt_n) * BM, n0 = (wg % nt_n) * BN;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // split-K (gridDim.y > 1): this block contracts k in [kb, ke) only
  const int kb = blockIdx.y * kchunk, ke = min(K, kb + kchunk);
  float va[8], vb[8];
  // A' tile rows = m, K contiguous iff !TA;  B' tile rows = n, K contiguous iff TB
  load_tile<ABF, !TA>(A, lda, M, ke, m0, kb, va);
  load_tile<BBF, TB>(Bm, ldb, N, ke, n0, kb, vb);
  for (int k0 = kb; k0 < ke; k0 += BK) {
    __syncthreads();
    store_tile<!TA>(As, va);
    store_tile<TB>(Bs, vb);
    __syncthreads();
    if (k0 + BK < ke) {  // prefetch next K tile into registers (branch is uniform)
      load_tile<ABF, !TA>(A, lda, M, ke, m0, k0 + BK, va);
      load_tile<BBF, TB>(Bm, ldb, N, ke, n0, k0 + BK, vb);
    }
    bf16x8 fa[2], fb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) fa[i] = ld_bf16x8(&As[(wr * 32 + i * 16 + lr) * LDK + lh * 8]);
#pragma unroll
    for (int j = 0; j < 2; ++j) fb[j] = ld_bf16x8(&Bs[(wc * 32 + j * 16 + lr) * LDK + lh * 8]);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mfma16x16x32(fa[i], fb[j], acc[i][j]);
  }

  // epilogue: lane holds rows 4*lh + r, column lr of each 16x16 tile
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wc * 32 + j * 16 + lr;
    const float bv = (bias != nullptr && n < N) ? bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr * 32 + i * 16 + 4 * lh + r;
        if (m < M && n < N) {
          if (gridDim.y > 1) {  // split-K: linear epilogue (host-checked), partial sums meet in fp32 C
            atomicAdd(reinterpret_cast<float*>(C) + (size_t)m * ldc + n,
                      alpha * acc[i][j][r] + (blockIdx.y == 0 ? bv : 0.f));
            continue;
          }
          float z = alpha * acc[i][j][r] + bv;
          const size_t o = (size_t)m * ldc + n;
          if (beta != 0.f) z += beta * (OBF ? bf2f(reinterpret_cast<uint16_t*>(C)[o]) : reinterpret_cast<float*>(C)[o]);
          if (Zout != nullptr) Zout[o] = z;
          const float y = apply_act(z, act);
          if constexpr (OBF) reinterpret_cast<uint16_t*>(C)[o] = f2bf(y);
          else reinterpret_cast<float*>(C)[o] = y;
        }
      }
    }
  }
}


// ---------------------------------------------------------------------------
// fp32 x fp32: exact-f32 MFMA path (v_mfma_f32_16x16x4_f32, one rounding per
// product, fp32 accumulate) -- fp32 operands are never rounded to bf16.  Same
// 64x64 tile / 2x2 waves / epilogue / split-K / XCD remap as the bf16 kernel;
// BK = 16, operands staged in LDS as fp32 [row][k] with a stride of 20 floats
// (16-byte rows for ds_write_b128; the 16 rows x 4 k of one fragment read land
// on 64 distinct banks).  A fragment (lane l): A'[row l&15][k = 4s + (l>>4)].
constexpr int FBK = 16, FLD = 20;

template <bool KCONT>
__device__ __forceinline__ void load_tile_f32(const float* base, int ld, int R, int K, int r0, int k0, float v[4]) {
  // 64 x 16 tile, 256 threads x 4 elements; KCONT: 4 consecutive k of one row,
  // else 4 consecutive rows of one k
  const int t = threadIdx.x;
  int outer, inner;
  bool full;
  if constexpr (KCONT) {
    outer = r0 + (t >> 2); inner = k0 + (t & 3) * 4;
    full = outer < R && inner + 4 <= K;
  } else {
    outer = k0 + (t >> 4); inner = r0 + (t & 15) * 4;
    full = outer < K && inner + 4 <= R;
  }
  const size_t off = (size_t)outer * ld + inner;
  if (full && ((reinterpret_cast<uintptr_t>(base + off) & 15) == 0)) {
    const float4 a = *reinterpret_cast<const float4*>(base + off);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    return;
  }
  const int oc = min(outer, (KCONT ? R : K) - 1);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int ic = min(inner + j, (KCONT ? K : R) - 1);
    const float x = base[(size_t)oc * ld + ic];
    v[j] = (outer < (KCONT ? R : K) && inner + j < (KCONT ? K : R)) ? x : 0.f;
  }
}

template <bool KCONT>
__device__ __forceinline__ void store_tile_f32(float* s, const float v[4]) {
  const int t = threadIdx.x;
  if constexpr (KCONT) {
    *reinterpret_cast<float4*>(&s[(t >> 2) * FLD + (t & 3) * 4]) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    const int k = t >> 4, r4 = (t & 15) * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) s[(r4 + j) * FLD + k] = v[j];
  }
}

template <bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_f32_bias_act(
    const float* __restrict__ A, int lda, const float* __restrict__ Bm, int ldb, float* __restrict__ C, int ldc,
    float* __restrict__ Zout, const float* __restrict__ bias, int M, int N, int K, float alpha, float beta, int act,
    int kchunk) {
  __shared__ __attribute__((aligned(16))) float As[BM * FLD];
  __shared__ __attribute__((aligned(16))) float Bs[BN * FLD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lh = lane >> 4;
  const int wr = wave >> 1, wc = wave & 1;
  const int nt_n = (N + BN - 1) / BN;
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig % 8, q = nwg / 8, rem = nwg % 8;
  const int wg = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + orig / 8;
  const int m0 = (wg / nt_n) * BM, n0 = (wg % nt_n) * BN;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int kb = blockIdx.y * kchunk, ke = min(K, kb + kchunk);
  float va[4], vb[4];
  load_tile_f32<!TA>(A, lda, M, ke, m0, kb, va);
  load_tile_f32<TB>(Bm, ldb, N, ke, n0, kb, vb);
  for (int k0 = kb; k0 < ke; k0 += FBK) {
    __syncthreads();
    store_tile_f32<!TA>(As, va);
    store_tile_f32<TB>(Bs, vb);
    __syncthreads();
    if (k0 + FBK < ke) {
      load_tile_f32<!TA>(A, lda, M, ke, m0, k0 + FBK, va);
      load_tile_f32<TB>(Bm, ldb, N, ke, n0, k0 + FBK, vb);
    }
#pragma unroll
    for (int s = 0; s < FBK / 4; ++s) {
      float fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = As[(wr * 32 + i * 16 + lr) * FLD + 4 * s + lh];
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = Bs[(wc * 32 + j * 16 + lr) * FLD + 4 * s + lh];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wc * 32 + j * 16 + lr;
    const float bv = (bias != nullptr && n < N) ? bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr * 32 + i * 16 + 4 * lh + r;
        if (m < M && n < N) {
          if (gridDim.y > 1) {
            atomicAdd(C + (size_t)m * ldc + n, alpha * acc[i][j][r] + (blockIdx.y == 0 ? bv : 0.f));
            continue;
          }
          float z = alpha * acc[i][j][r] + bv;
          const size_t o = (size_t)m * ldc + n;
          if (beta != 0.f) z += beta * C[o];
          if (Zout != nullptr) Zout[o] = z;
          C[o] = apply_act(z, act);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// N == 1 (matrix-vector) fp32 products -- the W&D tower's 256 -> 1 head and its
// weight gradient went through 64x64 MFMA tiles with one useful column (16-19
// us for 4 MB of reads).  b(k) = B[k * ldbk].
// Row form (A' rows contiguous): one wave per output row, lanes over k.
__global__ __launch_bounds__(256) void gemv_rows_f32(const float* __restrict__ A, int lda,
                                                     const float* __restrict__ Bv, int ldbk, float* __restrict__ C,
                                                     int ldc, float* __restrict__ Zout, const float* __restrict__ bias,
                                                     int M, int K, float alpha, float beta, int act) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= M) return;   // wave-uniform
  const float* a = A + (size_t)i * lda;
  float s0 = 0.f, s1 = 0.f;
  int k = lane;
  for (; k + 64 < K; k += 128) {
    s0 += a[k] * Bv[(size_t)k * ldbk];
    s1 += a[k + 64] * Bv[(size_t)(k + 64) * ldbk];
  }
  if (k < K) s0 += a[k] * Bv[(size_t)k * ldbk];
  const float t = wave_sum(s0 + s1);
  if (lane == 0) {
    float z = alpha * t + (bias != nullptr ? bias[0] : 0.f);
    const size_t o = (size_t)i * ldc;
    if (beta != 0.f) z += beta * C[o];
    if (Zout != nullptr) Zout[o] = z;
    C[o] = apply_act(z, act);
  }
}

// Column form (A' = A^T, A stored [K, M]): out[i] = sum_k A[k, i] b(k), a
// b-weighted column sum -- 64 columns x 4 k-groups per block, grid.y k-chunks
// meeting by atomics (linear epilogue only; C pre-zeroed or accumulated into).
__global__ __launch_bounds__(256) void gemv_cols_f32(const float* __restrict__ A, int lda,
                                                     const float* __restrict__ Bv, int ldbk, float* __restrict__ C,
                                                     int ldc, const float* __restrict__ bias, int M, int K,
                                                     float alpha, int kchunk) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), g = threadIdx.x >> 6;
  const int k0 = blockIdx.y * kchunk, k1 = min(K, k0 + kchunk);
  float s = 0.f;
  if (c < M)
    for (int k = k0 + g; k < k1; k += 4) s += A[(size_t)k * lda + c] * Bv[(size_t)k * ldbk];
  red[g][threadIdx.x & 63] = s;
  __syncthreads();
  if (g == 0 && c < M) {
    const float t = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    atomicAdd(C + (size_t)c * ldc, alpha * t + (blockIdx.y == 0 && bias != nullptr ? bias[0] : 0.f));
  }
}
}  // namespace gemm
}  // namespace dtfk

extern "C" hipError_t dtfk_gemm(const void* A, int a_bf16, int lda, int transA, const void* B,
                                int b_bf16, int ldb, int transB, void* C, int c_bf16, int ldc,
                                float* Z, const float* bias, int M, int N, int K, float alpha,
                                float beta, int act, hipStream_t stream) {
  using namespace dtfk::gemm;
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (tiles == 0) return hipSuccess;
  if (!a_bf16 && !b_bf16 && !c_bf16 && N == 1) {
    // matrix-vector forms (b(k) = B[k * ldbk]: B is [K, 1] or [1, K])
    const float* Af = static_cast<const float*>(A);
    const float* Bf = static_cast<const float*>(B);
    float* Cf = static_cast<float*>(C);
    const int ldbk = transB ? 1 : ldb;
    if (!transA) {
      hipLaunchKernelGGL(gemv_rows_f32, dim3((M + 3) / 4), dim3(256), 0, stream, Af, lda, Bf, ldbk, Cf, ldc, Z, bias,
                         M, K, alpha, beta, act);
      return hipGetLastError();
    }
    if (act == ACT_NONE && Z == nullptr && (beta == 0.f || beta == 1.f)) {
      const int bx = (M + 63) / 64;
      int gy = std::max(1, std::min((K + 63) / 64, 512 / bx));
      const int kc = (K + gy - 1) / gy;
      gy = (K + kc - 1) / kc;
      if (beta == 0.f) {
        const hipError_t e = dtfk::zero2d_f32(Cf, ldc, M, 1, stream);
        if (e != hipSuccess) return e;
      }
      hipLaunchKernelGGL(gemv_cols_f32, dim3(bx, gy), dim3(256), 0, stream, Af, lda, Bf, ldbk, Cf, ldc, bias, M, K,
                         alpha, kc);
      return hipGetLastError();
    }
  }
  // Split-K when the output has too few 64x64 tiles to fill 256 CUs and K is
  // long -- the weight gradients X^T dZ (M x N = fan_in x fan_out, K = batch).
  // Only for a linear fp32 epilogue: the partial products meet by atomics.
  int split = 1, kchunk = K;
  if (act == ACT_NONE && Z == nullptr && !c_bf16 && (beta == 0.f || beta == 1.f) && tiles < 256 && K >= 512) {
    split = (512 + tiles - 1) / tiles;
    if (split > K / 256) split = K / 256;
    if (split > 1) {
      kchunk = ((K + split - 1) / split + BK - 1) / BK * BK;
      split = (K + kchunk - 1) / kchunk;
    }
    if (split <= 1) { split = 1; kchunk = K; }
  }
  if (split > 1 && beta == 0.f) {
    const hipError_t e = dtfk::zero2d_f32(static_cast<float*>(C), ldc, M, N, stream);
    if (e != hipSuccess) return e;
  }
  const dim3 grid(tiles, split), block(256);
  if (!a_bf16 && !b_bf16 && !c_bf16) {
    // fp32 operands stay fp32 (exact-f32 MFMA); split-K chunks on the fp32 K-step
    if (split > 1) kchunk = (kchunk + FBK - 1) / FBK * FBK;
    const float* Af = static_cast<const float*>(A);
    const float* Bf = static_cast<const float*>(B);
    float* Cf = static_cast<float*>(C);
#define DTFK_F(TA, TB) \
  hipLaunchKernelGGL((gemm_f32_bias_act<TA, TB>), grid, block, 0, stream, Af, lda, Bf, ldb, Cf, ldc, Z, bias, M, N, \
                     K, alpha, beta, act, kchunk)
    if (transA) {
      if (transB) DTFK_F(true, true); else DTFK_F(true, false);
    } else {
      if (transB) DTFK_F(false, true); else DTFK_F(false, false);
    }
#undef DTFK_F
    return hipGetLastError();
  }
#define DTFK_G(AB, BB, TA, TB, OB)                                                               \
  hipLaunchKernelGGL((gemm_bias_act<AB, BB, TA, TB, OB>), grid, block, 0, stream, A, lda, B, ldb, \
                     C, ldc, Z, bias, M, N, K, alpha, beta, act, kchunk)
#define DTFK_G_OB(AB, BB, TA, TB) \
  if (c_bf16) DTFK_G(AB, BB, TA, TB, true); else DTFK_G(AB, BB, TA, TB, false)
#define DTFK_G_TB(AB, BB, TA) \
  if (transB) { DTFK_G_OB(AB, BB, TA, true); } else { DTFK_G_OB(AB, BB, TA, false); }
#define DTFK_G_TA(AB, BB) \
  if (transA) { DTFK_G_TB(AB, BB, true); } else { DTFK_G_TB(AB, BB, false); }
  if (a_bf16) {
    if (b_bf16) { DTFK_G_TA(true, true); } else { DTFK_G_TA(true, false); }
  } else {
    if (b_bf16) { DTFK_G_TA(false, true); } else { DTFK_G_TA(false, false); }
  }
#undef DTFK_G_TA
#undef DTFK_G_TB
#undef DTFK_G_OB
#undef DTFK_G
  return hipGetLastError();
}
