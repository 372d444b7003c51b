// Reached by: ops/big_gemm.py (BERT-base linears, ResNet-50 1x1 convs); tests/test_gemm_big_gpu.py
// Large-tile bf16 MFMA GEMM for the transformer-size products (BERT-base:
// T = B*S = 16384 token rows, 768 / 2304 / 3072 wide):
//
//   C[M,N] = act(alpha * A'[M,K] B'[K,N] + bias[N]) (+ beta * C)      fp32 accumulate
//
// A' = A (row-major [M,K], K contiguous) or A^T (A stored [K,M], M contiguous);
// B' = B^T (B stored [N,K], K contiguous) or B (stored [K,N], N contiguous).
// That covers all three products of a linear layer without a transpose copy:
// forward y = x W^T (K-contig x K-contig), input gradient dX = dY W (K-contig x
// N-contig) and weight gradient dW = dY^T X (M-contig x N-contig).
//
// CDNA4 design (cdna_hip_programming.md s5):
//  * 512-thread workgroup = 8 waves (2 along M x 4 along N), output tile BM x 256
//    (BM = 256: each wave owns 128x64 = 8x4 MFMA 16x16x32 accumulators, 128
//    VGPRs of fp32), K-step 64.
//  * Operands go HBM -> LDS with LDS-DMA (`global_load_lds_dwordx4`), never
//    through VGPRs: each wave instruction fills 1 KiB of lane-linear LDS, so the
//    bank-conflict swizzle is applied to the per-lane GLOBAL source address and
//    undone on the read (rule 21: linear destination, swizzled source + read).
//  * An S-stage ring of BK-deep K tiles in ONE __shared__ array (forward: BK 32,
//    S 5 = 160 KiB at BM = 256; transposed-read layouts: BK 64, S 2): while
//    tile t is multiplied, tiles t+1 .. t+S-1 are in flight; the wait is a
//    counted `s_waitcnt vmcnt(N)` and a raw s_barrier, so the prefetch
//    survives the barrier (a workgroup LDS fence would drain it: the DMA is a
//    pending LDS write on the vector-memory counter).
//  * Measured: the round-2 single-phase loop (rocprofv3 PMC, 16384x3072x768:
//    ~8 B/clk/CU of LDS-DMA fill, 77 % L2 hit rate, ~25 % MFMA utilisation) was
//    operand-delivery bound at ~0.5x hipBLASLt; the 8-phase schedule (gemm_8ph)
//    runs BERT-base's forward / input-gradient shapes at 0.93-1.09x hipBLASLt
//    and its weight gradients at 0.82-1.03x (profiles/gemm_8ph_r3.txt).  Models
//    pick per shape with hysteresis (ops/big_gemm.py: use_native keeps this
//    kernel unless hipBLASLt wins by more than DTF_BIG_GEMM_MARGIN).
//  * K-contiguous images are [rows][BK] with a 16-byte chunk XOR that puts the
//    16 lanes of a ds_read_b128 group on 16 distinct slots of a bank row.
//  * M/N-contiguous images are [BK k][rows] and are read with the hardware
//    transpose `ds_read_b64_tr_b16` (two per fragment); 32-byte groups XOR
//    (k&3 | (k>>3&1)<<2) keep the 8 k-rows of a 32-lane half on distinct banks.
//  * XCD-aware tile order (bijective remap): a row band's tiles share one L2.
//  * Split-K over gridDim.y for the few-tile, long-K weight gradients: fp32
//    partial tiles meet by atomics in C (which may already hold the gradient
//    to accumulate into -- beta = 1 is free).
// Shape contract (checked on the host): K % 64 == 0; 16-byte aligned bases and
// leading dimensions; an M/N-contiguous operand's M (or N) is a multiple of 8.
// Row/column tails are clamped (their products only reach unstored outputs).
#include "common.h"

#include <cstdlib>

namespace dtfk {
namespace gemm2 {

constexpr int BN = 256, NTHR = 512;
constexpr int KQ = 64;   // K granule of the shape contract / split-K chunks

typedef __attribute__((address_space(3))) void lvoid;
typedef __attribute__((address_space(1))) void gvoid;
typedef __attribute__((ext_vector_type(4))) short v4s;
typedef __attribute__((address_space(3))) v4s lds_v4s;

enum Act { ACT_NONE = 0, ACT_RELU = 1, ACT_SIGMOID = 2, ACT_TANH = 3, ACT_GELU = 4 };

// out of line: one call per output element keeps 128 inlined erff/tanhf
// copies out of every instantiation's epilogue
__device__ __attribute__((noinline)) float apply_act_slow(float z, int act) {
  switch (act) {
    case ACT_RELU: return fmaxf(z, 0.f);
    case ACT_SIGMOID: return 1.f / (1.f + __expf(-z));
    case ACT_TANH: return tanhf(z);
    case ACT_GELU: return 0.5f * z * (1.f + erff(z * 0.70710678118654752f));
    default: return z;
  }
}
__device__ __forceinline__ float gelu_fwd_f(float z) {
  float cdf, pdf;
  gelu_cdf_pdf(z, cdf, pdf);
  return z * cdf;
}
__device__ __forceinline__ float gelu_grad_f(float z) {
  float cdf, pdf;
  gelu_cdf_pdf(z, cdf, pdf);
  return fmaf(z, pdf, cdf);
}
// gelu'(z) for two values at once: the polynomial / scaling work as packed
// fp32 (v_pk_fma_f32 / v_pk_mul_f32 on float2), the rcp / exp per value --
// the fused GELU-backward epilogue is VALU-bound on this math
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu_grad2(f32x2 z) {
  const f32x2 x = f32x2{fabsf(z.x), fabsf(z.y)} * 0.70710678118654752f;
  const f32x2 d = x * 0.3275911f + 1.f;
  const f32x2 t = f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 poly = t * 0.5f * 1.061405429f + 0.5f * -1.453152027f;
  poly = t * poly + 0.5f * 1.421413741f;
  poly = t * poly + 0.5f * -0.284496736f;
  poly = t * poly + 0.5f * 0.254829592f;
  poly = t * poly;                                   // 0.5 * (1 - erf(|z| / sqrt2)) / exp(-z^2 / 2)
  const f32x2 a = z * z * -0.5f;
  const f32x2 e = f32x2{__expf(a.x), __expf(a.y)};
  const f32x2 tail = poly * e;
  const f32x2 cdf = f32x2{z.x >= 0.f ? 1.f - tail.x : tail.x, z.y >= 0.f ? 1.f - tail.y : tail.y};
  return z * (e * 0.3989422804014327f) + cdf;
}
__device__ __forceinline__ float apply_act(float z, int act) { return act == ACT_NONE ? z : apply_act_slow(z, act); }

// ---- LDS images ----------------------------------------------------------
// K-contiguous [R][BK] bf16 (BK*2-byte rows, CPR 16-byte chunks per row): the
// chunk XOR (r / (16/CPR)) & (CPR-1) puts the 16 rows of a ds_read_b128 lane
// group on 16 distinct 16-byte slots of a 256-byte bank row.
template <int BK>
__device__ __forceinline__ int kc_off(int r, int c) {
  constexpr int CPR = BK / 8;
  return r * (BK * 2) + ((c ^ ((r / (16 / CPR)) & (CPR - 1))) << 4);
}
// M/N-contiguous [BK][R] bf16: byte offset of (k, 16-byte chunk ch = mn/8).
// A transposed fragment read (frag, ds_read_b64_tr_b16) takes a 32-byte
// segment from each of 16 k-rows (k = 32 s + {0..3, 8..11, 16..19, 24..27});
// the chunk XOR spreads them over the bank row.  R >= 128 (rows >= 256 B):
// k bits 0, 1, 3 pick one of 8 segments.  R = 64 (128-byte rows, two per
// 256-byte bank row): k bit 0 already picks the half, so the XOR takes bits 1
// and 3 -- the masked R >= 128 XOR there (2 (k & 3)) collided with bit 0 and
// left half the banks unused: 2x the LDS cycles of every B read of a 192-wide
// tile's second quadrant column (SQ_LDS_BANK_CONFLICT 5x, profiles/gemm_layout_ab_r6.txt).
__device__ __forceinline__ int mn_swz(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }
template <int R>
__device__ __forceinline__ int mn_sw(int k) {
  if constexpr (R == 64) return (((k >> 1) & 1) | (((k >> 3) & 1) << 1)) << 1;
  else return (mn_swz(k) << 1) & (R / 8 - 1);
}
template <int R>
__device__ __forceinline__ int mn_off(int k, int ch) {
  return k * (2 * R) + ((ch ^ mn_sw<R>(k)) << 4);
}

// Stage one operand tile (R rows of the output dimension x BK k) into `img`.
// KC: src element (row, k) at base[row * ld + k]; else at base[k * ld + row].
template <int R, int BK, bool KC>
__device__ __forceinline__ void stage(const uint16_t* __restrict__ base, int ld, int rows, int r0, int k0,
                                      uint8_t* img, int wave, int lane) {
  constexpr int CPR = BK / 8;
#pragma unroll
  for (int j = 0; j < R * BK / 4096; ++j) {
    const int wbase = (j * 8 + wave) << 10;    // this wave instruction's 1 KiB
    const int o = wbase + (lane << 4);
    const uint16_t* src;
    if constexpr (KC) {
      const int r = o / (BK * 2), c = ((o >> 4) % CPR) ^ ((r / (16 / CPR)) & (CPR - 1));
      src = base + (size_t)min(r0 + r, rows - 1) * ld + k0 + c * 8;
    } else {
      const int k = o / (2 * R), ch = ((o % (2 * R)) >> 4) ^ mn_sw<R>(k);
      src = base + (size_t)(k0 + k) * ld + min(r0 + ch * 8, rows - 8);
    }
    __builtin_amdgcn_global_load_lds((gvoid*)src, (lvoid*)(img + wbase), 16, 0, 0);
  }
}

// Register-staged alternative to stage(): the same lane-linear image, loaded
// into VGPRs first (global_load_dwordx4) and written with ds_write_b128.
template <int R, int BK, bool KC>
__device__ __forceinline__ void gload(const uint16_t* __restrict__ base, int ld, int rows, int r0, int k0, int wave,
                                      int lane, uint4* v) {
  constexpr int CPR = BK / 8;
#pragma unroll
  for (int j = 0; j < R * BK / 4096; ++j) {
    const int o = ((j * 8 + wave) << 10) + (lane << 4);
    const uint16_t* src;
    if constexpr (KC) {
      const int r = o / (BK * 2), c = ((o >> 4) % CPR) ^ ((r / (16 / CPR)) & (CPR - 1));
      src = base + (size_t)min(r0 + r, rows - 1) * ld + k0 + c * 8;
    } else {
      const int k = o / (2 * R), ch = ((o % (2 * R)) >> 4) ^ mn_sw<R>(k);
      src = base + (size_t)(k0 + k) * ld + min(r0 + ch * 8, rows - 8);
    }
    v[j] = *reinterpret_cast<const uint4*>(src);
  }
}
template <int R, int BK>
__device__ __forceinline__ void lstore(uint8_t* img, int wave, int lane, const uint4* v) {
#pragma unroll
  for (int j = 0; j < R * BK / 4096; ++j)
    *reinterpret_cast<uint4*>(img + ((j * 8 + wave) << 10) + (lane << 4)) = v[j];
}

// MFMA 16x16x32 operand fragment of rows [rb, rb+16), k-sub s (k = 32 s ...):
// lane l gets (row rb + (l&15), k = 32 s + 8 (l>>4) + j), j = 0..7.
template <int R, int BK, bool KC>
__device__ __forceinline__ bf16x8 frag(const uint8_t* img, int rb, int s, int lane) {
  if constexpr (KC) {
    return *reinterpret_cast<const bf16x8*>(img + kc_off<BK>(rb + (lane & 15), s * 4 + (lane >> 4)));
  } else {
    // ds_read_b64_tr_b16: lane 4q+p of a 16-lane group addresses row k0+q,
    // columns 4p..4p+3 of the 4x16 block; lane i receives column i, row q in q
    const int k = s * 32 + 8 * (lane >> 4) + ((lane & 15) >> 2);
    const int mn = rb + 4 * (lane & 3);
    const int off = mn_off<R>(k, mn >> 3) + ((mn & 7) << 1);
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(img + off));
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(img + off + 4 * 2 * R));
    typedef __attribute__((ext_vector_type(8))) short v8s;
    const v8s v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, v);
  }
}

__device__ __forceinline__ void lds_sync() {
  // raw barrier: this wave's ds_reads retired, an in-flight DMA (vmcnt) is NOT
  // drained (a workgroup-scope LDS fence would wait vmcnt(0): the DMA counts
  // as a pending LDS write).  The asm statements pin LDS accesses on their side.
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// wait until at most `ahead` stages (ND DMA instructions each) are in flight
template <int ND>
__device__ __forceinline__ void wait_stages(int ahead) {
  switch (ahead) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ND) : "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * ND) : "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * ND) : "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * ND) : "memory"); break;
  }
}

// S-stage ring of BK-deep K tiles: while tile t is multiplied, tiles t+1 ..
// t+S-1 are in flight (S-1 stages of DMA bytes hide the HBM/L2 latency).
template <int BM, int BK, int S, bool AKC, bool BKC, bool OBF, int VAR = 0>
__global__ __launch_bounds__(NTHR) void gemm_big(const uint16_t* __restrict__ A, int lda,
                                                 const uint16_t* __restrict__ B, int ldb, void* __restrict__ C,
                                                 int ldc, const float* __restrict__ bias, int M, int N, int K,
                                                 float alpha, float beta, int act, int kchunk) {
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int MT = BM / 32, NT = 4;                    // 16x16 tiles per wave (2 x 4 waves)
  constexpr int NDMA = (BM + BN) * BK / 4096;            // DMA instructions per stage per thread
  static_assert(S >= 2 && S <= 5 && S * STAGE <= 160 * 1024, "LDS ring");
  __shared__ __attribute__((aligned(1024))) uint8_t smem[S * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;

  const int nt_n = (N + BN - 1) / BN;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig % 8, q = nwg / 8, rem = nwg % 8;
  const int wg = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + orig / 8;
  const int m0 = (wg / nt_n) * BM, n0 = (wg % nt_n) * BN;
  const int kb = blockIdx.y * kchunk, ke = min(K, kb + kchunk);
  const int nk = (ke - kb) / BK;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if constexpr (VAR == 4) {
    // one barrier per K tile (T3 minimum 2-phase): issue tile t+1's DMA, multiply
    // tile t, then wait for t+1 and barrier -- that barrier both publishes t+1
    // and retires every wave's reads of t before t+2 is staged into its buffer
    static_assert(S == 2, "two LDS buffers");
    if (nk > 0) {
      stage<BM, BK, AKC>(A, lda, M, m0, kb, smem, wave, lane);
      stage<BN, BK, BKC>(B, ldb, N, n0, kb, smem + A_BYTES, wave, lane);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_sync();
    for (int t = 0; t < nk; ++t) {
      const uint8_t* ia = smem + (t & 1) * STAGE;
      const uint8_t* ib = ia + A_BYTES;
      if (t + 1 < nk) {
        uint8_t* nx = smem + ((t + 1) & 1) * STAGE;
        stage<BM, BK, AKC>(A, lda, M, m0, kb + (t + 1) * BK, nx, wave, lane);
        stage<BN, BK, BKC>(B, ldb, N, n0, kb + (t + 1) * BK, nx + A_BYTES, wave, lane);
      }
#pragma unroll
      for (int s = 0; s < BK / 32; ++s) {
        bf16x8 fb[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) fb[j] = frag<BN, BK, BKC>(ib, wc * 64 + j * 16, s, lane);
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          const bf16x8 fa = frag<BM, BK, AKC>(ia, wr * (BM / 2) + i * 16, s, lane);
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[i][j] = mfma16x16x32(fa, fb[j], acc[i][j]);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_sync();
    }
  } else if constexpr (VAR == 3) {
    // register-staged double buffer: tile t+1's global loads are in flight
    // while tile t is multiplied, then written to the other LDS buffer
    static_assert(S == 2, "register staging uses two LDS buffers");
    uint4 va[BM * BK / 4096], vb[BN * BK / 4096];
    if (nk > 0) {
      gload<BM, BK, AKC>(A, lda, M, m0, kb, wave, lane, va);
      gload<BN, BK, BKC>(B, ldb, N, n0, kb, wave, lane, vb);
      lstore<BM, BK>(smem, wave, lane, va);
      lstore<BN, BK>(smem + A_BYTES, wave, lane, vb);
    }
    __syncthreads();
    for (int t = 0; t < nk; ++t) {
      const uint8_t* ia = smem + (t & 1) * STAGE;
      const uint8_t* ib = ia + A_BYTES;
      if (t + 1 < nk) {
        gload<BM, BK, AKC>(A, lda, M, m0, kb + (t + 1) * BK, wave, lane, va);
        gload<BN, BK, BKC>(B, ldb, N, n0, kb + (t + 1) * BK, wave, lane, vb);
      }
#pragma unroll
      for (int s = 0; s < BK / 32; ++s) {
        bf16x8 fb[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) fb[j] = frag<BN, BK, BKC>(ib, wc * 64 + j * 16, s, lane);
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          const bf16x8 fa = frag<BM, BK, AKC>(ia, wr * (BM / 2) + i * 16, s, lane);
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[i][j] = mfma16x16x32(fa, fb[j], acc[i][j]);
        }
      }
      if (t + 1 < nk) {
        uint8_t* nx = smem + ((t + 1) & 1) * STAGE;
        lstore<BM, BK>(nx, wave, lane, va);
        lstore<BN, BK>(nx + A_BYTES, wave, lane, vb);
      }
      __syncthreads();
    }
  } else {
#pragma unroll
  for (int p = 0; p < S - 1; ++p) {
    if (p < nk) {
      stage<BM, BK, AKC>(A, lda, M, m0, kb + p * BK, smem + p * STAGE, wave, lane);
      stage<BN, BK, BKC>(B, ldb, N, n0, kb + p * BK, smem + p * STAGE + A_BYTES, wave, lane);
    }
  }
  for (int t = 0; t < nk; ++t) {
    const uint8_t* cur = smem + (t % S) * STAGE;
    const int tn = t + S - 1;      // its buffer was last read in iteration t-1 (closing barrier)
    if (tn < nk) {
      uint8_t* nxt = smem + (tn % S) * STAGE;
      stage<BM, BK, AKC>(A, lda, M, m0, kb + tn * BK, nxt, wave, lane);
      stage<BN, BK, BKC>(B, ldb, N, n0, kb + tn * BK, nxt + A_BYTES, wave, lane);
    }
    wait_stages<NDMA>(min(S - 1, nk - 1 - t));   // tile t landed; later tiles stay in flight
    lds_sync();
    const uint8_t* ia = cur;
    const uint8_t* ib = cur + A_BYTES;
    if constexpr (VAR == 1) {
      // all fragments of the tile first (ds_reads back to back), then the MFMA
      // cluster at raised priority: the partner wave's reads overlap our MFMAs
      bf16x8 fa[BK / 32][MT], fb[BK / 32][NT];
#pragma unroll
      for (int s = 0; s < BK / 32; ++s) {
#pragma unroll
        for (int j = 0; j < NT; ++j) fb[s][j] = frag<BN, BK, BKC>(ib, wc * 64 + j * 16, s, lane);
#pragma unroll
        for (int i = 0; i < MT; ++i) fa[s][i] = frag<BM, BK, AKC>(ia, wr * (BM / 2) + i * 16, s, lane);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s = 0; s < BK / 32; ++s)
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[i][j] = mfma16x16x32(fa[s][i], fb[s][j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    } else {
#pragma unroll
      for (int s = 0; s < BK / 32; ++s) {
        bf16x8 fb[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) fb[j] = frag<BN, BK, BKC>(ib, wc * 64 + j * 16, s, lane);
        if constexpr (VAR == 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          const bf16x8 fa = frag<BM, BK, AKC>(ia, wr * (BM / 2) + i * 16, s, lane);
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[i][j] = mfma16x16x32(fa, fb[j], acc[i][j]);
        }
        if constexpr (VAR == 2) __builtin_amdgcn_s_setprio(0);
      }
    }
    lds_sync();   // every wave done reading `cur` before a later iteration restages it
  }
  }

  // epilogue: lane holds rows 4*(lane>>4) + r, column lane&15 of each 16x16 tile
  const bool split = gridDim.y > 1;
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int n = n0 + wc * 64 + j * 16 + (lane & 15);
    if (n >= N) continue;
    const float bv = (bias != nullptr) ? bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr * (BM / 2) + i * 16 + 4 * (lane >> 4) + r;
        if (m >= M) continue;
        const size_t o = (size_t)m * ldc + n;
        if (split) {   // linear fp32 epilogue (host-checked): partial sums meet in C
          atomicAdd(reinterpret_cast<float*>(C) + o, alpha * acc[i][j][r] + (blockIdx.y == 0 ? bv : 0.f));
          continue;
        }
        float z = alpha * acc[i][j][r] + bv;
        if (beta != 0.f)
          z += beta * (OBF ? bf2f(reinterpret_cast<const uint16_t*>(C)[o]) : reinterpret_cast<const float*>(C)[o]);
        const float y = apply_act(z, act);
        if constexpr (OBF) reinterpret_cast<uint16_t*>(C)[o] = f2bf(y);
        else reinterpret_cast<float*>(C)[o] = y;
      }
    }
  }
}

// ---- 8-phase schedule (cdna_hip_programming.md s5 "The 256^2 8-phase template") ----
// Same 256 x 256 tile, 8 waves (2 along M x 4 along N, 128 x 64 outputs each),
// BK 64 and LDS images as gemm_big, but every K tile is split into FOUR
// half-tiles, one per output quadrant half:
//   A_q = tile rows [64q, 64q+64) and [128+64q, 128+64q+64)   (quadrant row qm = q of both wave rows)
//   B_q = tile cols [64c+32q, 64c+32q+32) for c = 0..3          (quadrant col qn = q of all wave columns)
// each a 128-row x 64-k image of 16 KiB (2 LDS-DMA instructions per thread).
// Two K tiles (even / odd LDS buffer, 64 KiB each) per loop iteration, 8
// phases; phase p multiplies one 64 x 32 quadrant of the wave's outputs over
// the whole K tile (16 MFMA 16x16x32):
//   phase   quadrant  ds_reads (this K tile)   DMA issued (half-tile, K tile)
//     1      (0,0)    B_q0 then A_q0            A_q1  of t+1   (odd buffer)
//     2      (0,1)    B_q1                      B_q0  of t+2   (even buffer)
//     3      (1,1)    A_q1                      A_q0  of t+2
//     4      (1,0)    --  (registers)           B_q1  of t+2,  vmcnt(6): t+1 landed
//   phases 5..8: the same on the odd buffer (DMA: A_q1 of t+2, then B_q0 /
//   A_q0 / B_q1 of t+3, vmcnt(6) at phase 8: t+2 landed).
// Three half-tiles (6 DMA instructions) stay in flight across every barrier;
// vmcnt is counted, never 0 inside the loop.  A buffer region is restaged two
// phases after its last ds_read, or one phase after when those reads were
// retired before the reading phase's first barrier (B_q0: its reads are
// issued first and retired by lgkmcnt(#A reads) before that barrier).
// The two wave rows run one barrier apart (`if (wr) s_barrier` before the
// loop): while one group multiplies, the other issues its reads and DMA.
// A buffer retired by the vmcnt at phase p is read from phase p+1 on (the
// staggered group passes one more barrier after the other group's wait).
// Shape contract on top of gemm_big's: the K range of a workgroup is a
// multiple of 128 (an even number of K tiles).
// half-tile local index -> tile row (A) / column (B).  B: WN = the wave's
// column count (64, or 48 for 192-wide tiles); quadrant column 0 is its first
// 32 columns, quadrant column 1 the remaining WN - 32.
template <bool IS_A, int WN>
__device__ __forceinline__ int half_row(int l, int q) {
  if constexpr (IS_A) {
    return ((l >> 6) << 7) + (q << 6) + (l & 63);
  } else {
    constexpr int W1 = WN - 32;
    return q == 0 ? (l >> 5) * WN + (l & 31) : (l / W1) * WN + 32 + (l % W1);
  }
}

// Stage one half-tile (R rows of the output dimension x 64 k, R / 64 LDS-DMA
// instructions per thread) of K tile k0 into `img`.
template <bool IS_A, bool KC, int R, int WN>
__device__ __forceinline__ void stage_half(const uint16_t* __restrict__ base, int ld, int rows, int r0, int k0, int q,
                                           uint8_t* img, int wave, int lane) {
#pragma unroll
  for (int j = 0; j < R / 64; ++j) {
    const int wbase = (j * 8 + wave) << 10;
    const int o = wbase + (lane << 4);
    const uint16_t* src;
    if constexpr (KC) {   // [R][64] image, kc_off<64> chunk XOR
      const int rl = o >> 7, c = ((o >> 4) & 7) ^ ((rl >> 1) & 7);
      src = base + (size_t)min(r0 + half_row<IS_A, WN>(rl, q), rows - 1) * ld + k0 + c * 8;
    } else {              // [64][R] image, mn_off<R>
      const int k = o / (2 * R), ch = ((o % (2 * R)) >> 4) ^ mn_sw<R>(k);
      src = base + (size_t)(k0 + k) * ld + min(r0 + half_row<IS_A, WN>(ch * 8, q), rows - 8);
    }
    __builtin_amdgcn_global_load_lds((gvoid*)src, (lvoid*)(img + wbase), 16, 0, 0);
  }
}

__device__ __forceinline__ void raw_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// Fused GELU epilogues (interior tiles of a bf16 256-wide product only -- host
// contracts in dtfk_gemm_dgelu / dtfk_gemm_gelu_aux), EP:
//   EP_DGELU     C = (A' B') * gelu'(aux + bias), aux the saved pre-activation
//                (bf16, ld = ldc; bias may be null), and the per-column sums of
//                that fp32 product over each wave row's 128 rows to
//                colpart[M / 128][N] (the bias gradient's partials, reduced by
//                colsum_partials);
//   EP_GELU_AUX  aux = A' B' + bias (the pre-activation the backward needs) and
//                C = gelu(A' B' + bias), both bf16 with ld = ldc;
//   EP_STATS     C = A' B' (bf16) and, per column, the sum and the sum of
//                squares of the STORED (bf16-rounded) values over each wave
//                row's 128 rows to colpart[2][P][N], P = ceil(M / 128): the
//                BatchNorm statistics partials of a 1x1 convolution's output
//                (csrc/kernels/bn.hip bn_fwd_parts), edge tiles included.
enum Epi { EP_PLAIN = 0, EP_DGELU = 1, EP_GELU_AUX = 2, EP_STATS = 3 };
template <bool AKC, bool BKC, bool OBF, bool SW, int BNT = 256, int EP = EP_PLAIN>
__global__ __launch_bounds__(NTHR) void gemm_8ph(const uint16_t* __restrict__ A, int lda,
                                                 const uint16_t* __restrict__ B, int ldb, void* __restrict__ C,
                                                 int ldc, const float* __restrict__ bias, int M, int N, int K,
                                                 float alpha, float beta, int act, int kchunk, long long slab = 0,
                                                 uint16_t* __restrict__ aux = nullptr,
                                                 float* __restrict__ colpart = nullptr) {
  constexpr bool DG = EP == EP_DGELU, GA = EP == EP_GELU_AUX, ST = EP == EP_STATS;
  static_assert(EP == EP_PLAIN || (OBF && SW && BNT == 256), "GELU epilogues: bf16 out, 256-wide tiles");
  // BNT = 256, or 192 (waves 128 x 48: quadrant column 1 is one 16-wide n tile,
  // its half-tile 64 rows / one DMA per thread) for N where 256 leaves CUs idle
  static_assert(BNT == 256 || BNT == 192, "tile width");
  constexpr int BM = 256, BK = 64, WN = BNT / 4, NJ = WN / 16, NQ1 = NJ - 2;
  constexpr int HALF = 128 * BK * 2, HB1 = 4 * 16 * NQ1 * BK * 2;       // A / B_q0 halves, B_q1
  constexpr int BUF = 3 * HALF + HB1;                                    // A_q0 A_q1 B_q0 B_q1
  constexpr int VMC = 4 + NQ1;   // DMA ops of the 3 half-tiles in flight: B_q0 (2) + A_q0 (2) + B_q1 (NQ1)
  constexpr int NA = AKC ? 8 : 16;                                       // LDS instructions of one A-fragment set
  // operand buffers; after the K loop, each wave's fp32 output half-tile (64
  // rows of EPI_ROW bytes: WN floats + 16 pad) for the row-contiguous store pass
  constexpr int EPI_ROW = 4 * WN + 16, EPI_WAVE = 64 * EPI_ROW;
  __shared__ __attribute__((aligned(1024))) uint8_t smem[(2 * BUF > 8 * EPI_WAVE) ? 2 * BUF : 8 * EPI_WAVE];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  const int nt_n = (N + BNT - 1) / BNT;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig % 8, q8 = nwg / 8, rem = nwg % 8;
  const int wg = (xcd < rem ? xcd * (q8 + 1) : rem * (q8 + 1) + (xcd - rem) * q8) + orig / 8;
  const int m0 = (wg / nt_n) * BM, n0 = (wg % nt_n) * BNT;
  const int kb = blockIdx.y * kchunk, ke = min(K, kb + kchunk);
  const int nk = (ke - kb) / BK;   // even (host contract)

  f32x4 acc[8][NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // half-tile h of K tile t: 0 B_q0, 1 A_q0, 2 B_q1, 3 A_q1 (staging order)
  auto stage = [&](int t, int h) {
    if (t >= nk) return;
    uint8_t* buf = smem + (t & 1) * BUF;
    const int k0 = kb + t * BK;
    if (h == 0) stage_half<false, BKC, 128, WN>(B, ldb, N, n0, k0, 0, buf + 2 * HALF, wave, lane);
    else if (h == 1) stage_half<true, AKC, 128, WN>(A, lda, M, m0, k0, 0, buf, wave, lane);
    else if (h == 2) stage_half<false, BKC, 64 * NQ1, WN>(B, ldb, N, n0, k0, 1, buf + 3 * HALF, wave, lane);
    else stage_half<true, AKC, 128, WN>(A, lda, M, m0, k0, 1, buf + HALF, wave, lane);
  };
  bf16x8 fa[2][4], fb[2][2][2];   // A: [k-sub][m-tile] of one quadrant row; B: [qn][k-sub][n-tile]
  auto read_a = [&](const uint8_t* buf, int qm) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[s][i] = frag<128, BK, AKC>(buf + qm * HALF, wr * 64 + i * 16, s, lane);
  };
  auto read_b = [&](const uint8_t* buf, int qn) {
    if (qn == 0) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 2; ++j) fb[0][s][j] = frag<128, BK, BKC>(buf + 2 * HALF, wc * 32 + j * 16, s, lane);
    } else {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < NQ1; ++j)
          fb[1][s][j] = frag<64 * NQ1, BK, BKC>(buf + 3 * HALF, wc * 16 * NQ1 + j * 16, s, lane);
    }
  };
  auto mma = [&](int qm, int qn) {
    raw_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if (qn == 0 || j < NQ1)
            acc[qm * 4 + i][qn * 2 + j] = SW ? mfma16x16x32(fb[qn][s][j], fa[s][i], acc[qm * 4 + i][qn * 2 + j])
                                             : mfma16x16x32(fa[s][i], fb[qn][s][j], acc[qm * 4 + i][qn * 2 + j]);
    __builtin_amdgcn_s_setprio(0);
    raw_barrier();
  };
  // phase 1 / 5 reads: B_q0 first, then A_q0; the B reads retire before the barrier
  auto read_first = [&](const uint8_t* buf) {
    read_b(buf, 0);
    __builtin_amdgcn_sched_barrier(0);
    read_a(buf, 0);
    if constexpr (NA <= 15) asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(NA) : "memory");
    else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };

  // prologue: K tile 0 whole, K tile 1 but its A_q1 (issued in phase 1)
#pragma unroll
  for (int h = 0; h < 4; ++h) stage(0, h);
#pragma unroll
  for (int h = 0; h < 3; ++h) stage(1, h);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VMC) : "memory");
  raw_barrier();
  if (wr) raw_barrier();   // the second wave row runs one barrier behind

  for (int t = 0; t < nk; t += 2) {
    const uint8_t* ev = smem;
    const uint8_t* od = smem + BUF;
    const bool last = t + 2 >= nk;
    // phases 1-4: even buffer (K tile t)
    read_first(ev);
    stage(t + 1, 3);
    mma(0, 0);
    read_b(ev, 1);
    stage(t + 2, 0);
    mma(0, 1);
    read_a(ev, 1);
    stage(t + 2, 1);
    mma(1, 1);
    stage(t + 2, 2);
    if (last) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VMC) : "memory");
    mma(1, 0);
    // phases 5-8: odd buffer (K tile t+1)
    read_first(od);
    stage(t + 2, 3);
    mma(0, 0);
    read_b(od, 1);
    stage(t + 3, 0);
    mma(0, 1);
    read_a(od, 1);
    stage(t + 3, 1);
    mma(1, 1);
    stage(t + 3, 2);
    if (!last) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VMC) : "memory");
    mma(1, 0);
  }
  if (!wr) raw_barrier();   // equal barrier counts for both wave rows
  // probes only (dtfk_gemm_big_cfg 11-13): -1 the loop without the epilogue,
  // -2 a quarter of the outputs stored, -3 every tile stored over tile (0, 0)
  const int probe = act < 0 ? -act : 0;
  if (probe == 1) return;
  if (probe) act = ACT_NONE;

  if constexpr (!SW) {
    // split-K (fp32, linear): accumulators in MFMA layout -- lane l holds rows
    // 4 (l >> 4) .. +3 of column (l & 15), so each atomic instruction covers
    // 16 consecutive columns of 4 rows (4 cache lines, not 16)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = n0 + wc * WN + j * 16 + (lane & 15);
      if (n >= N) continue;
      const float bv = (bias != nullptr && blockIdx.y == 0) ? bias[n] : 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wr * 128 + i * 16 + 4 * (lane >> 4) + r;
          if (m < M) atomicAdd(reinterpret_cast<float*>(C) + (size_t)m * ldc + n, alpha * acc[i][j][r] + bv);
        }
    }
    return;
  }
  // split-K into slabs (fp32 partial products, summed by slab_reduce): this
  // K range's partial tile is a plain tile of slab blockIdx.y
  if (slab > 0) C = reinterpret_cast<float*>(C) + blockIdx.y * slab;
  // The MFMAs ran with swapped operands (B fragment first): each accumulator
  // is the 16x16 tile TRANSPOSED, so lane l holds output row (l & 15) and the
  // 4 consecutive columns 4 (l >> 4) .. +3 -- one 8-byte (bf16) / 16-byte
  // (fp32) store per tile instead of four 2- / 4-byte ones.
  const bool vec = (ldc & 7) == 0 && (reinterpret_cast<uintptr_t>(C) & 15) == 0;
  const int mrow = m0 + wr * 128 + (lane & 15), ncol = n0 + wc * WN + 4 * (lane >> 4);
  if (vec && m0 + BM <= M && n0 + BNT <= N && probe == 0) {
    // Interior tile: the wave's 128 x 64 outputs go through its private LDS
    // region (free after the loop's last barrier) in two halves of 64 rows,
    // as fp32 (alpha acc + bias); read back as 8 consecutive columns per lane
    // (+ beta C, activation, conversion) and stored as whole row segments:
    // each store instruction writes 8 rows x 128 (bf16) / 256 (fp32) bytes =
    // full cache lines, instead of 16 rows x 32 / 64 bytes.  Measured: the
    // end-of-tile store burst was the kernel's largest cost (profiles/gemm_8ph_r3.txt).
    uint8_t* ep = smem + wave * EPI_WAVE;
    float bv[NJ][4];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[j][r] = (bias != nullptr && !DG) ? bias[ncol + j * 16 + r] : 0.f;
    // read-back: row rsub (+8 it), columns c8 .. c8+7; WN / 8 lanes per row (48-wide: lanes >= 48 idle)
    constexpr int LPR = WN / 8;
    const int rsub = lane / LPR, c8 = (lane % LPR) * 8;
    const bool rb_on = lane < 8 * LPR;
    // DG: the pre-activation's bias for this lane's 8 columns; their column sums
    // (ST: the column sums and sums of squares of the stored values)
    float ab[8], cs[8], cq[8];
    if constexpr (DG) {
#pragma unroll
      for (int q = 0; q < 8; ++q) { ab[q] = bias != nullptr ? bias[n0 + wc * WN + c8 + q] : 0.f; cs[q] = 0.f; }
    }
    if constexpr (ST) {
#pragma unroll
      for (int q = 0; q < 8; ++q) { cs[q] = 0.f; cq[q] = 0.f; }
    }
    typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
    // DG: the saved pre-activation of BOTH halves requested up front (16 loads
    // in flight; the operand-fragment registers are free after the loop)
    u32x4 apre[DG ? 16 : 1];
    if constexpr (DG) {
#pragma unroll
      for (int q = 0; q < 16; ++q)
        apre[q] = *reinterpret_cast<const u32x4*>(
            aux + (size_t)(m0 + wr * 128 + (q >> 3) * 64 + (q & 7) * 8 + rsub) * ldc + n0 + wc * WN + c8);
    }
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      // beta != 0: this half's C chunks are loaded first, all at once (the
      // operand-fragment registers are free after the loop), so their latency
      // hides under the LDS round trip instead of one load per store
      u32x4 cpre[OBF ? 8 : 16];
      if (!DG && beta != 0.f && rb_on) {
#pragma unroll
        for (int it = 0; it < 8; ++it) {
          const size_t o = (size_t)(m0 + wr * 128 + half * 64 + it * 8 + rsub) * ldc + n0 + wc * WN + c8;
          if constexpr (OBF) {
            cpre[it] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const uint16_t*>(C) + o);
          } else {
            cpre[2 * it] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const float*>(C) + o);
            cpre[2 * it + 1] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const float*>(C) + o + 4);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int row = i * 16 + (lane & 15), col = j * 16 + 4 * (lane >> 4);
          const f32x4 a4 = acc[half * 4 + i][j];
          *reinterpret_cast<f32x4*>(ep + row * EPI_ROW + col * 4) =
              f32x4{alpha * a4[0] + bv[j][0], alpha * a4[1] + bv[j][1], alpha * a4[2] + bv[j][2],
                    alpha * a4[3] + bv[j][3]};
        }
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        if (!rb_on) break;
        const int lrow = it * 8 + rsub;
        const f32x4 lo = *reinterpret_cast<const f32x4*>(ep + lrow * EPI_ROW + c8 * 4);
        const f32x4 hi = *reinterpret_cast<const f32x4*>(ep + lrow * EPI_ROW + c8 * 4 + 16);
        float z[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const size_t o = (size_t)(m0 + wr * 128 + half * 64 + lrow) * ldc + n0 + wc * WN + c8;
        if constexpr (DG) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t u2 = apre[half * 8 + it][q];
            const f32x2 g2 = gelu_grad2(f32x2{bf2f((uint16_t)(u2 & 0xffff)), bf2f((uint16_t)(u2 >> 16))} +
                                        f32x2{ab[2 * q], ab[2 * q + 1]});
            z[2 * q] *= g2.x;
            z[2 * q + 1] *= g2.y;
          }
#pragma unroll
          for (int q = 0; q < 8; ++q) cs[q] += z[q];
        } else if (beta != 0.f) {
          if constexpr (OBF) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              z[2 * q] += beta * bf2f((uint16_t)(cpre[it][q] & 0xffff));
              z[2 * q + 1] += beta * bf2f((uint16_t)(cpre[it][q] >> 16));
            }
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              z[q] += beta * __uint_as_float(cpre[2 * it][q]);
              z[4 + q] += beta * __uint_as_float(cpre[2 * it + 1][q]);
            }
          }
        }
        if constexpr (GA) {
          *reinterpret_cast<uint4*>(aux + o) =
              make_uint4(pack2bf(z[0], z[1]), pack2bf(z[2], z[3]), pack2bf(z[4], z[5]), pack2bf(z[6], z[7]));
#pragma unroll
          for (int q = 0; q < 8; ++q) z[q] = gelu_fwd_f(z[q]);
        }
        if (act != ACT_NONE) {
#pragma unroll
          for (int q = 0; q < 8; ++q) z[q] = apply_act_slow(z[q], act);
        }
        if constexpr (ST) {
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const float r = bf2f(f2bf(z[q]));
            cs[q] += r;
            cq[q] += r * r;
          }
        }
        if constexpr (OBF) {
          *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(C) + o) =
              make_uint4(pack2bf(z[0], z[1]), pack2bf(z[2], z[3]), pack2bf(z[4], z[5]), pack2bf(z[6], z[7]));
        } else {
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + o) = make_float4(z[0], z[1], z[2], z[3]);
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + o + 4) = make_float4(z[4], z[5], z[6], z[7]);
        }
      }
    }
    if constexpr (DG) {
      // lanes of one column group (lane % 8) hold 8 rows each of the 16 x 8 it/half rows: butterfly over the
      // row index, then the rsub == 0 lanes store the wave row's 128-row column sums
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        cs[q] += __shfl_xor(cs[q], 8);
        cs[q] += __shfl_xor(cs[q], 16);
        cs[q] += __shfl_xor(cs[q], 32);
      }
      if (rsub == 0) {
        float* p = colpart + (size_t)((m0 >> 7) + wr) * N + n0 + wc * WN + c8;
        *reinterpret_cast<float4*>(p) = make_float4(cs[0], cs[1], cs[2], cs[3]);
        *reinterpret_cast<float4*>(p + 4) = make_float4(cs[4], cs[5], cs[6], cs[7]);
      }
    }
    if constexpr (ST) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        cs[q] += __shfl_xor(cs[q], 8);
        cs[q] += __shfl_xor(cs[q], 16);
        cs[q] += __shfl_xor(cs[q], 32);
        cq[q] += __shfl_xor(cq[q], 8);
        cq[q] += __shfl_xor(cq[q], 16);
        cq[q] += __shfl_xor(cq[q], 32);
      }
      if (rsub == 0) {
        const size_t P = (size_t)((M + 127) >> 7);
        float* p = colpart + (size_t)((m0 >> 7) + wr) * N + n0 + wc * WN + c8;
        *reinterpret_cast<float4*>(p) = make_float4(cs[0], cs[1], cs[2], cs[3]);
        *reinterpret_cast<float4*>(p + 4) = make_float4(cs[4], cs[5], cs[6], cs[7]);
        *reinterpret_cast<float4*>(p + P * N) = make_float4(cq[0], cq[1], cq[2], cq[3]);
        *reinterpret_cast<float4*>(p + P * N + 4) = make_float4(cq[4], cq[5], cq[6], cq[7]);
      }
    }
    return;
  }
  if constexpr (ST) {
    // edge tile (rows past M or columns past N): bf16 stores with bounds, and the
    // per-column partials of this wave row's 128 rows -- each lane sums its 4
    // columns over its rows, then a butterfly over the 16 row lanes
    float ps[NJ][4], pq[NJ][4];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) { ps[j][r] = 0.f; pq[j][r] = 0.f; }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + wr * 128 + i * 16 + (lane & 15);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n = n0 + wc * WN + j * 16 + 4 * (lane >> 4);
        if (m >= M || n >= N) continue;
        const size_t o = (size_t)m * ldc + n;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (n + r >= N) continue;
          const uint16_t h = f2bf(alpha * acc[i][j][r]);
          reinterpret_cast<uint16_t*>(C)[o + r] = h;
          const float v = bf2f(h);
          ps[j][r] += v;
          pq[j][r] += v * v;
        }
      }
    }
    const size_t P = (size_t)((M + 127) >> 7);
    const int prow = (m0 >> 7) + wr;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float a = ps[j][r], b = pq[j][r];
        a += __shfl_xor(a, 1); a += __shfl_xor(a, 2); a += __shfl_xor(a, 4); a += __shfl_xor(a, 8);
        b += __shfl_xor(b, 1); b += __shfl_xor(b, 2); b += __shfl_xor(b, 4); b += __shfl_xor(b, 8);
        const int n = n0 + wc * WN + j * 16 + 4 * (lane >> 4) + r;
        if ((lane & 15) == 0 && n < N && prow < (int)P) {
          colpart[(size_t)prow * N + n] = a;
          colpart[(P + prow) * N + n] = b;
        }
      }
    return;
  }
  if (vec && m0 + BM <= M && n0 + BNT <= N) {
    // interior tile: no per-lane bounds, only wave-uniform branches (an
    // exec-masked branch per element costs more than the stores themselves)
    float bv[NJ][4];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[j][r] = bias != nullptr ? bias[ncol + j * 16 + r] : 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if (probe == 2 && j != 0) continue;
        const size_t o = (size_t)(mrow + i * 16) * ldc + ncol + j * 16 - (probe == 3 ? (size_t)m0 * ldc + n0 : 0);
        float z[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) z[r] = alpha * acc[i][j][r] + bv[j][r];
        if (beta != 0.f) {
          if constexpr (OBF) {
            const uint2 c = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(C) + o);
            z[0] += beta * bf2f((uint16_t)(c.x & 0xffff));
            z[1] += beta * bf2f((uint16_t)(c.x >> 16));
            z[2] += beta * bf2f((uint16_t)(c.y & 0xffff));
            z[3] += beta * bf2f((uint16_t)(c.y >> 16));
          } else {
            const float4 c = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(C) + o);
            z[0] += beta * c.x; z[1] += beta * c.y; z[2] += beta * c.z; z[3] += beta * c.w;
          }
        }
        if (act != ACT_NONE) {
#pragma unroll
          for (int r = 0; r < 4; ++r) z[r] = apply_act_slow(z[r], act);
        }
        // (non-temporal stores measured 1.2-1.4x slower here: profiles/gemm_8ph_r3.txt)
        if constexpr (OBF)
          *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(C) + o) = make_uint2(pack2bf(z[0], z[1]), pack2bf(z[2], z[3]));
        else
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + o) = make_float4(z[0], z[1], z[2], z[3]);
      }
    return;
  }
  const bool split = false;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = m0 + wr * 128 + i * 16 + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = n0 + wc * WN + j * 16 + 4 * (lane >> 4);
      if (n >= N) continue;
      const size_t o = (size_t)m * ldc + n;
      const bool full = vec && n + 3 < N;
      float z[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float bv = (bias != nullptr && n + r < N && (!split || blockIdx.y == 0)) ? bias[n + r] : 0.f;
        z[r] = alpha * acc[i][j][r] + bv;
      }
      if (split) {   // linear fp32 epilogue (host-checked): partial sums meet in C
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (n + r < N) atomicAdd(reinterpret_cast<float*>(C) + o + r, z[r]);
        continue;
      }
      if (beta != 0.f) {
        if constexpr (OBF) {
          if (full) {
            const uint2 c = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(C) + o);
            z[0] += beta * bf2f((uint16_t)(c.x & 0xffff));
            z[1] += beta * bf2f((uint16_t)(c.x >> 16));
            z[2] += beta * bf2f((uint16_t)(c.y & 0xffff));
            z[3] += beta * bf2f((uint16_t)(c.y >> 16));
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (n + r < N) z[r] += beta * bf2f(reinterpret_cast<const uint16_t*>(C)[o + r]);
          }
        } else {
          if (full) {
            const float4 c = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(C) + o);
            z[0] += beta * c.x; z[1] += beta * c.y; z[2] += beta * c.z; z[3] += beta * c.w;
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (n + r < N) z[r] += beta * reinterpret_cast<const float*>(C)[o + r];
          }
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) z[r] = apply_act(z[r], act);
      if constexpr (OBF) {
        if (full) {
          uint2 c;
          c.x = (uint32_t)f2bf(z[0]) | ((uint32_t)f2bf(z[1]) << 16);
          c.y = (uint32_t)f2bf(z[2]) | ((uint32_t)f2bf(z[3]) << 16);
          *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(C) + o) = c;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n + r < N) reinterpret_cast<uint16_t*>(C)[o + r] = f2bf(z[r]);
        }
      } else {
        if (full) {
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + o) = make_float4(z[0], z[1], z[2], z[3]);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n + r < N) reinterpret_cast<float*>(C)[o + r] = z[r];
        }
      }
    }
  }
}

// C[m, n] = sum_s ws[s][m, n] + bias[n] + beta * C[m, n]: the split-K slabs of
// gemm_8ph summed in slab order (deterministic), 4 columns per thread.
__global__ __launch_bounds__(256) void slab_reduce(const float* __restrict__ ws, int S, long long slab,
                                                   float* __restrict__ C, int ldc, int M, int N,
                                                   const float* __restrict__ bias, float beta) {
  const int nq = N / 4;
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long long)M * nq) return;
  const int m = (int)(e / nq), n = (int)(e - (long long)m * nq) * 4;
  const float* src = ws + (size_t)m * N + n;
  f32x4 z = *reinterpret_cast<const f32x4*>(src);
  for (int s = 1; s < S; ++s) z += *reinterpret_cast<const f32x4*>(src + s * slab);
  if (bias != nullptr) z += f32x4{bias[n], bias[n + 1], bias[n + 2], bias[n + 3]};
  float* dst = C + (size_t)m * ldc + n;
  if (beta != 0.f) {
#pragma unroll
    for (int r = 0; r < 4; ++r) z[r] += beta * dst[r];
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) dst[r] = z[r];
}

// Split-K plan of one product: {split, kchunk, slab mode}.  Slab mode (the
// 8-phase kernel, fp32 linear output, N % 4 == 0): ~one workgroup per CU,
// partial tiles to a [split, M, N] fp32 workspace + slab_reduce -- plain
// vector stores instead of per-element atomics.  Otherwise the atomic split
// of gemm_big (partial tiles meet in C).
struct SplitPlan { int split, kchunk, slabs; };
static SplitPlan plan_split(int M, int N, int K, int c_bf16, float beta, int act, int split_k, bool ph8) {
  using namespace dtfk::gemm2;
  const int kq = ph8 ? 2 * KQ : KQ;
  const long long tiles = (long long)((M + 255) / 256) * ((N + BN - 1) / BN);
  const bool linear = act == ACT_NONE && !c_bf16 && (beta == 0.f || beta == 1.f);
  SplitPlan p{1, K, 0};
  if (!(split_k > 1 || (split_k <= 0 && linear && tiles < 256 && K >= 2048))) return p;
  const bool slabs = ph8 && linear && N % 4 == 0;
  // slab mode's workgroup target (DTF_GEMM_SLAB_WGS, default 256: ~one per CU);
  // fewer means fewer, longer splits and less fp32 slab traffic
  static const long long slab_wgs = [] {
    const char* e = getenv("DTF_GEMM_SLAB_WGS");
    const long long v = e ? atoll(e) : 0LL;
    return v > 0 ? v : 256LL;
  }();
  int split = split_k > 1 ? split_k : (slabs ? (int)max(2LL, slab_wgs / tiles) : (int)((512 + tiles - 1) / tiles));
  split = min(split, K / (slabs ? 256 : 512) > 0 ? K / (slabs ? 256 : 512) : 1);
  p.kchunk = ((K + split - 1) / split + kq - 1) / kq * kq;
  p.split = (K + p.kchunk - 1) / p.kchunk;
  p.slabs = slabs && p.split > 1;
  return p;
}

}  // namespace gemm2
}  // namespace dtfk

// Bytes of fp32 workspace dtfk_gemm_big needs for this product (0: none).
extern "C" long long dtfk_gemm_big_workspace(int M, int N, int K, int c_bf16, float beta, int act, int split_k,
                                             int variant) {
  const bool ph8 = variant >= 8 || (variant == 0 && K % 128 == 0);
  const dtfk::gemm2::SplitPlan p = dtfk::gemm2::plan_split(M, N, K, c_bf16, beta, act, split_k, ph8);
  return p.slabs ? (long long)p.split * M * N * 4 : 0;
}

// The shape / alignment contract of dtfk_gemm_big, checked on the host before
// any launch: callers pick another GEMM when it fails, and every error the
// launch itself returns is a real error (never mistaken for "unsupported").
extern "C" int dtfk_gemm_big_supported(const void* A, int lda, int transA, const void* B, int ldb, int transB,
                                       int c_bf16, int M, int N, int K, float beta, int act, int split_k) {
  using namespace dtfk::gemm2;
  const bool akc = !transA, bkc = transB != 0;
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (M <= 0 || N <= 0 || K <= 0 || K % KQ != 0 || !al16(A) || !al16(B) || lda % 8 || ldb % 8) return 0;
  if ((!akc && M % 8) || (!bkc && N % 8) || (akc && lda < K) || (bkc && ldb < K) || (!akc && lda < M) ||
      (!bkc && ldb < N))
    return 0;
  const long long tiles = (long long)((M + 255) / 256) * ((N + BN - 1) / BN);
  if (tiles > 0x7fffffff) return 0;
  const bool linear = act == ACT_NONE && !c_bf16 && (beta == 0.f || beta == 1.f);
  if (split_k > 1 && !linear) return 0;
  return 1;
}

// Returns hipErrorInvalidValue (launching nothing) when the shape contract
// (dtfk_gemm_big_supported) does not hold.  split_k <= 0: automatic.
// variant: 0 = automatic (the 8-phase schedule whenever every workgroup's K
// range is a multiple of 128 -- 192-wide tiles where they fill the CUs better
// -- else the one-barrier loop), 4 = one-barrier loop (gemm_big VAR 4), 8 =
// 8-phase 256-wide, 9 = 8-phase 192-wide where unsplit (hipErrorInvalidValue if K % 128).
extern "C" hipError_t dtfk_gemm_big(const void* A, int lda, int transA, const void* B, int ldb, int transB,
                                    void* C, int c_bf16, int ldc, const float* bias, int M, int N, int K,
                                    float alpha, float beta, int act, int split_k, int variant, void* ws,
                                    hipStream_t stream) {
  using namespace dtfk::gemm2;
  const bool akc = !transA, bkc = transB != 0;
  if (!dtfk_gemm_big_supported(A, lda, transA, B, ldb, transB, c_bf16, M, N, K, beta, act, split_k))
    return hipErrorInvalidValue;
  if (variant != 0 && variant != 4 && variant != 8 && variant != 9) return hipErrorInvalidValue;
  const bool ph8 = variant >= 8 || (variant == 0 && K % 128 == 0);
  if (ph8 && K % 128) return hipErrorInvalidValue;
  const int tn = (N + BN - 1) / BN;
  // 256 x 256 tiles even when they leave CUs idle (N = 768: 192 tiles): measured
  // faster than 128 x 256 at every BERT shape (scripts/probes/gemm_big_cfg.py)
  const long long tiles = (long long)((M + 255) / 256) * tn;
  const SplitPlan plan = plan_split(M, N, K, c_bf16, beta, act, split_k, ph8);
  const int split = plan.split, kchunk = plan.kchunk;
  if (plan.slabs && ws == nullptr) return hipErrorInvalidValue;   // dtfk_gemm_big_workspace bytes needed
  if (plan.slabs) {
    const long long slab = (long long)M * N;
    const dim3 grid((unsigned)tiles, split), block(NTHR);
    const uint16_t* a = static_cast<const uint16_t*>(A);
    const uint16_t* b = static_cast<const uint16_t*>(B);
#define DTFK_GS(AK, BKk)                                                                                       \
  hipLaunchKernelGGL((gemm_8ph<AK, BKk, false, true>), grid, block, 0, stream, a, lda, b, ldb, ws, N, nullptr, M, \
                     N, K, alpha, 0.f, 0, kchunk, slab)
    if (akc) {
      if (bkc) DTFK_GS(true, true); else DTFK_GS(true, false);
    } else {
      if (bkc) DTFK_GS(false, true); else DTFK_GS(false, false);
    }
#undef DTFK_GS
    const long long work = (long long)M * (N / 4);
    hipLaunchKernelGGL(slab_reduce, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, stream,
                       static_cast<const float*>(ws), split, slab, static_cast<float*>(C), ldc, M, N, bias, beta);
    return hipGetLastError();
  }
  if (split > 1 && beta == 0.f) {
    const hipError_t e = dtfk::zero2d_f32(static_cast<float*>(C), ldc, M, N, stream);
    if (e != hipSuccess) return e;
  }
  // 192-wide tiles when 256-wide ones leave a wave of tiles partly empty
  // (BERT-base: N = 768 -> 192 tiles for 256 CUs, N = 2304 -> 2.25 waves)
  const long long tiles192 = (long long)((M + 255) / 256) * ((N + 191) / 192);
  auto fill = [](long long t) { return (double)t / (double)(((t + 255) / 256) * 256); };
  const bool w192 = ph8 && split == 1 && (variant == 9 || (variant == 0 && fill(tiles192) > fill(tiles) + 0.1));
  const dim3 grid192((unsigned)tiles192, 1);
  const dim3 grid((unsigned)tiles, split), block(NTHR);
  const uint16_t* a = static_cast<const uint16_t*>(A);
  const uint16_t* b = static_cast<const uint16_t*>(B);
// 64-deep tiles, 2 stages, one barrier per tile (VAR 4) for every layout: the
// 32-deep 5-stage ring, 128-row tiles, register staging and the two-barrier
// loop measured slower (profiles/gemm_big_cfg_r2.jsonl)
#define DTFK_GB(AK, BKk, OB)                                                                                      \
  if (ph8 && split > 1)                                                                                          \
    hipLaunchKernelGGL((gemm_8ph<AK, BKk, false, false>), grid, block, 0, stream, a, lda, b, ldb, C, ldc, bias, M, \
                       N, K, alpha, 1.f, act, kchunk);                                                           \
  else if (w192)                                                                                                 \
    hipLaunchKernelGGL((gemm_8ph<AK, BKk, OB, true, 192>), grid192, block, 0, stream, a, lda, b, ldb, C, ldc, bias, \
                       M, N, K, alpha, beta, act, kchunk);                                                       \
  else if (ph8)                                                                                                  \
    hipLaunchKernelGGL((gemm_8ph<AK, BKk, OB, true>), grid, block, 0, stream, a, lda, b, ldb, C, ldc, bias, M, N, \
                       K, alpha, beta, act, kchunk);                                                             \
  else                                                                                                           \
    hipLaunchKernelGGL((gemm_big<256, 64, 2, AK, BKk, OB, 4>), grid, block, 0, stream, a, lda, b, ldb, C, ldc, bias, \
                       M, N, K, alpha, split > 1 ? 1.f : beta, act, kchunk)
#define DTFK_GB_O(AK, BKk) \
  if (c_bf16) { DTFK_GB(AK, BKk, true); } else { DTFK_GB(AK, BKk, false); }
#define DTFK_GB_B(AK) \
  if (bkc) { DTFK_GB_O(AK, true); } else { DTFK_GB_O(AK, false); }
  if (akc) { DTFK_GB_B(true); } else { DTFK_GB_B(false); }
#undef DTFK_GB_B
#undef DTFK_GB_O
#undef DTFK_GB
  return hipGetLastError();
}

// dU[M,N] = (A' B') * gelu'(aux + bias) in bf16 and colpart[M/128][N] = its
// fp32 column sums per 128 rows: the input gradient of a linear layer fed by
// bias + GELU (BERT's FFN-down dX) with the GELU backward and the bias
// gradient's first reduction in the epilogue.  Contract (else
// hipErrorInvalidValue, nothing launched): M % 256 == 0, N % 256 == 0,
// K % 128 == 0, 16-byte aligned bases / leading dims, aux with ld = ldc.
extern "C" hipError_t dtfk_gemm_dgelu(const void* A, int lda, int transA, const void* B, int ldb, int transB,
                                      void* C, int ldc, const void* aux, const float* bias, float* colpart, int M,
                                      int N, int K, hipStream_t stream) {
  using namespace dtfk::gemm2;
  if (M % 256 || N % 256 || K % 128 || ldc % 8 || (reinterpret_cast<uintptr_t>(C) & 15) ||
      (reinterpret_cast<uintptr_t>(aux) & 15) || (reinterpret_cast<uintptr_t>(colpart) & 15) ||
      !dtfk_gemm_big_supported(A, lda, transA, B, ldb, transB, 1, M, N, K, 0.f, 0, 1))
    return hipErrorInvalidValue;
  const dim3 grid((unsigned)((M / 256) * (N / BN)), 1), block(NTHR);
  const uint16_t* a = static_cast<const uint16_t*>(A);
  const uint16_t* b = static_cast<const uint16_t*>(B);
  uint16_t* x = const_cast<uint16_t*>(static_cast<const uint16_t*>(aux));   // read only (EP_DGELU)
#define DTFK_DG(AK, BKk)                                                                                          \
  hipLaunchKernelGGL((gemm_8ph<AK, BKk, true, true, 256, EP_DGELU>), grid, block, 0, stream, a, lda, b, ldb, C,  \
                     ldc, bias, M, N, K, 1.f, 0.f, 0, K, 0LL, x, colpart)
  const bool akc = !transA, bkc = transB != 0;
  if (akc) {
    if (bkc) DTFK_DG(true, true); else DTFK_DG(true, false);
  } else {
    if (bkc) DTFK_DG(false, true); else DTFK_DG(false, false);
  }
#undef DTFK_DG
  return hipGetLastError();
}

// aux = A' B' + bias and C = gelu(aux), bf16 [M,N] with ld = ldc: the forward of
// a linear layer followed by bias + GELU (BERT's FFN-up) writing the saved
// pre-activation and the activation in one epilogue.  Contract as
// dtfk_gemm_dgelu (else hipErrorInvalidValue, nothing launched).
extern "C" hipError_t dtfk_gemm_gelu_aux(const void* A, int lda, int transA, const void* B, int ldb, int transB,
                                         void* C, int ldc, void* aux, const float* bias, int M, int N, int K,
                                         hipStream_t stream) {
  using namespace dtfk::gemm2;
  if (M % 256 || N % 256 || K % 128 || ldc % 8 || (reinterpret_cast<uintptr_t>(C) & 15) ||
      (reinterpret_cast<uintptr_t>(aux) & 15) ||
      !dtfk_gemm_big_supported(A, lda, transA, B, ldb, transB, 1, M, N, K, 0.f, 0, 1))
    return hipErrorInvalidValue;
  const dim3 grid((unsigned)((M / 256) * (N / BN)), 1), block(NTHR);
  const uint16_t* a = static_cast<const uint16_t*>(A);
  const uint16_t* b = static_cast<const uint16_t*>(B);
  uint16_t* x = static_cast<uint16_t*>(aux);
#define DTFK_GA(AK, BKk)                                                                                         \
  hipLaunchKernelGGL((gemm_8ph<AK, BKk, true, true, 256, EP_GELU_AUX>), grid, block, 0, stream, a, lda, b, ldb, \
                     C, ldc, bias, M, N, K, 1.f, 0.f, 0, K, 0LL, x, nullptr)
  const bool akc = !transA, bkc = transB != 0;
  if (akc) {
    if (bkc) DTFK_GA(true, true); else DTFK_GA(true, false);
  } else {
    if (bkc) DTFK_GA(false, true); else DTFK_GA(false, false);
  }
#undef DTFK_GA
  return hipGetLastError();
}

// Partial rows of dtfk_gemm_bn_stats' colpart: [2][P][N] floats
extern "C" int dtfk_gemm_bn_stat_rows(int M) { return (M + 127) / 128; }

// C = op(A) op(B) in bf16 (ld = ldc) and the BatchNorm statistics partials of C
// (per-column sums and sums of squares of the stored values per 128 rows) in
// colpart[2][ceil(M / 128)][N]: a 1x1 convolution's forward whose output feeds
// a BatchNorm (csrc/kernels/bn.hip bn_fwd_parts finalizes them).  Contract
// (else hipErrorInvalidValue, nothing launched): dtfk_gemm_big_supported for a
// bf16 output, K % 128 == 0, N % 8 == 0, ldc % 8 == 0, 16-byte aligned colpart.
extern "C" hipError_t dtfk_gemm_bn_stats(const void* A, int lda, int transA, const void* B, int ldb, int transB,
                                         void* C, int ldc, float* colpart, int M, int N, int K, hipStream_t stream) {
  using namespace dtfk::gemm2;
  if (K % 128 || N % 8 || ldc % 8 || (reinterpret_cast<uintptr_t>(colpart) & 15) ||
      !dtfk_gemm_big_supported(A, lda, transA, B, ldb, transB, 1, M, N, K, 0.f, 0, 1))
    return hipErrorInvalidValue;
  const dim3 grid((unsigned)(((M + 255) / 256) * ((N + BN - 1) / BN)), 1), block(NTHR);
  const uint16_t* a = static_cast<const uint16_t*>(A);
  const uint16_t* b = static_cast<const uint16_t*>(B);
#define DTFK_ST(AK, BKk)                                                                                         \
  hipLaunchKernelGGL((gemm_8ph<AK, BKk, true, true, 256, EP_STATS>), grid, block, 0, stream, a, lda, b, ldb, C, \
                     ldc, nullptr, M, N, K, 1.f, 0.f, 0, K, 0LL, nullptr, colpart)
  const bool akc = !transA, bkc = transB != 0;
  if (akc) {
    if (bkc) DTFK_ST(true, true); else DTFK_ST(true, false);
  } else {
    if (bkc) DTFK_ST(false, true); else DTFK_ST(false, false);
  }
#undef DTFK_ST
  return hipGetLastError();
}

// Tiling experiments (scripts/probes/gemm_big_cfg.py): the forward layout
// (K-contiguous x K-contiguous, bf16 out, no epilogue) at a chosen
// (BM, BK, stages).  Not used by the framework's dispatch above.
extern "C" hipError_t dtfk_gemm_big_cfg(int cfg, const void* A, int lda, const void* B, int ldb, void* C, int ldc,
                                        int M, int N, int K, hipStream_t stream) {
  using namespace dtfk::gemm2;
  if (K % KQ || M % 256 || N % 256 || lda % 8 || ldb % 8) return hipErrorInvalidValue;
  const uint16_t* a = static_cast<const uint16_t*>(A);
  const uint16_t* b = static_cast<const uint16_t*>(B);
  const int tn = N / BN;
#define DTFK_CFG(BMV, BKV, SV, ...)                                                                               \
  hipLaunchKernelGGL((gemm_big<BMV, BKV, SV, true, true, true, ##__VA_ARGS__>), dim3((M / BMV) * tn, 1), dim3(NTHR), 0, stream, \
                     a, lda, b, ldb, C, ldc, nullptr, M, N, K, 1.f, 0.f, 0, K)
  switch (cfg) {
    case 0: DTFK_CFG(256, 32, 5); break;
    case 1: DTFK_CFG(256, 64, 2); break;
    case 2: DTFK_CFG(128, 64, 3); break;
    case 3: DTFK_CFG(128, 32, 5); break;
    case 4: DTFK_CFG(256, 32, 3); break;
    case 5: DTFK_CFG(128, 64, 2); break;
    case 6: DTFK_CFG(256, 64, 2, 1); break;
    case 7: DTFK_CFG(256, 64, 2, 2); break;
    case 8: DTFK_CFG(256, 64, 2, 3); break;
    case 9: DTFK_CFG(256, 64, 2, 4); break;
    case 10:
    case 11:   // 11-13: epilogue probes (11: none, 12: a quarter of C, 13: all tiles onto tile (0, 0))
    case 12:
    case 13:
      if (K % 128) return hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_8ph<true, true, true, true>), dim3((M / 256) * tn, 1), dim3(NTHR), 0, stream, a, lda, b, ldb,
                         C, ldc, nullptr, M, N, K, 1.f, 0.f, cfg == 10 ? 0 : 10 - cfg, K);
      break;
    case 14:   // 192-wide 8-phase tiles (N % 192 == 0)
      if (K % 128 || N % 192) return hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_8ph<true, true, true, true, 192>), dim3((M / 256) * (N / 192), 1), dim3(NTHR), 0,
                         stream, a, lda, b, ldb, C, ldc, nullptr, M, N, K, 1.f, 0.f, 0, K);
      break;
    default: return hipErrorInvalidValue;
  }
#undef DTFK_CFG
  return hipGetLastError();
}
