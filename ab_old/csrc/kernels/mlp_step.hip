// Reached by: models/mlp.py FusedMLPTrainer (bench.py 3-launch fallback chain, examples --fused, smoke()); tests/test_mlp_fused_gpu.py, test_ipc_gpu.py
// Fused training step for the reference's 784-100-10 MLP
// (reference: example.py:84-118 -- x*W1+b1 -> sigmoid -> *W2+b2 -> softmax ->
// -sum(y log y_hat) mean -> GradientDescentOptimizer.minimize).
//
// MI355X design (not a translation of the TF graph).  At batch 100 the step is
// ~32 MFLOP: pure latency on this chip.  In-kernel s_memrealtime/s_memtime
// stamps (scripts/prof_mlp.py) drove the structure:
//  * every global load of a launch is issued up front and is branch-free
//    (clamped addresses, masking after the load): hipcc otherwise branches
//    around each conditional load and waits vmcnt(0) per element, turning one
//    round trip into ~14 (measured 3.4 us -> one round trip);
//  * bytes per workgroup stay small (~40 KB) and are spread over ~50 CUs, since
//    a single workgroup reads freshly written data at only ~50 GB/s;
//  * everything GEMM-shaped is on 16x16x32 bf16 MFMA (including the head's
//    backward), row reductions are DPP rotates, not LDS-latency shuffles.
//
//   A1 mlp_l1_fwd     grid (7 column tiles x 2 K-halves x B/16 row blocks) = 98
//                     workgroups at B=100, 4 waves split K.  Each pulls a 16-row
//                     x slice (uint8 pixels converted to bf16 in registers) and
//                     half of one 16-column tile of the bf16 W1 shadow (stored
//                     K-contiguous: every B fragment is one 16-byte load);
//                     cross-wave reduction in LDS; writes partial z2 (fp32).
//   A2 mlp_head_bwd   one 8-wave workgroup per 16 rows: sums the K-halves, bias +
//                     sigmoid/ReLU, layer 2 (MFMA), softmax cross-
//                     entropy on the MFMA accumulator layout with DPP row
//                     reductions (stable log-sum-exp, or the reference's naive
//                     -sum(y log p)), argmax accuracy, dz3; dz2 = dz3 W2^T *
//                     act'(z2) and dW2^T = dz3^T a2 on MFMA; dz2^T (bf16,
//                     batch-contiguous) stored straight from the accumulators;
//                     per-block partial dW2/db1/db2/loss/correct slab.
//   B  mlp_wgrad      dW1 = x^T dz2: one wave per 16x16 tile of dW1 (343 tiles);
//                     the wave transposes its 16-column x strip through LDS and
//                     runs B/32 MFMAs.  FUSED (1 GPU): SGD in
//                     the epilogue + bf16 shadow refresh, no gradient round trip.
//                     GRAD: gradients to one flat bucket (fp32|bf16) for the
//                     RCCL all-reduce.  Four reducer workgroups sum A2's slabs in
//                     a fixed order (deterministic, no float atomics); the last
//                     writes loss/accuracy into the device metrics ring and bumps
//                     the device global_step.
//   C  mlp_apply_flat after the all-reduce: p -= lr*scale*g over the flat bucket +
//                     shadow refresh (also builds shadows after init/restore).
//
// Flat parameter layout == TF variable order of example.py:
//   W1 [784,100] @0, W2 [100,10] @78400, b1 [100] @79400, b2 [10] @79500.
// bf16 shadows: W1T [112][800] (n-major, k contiguous), W2T [16][128] (class-
// major, hidden contiguous), W2N [112][32] (hidden-major, class contiguous).
#include "common.h"

namespace dtfk {
namespace mlp {

constexpr int DIN = 784, DINP = 800;   // K of layer 1, padded to 25*32
constexpr int HID = 100, HIDP = 112;   // N of layer 1 (7 MFMA col tiles)
constexpr int HIDK = 128;              // K of layer 2 padded to 4*32
constexpr int NCLS = 10;
constexpr int OFF_W1 = 0, OFF_W2 = 78400, OFF_B1 = 79400, OFF_B2 = 79500;
constexpr int NPARAM = 79510;
constexpr int PART = 1112;             // dW2(1000) db1(100) db2(10) loss correct
constexpr int A2S = 136;               // LDS row stride (bf16) of a2
constexpr int D3S = 40;                // LDS row stride (bf16) of dz3
constexpr int ROWS = 16;
constexpr int NSTRIP = DIN / 16;       // 49 dW1 row strips
constexpr int NRED = 4;                // reducer workgroups in B
constexpr int RCH = (PART + NRED - 1) / NRED;  // 278 slab entries per reducer
constexpr int KSPLIT = 2;              // layer-1 K halves (spreads W1 reads over 2x CUs)
constexpr int KS_PER = 13;             // k-steps per half: [0,13) and [13,25)
constexpr int KJ = (KS_PER + 3) / 4;   // k-steps per wave
// IPC exchange buffer: [flag area][grad slot 0][grad slot 1]; flag area holds
// the step flag (offset 0) and one flag per wgrad workgroup (offset 64 + 8*wg)
constexpr int IPC_FLAG_BYTES = 4096;
constexpr int IPC_WG_FLAG0 = 64;

// debug stamps: slot ph = s_memrealtime (100 MHz), slot 8+ph = s_memtime (core clock)
#define TS(ph)                                                                       \
  if (ts != nullptr && threadIdx.x == 0) {                                           \
    long long* t_ = ts + (blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) * 16; \
    t_[(ph)] = (long long)__builtin_amdgcn_s_memrealtime();                          \
    t_[8 + (ph)] = (long long)__builtin_amdgcn_s_memtime();                          \
  }

// 8 consecutive input features of one row as fp32 (XK: 0 u8/255, 1 fp32, 2 bf16)
template <int XK>
__device__ __forceinline__ void load_x8(const uint8_t* __restrict__ xin, size_t e, float v[8]) {
  if constexpr (XK == 0) {
    const uint2 u = *reinterpret_cast<const uint2*>(xin + e);
    const float s = 1.f / 255.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = (float)((u.x >> (8 * j)) & 255u) * s;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[4 + j] = (float)((u.y >> (8 * j)) & 255u) * s;
  } else if constexpr (XK == 1) {
    const float4* f = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(xin) + e);
    const float4 a = f[0], b = f[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
    const uint4 u = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(xin) + e);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[2 * j] = bf2f(w[j] & 0xffff); v[2 * j + 1] = bf2f(w[j] >> 16); }
  }
}

__device__ __forceinline__ bf16x8 to_bf16x8(const float v[8], bool keep) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = static_cast<__bf16>(keep ? v[j] : 0.f);
  return r;
}

// ---------------------------------------------------------------------- A1
// grid (7 column tiles, KSPLIT K-halves, B/16 row blocks); writes the partial
// pre-activation z2 of its K-half: z2p[ksplit][row][n] (fp32).
template <int XK>
__global__ __launch_bounds__(256) void mlp_l1_fwd(
    const uint8_t* __restrict__ xin, int B, const uint16_t* __restrict__ W1T,
    float* __restrict__ z2p, long long* __restrict__ ts) {
  TS(0);
  __shared__ float red[4][16][17];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lh = lane >> 4;
  const int ct = blockIdx.x;                 // column tile of W1 / z2
  const int ks0 = blockIdx.y * KS_PER;       // first k-step of this K-half
  const int ks1 = min(25, ks0 + KS_PER);
  const int r0 = blockIdx.z * ROWS;          // first batch row
  const int row = r0 + lr;
  const bool rv = row < B;
  const size_t xrow = (size_t)min(row, B - 1) * DIN;

  // all global loads first, branch-free: k-steps ks = ks0 + wave + 4*j,
  // clamped into range and masked at use
  bf16x8 bw[KJ];
  float xv[KJ][8];
  const uint16_t* pw = W1T + (size_t)(ct * 16 + lr) * DINP + lh * 8;
#pragma unroll
  for (int j = 0; j < KJ; ++j) {
    const int ks = ks0 + wave + 4 * j;
    bw[j] = ld_bf16x8(pw + min(ks, 24) * 32);
    load_x8<XK>(xin, xrow + min(ks * 32 + lh * 8, DIN - 8), xv[j]);
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < KJ; ++j) {
    const int ks = ks0 + wave + 4 * j;
    const bool keep = rv && ks < ks1 && ks * 32 + lh * 8 < DIN;
    acc = mfma16x16x32(to_bf16x8(xv[j], keep), bw[j], acc);
  }
  TS(1);
#pragma unroll
  for (int i = 0; i < 4; ++i) red[wave][4 * lh + i][lr] = acc[i];
  __syncthreads();
  TS(2);
  {
    const int r = tid >> 4, c = tid & 15;
    const size_t nrows = (size_t)gridDim.z * ROWS;
    z2p[((size_t)blockIdx.y * nrows + r0 + r) * HIDP + ct * 16 + c] =
        red[0][r][c] + red[1][r][c] + red[2][r][c] + red[3][r][c];
  }
  TS(3);
}

// ---------------------------------------------------------------------- A2
// agent-coherent (L2-bypassing, sc1) loads of a float4 written by another XCD
__device__ __forceinline__ float4 ld_coherent4(const float* p) {
  float4 r;
  r.x = __hip_atomic_load(p + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  r.y = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  r.z = __hip_atomic_load(p + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  r.w = __hip_atomic_load(p + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return r;
}

// one 512-thread workgroup per 16 batch rows (row block rb of nblk).
// COHERENT_Z: z2p was produced by other workgroups of the SAME launch (merged
// kernel) -> read it with agent-coherent loads instead of plain cached loads.
template <bool COHERENT_Z>
__device__ __forceinline__ void head_bwd_block(
    int rb, int nblk, const float* __restrict__ z2p, const uint8_t* __restrict__ labels, int B,
    const uint16_t* __restrict__ W2T, const uint16_t* __restrict__ W2N,
    const float* __restrict__ params, uint16_t* __restrict__ dz2T, int BP,
    float* __restrict__ partials, float inv_batch, int act, int naive_loss,
    long long* __restrict__ gstep, long long* __restrict__ ts) {
  __shared__ __attribute__((aligned(16))) float a2f[ROWS * HIDP];      // [r][n] fp32
  __shared__ __attribute__((aligned(16))) uint16_t a2b[ROWS * A2S];    // [r][n] bf16, n<128
  __shared__ __attribute__((aligned(16))) uint16_t a2T[HIDP * D3S];    // [n][r] bf16, r<32
  __shared__ __attribute__((aligned(16))) uint16_t dz3b[ROWS * D3S];   // [r][c] bf16, c<32
  __shared__ __attribute__((aligned(16))) uint16_t dz3T[ROWS * D3S];   // [c][r] bf16, r<32
  __shared__ float wred[4][18];                                        // db2[16], loss, correct

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lh = lane >> 4;
  const int r0 = rb * ROWS;
  const size_t nrows = (size_t)nblk * ROWS;
  float* part = partials + (size_t)rb * PART;

  // ---- all global loads up front (branch-free) ----
  const int qi = min(tid, ROWS * HIDP / 4 - 1);  // float4 index in the 16x112 slice
  const int qr = (4 * qi) / HIDP, qc = (4 * qi) % HIDP;
  float4 zq = COHERENT_Z ? ld_coherent4(z2p + (size_t)r0 * HIDP + 4 * qi)
                         : reinterpret_cast<const float4*>(z2p + (size_t)r0 * HIDP)[qi];
#pragma unroll
  for (int k = 1; k < KSPLIT; ++k) {
    const float4 z = COHERENT_Z ? ld_coherent4(z2p + ((size_t)k * nrows + r0) * HIDP + 4 * qi)
                                : reinterpret_cast<const float4*>(z2p + ((size_t)k * nrows + r0) * HIDP)[qi];
    zq.x += z.x; zq.y += z.y; zq.z += z.z; zq.w += z.w;
  }
  float b1q[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) b1q[j] = params[OFF_B1 + min(qc + j, HID - 1)];
  bf16x8 bw2[HIDK / 32];
#pragma unroll
  for (int ks = 0; ks < HIDK / 32; ++ks) bw2[ks] = ld_bf16x8(W2T + lr * HIDK + ks * 32 + lh * 8);
  const float b2v = params[OFF_B2 + min(lr, NCLS - 1)];
  const int srow = 4 * lh + (wave & 3);  // softmax row of this lane (waves 0..3)
  int y = labels[min(r0 + srow, B - 1)];
  y = y < NCLS ? y : 0;  // corrupt label ids cannot index out of the row
  const bf16x8 bn = ld_bf16x8(W2N + (min(wave, 6) * 16 + lr) * 32 + lh * 8);

  // ---- a2 = act(z2 + b1) in three LDS layouts; zero the MFMA K-pads ----
  if (tid < ROWS * HIDP / 4) {
    float zz[4] = {zq.x, zq.y, zq.z, zq.w};
    float a[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float z = zz[j] + b1q[j];
      a[j] = act == 0 ? sigmoidf_(z) : fmaxf(z, 0.f);
      if (qc + j >= HID || r0 + qr >= B) a[j] = 0.f;
      a2T[(qc + j) * D3S + qr] = f2bf(a[j]);
    }
    reinterpret_cast<float4*>(a2f)[tid] = make_float4(a[0], a[1], a[2], a[3]);
    *reinterpret_cast<uint2*>(&a2b[qr * A2S + qc]) = make_uint2(pack2bf(a[0], a[1]), pack2bf(a[2], a[3]));
  } else {
    const int q = tid - ROWS * HIDP / 4;  // 64 threads
    *reinterpret_cast<uint2*>(&a2b[(q >> 2) * A2S + HIDP + (q & 3) * 4]) = make_uint2(0u, 0u);
    const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int u = 0; u < 4; ++u) {  // a2T rows 16..31 for all 112 hidden units (224 uint4)
      const int e = q + 64 * u;
      if (e < 2 * HIDP) *reinterpret_cast<uint4*>(&a2T[(e >> 1) * D3S + 16 + 8 * (e & 1)]) = z4;
    }
    if (q < 32) *reinterpret_cast<uint4*>(&dz3b[(q >> 1) * D3S + 16 + 8 * (q & 1)]) = z4;
    else *reinterpret_cast<uint4*>(&dz3T[((q - 32) >> 1) * D3S + 16 + 8 * (q & 1)]) = z4;
  }
  __syncthreads();
  TS(1);

  // ---- layer 2 + softmax cross-entropy (waves 0..3, one accumulator row each) ----
  // lane: class c = lr; wave w handles rows 4*lh + w.  Row reductions are over
  // the 16 lanes of a DPP row (= the 16 classes of one batch row).
  if (wave < 4) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < HIDK / 32; ++ks)
      acc = mfma16x16x32(ld_bf16x8(a2b + lr * A2S + ks * 32 + lh * 8), bw2[ks], acc);
    const int c = lr;
    const bool cv = c < NCLS;
    const bool valid = r0 + srow < B;
    const float z = (wave == 0 ? acc[0] : wave == 1 ? acc[1] : wave == 2 ? acc[2] : acc[3]) + b2v;
    const float v = cv ? z : -3.0e38f;
    const float m = row16_max(v);
    const float e = cv ? __expf(v - m) : 0.f;
    const float ssum = row16_sum(e);
    const float p = e * __frcp_rn(ssum);
    const float zy = row16_sum(c == y ? z : 0.f);
    const float am = row16_min((cv && v == m) ? (float)c : 1e9f);  // tf.argmax: first max
    const float loss = naive_loss ? -__logf(row16_sum(c == y ? p : 0.f)) : (m + __logf(ssum) - zy);
    const float d = (valid && cv) ? (p - (c == y ? 1.f : 0.f)) * inv_batch : 0.f;
    const uint16_t db = f2bf(d);
    dz3b[srow * D3S + c] = db;
    dz3T[c * D3S + srow] = db;
    float db2 = d;
    db2 += __shfl_xor(db2, 16, 64);
    db2 += __shfl_xor(db2, 32, 64);
    const float lsum = wave_sum((c == 0 && valid) ? loss : 0.f);
    const float csum = wave_sum((c == 0 && valid && (int)am == y) ? 1.f : 0.f);
    if (lh == 0) wred[wave][c] = db2;
    if (lane == 0) { wred[wave][16] = lsum; wred[wave][17] = csum; }
  }
  __syncthreads();
  TS(2);

  if (wave < 7) {
    // ---- hidden tile t = wave: dz2 = (dz3 W2^T) * act'(a2), dW2^T = dz3^T a2 ----
    const int n = wave * 16 + lr;
    const f32x4 acc = mfma16x16x32(ld_bf16x8(dz3b + lr * D3S + lh * 8), bn, f32x4{0.f, 0.f, 0.f, 0.f});
    float d[4], sdb = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float a = a2f[(4 * lh + i) * HIDP + n];  // 0 for pad rows/cols -> d = 0
      d[i] = act == 0 ? acc[i] * a * (1.f - a) : (a > 0.f ? acc[i] : 0.f);
      sdb += d[i];
    }
    *reinterpret_cast<uint2*>(&dz2T[(size_t)n * BP + r0 + 4 * lh]) =
        make_uint2(pack2bf(d[0], d[1]), pack2bf(d[2], d[3]));
    sdb += __shfl_xor(sdb, 16, 64);
    sdb += __shfl_xor(sdb, 32, 64);
    if (lh == 0 && n < HID) part[1000 + n] = sdb;
    const f32x4 w = mfma16x16x32(ld_bf16x8(dz3T + lr * D3S + lh * 8),
                                 ld_bf16x8(a2T + n * D3S + lh * 8), f32x4{0.f, 0.f, 0.f, 0.f});
    if (n < HID) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = 4 * lh + i;
        if (c < NCLS) part[n * NCLS + c] = w[i];
      }
    }
  } else if (lane < 18) {
    const float v = wred[0][lane] + wred[1][lane] + wred[2][lane] + wred[3][lane];
    if (lane < NCLS) part[1100 + lane] = v;
    else if (lane >= 16) part[1110 + (lane - 16)] = v;
  }
  // the device global step advances here (not in B), so B -- and the IPC
  // exchange inside it -- sees one stable epoch value
  if (rb == 0 && tid == 0) *gstep += 1;
}

__global__ __launch_bounds__(512) void mlp_head_bwd(
    const float* __restrict__ z2p, const uint8_t* __restrict__ labels, int B,
    const uint16_t* __restrict__ W2T, const uint16_t* __restrict__ W2N,
    const float* __restrict__ params, uint16_t* __restrict__ dz2T, int BP,
    float* __restrict__ partials, float inv_batch, int act, int naive_loss,
    long long* __restrict__ gstep, long long* __restrict__ ts) {
  TS(0);
  head_bwd_block<false>(blockIdx.x, gridDim.x, z2p, labels, B, W2T, W2N, params, dz2T, BP, partials, inv_batch,
                        act, naive_loss, gstep, ts);
  TS(3);
}

// ---------------------------------------------------------------------- A (A1 + A2 in one launch)
// Same layer-1 tiling as A1 with 8 waves per workgroup; the LAST of the
// 7 x KSPLIT workgroups of a row block to finish (device-scope counter,
// release/acquire fences) runs that row block's head/backward (A2) in place.
// Removes the A1 -> A2 kernel boundary (~2.6 us of launch gap measured with
// s_memrealtime stamps) and lets early row blocks start A2 while others still
// run layer 1.  The counter is reset by its last arriver (graph-replay safe).
constexpr int KJ8 = (KS_PER + 7) / 8;   // k-steps per wave with 8 waves

template <int XK>
__global__ __launch_bounds__(512) void mlp_fwd_head(
    const uint8_t* __restrict__ xin, int B, const uint16_t* __restrict__ W1T, float* __restrict__ z2p,
    const uint8_t* __restrict__ labels, const uint16_t* __restrict__ W2T, const uint16_t* __restrict__ W2N,
    const float* __restrict__ params, uint16_t* __restrict__ dz2T, int BP, float* __restrict__ partials,
    float inv_batch, int act, int naive_loss, int* __restrict__ counters, long long* __restrict__ gstep) {
  __shared__ float red8[8][16][17];
  __shared__ int last;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lh = lane >> 4;
  const int ct = blockIdx.x;
  const int ks0 = blockIdx.y * KS_PER;
  const int ks1 = min(25, ks0 + KS_PER);
  const int rb = blockIdx.z;
  const int r0 = rb * ROWS;
  const int row = r0 + lr;
  const bool rv = row < B;
  const size_t xrow = (size_t)min(row, B - 1) * DIN;

  bf16x8 bw[KJ8];
  float xv[KJ8][8];
  const uint16_t* pw = W1T + (size_t)(ct * 16 + lr) * DINP + lh * 8;
#pragma unroll
  for (int j = 0; j < KJ8; ++j) {
    const int ks = ks0 + wave + 8 * j;
    bw[j] = ld_bf16x8(pw + min(ks, 24) * 32);
    load_x8<XK>(xin, xrow + min(ks * 32 + lh * 8, DIN - 8), xv[j]);
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < KJ8; ++j) {
    const int ks = ks0 + wave + 8 * j;
    const bool keep = rv && ks < ks1 && ks * 32 + lh * 8 < DIN;
    acc = mfma16x16x32(to_bf16x8(xv[j], keep), bw[j], acc);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) red8[wave][4 * lh + i][lr] = acc[i];
  __syncthreads();
  if (tid < 256) {
    const int r = tid >> 4, c = tid & 15;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) v += red8[w][r][c];
    // agent-coherent write-through store (sc1): visible to the other XCDs
    // without a full-L2 writeback (a __threadfence() release here costs a
    // buffer_wbl2 per workgroup: measured 13 -> 31 us per step)
    __hip_atomic_store(&z2p[((size_t)blockIdx.y * gridDim.z * ROWS + r0 + r) * HIDP + ct * 16 + c], v,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __builtin_amdgcn_s_waitcnt(0);   // this thread's stores acknowledged
  __syncthreads();                 // ... for every thread of the block
  if (tid == 0) {
    const int prev = __hip_atomic_fetch_add(&counters[rb], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = prev == (int)(gridDim.x * gridDim.y) - 1;
    if (last) __hip_atomic_store(&counters[rb], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!last) return;
  head_bwd_block<true>(rb, gridDim.z, z2p, labels, B, W2T, W2N, params, dz2T, BP, partials, inv_batch, act,
                       naive_loss, gstep, nullptr);
}

// ---------------------------------------------------------------------- IPC (in-B exchange)
struct IpcArgs {
  void* const* peer_base;   // W base pointers of the exchange buffers (own + mapped peers)
  int W, rank, parity;
  long long slot_bytes;
  float scale;              // 1 / W
  int* err;
  long long timeout;        // s_memrealtime ticks
};

__device__ __forceinline__ uint16_t* ipc_slot(const IpcArgs& a, int r) {
  return reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(a.peer_base[r]) + IPC_FLAG_BYTES +
                                     (long long)a.parity * a.slot_bytes);
}

// Single-wave workgroup `wg` publishes its epoch flag after its gradient
// stores (uncached exchange memory: completion == visibility, no L2 writeback
// needed), then lane r waits for peer r's flag of the same workgroup -- the W
// remote polls overlap.  Returns false (and raises err) on timeout.
// Ordering: the asm wait is both the hardware drain (every slot store of this
// wave acknowledged by the fabric) and a compiler memory barrier (the
// `__builtin_amdgcn_s_waitcnt` builtin is IntrNoMem and let the flag store be
// scheduled above the payload stores).  The consumer side ends its poll with a
// second asm barrier so no slot load is hoisted above the flag match; its slot
// loads are non-temporal loads of uncached memory (the guide's sc1-load form
// of the acquire, MI355X_MICROARCH.md "Valid forms").
// Publication order: the slot buffers are hipDeviceMallocUncached (ipc_peer.cpp),
// so a gradient store's vmcnt completes only once the write has reached memory;
// the waitcnt below (an asm with a "memory" clobber, so also a compiler barrier)
// retires every slot store before the flag store issues, and peers read the
// slots with system-scope loads after seeing the flag.  A release store would
// add an L2 writeback (buffer_wbl2) that uncached data does not need.
__device__ __forceinline__ bool ipc_wg_sync(const IpcArgs& a, int wg, unsigned long long epoch, int lane) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const long long off = IPC_WG_FLAG0 + 8LL * wg;
  if (lane == 0)
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(a.peer_base[a.rank]) + off),
                       epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  int good = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
  if (good && lane < a.W && lane != a.rank) {
    const unsigned long long* f =
        reinterpret_cast<const unsigned long long*>(reinterpret_cast<const char*>(a.peer_base[lane]) + off);
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      __builtin_amdgcn_s_sleep(1);
      if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) {
        atomicOr(a.err, 1);
        good = 0;
        break;
      }
    }
  }
  const bool all_good = __all(good);
  asm volatile("" ::: "memory");   // no peer-slot load above the flag match
  return all_good;
}

// ---------------------------------------------------------------------- B
// grid: NSTRIP*7 tile workgroups (16-row strip of dW1 x 16-column tile) + NRED
// MODE 0: fused SGD (1 GPU); 1: gradients to a flat bucket (RCCL); 2: IPC --
// every workgroup exchanges its own gradient block with the same workgroup on
// all peer GPUs and applies SGD in place (no separate all-reduce/apply launch).
template <int KSTEPS, int XK, int MODE>  // KSTEPS > 0: K = 32*KSTEPS; 0: runtime BP
__global__ __launch_bounds__(64) void mlp_wgrad(
    const uint8_t* __restrict__ xin, const uint16_t* __restrict__ dz2T, int BP, int B,
    const float* __restrict__ partials, int nblk_rows, float* __restrict__ params,
    uint16_t* __restrict__ W1T, uint16_t* __restrict__ W2T, uint16_t* __restrict__ W2N,
    void* __restrict__ grads, int grad_bf16, const float* __restrict__ lr_ptr,
    float* __restrict__ metrics, long long* __restrict__ gstep, int ring,
    long long* __restrict__ ts, IpcArgs ipc) {
  constexpr bool FUSED = MODE == 0;
  constexpr bool NEEDP = MODE != 1;     // master params read for an in-kernel update
  TS(0);
  extern __shared__ __attribute__((aligned(16))) uint16_t xt[];  // [16][BP + 8] bf16
  const int lane = threadIdx.x;
  const int lr = lane & 15, lh = lane >> 4;
  constexpr int NTILE = NSTRIP * 7;

  if ((int)blockIdx.x < NTILE) {
    const int strip = blockIdx.x / 7, t = blockIdx.x % 7;
    const int k0 = strip * 16;
    const int kr = k0 + 4 * lh;
    const int n = t * 16 + lr;
    const int XTS = BP + 8;
    float pm[4];
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if constexpr (NEEDP) {  // master W1 for the SGD epilogue, issued first
#pragma unroll
      for (int i = 0; i < 4; ++i) pm[i] = params[OFF_W1 + (kr + i) * HID + min(n, HID - 1)];
    }
    const uint16_t* pb = dz2T + (size_t)n * BP + lh * 8;
    if constexpr (KSTEPS > 0) {
      bf16x8 b[KSTEPS];
#pragma unroll
      for (int s = 0; s < KSTEPS; ++s) b[s] = ld_bf16x8(pb + s * 32);
      constexpr int NQ = (KSTEPS * 32 + 63) / 64;
      float v[NQ][16];
#pragma unroll
      for (int q = 0; q < NQ; ++q) {  // lane = batch row of the x strip
        const size_t e = (size_t)min(lane + 64 * q, B - 1) * DIN + k0;
        load_x8<XK>(xin, e, v[q]);
        load_x8<XK>(xin, e + 8, v[q] + 8);
      }
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int bq = lane + 64 * q;
        if (bq < BP) {
#pragma unroll
          for (int j = 0; j < 16; ++j) xt[j * XTS + bq] = f2bf(bq < B ? v[q][j] : 0.f);
        }
      }
      __syncthreads();
      TS(1);
#pragma unroll
      for (int s = 0; s < KSTEPS; ++s) acc = mfma16x16x32(ld_bf16x8(xt + lr * XTS + s * 32 + lh * 8), b[s], acc);
    } else {
      for (int bq = lane; bq < BP; bq += 64) {
        float v[16];
        const size_t e = (size_t)min(bq, B - 1) * DIN + k0;
        load_x8<XK>(xin, e, v);
        load_x8<XK>(xin, e + 8, v + 8);
#pragma unroll
        for (int j = 0; j < 16; ++j) xt[j * XTS + bq] = f2bf(bq < B ? v[j] : 0.f);
      }
      __syncthreads();
      TS(1);
      for (int kb = 0; kb < BP; kb += 32)
        acc = mfma16x16x32(ld_bf16x8(xt + lr * XTS + kb + lh * 8), ld_bf16x8(pb + kb), acc);
    }
    TS(2);
    if constexpr (MODE == 2) {
      const unsigned long long epoch = (unsigned long long)(*gstep);
      const int nc = min(n, HID - 1);
      uint16_t gb[4];
      uint16_t* mine = ipc_slot(ipc, ipc.rank);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        gb[i] = f2bf(acc[i]);
        if (n < HID) mine[OFF_W1 + (kr + i) * HID + n] = gb[i];
      }
      if (!ipc_wg_sync(ipc, blockIdx.x, epoch, lane)) return;
      float g[4] = {0.f, 0.f, 0.f, 0.f};
      for (int r = 0; r < ipc.W; ++r) {   // rank order: identical sums on every GPU
        const uint16_t* src = ipc_slot(ipc, r);
#pragma unroll
        for (int i = 0; i < 4; ++i)
          g[i] += bf2f(r == ipc.rank ? gb[i] : ld_sys_u16(src + OFF_W1 + (kr + i) * HID + nc));
      }
      if (n < HID) {
        const float step = (*lr_ptr) * ipc.scale;
        float p[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          p[i] = pm[i] - step * g[i];
          params[OFF_W1 + (kr + i) * HID + n] = p[i];
        }
        *reinterpret_cast<uint2*>(&W1T[(size_t)n * DINP + kr]) = make_uint2(pack2bf(p[0], p[1]), pack2bf(p[2], p[3]));
      }
      TS(3);
      return;
    }
    if (n < HID) {
      if constexpr (FUSED) {
        const float lrate = *lr_ptr;
        float p[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          p[i] = pm[i] - lrate * acc[i];
          params[OFF_W1 + (kr + i) * HID + n] = p[i];
        }
        *reinterpret_cast<uint2*>(&W1T[(size_t)n * DINP + kr]) =
            make_uint2(pack2bf(p[0], p[1]), pack2bf(p[2], p[3]));
      } else if (grad_bf16) {
        uint16_t* g = reinterpret_cast<uint16_t*>(grads);
#pragma unroll
        for (int i = 0; i < 4; ++i) g[OFF_W1 + (kr + i) * HID + n] = f2bf(acc[i]);
      } else {
        float* g = reinterpret_cast<float*>(grads);
#pragma unroll
        for (int i = 0; i < 4; ++i) g[OFF_W1 + (kr + i) * HID + n] = acc[i];
      }
    }
    TS(3);
    return;
  }

  // ---- reducer workgroups: small-parameter gradients (+ metrics, step) ----
  const int jr = blockIdx.x - NTILE;
  const int lo = jr * RCH, hi = min(PART, lo + RCH);
  constexpr int NU = (RCH + 63) / 64;  // 5 entries per lane
  float s[NU];
  float pv[NU];
  if constexpr (KSTEPS > 0) {
    constexpr int NBM = 2 * KSTEPS;  // row blocks <= BP/16
    float v[NU][NBM];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int i = min(lo + lane + 64 * u, PART - 1);
#pragma unroll
      for (int b = 0; b < NBM; ++b) v[u][b] = partials[(size_t)min(b, nblk_rows - 1) * PART + i];
      if constexpr (NEEDP) pv[u] = params[OFF_W2 + min(i, 1109)];
    }
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      s[u] = 0.f;
#pragma unroll
      for (int b = 0; b < NBM; ++b) s[u] += b < nblk_rows ? v[u][b] : 0.f;
    }
  } else {
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int i = min(lo + lane + 64 * u, PART - 1);
      s[u] = 0.f;
      for (int b = 0; b < nblk_rows; ++b) s[u] += partials[(size_t)b * PART + i];
      if constexpr (NEEDP) pv[u] = params[OFF_W2 + min(i, 1109)];
    }
  }
  float* lred = reinterpret_cast<float*>(xt);
  const float lrate = *lr_ptr;
  if constexpr (MODE == 2) {   // exchange the small-parameter gradients of this reducer's range
    const unsigned long long epoch = (unsigned long long)(*gstep);
    uint16_t* mine = ipc_slot(ipc, ipc.rank);
    uint16_t gb[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int i = lo + lane + 64 * u;
      gb[u] = f2bf(s[u]);
      if (i < hi && i < 1110) mine[OFF_W2 + i] = gb[u];
    }
    const bool ok = ipc_wg_sync(ipc, blockIdx.x, epoch, lane);
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int i = lo + lane + 64 * u;
      const int ic = min(i, 1109);
      float g = 0.f;
      for (int r = 0; r < ipc.W; ++r)
        g += bf2f(r == ipc.rank ? gb[u] : ld_sys_u16(ipc_slot(ipc, r) + OFF_W2 + ic));
      if (i >= hi) continue;
      if (i >= 1110) { lred[i - 1110] = s[u]; continue; }
      if (!ok) continue;
      const float p = pv[u] - lrate * ipc.scale * g;
      params[OFF_W2 + i] = p;
      if (i < 1000) {
        W2T[(i % NCLS) * HIDK + i / NCLS] = f2bf(p);
        W2N[(i / NCLS) * 32 + i % NCLS] = f2bf(p);
      }
    }
  } else {
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int i = lo + lane + 64 * u;
    if (i >= hi) continue;
    if (i >= 1110) { lred[i - 1110] = s[u]; continue; }
    if constexpr (FUSED) {
      const float p = pv[u] - lrate * s[u];
      params[OFF_W2 + i] = p;
      if (i < 1000) {
        W2T[(i % NCLS) * HIDK + i / NCLS] = f2bf(p);
        W2N[(i / NCLS) * 32 + i % NCLS] = f2bf(p);
      }
    } else if (grad_bf16) {
      reinterpret_cast<uint16_t*>(grads)[OFF_W2 + i] = f2bf(s[u]);
    } else {
      reinterpret_cast<float*>(grads)[OFF_W2 + i] = s[u];
    }
  }
  }
  if (hi == PART) {
    __syncthreads();
    if (lane == 0) {
      const long long st = *gstep - 1;   // the head kernel already advanced the step
      const int slot = (int)(st % ring);
      metrics[2 * slot] = lred[0] / (float)B;
      metrics[2 * slot + 1] = lred[1] / (float)B;
    }
  }
  TS(3);
}

// ---------------------------------------------------------------------- C
__global__ __launch_bounds__(256) void mlp_apply_flat(
    float* __restrict__ params, const void* __restrict__ grads, int grad_bf16,
    const float* __restrict__ lr_ptr, float scale, uint16_t* __restrict__ W1T,
    uint16_t* __restrict__ W2T, uint16_t* __restrict__ W2N) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= NPARAM) return;
  float p = params[i];
  if (grads != nullptr) {
    const float g = grad_bf16 ? bf2f(reinterpret_cast<const uint16_t*>(grads)[i])
                              : reinterpret_cast<const float*>(grads)[i];
    p -= (*lr_ptr) * scale * g;
    params[i] = p;
  }
  if (i < OFF_W2) {
    W1T[(size_t)(i % HID) * DINP + i / HID] = f2bf(p);
  } else if (i < OFF_B1) {
    const int j = i - OFF_W2;
    W2T[(j % NCLS) * HIDK + j / NCLS] = f2bf(p);
    W2N[(j / NCLS) * 32 + j % NCLS] = f2bf(p);
  }
}
// ---------------------------------------------------------------------- C'
// One-shot all-reduce fused into the SGD apply, for N GPUs of one node.
// Every rank's wgrad (GRAD mode, bf16) wrote its gradient into its own
// IPC-exported uncached buffer (parity slot); peers' buffers are mapped.
//   1. each block's thread 0 publishes this rank's epoch (= device global
//      step, bumped by wgrad) in its flag word -- idempotent, so no block
//      depends on another being scheduled;
//   2. it waits (bounded, s_memrealtime) until every peer's flag reached the
//      epoch: all gradients of this step are complete and visible;
//   3. the block sums the N gradients in rank order (identical on every rank
//      -> replicas stay bit-identical), p -= lr*scale*sum, refreshes shadows.
// Each rank reads (N-1) x 159 KB over its xGMI links in parallel instead of a
// ring's 2(N-1) latency-bound hops.  Double-buffered by step parity: a rank
// rewrites slot p only after its next apply saw every peer's flag for the
// step in between, i.e. after every peer finished reading slot p.
__global__ __launch_bounds__(256) void mlp_ipc_reduce_apply(
    float* __restrict__ params, void* const* __restrict__ peer_base, int W, int rank, int parity,
    long long slot_bytes, const long long* __restrict__ gstep, const float* __restrict__ lr_ptr, float scale,
    uint16_t* __restrict__ W1T, uint16_t* __restrict__ W2T, uint16_t* __restrict__ W2N, int* __restrict__ err,
    long long timeout_ticks) {
  __shared__ int ok;
  const unsigned long long epoch = (unsigned long long)(*gstep);
  if (threadIdx.x == 0) {
    ok = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;  // fail fast after a timeout
    __threadfence_system();
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(peer_base[rank]), epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  // lane r polls peer r's flag: the W remote round trips overlap instead of
  // running back to back (~1 us each over xGMI)
  if (ok && threadIdx.x < W) {
    const unsigned long long* f = reinterpret_cast<const unsigned long long*>(peer_base[threadIdx.x]);
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    // relaxed polls (an acquire load is an L2 invalidate per poll), one acquire after
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      __builtin_amdgcn_s_sleep(1);
      if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
        atomicOr(err, 1);
        ok = 0;
        break;
      }
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
  }
  __syncthreads();
  if (!ok) return;
  const int i0 = (blockIdx.x * blockDim.x + threadIdx.x) * 2;   // 2 params per thread (4-byte loads)
  if (i0 >= NPARAM) return;
  const long long off = IPC_FLAG_BYTES + (long long)parity * slot_bytes;
  float g0 = 0.f, g1 = 0.f;
  for (int r = 0; r < W; ++r) {
    const uint32_t u = ld_sys_u32(
        reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(peer_base[r]) + off) + (i0 >> 1));
    g0 += bf2f(u & 0xFFFF);
    g1 += bf2f(u >> 16);
  }
  const float step = (*lr_ptr) * scale;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int i = i0 + j;
    const float p = params[i] - step * (j == 0 ? g0 : g1);
    params[i] = p;
    if (i < OFF_W2) {
      W1T[(size_t)(i % HID) * DINP + i / HID] = f2bf(p);
    } else if (i < OFF_B1) {
      const int q = i - OFF_W2;
      W2T[(q % NCLS) * HIDK + q / NCLS] = f2bf(p);
      W2N[(q / NCLS) * 32 + q % NCLS] = f2bf(p);
    }
  }
}

#undef TS

}  // namespace mlp
}  // namespace dtfk

// ---------------------------------------------------------------- launchers
extern "C" {

int dtfk_mlp_ksplit() { return dtfk::mlp::KSPLIT; }

hipError_t dtfk_mlp_l1_fwd(const void* x, int x_kind, int B, const void* W1T, float* z2p,
                           long long* ts, hipStream_t stream) {
  using namespace dtfk::mlp;
  const dim3 grid(HIDP / 16, KSPLIT, (B + 15) / 16);
  const uint8_t* xp = (const uint8_t*)x;
  const uint16_t* w = (const uint16_t*)W1T;
  switch (x_kind) {
    case 0: hipLaunchKernelGGL(mlp_l1_fwd<0>, grid, dim3(256), 0, stream, xp, B, w, z2p, ts); break;
    case 1: hipLaunchKernelGGL(mlp_l1_fwd<1>, grid, dim3(256), 0, stream, xp, B, w, z2p, ts); break;
    default: hipLaunchKernelGGL(mlp_l1_fwd<2>, grid, dim3(256), 0, stream, xp, B, w, z2p, ts); break;
  }
  return hipGetLastError();
}

hipError_t dtfk_mlp_fwd_head(const void* x, int x_kind, int B, const void* W1T, float* z2p, const void* labels,
                             const void* W2T, const void* W2N, const float* params, void* dz2T, int BP,
                             float* partials, float inv_batch, int act, int naive_loss, int* counters,
                             long long* gstep, hipStream_t stream) {
  using namespace dtfk::mlp;
  const dim3 grid(HIDP / 16, KSPLIT, (B + 15) / 16);
  const uint8_t* xp = (const uint8_t*)x;
#define DTFK_FH(XK)                                                                                        \
  hipLaunchKernelGGL(mlp_fwd_head<XK>, grid, dim3(512), 0, stream, xp, B, (const uint16_t*)W1T, z2p,       \
                     (const uint8_t*)labels, (const uint16_t*)W2T, (const uint16_t*)W2N, params,            \
                     (uint16_t*)dz2T, BP, partials, inv_batch, act, naive_loss, counters, gstep)
  switch (x_kind) {
    case 0: DTFK_FH(0); break;
    case 1: DTFK_FH(1); break;
    default: DTFK_FH(2); break;
  }
#undef DTFK_FH
  return hipGetLastError();
}

hipError_t dtfk_mlp_head_bwd(const float* z2p, const void* labels, int B, const void* W2T,
                             const void* W2N, const float* params, void* dz2T, int BP,
                             float* partials, float inv_batch, int act, int naive_loss,
                             long long* gstep, long long* ts, hipStream_t stream) {
  using namespace dtfk::mlp;
  hipLaunchKernelGGL(mlp_head_bwd, dim3((B + 15) / 16), dim3(512), 0, stream, z2p,
                     (const uint8_t*)labels, B, (const uint16_t*)W2T, (const uint16_t*)W2N, params,
                     (uint16_t*)dz2T, BP, partials, inv_batch, act, naive_loss, gstep, ts);
  return hipGetLastError();
}

// grad_kind: 0 fused SGD, 1 fp32 grads, 2 bf16 grads, 3 IPC exchange + SGD (ipc_* args)
hipError_t dtfk_mlp_wgrad(const void* x, int x_kind, const void* dz2T, int BP, int B,
                          const float* partials, float* params, void* W1T, void* W2T, void* W2N,
                          void* grads, int grad_kind, const float* lr, float* metrics,
                          long long* gstep, int ring, long long* ts, void* const* ipc_table, int ipc_W,
                          int ipc_rank, int ipc_parity, long long ipc_slot_bytes, int* ipc_err,
                          long long ipc_timeout, hipStream_t stream) {
  using namespace dtfk::mlp;
  const dim3 grid(NSTRIP * 7 + NRED), block(64);
  const size_t lds = (size_t)16 * (BP + 8) * sizeof(uint16_t);
  const int gb = grad_kind == 2 ? 1 : 0;
  IpcArgs ipc{ipc_table, ipc_W, ipc_rank, ipc_parity, ipc_slot_bytes, ipc_W > 0 ? 1.f / ipc_W : 1.f, ipc_err,
              ipc_timeout};
#define DTFK_WG(KS, XK, M)                                                                        \
  hipLaunchKernelGGL((mlp_wgrad<KS, XK, M>), grid, block, lds, stream, (const uint8_t*)x,         \
                     (const uint16_t*)dz2T, BP, B, partials, (B + 15) / 16, params,               \
                     (uint16_t*)W1T, (uint16_t*)W2T, (uint16_t*)W2N, grads, gb, lr, metrics, gstep, \
                     ring, ts, ipc)
#define DTFK_WG_F(KS, XK) \
  if (grad_kind == 0) DTFK_WG(KS, XK, 0); else if (grad_kind == 3) DTFK_WG(KS, XK, 2); else DTFK_WG(KS, XK, 1)
#define DTFK_WG_X(KS)                         \
  switch (x_kind) {                           \
    case 0: DTFK_WG_F(KS, 0); break;          \
    case 1: DTFK_WG_F(KS, 1); break;          \
    default: DTFK_WG_F(KS, 2); break;         \
  }
  switch (BP / 32) {
    case 1: DTFK_WG_X(1); break;
    case 2: DTFK_WG_X(2); break;
    case 3: DTFK_WG_X(3); break;
    case 4: DTFK_WG_X(4); break;
    default: DTFK_WG_X(0); break;
  }
#undef DTFK_WG_X
#undef DTFK_WG_F
#undef DTFK_WG
  return hipGetLastError();
}

hipError_t dtfk_mlp_apply_flat(float* params, const void* grads, int grad_kind, const float* lr,
                               float scale, void* W1T, void* W2T, void* W2N, hipStream_t stream) {
  using namespace dtfk::mlp;
  hipLaunchKernelGGL(mlp_apply_flat, dim3((NPARAM + 255) / 256), dim3(256), 0, stream, params,
                     grads, grad_kind == 2 ? 1 : 0, lr, scale, (uint16_t*)W1T, (uint16_t*)W2T,
                     (uint16_t*)W2N);
  return hipGetLastError();
}

int dtfk_mlp_ipc_flag_bytes() { return dtfk::mlp::IPC_FLAG_BYTES; }

hipError_t dtfk_mlp_ipc_reduce_apply(float* params, void* const* peer_table, int W, int rank, int parity,
                                     long long slot_bytes, const long long* gstep, const float* lr, float scale,
                                     void* W1T, void* W2T, void* W2N, int* err, long long timeout_ticks,
                                     hipStream_t stream) {
  using namespace dtfk::mlp;
  hipLaunchKernelGGL(mlp_ipc_reduce_apply, dim3((NPARAM / 2 + 255) / 256), dim3(256), 0, stream, params, peer_table,
                     W, rank, parity, slot_bytes, gstep, lr, scale, (uint16_t*)W1T, (uint16_t*)W2T, (uint16_t*)W2N,
                     err, timeout_ticks);
  return hipGetLastError();
}

}  // extern "C"
