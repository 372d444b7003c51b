// Reached by: compat Session's lowered MLP step (compat/lowering.py GraphStepPlan: float feeds, other shapes, and N synchronous workers with the IPC reduce-SGD); tests/test_lowering_gpu.py, test_compat_ipc_gpu.py
// fp32 lowering of the reference graph's training step, for the compat
// Session (compat/lowering.py): the graph
//   a2 = act(x W1 + b1); y = softmax(a2 W2 + b2)
//   loss = mean(-sum(y_ * log(y), 1))         (example.py:93-103, "naive")
//        | mean(softmax_cross_entropy_with_logits(y_, z3))     ("stable")
//   train_op = GradientDescentOptimizer(lr).minimize(loss, global_step)
//   accuracy = mean(cast(equal(argmax(y, 1), argmax(y_, 1))))
// is matched on the deferred graph and run as two launches instead of ~25
// eager ops, with every product on the exact-fp32 matrix core path
// (v_mfma_f32_16x16x4_f32, fp32 accumulate): the numbers are the fp32 graph's,
// only the summation order differs.
//
//   L1 graph_mlp_l1h    a2 = act(x W1 + b1): one workgroup per 16x16 tile of
//                       a2, its 8 waves take interleaved 16-deep K blocks
//                       (lane group g holds k = 16j + 4g .. +3 as one float4
//                       of x, so the 4 MFMAs of a block need no shuffles),
//                       partial tiles summed through LDS; rows >= B and
//                       columns >= H are written as 0.  The LAST workgroup of
//                       each 16-row tile to finish (arrival counter) then runs
//                       that row tile's head (L2) in the same launch:
//   L2 head_tile        z3 = a2 W2 + b2 (MFMA), softmax per row with 16-lane
//                       reductions (one row element per wave), loss, argmax
//                       accuracy, dz3; da2 = dz3 W2^T (MFMA), dz2 = da2 act'(a2);
//                       the row tile's dW2 partial a2^T dz3 and loss sums.
//   L3 graph_mlp_wgrad  [dW1; db1] = [x 1]^T dz2, one workgroup per 16x16
//                       tile, batch split over its 4 waves, fused W1 -= lr dW1,
//                       b1 -= lr db1 (or gradients out).
// Biases ride along as ones columns (a2's column H gives db2 in L2's dW2
// tile, x's virtual column K gives db1 in L3), so no serial column sums.
// Shapes: any B <= 256 with B*HP <= 16384 (HP = H + 1 rounded up to 16),
// K >= 1, H <= 128, C <= 16.
#include "common.h"

#include <algorithm>

namespace dtfk {
namespace gmlp {

constexpr int MAXB = 256;
constexpr int MAXH = 128;
constexpr int CP = 16;                  // classes padded to one MFMA tile
constexpr int A2_LDS = 16384;           // floats of a2 / dz2 staged in L2's LDS

// Pins a loaded value in a register at this point: the load above it is then
// issued unconditionally instead of being sunk into a branch around its use.
__device__ __forceinline__ float pin(float v) {
  asm volatile("" : "+v"(v));
  return v;
}

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float act_fwd(float z, int act) {
  return act == 0 ? 1.f / (1.f + expf(-z)) : fmaxf(z, 0.f);
}
// derivative from the activation's output (sigmoid: a(1-a); relu: a > 0)
__device__ __forceinline__ float act_bwd(float a, int act) {
  return act == 0 ? a * (1.f - a) : (a > 0.f ? 1.f : 0.f);
}

// ---------------------------------------------------------------- L1
constexpr int L1W = 8;     // waves per a2 tile (interleaved 16-deep K blocks)
constexpr int PF = 8;      // K blocks per wave whose loads are issued before any MFMA

// A uint8 pixel as the float32 the MNIST loader feeds: k / 255 correctly rounded
// (numpy's float32 division; data/mnist.py), so a uint8 feed is bit-identical to
// the float one.
__device__ __forceinline__ float px255(uint32_t k) { return __fdiv_rn((float)k, 255.f); }

// VEC: K % 4 == 0 and x 16-byte aligned -> x as float4s.  U8: x is uint8 pixels
// (xu, 4-byte aligned rows, K % 4 == 0), 4 per 32-bit load, converted by px255.
template <bool VEC, bool U8 = false>
__device__ __forceinline__ void l1_tile(const float* __restrict__ x, const uint8_t* __restrict__ xu,
                                        const float* __restrict__ W1,
                                        const float* __restrict__ b1, float* __restrict__ a2,
                                        int B, int K, int H, int HP, int act) {
  __shared__ f32x4 part[L1W][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int nct = HP / 16;
  const int r0 = (blockIdx.x / nct) * 16, c0 = (blockIdx.x % nct) * 16;
  const int row = r0 + r, col = c0 + r;
  const bool rv = row < B, cv = col < H;
  const float* xr = x + (size_t)min(row, B - 1) * K;
  const uint8_t* xur = xu + (size_t)min(row, B - 1) * K;
  const float* wc = W1 + min(col, H - 1);
  const float bv = pin(b1[min(col, H - 1)]);   // issued with the operand loads, not after the barrier
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const int nkb = (K + 15) / 16;
  for (int base = w; base < nkb; base += L1W * PF) {
    // every load of this chunk first, branch-free (clamped addresses, masked
    // values): one memory round trip, then the MFMAs
    float xa[PF][4], wb[PF][4];
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      const int k = (base + j * L1W) * 16 + 4 * g;
      if constexpr (U8) {
        const uint32_t v = *reinterpret_cast<const uint32_t*>(xur + min(k, K - 4));
        const bool ok = k < K;
#pragma unroll
        for (int s = 0; s < 4; ++s) xa[j][s] = ok ? px255((v >> (8 * s)) & 255u) : 0.f;
      } else if constexpr (VEC) {
        const float4 v = *reinterpret_cast<const float4*>(xr + min(k, K - 4));
        const bool ok = k < K;                     // K % 4 == 0: the float4 is all in or all out
        xa[j][0] = ok ? v.x : 0.f; xa[j][1] = ok ? v.y : 0.f; xa[j][2] = ok ? v.z : 0.f; xa[j][3] = ok ? v.w : 0.f;
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const float v = xr[min(k + s, K - 1)];
          xa[j][s] = k + s < K ? v : 0.f;
        }
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const float v = wc[(size_t)min(k + s, K - 1) * H];
        wb[j][s] = k + s < K ? v : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < PF; ++j)
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = mfma4(rv ? xa[j][s] : 0.f, cv ? wb[j][s] : 0.f, acc);
  }
  part[w][lane] = acc;
  __syncthreads();
  if (w == 0) {
    f32x4 t = part[0][lane];
#pragma unroll
    for (int q = 1; q < L1W; ++q) {
      const f32x4 p = part[q][lane];
      t[0] += p[0]; t[1] += p[1]; t[2] += p[2]; t[3] += p[3];
    }
    // C layout: lane holds rows 4g + i, column r.  Column H carries 1 for
    // valid rows: L2's dW2 tile then yields db2 = colsum(dz3) as its row H.
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = r0 + 4 * g + i;
      const float z = t[i] + (cv ? bv : 0.f);
      // write-through (sc1) store: the row tile's head (another workgroup, maybe
      // another XCD) reads it with sc1 loads -- no L2 write-back fence needed
      __hip_atomic_store(a2 + (size_t)m * HP + col, m < B ? (cv ? act_fwd(z, act) : (col == H ? 1.f : 0.f)) : 0.f,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---------------------------------------------------------------- L2
// One workgroup (4 waves) per 16-row tile of the batch: z3 = a2 W2 + b2 (split-K
// over the 4 waves), softmax / loss / accuracy / dz3 (wave 0, 16-lane
// reductions), then per hidden tile (spread over the waves) da2 = dz3 W2^T ->
// dz2 = da2 act'(a2) and this row tile's dW2 partial a2^T dz3 (row H of it is
// db2: a2's ones column).  The partials and the loss / accuracy sums go to a
// global scratch; L3's finalize workgroups reduce them in fixed row-tile order
// (deterministic) and update W2 / b2.  It replaces ONE 512-thread workgroup that
// walked the whole batch serially (~18 us; profiles/mnist_graph_lowered_*).
struct HeadArgs {
  const float* a2;      // [BP][HP] from L1
  const float* ylab;    // [B][C]
  const float* W2;      // [H][C] (read only here: L3 updates it)
  const float* b2;      // [C]
  float* dz2;           // [BP][HP] out
  float* part;          // [NRT][HP][CP] dW2 partials (row H = db2), then [NRT][2] loss / correct
  int B, H, HP, C, act, naive;
};

constexpr int HW = 4;   // waves of the z3 split-K and of the softmax rows

// The head of batch-row tile rt, run by the LAST of L1's workgroups of that row
// tile to finish (NW waves; every thread of the block calls it: it has barriers).
template <int NW>
__device__ void head_tile(const HeadArgs& a, const int rt) {
  __shared__ float a2s[16 * MAXH + 16];       // this tile's a2 rows [16][HP]
  __shared__ float w2s[(MAXH + 16) * CP];     // W2 [HP][CP], zero padded
  __shared__ float dz3s[16 * CP];             // dz3 / B of the tile [16][CP]
  __shared__ f32x4 zp[HW][64];                // split-K partials of z3
  const int B = a.B, H = a.H, HP = a.HP, C = a.C;
  const int NRT = (B + 15) / 16;
  const int rb = rt * 16;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  // the softmax operands first (waves < HW: element i = w of the lane's rows; b2):
  // issued before the staging below so their latency is not a separate round trip
  const float labw = pin(a.ylab[(size_t)min(rb + 4 * g + (w & 3), B - 1) * C + min(r, C - 1)]);
  const float b2p = pin(a.b2[min(r, C - 1)]);
  // operands, branch-free (clamped + masked): a2 tile, W2 -- every load issued
  // before the first LDS store (a load -> store loop waits one round trip per
  // iteration: ~1 us each)
  constexpr int A2N = (16 * (MAXH + 16) / 4 + NW * 64 - 1) / (NW * 64);   // float4s per thread
  constexpr int W2N = ((MAXH + 16) * CP + NW * 64 - 1) / (NW * 64);       // floats per thread
  float4 av4[A2N];
  float wv[W2N];
  // a2 rows of the tile: written (sc1) by the other workgroups of this launch ->
  // L1-bypassing sc1 loads through a buffer resource
  const __amdgpu_buffer_rsrc_t a2r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.a2 + (size_t)rb * HP), 0, 16 * HP * 4, 0x00020000);
  const int na2 = 16 * HP / 4;
#pragma unroll
  for (int j = 0; j < A2N; ++j)
    av4[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(a2r, 16 * min(tid + j * NW * 64, na2 - 1), 0, 16));
#pragma unroll
  for (int j = 0; j < W2N; ++j) {
    const int i = tid + j * NW * 64, h = i / CP, c = i % CP;
    wv[j] = a.W2[min(h, H - 1) * C + min(c, C - 1)];
  }
#pragma unroll
  for (int j = 0; j < A2N; ++j)
    if (tid + j * NW * 64 < na2) reinterpret_cast<float4*>(a2s)[tid + j * NW * 64] = av4[j];
#pragma unroll
  for (int j = 0; j < W2N; ++j) {
    const int i = tid + j * NW * 64, h = i / CP, c = i % CP;
    if (i < HP * CP) w2s[i] = (h < H && c < C) ? wv[j] : 0.f;
  }
  __syncthreads();
  // z3 tile, K = HP split over HW waves
  if (w < HW) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k = 4 * w; k < HP; k += 4 * HW) acc = mfma4(a2s[r * HP + k + g], w2s[(k + g) * CP + r], acc);
    zp[w][lane] = acc;
  }
  __syncthreads();
  // softmax / loss / dz3: wave w takes element i = w of every lane's 4 rows (the
  // 16-lane reductions of the 16 rows run on all 4 waves instead of serially on one)
  __shared__ float lcs[HW][2];
  if (w < HW) {
    f32x4 acc = zp[0][lane];
#pragma unroll
    for (int q = 1; q < HW; ++q) acc += zp[q][lane];
    const float b2v = r < C ? b2p : 0.f;
    float loss_part = 0.f, corr_part = 0.f;
    {
      const int i = w;
      const int m = rb + 4 * g + i;               // row; column = r (class)
      const bool valid = m < B;
      const bool cl = r < C;
      const float lab = (valid && cl) ? labw : 0.f;
      const float ai = w == 0 ? acc[0] : (w == 1 ? acc[1] : (w == 2 ? acc[2] : acc[3]));   // no dynamic index
      const float z = cl ? ai + b2v : -INFINITY;
      const float mx = row16_max(z);
      const float e = cl ? expf(z - mx) : 0.f;
      const float s = row16_sum(e);
      const float y = e / s;
      const float lsum = row16_sum(lab);
      // loss term: naive -y_ log(softmax) exactly as the graph computes it
      // (0 * log(0) = NaN like TF); stable -y_ (z - max - log sum exp)
      const float lt = cl ? -lab * (a.naive ? logf(y) : (z - mx - logf(s))) : 0.f;
      const float lrow = row16_sum(lt);
      // first-max argmax of y and of y_
      const float ym = row16_max(cl ? y : -INFINITY);
      const float pi = row16_min(cl && y == ym ? (float)r : 1e9f);
      const float lm = row16_max(cl ? lab : -INFINITY);
      const float li = row16_min(cl && lab == lm ? (float)r : 1e9f);
      if (r == 0 && valid) {
        loss_part += lrow;
        corr_part += pi == li ? 1.f : 0.f;
      }
      const float d = a.naive ? (y * lsum - lab) : (y - lab);
      dz3s[(4 * g + i) * CP + r] = (valid && cl) ? d / (float)B : 0.f;
    }
    // (lanes with r == 0 hold the partial sums of their row)
    loss_part += __shfl_xor(loss_part, 16, 64);
    loss_part += __shfl_xor(loss_part, 32, 64);
    corr_part += __shfl_xor(corr_part, 16, 64);
    corr_part += __shfl_xor(corr_part, 32, 64);
    if (lane == 0) {
      lcs[w][0] = loss_part;
      lcs[w][1] = corr_part;
    }
  }
  __syncthreads();
  if (tid == 0) {   // the tile's sums in fixed wave order
    float* lc = a.part + (size_t)NRT * HP * CP;
    lc[2 * rt] = ((lcs[0][0] + lcs[1][0]) + lcs[2][0]) + lcs[3][0];
    lc[2 * rt + 1] = ((lcs[0][1] + lcs[1][1]) + lcs[2][1]) + lcs[3][1];
  }
  // per hidden tile: da2 = dz3 W2^T -> dz2 rows; dW2 partial = a2^T dz3
  const int nht = HP / 16;
  for (int ht = w; ht < nht; ht += NW) {
    const int hb = ht * 16;
    f32x4 da = {0.f, 0.f, 0.f, 0.f}, dw = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < CP; k += 4) da = mfma4(dz3s[r * CP + k + g], w2s[(hb + r) * CP + k + g], da);
#pragma unroll
    for (int k = 0; k < 16; k += 4) dw = mfma4(a2s[(k + g) * HP + hb + r], dz3s[(k + g) * CP + r], dw);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = 4 * g + i, h = hb + r;         // da: row m, column h
      const float av = a2s[m * HP + h];
      a.dz2[(size_t)(rb + m) * HP + h] = (rb + m < B && h < H) ? da[i] * act_bwd(av, a.act) : 0.f;
      // dw: row hb + 4g + i (hidden), column r (class)
      a.part[((size_t)rt * HP + hb + 4 * g + i) * CP + r] = dw[i];
    }
  }
}

// L1 + L2 in one launch: every workgroup computes its a2 tile; the last of the
// row tile's HP / 16 workgroups to finish (a per-row-tile arrival counter,
// reset by that workgroup for the next step) runs the row tile's head -- no
// second launch and no grid-wide wait.
template <bool VEC, bool U8 = false>
__global__ __launch_bounds__(512) void graph_mlp_l1h(const float* __restrict__ x, const uint8_t* __restrict__ xu,
                                                     const float* __restrict__ W1,
                                                     const float* __restrict__ b1, HeadArgs h, int K, int* cnt) {
  __shared__ int last;
  l1_tile<VEC, U8>(x, xu, W1, b1, const_cast<float*>(h.a2), h.B, K, h.H, h.HP, h.act);
  const int nct = h.HP / 16, rt = blockIdx.x / nct;
  if (threadIdx.x < 64) {   // wave 0 stored the tile (write-through): wait for the stores, then arrive
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x == 0) {
      const int old = atomicAdd(cnt + rt, 1);
      last = old == nct - 1;
      if (last) cnt[rt] = 0;   // nobody else touches it until the next launch
    }
  }
  __syncthreads();
  if (!last) return;
  head_tile<8>(h, rt);      // reads the other workgroups' a2 rows with sc1 loads
}

// ---------------------------------------------------------------- L3
// One workgroup per 16x16 tile of [dW1; db1] ((K+1) x H: row K is db1, from a
// virtual x column of ones); its 4 waves split the batch and prefetch all of
// their operands (<= 16 batch blocks each) before the MFMAs.
constexpr int L3PF = 16;
struct WgradArgs {
  const float* x;
  const uint8_t* xu;    // uint8 pixels instead of x (px255), or null
  const float* dz2;
  float* W1;
  float* b1;
  float* W2;
  float* b2;
  float* gW1;           // gradient outputs (sgd == 0)
  float* gb1;
  float* gW2;
  float* gb2;
  const float* hpart;   // L2's dW2 partials + loss / correct sums
  float* metrics;       // [0] loss, [1] accuracy, [2] global_step after the step
  float* host_metrics;  // the same three in pinned host memory (nullptr: none) -- no copy-back op
  void* gstep;          // global_step storage or nullptr
  int gstep_kind;       // 0 f32, 1 i64, 2 i32, 3 f64
  const float* lr_ptr;  // device learning rate (a captured step reads the current one)
  int B, K, H, HP, C, sgd, tiles;
};

// Workgroups >= tiles: one per hidden tile of W2 / b2 -- the sum of L2's row-tile
// partials in fixed order, the update (or gradients out); the first of them also
// finalizes loss / accuracy and bumps global_step.
__device__ void graph_mlp_w2_final(const WgradArgs& a, int ht) {
  const int tid = threadIdx.x;
  const int HP = a.HP, H = a.H, C = a.C, NRT = (a.B + 15) / 16;
  const float lr = *a.lr_ptr;
  for (int e = tid; e < 16 * CP; e += blockDim.x) {
    const int h = ht * 16 + e / CP, c = e % CP;
    float s = 0.f;
    for (int rt = 0; rt < NRT; ++rt) s += a.hpart[((size_t)rt * HP + h) * CP + c];
    if (c < C) {
      if (h < H) {
        if (a.sgd) a.W2[h * C + c] -= lr * s;
        else a.gW2[h * C + c] = s;
      } else if (h == H) {
        if (a.sgd) a.b2[c] -= lr * s;
        else a.gb2[c] = s;
      }
    }
  }
  if (ht == 0 && tid == 0) {
    const float* lc = a.hpart + (size_t)NRT * HP * CP;
    float ls = 0.f, cr = 0.f;
    for (int rt = 0; rt < NRT; ++rt) { ls += lc[2 * rt]; cr += lc[2 * rt + 1]; }
    a.metrics[0] = ls / (float)a.B;
    a.metrics[1] = cr / (float)a.B;
    if (a.gstep != nullptr) {
      float now;
      switch (a.gstep_kind) {
        case 0: now = (*reinterpret_cast<float*>(a.gstep) += 1.f); break;
        case 1: now = (float)(*reinterpret_cast<long long*>(a.gstep) += 1); break;
        case 2: now = (float)(*reinterpret_cast<int*>(a.gstep) += 1); break;
        default: now = (float)(*reinterpret_cast<double*>(a.gstep) += 1.0); break;
      }
      a.metrics[2] = now;                 // post-increment value, read back with the loss
    }
    if (a.host_metrics != nullptr) {      // system-scope (write-through) stores over PCIe
#pragma unroll
      for (int i = 0; i < 3; ++i)
        __hip_atomic_store(a.host_metrics + i, a.metrics[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      // acknowledged before the wave ends (the kernel's completion signal follows);
      // a __threadfence_system() here wrote back the whole L2 first
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
}

__global__ __launch_bounds__(256) void graph_mlp_wgrad(WgradArgs a) {
  __shared__ f32x4 part[4][64];
  if ((int)blockIdx.x >= a.tiles) {
    graph_mlp_w2_final(a, (int)blockIdx.x - a.tiles);
    return;
  }
  const float* __restrict__ x = a.x;
  const float* __restrict__ dz2 = a.dz2;
  const int B = a.B, K = a.K, H = a.H, HP = a.HP, sgd = a.sgd;
  const float lr = *a.lr_ptr;
  float* W1 = a.W1;
  float* b1 = a.b1;
  float* gW1 = a.gW1;
  float* gb1 = a.gb1;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int nht = HP / 16;
  const int k0 = (blockIdx.x / nht) * 16, h0 = (blockIdx.x % nht) * 16;
  const int kk = k0 + r;
  const int kc = min(kk, K - 1);
  const int nbb = ((B + 15) & ~15) / 4;            // batch blocks of 4
  float xv[L3PF], dv[L3PF];
#pragma unroll
  for (int t = 0; t < L3PF; ++t) {
    const int m = (w + 4 * t) * 4 + g;             // batch row supplied by this lane
    const int mc = min(m, B - 1);
    const float xr = a.xu != nullptr ? px255(a.xu[(size_t)mc * K + kc]) : x[(size_t)mc * K + kc];
    const float d = dz2[(size_t)min(m, nbb * 4 - 1) * HP + h0 + r];   // rows >= B are 0
    const bool ok = m < B && (w + 4 * t) < nbb;
    xv[t] = ok ? (kk < K ? xr : (kk == K ? 1.f : 0.f)) : 0.f;
    dv[t] = ok ? d : 0.f;
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < L3PF; ++t) acc = mfma4(xv[t], dv[t], acc);
  part[w][lane] = acc;
  __syncthreads();
  if (w == 0) {
    f32x4 s4 = part[0][lane];
#pragma unroll
    for (int q = 1; q < 4; ++q) {
      const f32x4 p = part[q][lane];
      s4[0] += p[0]; s4[1] += p[1]; s4[2] += p[2]; s4[3] += p[3];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = k0 + 4 * g + i, h = h0 + r;
      if (h < H) {
        if (k < K) {
          const size_t o = (size_t)k * H + h;
          if (sgd) W1[o] -= lr * s4[i];
          else gW1[o] = s4[i];
        } else if (k == K) {
          if (sgd) b1[h] -= lr * s4[i];
          else gb1[h] = s4[i];
        }
      }
    }
  }
}

// Feed ingest: the step's packed feed (x | y_ | lr) read straight from the
// pinned host staging slot over PCIe by many workgroups (16-byte loads), instead
// of a copy-engine transfer -- for a ~0.3 MB feed the DMA's setup / completion
// latency is most of its time.  n4: 16-byte chunks (the tail pads to a chunk).
// The slot is rewritten by the host every other step: system-scope loads (no
// stale cached copy of the previous use).
__global__ __launch_bounds__(256) void feed_ingest(const uint4* __restrict__ host, uint4* __restrict__ dev,
                                                   long long n4) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    const unsigned long long lo = ld_sys_u64(host + i), hi = ld_sys_u64(reinterpret_cast<const char*>(host + i) + 8);
    dev[i] = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
  }
}

}  // namespace gmlp
}  // namespace dtfk

extern "C" hipError_t dtfk_graph_feed_ingest(const void* host, void* dev, long long bytes, hipStream_t stream) {
  if (bytes <= 0) return hipSuccess;
  if ((reinterpret_cast<uintptr_t>(host) | reinterpret_cast<uintptr_t>(dev) | (uintptr_t)bytes) & 15)
    return hipErrorInvalidValue;
  const long long n4 = bytes / 16;
  const unsigned grid = (unsigned)std::min<long long>(160, (n4 + 255) / 256);
  hipLaunchKernelGGL(dtfk::gmlp::feed_ingest, dim3(grid), dim3(256), 0, stream, static_cast<const uint4*>(host),
                     static_cast<uint4*>(dev), n4);
  return hipGetLastError();
}

// Device scratch (floats) the step needs besides a2 / dz2: L2's partials + loss
// sums + the per-row-tile arrival counters (int).  Must be ZERO when first used.
extern "C" long long dtfk_graph_mlp_part_floats(int B, int H) {
  const int HP = (H + 16) & ~15, NRT = (B + 15) / 16;
  return (long long)NRT * HP * dtfk::gmlp::CP + 3LL * NRT;
}

// xu (uint8 pixels, K % 4 == 0, 4-byte aligned) replaces x when non-null.
extern "C" hipError_t dtfk_graph_mlp_step(const float* x, const uint8_t* xu, const float* ylab, float* W1, float* b1,
                                          float* W2,
                                          float* b2, float* a2buf, float* dz2buf, float* part, float* gW1, float* gb1,
                                          float* gW2, float* gb2, float* metrics, float* host_metrics, void* gstep,
                                          int gstep_kind, const float* lr_ptr, int B, int K, int H, int C, int act,
                                          int naive, int sgd, hipStream_t stream) {
  using namespace dtfk::gmlp;
  if (B < 1 || B > MAXB || H < 1 || H > MAXH || C < 1 || C > CP || K < 1 || lr_ptr == nullptr)
    return hipErrorInvalidValue;
  const int HP = (H + 16) & ~15, BP = (B + 15) & ~15;   // >= H + 1 (ones column)
  if (BP * HP > A2_LDS) return hipErrorInvalidValue;
  if (xu != nullptr && ((K & 3) || (reinterpret_cast<uintptr_t>(xu) & 3))) return hipErrorInvalidValue;
  const bool vec = (K & 3) == 0 && K >= 4 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  HeadArgs h{a2buf, ylab, W2, b2, dz2buf, part, B, H, HP, C, act, naive};
  // per-row-tile arrival counters behind the partials (zero at allocation, reset by their last arriver)
  int* cnt = reinterpret_cast<int*>(part + (size_t)(BP / 16) * HP * CP + 2 * (BP / 16));
  const dim3 g1((BP / 16) * (HP / 16));
  if (xu != nullptr)
    hipLaunchKernelGGL((graph_mlp_l1h<true, true>), g1, dim3(512), 0, stream, x, xu, W1, b1, h, K, cnt);
  else if (vec)
    hipLaunchKernelGGL((graph_mlp_l1h<true, false>), g1, dim3(512), 0, stream, x, xu, W1, b1, h, K, cnt);
  else
    hipLaunchKernelGGL((graph_mlp_l1h<false, false>), g1, dim3(512), 0, stream, x, xu, W1, b1, h, K, cnt);
  const int tiles = ((K + 1 + 15) / 16) * (HP / 16);
  WgradArgs wa{x, xu, dz2buf, W1, b1, W2, b2, gW1, gb1, gW2, gb2, part, metrics, host_metrics, gstep, gstep_kind,
               lr_ptr, B, K, H, HP, C, sgd, tiles};
  hipLaunchKernelGGL(graph_mlp_wgrad, dim3(tiles + HP / 16), dim3(256), 0, stream, wa);
  return hipGetLastError();
}
