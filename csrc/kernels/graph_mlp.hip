// fp32 lowering of the reference graph's training step, for the compat
// Session (compat/lowering.py): the graph
//   a2 = act(x W1 + b1); y = softmax(a2 W2 + b2)
//   loss = mean(-sum(y_ * log(y), 1))         (example.py:93-103, "naive")
//        | mean(softmax_cross_entropy_with_logits(y_, z3))     ("stable")
//   train_op = GradientDescentOptimizer(lr).minimize(loss, global_step)
//   accuracy = mean(cast(equal(argmax(y, 1), argmax(y_, 1))))
// is matched on the deferred graph and run as three kernels instead of ~25
// eager ops, with every product on the exact-fp32 matrix core path
// (v_mfma_f32_16x16x4_f32, fp32 accumulate): the numbers are the fp32 graph's,
// only the summation order differs.
//
//   L1 graph_mlp_l1     a2 = act(x W1 + b1): one workgroup per 16x16 tile of
//                       a2, its 4 waves take interleaved 16-deep K blocks
//                       (lane group g holds k = 16j + 4g .. +3 as one float4
//                       of x, so the 4 MFMAs of a block need no shuffles),
//                       partial tiles summed through LDS; rows >= B and
//                       columns >= H are written as 0.
//   L2 graph_mlp_head   one 512-thread workgroup for the whole batch (B <= 256):
//                       z3 = a2 W2 + b2 (MFMA), softmax per row with 16-lane
//                       reductions, loss, argmax accuracy, dz3; dW2 = a2^T dz3,
//                       db2, da2 = dz3 W2^T (MFMA), dz2 = da2 act'(a2);
//                       SGD on W2/b2 (or gradients out), metrics, and
//                       global_step += 1.
//   L3 graph_mlp_wgrad  [dW1; db1] = [x 1]^T dz2, one workgroup per 16x16
//                       tile, batch split over its 4 waves, fused W1 -= lr dW1,
//                       b1 -= lr db1 (or gradients out).
// Biases ride along as ones columns (a2's column H gives db2 in L2's dW2
// tile, x's virtual column K gives db1 in L3), so no serial column sums.
// Shapes: any B <= 256 with B*HP <= 16384 (HP = H + 1 rounded up to 16),
// K >= 1, H <= 128, C <= 16.
#include "common.h"

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

template <bool VEC>   // VEC: K % 4 == 0 and x 16-byte aligned -> x as float4s
__global__ __launch_bounds__(512) void graph_mlp_l1(const float* __restrict__ x, const float* __restrict__ W1,
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
  const float* wc = W1 + min(col, H - 1);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const int nkb = (K + 15) / 16;
  for (int base = w; base < nkb; base += L1W * PF) {
    // every load of this chunk first, branch-free (clamped addresses, masked
    // values): one memory round trip, then the MFMAs
    float xa[PF][4], wb[PF][4];
#pragma unroll
    for (int j = 0; j < PF; ++j) {
      const int k = (base + j * L1W) * 16 + 4 * g;
      if constexpr (VEC) {
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
    const float bv = cv ? b1[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = r0 + 4 * g + i;
      const float z = t[i] + bv;
      a2[(size_t)m * HP + col] = m < B ? (cv ? act_fwd(z, act) : (col == H ? 1.f : 0.f)) : 0.f;
    }
  }
}

// ---------------------------------------------------------------- L2
struct HeadArgs {
  const float* a2;      // [BP][HP] from L1
  const float* ylab;    // [B][C]
  float* W2;            // [H][C]
  float* b1;            // [H]
  float* b2;            // [C]
  float* dz2;           // [BP][HP] out
  float* gW2;           // gradient outputs (mode GRAD) or nullptr
  float* gb1;
  float* gb2;
  float* metrics;       // [0] loss, [1] accuracy, [2] global_step after the step
  void* gstep;          // global_step storage or nullptr
  int gstep_kind;       // 0 f32, 1 i64, 2 i32, 3 f64
  float lr;
  int B, H, HP, C, act, naive, sgd;
};

__global__ __launch_bounds__(512) void graph_mlp_head(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int B = a.B, H = a.H, HP = a.HP, C = a.C;
  const int BP = (B + 15) & ~15;
  float* a2s = sm;                       // [BP][HP] -> later dz2
  float* w2s = a2s + BP * HP;            // [HP][CP]
  float* dz3s = w2s + HP * CP;           // [BP][CP]
  float* labs = dz3s + BP * CP;          // [BP][CP] labels
  float* red = labs + BP * CP;           // [64] reductions
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nw = blockDim.x >> 6;
  const int r = lane & 15, g = lane >> 4;

  {
    // every global operand in one round trip: a2 (<= 16384 floats, as
    // float4s), W2 (<= 2048), labels (<= 4096), b2 -- clamped, masked, no branches
    const int n4 = BP * HP / 4, nw2 = HP * CP, nl = BP * CP;
    const float4* src = reinterpret_cast<const float4*>(a.a2);
    float4 v[8];
    float wv[4], lv[8];
    // indices are clamped and stores unconditional (a clamped lane rewrites
    // the last element with the same value): no branch the compiler could
    // sink a load into
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = src[min(tid + j * 512, n4 - 1)];
    float wt[4], lt[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = min(tid + j * 512, nw2 - 1), h = i / CP, c = i % CP;
      wt[j] = a.W2[min(h, H - 1) * C + min(c, C - 1)];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = min(tid + j * 512, nl - 1), m = i / CP, c = i % CP;
      lt[j] = a.ylab[(size_t)min(m, B - 1) * C + min(c, C - 1)];
    }
    // all loads are in flight; only now mask (pin keeps each load unconditional)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = min(tid + j * 512, nw2 - 1), h = i / CP, c = i % CP;
      const float t = pin(wt[j]);
      wv[j] = (h < H && c < C) ? t : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = min(tid + j * 512, nl - 1), m = i / CP, c = i % CP;
      const float t = pin(lt[j]);
      lv[j] = (m < B && c < C) ? t : 0.f;
    }
    float4* dst = reinterpret_cast<float4*>(a2s);
#pragma unroll
    for (int j = 0; j < 8; ++j) dst[min(tid + j * 512, n4 - 1)] = v[j];
#pragma unroll
    for (int j = 0; j < 4; ++j) w2s[min(tid + j * 512, nw2 - 1)] = wv[j];
#pragma unroll
    for (int j = 0; j < 8; ++j) labs[min(tid + j * 512, nl - 1)] = lv[j];
  }
  if (tid < 2) red[tid] = 0.f;
  __syncthreads();

  // z3 = a2 W2 + b2 -> softmax, loss, accuracy, dz3 (one 16-row tile per wave pass)
  float loss_part = 0.f, corr_part = 0.f;
  const float b2v = r < C ? a.b2[r] : 0.f;
  for (int rt = w; rt < BP / 16; rt += nw) {
    const int rb = rt * 16;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < HP; k += 4)
      acc = mfma4(a2s[(rb + r) * HP + k + g], w2s[(k + g) * CP + r], acc);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = rb + 4 * g + i;               // row; column = r (class)
      const bool valid = m < B;
      const bool cl = r < C;
      const float z = cl ? acc[i] + b2v : -INFINITY;
      const float mx = row16_max(z);
      const float e = cl ? expf(z - mx) : 0.f;
      const float s = row16_sum(e);
      const float y = e / s;
      const float lab = labs[m * CP + r];
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
      dz3s[m * CP + r] = (valid && cl) ? d / (float)B : 0.f;
    }
  }
  loss_part = wave_sum(loss_part);
  corr_part = wave_sum(corr_part);
  if (lane == 0) {
    atomicAdd(&red[0], loss_part);      // LDS atomics: 8 waves
    atomicAdd(&red[1], corr_part);
  }
  __syncthreads();

  // dW2 = a2^T dz3 ([HP x CP] over BP); row H of the product is db2 (a2's ones column)
  for (int ht = w; ht < HP / 16; ht += nw) {
    const int hb = ht * 16;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < BP; k += 4) acc = mfma4(a2s[(k + g) * HP + hb + r], dz3s[(k + g) * CP + r], acc);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int h = hb + 4 * g + i;
      if (r < C) {
        if (h < H) {
          if (a.sgd) a.W2[h * C + r] = w2s[h * CP + r] - a.lr * acc[i];
          else a.gW2[h * C + r] = acc[i];
        } else if (h == H) {
          if (a.sgd) a.b2[r] = a.b2[r] - a.lr * acc[i];
          else a.gb2[r] = acc[i];
        }
      }
    }
  }
  __syncthreads();   // every wave is done reading a2s as a2 before it becomes dz2

  // da2 = dz3 W2^T ([BP x HP] over CP), dz2 = da2 * act'(a2) (in place)
  const int nht = HP / 16;
  for (int t = w; t < (BP / 16) * nht; t += nw) {
    const int rb = (t / nht) * 16, hb = (t % nht) * 16;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < CP; k += 4) acc = mfma4(dz3s[(rb + r) * CP + k + g], w2s[(hb + r) * CP + k + g], acc);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = rb + 4 * g + i, h = hb + r;
      const float av = a2s[m * HP + h];
      const float d = (m < B && h < H) ? acc[i] * act_bwd(av, a.act) : 0.f;
      a2s[m * HP + h] = d;
      a.dz2[(size_t)m * HP + h] = d;
    }
  }
  if (tid == 0) {
    a.metrics[0] = red[0] / (float)B;
    a.metrics[1] = red[1] / (float)B;
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
  }
}

// ---------------------------------------------------------------- L3
// One workgroup per 16x16 tile of [dW1; db1] ((K+1) x H: row K is db1, from a
// virtual x column of ones); its 4 waves split the batch and prefetch all of
// their operands (<= 16 batch blocks each) before the MFMAs.
constexpr int L3PF = 16;
__global__ __launch_bounds__(256) void graph_mlp_wgrad(const float* __restrict__ x, const float* __restrict__ dz2,
                                                       float* __restrict__ W1, float* __restrict__ b1,
                                                       float* __restrict__ gW1, float* __restrict__ gb1, float lr,
                                                       int B, int K, int H, int HP, int sgd) {
  __shared__ f32x4 part[4][64];
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
    const float xr = x[(size_t)mc * K + kc];
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

}  // namespace gmlp
}  // namespace dtfk

// Shared-memory bytes L2 needs (host check before launch).
extern "C" long long dtfk_graph_mlp_lds(int B, int HP) {
  const int BP = (B + 15) & ~15;
  return 4LL * ((long long)BP * HP + HP * dtfk::gmlp::CP + 2LL * BP * dtfk::gmlp::CP + 64);
}

extern "C" hipError_t dtfk_graph_mlp_step(const float* x, const float* ylab, float* W1, float* b1, float* W2,
                                          float* b2, float* a2buf, float* dz2buf, float* gW1, float* gb1, float* gW2,
                                          float* gb2, float* metrics, void* gstep, int gstep_kind, float lr, int B,
                                          int K, int H, int C, int act, int naive, int sgd, hipStream_t stream) {
  using namespace dtfk::gmlp;
  if (B < 1 || B > MAXB || H < 1 || H > MAXH || C < 1 || C > CP || K < 1) return hipErrorInvalidValue;
  const int HP = (H + 16) & ~15, BP = (B + 15) & ~15;   // >= H + 1 (ones column)
  if (BP * HP > A2_LDS) return hipErrorInvalidValue;
  const bool vec = (K & 3) == 0 && K >= 4 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  if (vec)
    hipLaunchKernelGGL(graph_mlp_l1<true>, dim3((BP / 16) * (HP / 16)), dim3(512), 0, stream, x, W1, b1, a2buf, B, K,
                       H, HP, act);
  else
    hipLaunchKernelGGL(graph_mlp_l1<false>, dim3((BP / 16) * (HP / 16)), dim3(512), 0, stream, x, W1, b1, a2buf, B,
                       K, H, HP, act);
  HeadArgs h{a2buf, ylab, W2, b1, b2, dz2buf, gW2, gb1, gb2, metrics, gstep, gstep_kind, lr, B, H, HP, C, act,
             naive, sgd};
  const size_t lds = (size_t)dtfk_graph_mlp_lds(B, HP);
  static bool lds_set = false;
  if (!lds_set) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&graph_mlp_head),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    lds_set = true;
  }
  hipLaunchKernelGGL(graph_mlp_head, dim3(1), dim3(512), lds, stream, h);
  const int tiles = ((K + 1 + 15) / 16) * (HP / 16);
  hipLaunchKernelGGL(graph_mlp_wgrad, dim3(tiles), dim3(256), 0, stream, x, dz2buf, W1, b1, gW1, gb1, lr, B, K, H,
                     HP, sgd);
  return hipGetLastError();
}
