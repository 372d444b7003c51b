// Reached by: ops/__init__.py and optim/ (every model: xent, embedding bags, AUC, fused optimizers, DDP buckets); tests/test_ops_gpu.py
// Fused elementwise / reduction / sparse kernels behind `distributed_tensorflow_example_amd.ops`
// and `.optim`:
//   act_backward      dZ = dY * act'(.)                    (SigmoidGrad / ReluGrad ...)
//   col_sum           db = sum_rows dZ                     (bias gradient, K2/K5)
//   bucket_{pack,unpack}_bf16  DDP bucket <-> bf16 comm buffer, 1/N folded in (K16)
//   softmax_xent      fused softmax cross-entropy fwd+bwd  (K6; stable or reference-naive)
//   sigmoid_xent      fused sigmoid cross-entropy fwd+bwd  (K11, lr2.py:391)
//   embedding_bag     CSR bag sum/mean with per-id weights (K10, embedding_lookup_sparse)
//   embedding_bag_bwd scatter-add / fused scatter-SGD      (K10 backward + K8 sparse apply)
//   argmax_correct    accuracy counter                     (K7)
//   auc_hist          streaming_auc confusion histograms   (K12)
//   multi-tensor SGD / momentum / Adam (TF epsilon-hat semantics) / AdamW   (K8, K9)
// Every kernel is wave64-native: one wave per row/bag where rows are
// independent, shuffles over 64 lanes, no warp-32 idioms.
#include "common.h"

namespace dtfk {
namespace ops {

__device__ __forceinline__ float act_grad(float dy, float y, float z, int act) {
  switch (act) {
    case 1: return y > 0.f ? dy : 0.f;                 // relu (from y)
    case 2: return dy * y * (1.f - y);                 // sigmoid (from y)
    case 3: return dy * (1.f - y * y);                 // tanh (from y)
    case 4: {                                          // gelu (from z)
      const float cdf = 0.5f * (1.f + erff(z * 0.70710678118654752f));
      const float pdf = 0.3989422804014327f * __expf(-0.5f * z * z);
      return dy * (cdf + z * pdf);
    }
    default: return dy;
  }
}

__global__ void act_backward(const float* __restrict__ dy, const float* __restrict__ y,
                             const float* __restrict__ z, float* __restrict__ dz, int64_t n, int act) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dz[i] = act_grad(dy[i], y ? y[i] : 0.f, z ? z[i] : 0.f, act);
}

// out[n] = sum_m X[m, n] (X row-major [M, N]); block = 256 threads covers 64
// columns x 4 row-groups, grid.y splits rows, partials atomically added.
__global__ void col_sum(const float* __restrict__ X, float* __restrict__ out, int M, int N,
                        int rows_per_block, int accum) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int g = threadIdx.x >> 6;
  const int r0 = blockIdx.y * rows_per_block, r1 = min(M, r0 + rows_per_block);
  float s = 0.f;
  if (c < N)
    for (int r = r0 + g; r < r1; r += 4) s += X[(size_t)r * N + c];
  red[g][threadIdx.x & 63] = s;
  __syncthreads();
  if (g == 0 && c < N) {
    const float t = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    if (gridDim.y == 1) out[c] = accum ? out[c] + t : t;
    else atomicAdd(&out[c], t);
  }
}

// N % 4 == 0: 16 lanes x float4 = 64 columns per block x 16 row groups, four
// rows in flight per thread; grid.y <= 32 row chunks, so each output column
// takes at most 32 atomics (a [4096, 512] bias gradient with 64 blocks of
// scalar loads was 15 us latency-bound; 256 row chunks of atomics on the same
// 512 addresses, 26 us contention-bound).
__global__ void col_sum4(const float4* __restrict__ X, float* __restrict__ out, int M, int N4,
                         int rows_per_block, int accum) {
  __shared__ float4 red[16][16];
  const int cl = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  const int r0 = blockIdx.y * rows_per_block, r1 = min(M, r0 + rows_per_block);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c < N4) {
    int r = r0 + g;
    for (; r + 48 < r1; r += 64) {
      const float4 a = X[(size_t)r * N4 + c], b = X[(size_t)(r + 16) * N4 + c];
      const float4 d = X[(size_t)(r + 32) * N4 + c], e = X[(size_t)(r + 48) * N4 + c];
      s.x += (a.x + b.x) + (d.x + e.x);
      s.y += (a.y + b.y) + (d.y + e.y);
      s.z += (a.z + b.z) + (d.z + e.z);
      s.w += (a.w + b.w) + (d.w + e.w);
    }
    for (; r < r1; r += 16) {
      const float4 a = X[(size_t)r * N4 + c];
      s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
    }
  }
  red[g][cl] = s;
  __syncthreads();
  if (g == 0 && c < N4) {
    float4 t = red[0][cl];
#pragma unroll
    for (int i = 1; i < 16; ++i) {
      t.x += red[i][cl].x; t.y += red[i][cl].y; t.z += red[i][cl].z; t.w += red[i][cl].w;
    }
    float* o = out + 4 * c;
    if (gridDim.y == 1) {
      if (accum) {
        const float4 p = *reinterpret_cast<const float4*>(o);
        t.x += p.x; t.y += p.y; t.z += p.z; t.w += p.w;
      }
      *reinterpret_cast<float4*>(o) = t;
    } else {
      atomicAdd(o, t.x); atomicAdd(o + 1, t.y); atomicAdd(o + 2, t.z); atomicAdd(o + 3, t.w);
    }
  }
}

// One wave per row. labels: int64 class ids (label_kind 0) or dense one-hot /
// probabilities [B, C] (label_kind 1, the reference's y_ placeholder).
// loss_rows[b]; grad = (softmax - y) * grad_scale.  naive=1 reproduces
// -sum(y * log(softmax)) (example.py:103) including its inf/NaN behaviour.
__global__ void softmax_xent(const float* __restrict__ logits, const int64_t* __restrict__ labels,
                             const float* __restrict__ ydense, float* __restrict__ loss_rows,
                             float* __restrict__ grad, int64_t* __restrict__ correct, int Bn, int Cn,
                             float grad_scale, int naive) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= Bn) return;
  const float* z = logits + (size_t)row * Cn;
  float m = -3.0e38f;
  int am = 0x7fffffff;
  for (int c = lane; c < Cn; c += 64) {
    const float v = z[c];
    if (v > m || (v == m && c < am)) { m = v; am = c; }
  }
  // wave argmax with first-index tie break
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float om = __shfl_xor(m, off, 64);
    const int oa = __shfl_xor(am, off, 64);
    if (om > m || (om == m && oa < am)) { m = om; am = oa; }
  }
  float s = 0.f;
  for (int c = lane; c < Cn; c += 64) s += __expf(z[c] - m);
  s = wave_sum(s);
  const float lse = m + __logf(s);
  float loss = 0.f;
  int y = -1;
  if (ydense == nullptr) {
    y = (int)labels[row];
    y = y < 0 ? 0 : (y >= Cn ? Cn - 1 : y);  // out-of-range ids cannot read past the row
    if (lane == 0) loss = naive ? -__logf(__expf(z[y] - m) / s) : lse - z[y];
  } else {
    float l = 0.f, ymax = -1.f;
    int ya = 0;
    for (int c = lane; c < Cn; c += 64) {
      const float yc = ydense[(size_t)row * Cn + c];
      if (naive) l += -yc * __logf(__expf(z[c] - m) / s);
      else l += yc * (lse - z[c]);
      if (yc > ymax) { ymax = yc; ya = c; }
    }
    loss = wave_sum(l);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const float om = __shfl_xor(ymax, off, 64);
      const int oa = __shfl_xor(ya, off, 64);
      if (om > ymax || (om == ymax && oa < ya)) { ymax = om; ya = oa; }
    }
    y = ya;
  }
  if (lane == 0) {
    loss_rows[row] = loss;
    if (correct) atomicAdd((unsigned long long*)correct, (unsigned long long)(am == y ? 1 : 0));
  }
  if (grad != nullptr) {
    for (int c = lane; c < Cn; c += 64) {
      const float p = __expf(z[c] - m) / s;
      const float t = ydense ? ydense[(size_t)row * Cn + c] : (c == y ? 1.f : 0.f);
      grad[(size_t)row * Cn + c] = (p - t) * grad_scale;
    }
  }
}

// bf16 logits (+ fp32 bias), int64 labels, one 256-thread block per row (vocab-
// sized rows: the MLM decoder's [masked tokens, 30522]).  Forward is one read
// with an online max/sum (lse and loss per row); backward recomputes
// softmax from lse and writes dlogits = (softmax - onehot) * scale * dloss in
// bf16 -- the upstream scalar gradient is read from device memory, so no
// separate scaling pass.  C must be even (4-byte = 2-logit accesses).
__device__ __forceinline__ void lse_combine(float& m, float& s, float om, float os) {
  const float nm = fmaxf(m, om);
  s = s * __expf(m - nm) + os * __expf(om - nm);
  m = nm;
}

// Vocab-sized rows (BERT's MLM decoder: [M, 30522] bf16, rows only 4-byte
// aligned): one block per row, two passes -- the row max, then the sum of
// exp(z - max) (the second read hits L2) -- one exp per element and no
// loop-carried rescale chain (the online form's 1.5 exps per element and
// dependent max/rescale updates ran this kernel at ~1.4 TB/s); 4 independent
// dword loads per thread per trip.
__device__ __forceinline__ float2 ld_bias2(const float* bias, int i) {
  return bias ? *reinterpret_cast<const float2*>(bias + 2 * i) : float2{0.f, 0.f};
}
__device__ __forceinline__ float block_max256(float v, float* sh) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  const float r = fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
  __syncthreads();
  return r;
}
__device__ __forceinline__ float block_sum256(float v, float* sh) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  const float r = (sh[0] + sh[1]) + (sh[2] + sh[3]);
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(256) void xent_fwd_bf16(const uint16_t* __restrict__ logits, const float* __restrict__ bias,
                                                     const int64_t* __restrict__ labels, float* __restrict__ lse_rows,
                                                     float* __restrict__ loss_rows, int Cn) {
  __shared__ float sh[4];
  const int row = blockIdx.x;
  const uint32_t* z = reinterpret_cast<const uint32_t*>(logits + (size_t)row * Cn);
  const int n2 = Cn >> 1;
  float m0 = -3.0e38f, m1 = -3.0e38f;
  int i = threadIdx.x;
  for (; i + 768 < n2; i += 1024) {
    uint32_t w[4];
    float2 bb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { w[u] = z[i + 256 * u]; bb[u] = ld_bias2(bias, i + 256 * u); }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      m0 = fmaxf(m0, bf2f(w[u] & 0xffff) + bb[u].x);
      m1 = fmaxf(m1, bf2f(w[u] >> 16) + bb[u].y);
    }
  }
  for (; i < n2; i += 256) {
    const uint32_t w = z[i];
    const float2 bb = ld_bias2(bias, i);
    m0 = fmaxf(m0, bf2f(w & 0xffff) + bb.x);
    m1 = fmaxf(m1, bf2f(w >> 16) + bb.y);
  }
  const float M = block_max256(fmaxf(m0, m1), sh);
  float s0 = 0.f, s1 = 0.f;
  i = threadIdx.x;
  for (; i + 768 < n2; i += 1024) {
    uint32_t w[4];
    float2 bb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { w[u] = z[i + 256 * u]; bb[u] = ld_bias2(bias, i + 256 * u); }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      s0 += __expf(bf2f(w[u] & 0xffff) + bb[u].x - M);
      s1 += __expf(bf2f(w[u] >> 16) + bb[u].y - M);
    }
  }
  for (; i < n2; i += 256) {
    const uint32_t w = z[i];
    const float2 bb = ld_bias2(bias, i);
    s0 += __expf(bf2f(w & 0xffff) + bb.x - M);
    s1 += __expf(bf2f(w >> 16) + bb.y - M);
  }
  const float S = block_sum256(s0 + s1, sh);
  if (threadIdx.x == 0) {
    const float lse = M + __logf(S);
    int y = (int)labels[row];
    y = y < 0 ? 0 : (y >= Cn ? Cn - 1 : y);
    const float zy = bf2f(logits[(size_t)row * Cn + y]) + (bias ? bias[y] : 0.f);
    lse_rows[row] = lse;
    loss_rows[row] = lse - zy;
  }
}

__global__ __launch_bounds__(256) void xent_bwd_bf16(const uint16_t* __restrict__ logits, const float* __restrict__ bias,
                                                     const int64_t* __restrict__ labels,
                                                     const float* __restrict__ lse_rows, const float* __restrict__ dloss,
                                                     uint16_t* __restrict__ grad, int Cn, float scale) {
  const int row = blockIdx.x;
  const uint32_t* z = reinterpret_cast<const uint32_t*>(logits + (size_t)row * Cn);
  uint32_t* gr = reinterpret_cast<uint32_t*>(grad + (size_t)row * Cn);
  const float lse = lse_rows[row];
  const float sc = scale * (dloss ? dloss[0] : 1.f);
  int y = (int)labels[row];
  y = y < 0 ? 0 : (y >= Cn ? Cn - 1 : y);
  const int n2 = Cn >> 1;
  auto one = [&](int k, uint32_t w, float2 bb) {
    const float a = bf2f(w & 0xffff) + bb.x, b = bf2f(w >> 16) + bb.y;
    const float ga = (__expf(a - lse) - (2 * k == y ? 1.f : 0.f)) * sc;
    const float gb = (__expf(b - lse) - (2 * k + 1 == y ? 1.f : 0.f)) * sc;
    gr[k] = pack2bf(ga, gb);
  };
  int i = threadIdx.x;
  for (; i + 768 < n2; i += 1024) {
    uint32_t w[4];
    float2 bb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { w[u] = z[i + 256 * u]; bb[u] = ld_bias2(bias, i + 256 * u); }
#pragma unroll
    for (int u = 0; u < 4; ++u) one(i + 256 * u, w[u], bb[u]);
  }
  for (; i < n2; i += 256) one(i, z[i], ld_bias2(bias, i));
}

// max(x,0) - x*t + log1p(exp(-|x|)); grad (sigmoid(x) - t) * scale
__global__ void sigmoid_xent(const float* __restrict__ x, const float* __restrict__ t,
                             float* __restrict__ loss, float* __restrict__ grad, int64_t n,
                             float grad_scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = x[i], z = t[i];
    loss[i] = fmaxf(v, 0.f) - v * z + log1pf(__expf(-fabsf(v)));
    if (grad) grad[i] = (1.f / (1.f + __expf(-v)) - z) * grad_scale;
  }
}

// Wide&Deep head, one workgroup: z = a[i] + b[i] + bias[0] (the wide part, the
// tower's output, the shared bias), loss = mean sigmoid-xent(z, t) and
// dz = (sigmoid(z) - t) / B -- the two adds, the xent and its mean of the
// unfused graph in one launch.
__global__ __launch_bounds__(1024) void logit3_xent(const float* __restrict__ a, const float* __restrict__ b,
                                                    const float* __restrict__ bias, const float* __restrict__ t,
                                                    float* __restrict__ loss, float* __restrict__ dz, int n) {
  __shared__ float scratch[16];
  const float c = bias[0], inv = 1.f / (float)n;
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float v = a[i] + b[i] + c, z = t[i];
    s += fmaxf(v, 0.f) - v * z + log1pf(__expf(-fabsf(v)));
    dz[i] = (1.f / (1.f + __expf(-v)) - z) * inv;
  }
  s = block_sum(s, scratch);
  if (threadIdx.x == 0) loss[0] = s * inv;
}
// its backward: d = dz * g (the gradient of both summands) and the bias
// gradient sum(d), stored or added to the bias's .grad (accum)
__global__ __launch_bounds__(1024) void logit3_xent_bwd(const float* __restrict__ dz, const float* __restrict__ g,
                                                        float* __restrict__ d, float* __restrict__ gbias, int accum,
                                                        int n) {
  __shared__ float scratch[16];
  const float gs = g[0];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float v = dz[i] * gs;
    d[i] = v;
    s += v;
  }
  s = block_sum(s, scratch);
  if (threadIdx.x == 0 && gbias != nullptr) gbias[0] = accum ? gbias[0] + s : s;
}

// Up to 8 device-to-device copies in one launch (a captured step's input
// refresh: one kernel instead of a copy-engine blit per input).
struct CopyList {
  const char* src[8];
  char* dst[8];
  long long bytes[8];
  int n;
};
__global__ __launch_bounds__(256) void multi_copy(CopyList c) {
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x, nth = (long long)gridDim.x * blockDim.x;
  for (int k = 0; k < c.n; ++k) {
    const char* s = c.src[k];
    char* d = c.dst[k];
    const long long nb = c.bytes[k];
    if (((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 15) == 0) {
      const long long n16 = nb >> 4;
      for (long long j = tid; j < n16; j += nth)
        reinterpret_cast<uint4*>(d)[j] = reinterpret_cast<const uint4*>(s)[j];
      for (long long j = (n16 << 4) + tid; j < nb; j += nth) d[j] = s[j];
    } else {
      for (long long j = tid; j < nb; j += nth) d[j] = s[j];
    }
  }
}

// out[b, :] = combine_{j in bag b} w_j * W[ids_j, :]   (mode 0 sum, 1 mean, 2 sqrtn)
// One wave per bag; lanes stride the embedding dim (D >= 64) or, for narrow
// tables (D < 64, e.g. the LR weight D = 1), lanes stride the bag's ids.
// remap (optional): ids index remap[] and remap[id] is the table row (a one-GPU
// sharded table reads its rows in place: W = the table, ids = the dedup
// inverse, remap = the unique ids -- no gathered [U, D] rows tensor)
__global__ void embedding_bag_fwd(const float* __restrict__ W, int64_t V, int D,
                                  const int64_t* __restrict__ ids, const int64_t* __restrict__ offsets,
                                  const float* __restrict__ psw, int Bn, int mode,
                                  float* __restrict__ out, int64_t* __restrict__ bad_ids,
                                  const int64_t* __restrict__ remap) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (b >= Bn) return;
  const int64_t s = offsets[b], e = offsets[b + 1];
  float wsum = 0.f;
  if (D < 64) {
    for (int d = 0; d < D; ++d) {
      float acc = 0.f, ws = 0.f;
      for (int64_t j = s + lane; j < e; j += 64) {
        int64_t id = ids[j];
        if (remap != nullptr) id = remap[id];
        const float w = psw ? psw[j] : 1.f;
        if (id < 0 || id >= V) { if (bad_ids && d == 0) atomicAdd((unsigned long long*)bad_ids, 1ull); continue; }
        acc += w * W[id * D + d];
        ws += mode == 2 ? w * w : w;
      }
      acc = wave_sum(acc);
      wsum = wave_sum(ws);
      if (lane == 0) {
        float scale = 1.f;
        if (mode == 1 && e > s) scale = 1.f / fmaxf(wsum, 1e-30f);
        if (mode == 2 && e > s) scale = rsqrtf(fmaxf(wsum, 1e-30f));
        out[(size_t)b * D + d] = acc * scale;
      }
    }
    return;
  }
  for (int d0 = blockIdx.y * 64; d0 < D; d0 += 64 * gridDim.y) {   // wide rows: one 64-column slice per blockIdx.y
    const int d = d0 + lane;
    float acc = 0.f, ws = 0.f;
    for (int64_t j = s; j < e; ++j) {
      const int64_t id = remap != nullptr ? remap[ids[j]] : ids[j];
      const float w = psw ? psw[j] : 1.f;
      if (id < 0 || id >= V) continue;
      if (d < D) acc += w * W[id * D + d];
      ws += mode == 2 ? w * w : w;
    }
    float scale = 1.f;
    if (mode == 1 && e > s) scale = 1.f / fmaxf(ws, 1e-30f);
    if (mode == 2 && e > s) scale = rsqrtf(fmaxf(ws, 1e-30f));
    if (d < D) out[(size_t)b * D + d] = acc * scale;
  }
}

// dW[ids_j, :] += w_j * scale_b * dOut[b, :]  (dense fp32 gradient table), or with
// lr != 0: W[ids_j, :] -= lr * (...) directly (fused sparse SGD apply; the
// reference applies IndexedSlices with ScatterSub on the ps).  Float atomics
// (execute at the memory side; duplicates within and across bags combine).
__global__ void embedding_bag_bwd(float* __restrict__ target, int64_t V, int D,
                                  const int64_t* __restrict__ ids, const int64_t* __restrict__ offsets,
                                  const float* __restrict__ psw, const float* __restrict__ dout, int Bn,
                                  int mode, float lr) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (b >= Bn) return;
  // offsets == nullptr: one id per bag (a row-wise scatter, e.g. the owner-side
  // sparse SGD of gradient rows) -- no arange offsets tensor to build
  const int64_t s = offsets != nullptr ? offsets[b] : b, e = offsets != nullptr ? offsets[b + 1] : b + 1;
  float ws = 0.f;
  if (mode != 0) {
    for (int64_t j = s + lane; j < e; j += 64) {
      const float w = psw ? psw[j] : 1.f;
      ws += mode == 2 ? w * w : w;
    }
    ws = wave_sum(ws);
  }
  float scale = 1.f;
  if (mode == 1 && e > s) scale = 1.f / fmaxf(ws, 1e-30f);
  if (mode == 2 && e > s) scale = rsqrtf(fmaxf(ws, 1e-30f));
  const float mul = lr != 0.f ? -lr * scale : scale;
  if (D < 64) {
    for (int64_t j = s + lane; j < e; j += 64) {
      const int64_t id = ids[j];
      if (id < 0 || id >= V) continue;
      const float w = (psw ? psw[j] : 1.f) * mul;
      for (int d = 0; d < D; ++d) atomicAdd(&target[id * D + d], w * dout[(size_t)b * D + d]);
    }
    return;
  }
  for (int64_t j = s; j < e; ++j) {
    const int64_t id = ids[j];
    if (id < 0 || id >= V) continue;
    const float w = (psw ? psw[j] : 1.f) * mul;
    for (int d = lane; d < D; d += 64) atomicAdd(&target[id * D + d], w * dout[(size_t)b * D + d]);
  }
}

// bag_of[j] = the bag of CSR position j (offsets [B + 1], non-decreasing): one
// binary search per position -- one kernel instead of repeat_interleave's five
__global__ __launch_bounds__(256) void bag_index(const int64_t* __restrict__ offsets, int B, int* __restrict__ bag_of,
                                                 int64_t N) {
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < N; j += (int64_t)gridDim.x * blockDim.x) {
    int lo = 0, hi = B;            // last b with offsets[b] <= j
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (offsets[mid] <= j) lo = mid; else hi = mid;
    }
    bag_of[j] = lo;
  }
}

// Sum-bag gradient without atomic pile-ups on hot ids.  Occurrences arrive
// sorted by target row (one radix sort per step, shared by every table that
// reads the same ids), each wave reduces 64 consecutive occurrences in
// registers and issues one atomic per (row run, column): a Zipf-hot row seen
// 10^4 times in a batch costs ~10^4/64 atomics instead of 10^4 serialised ones.
//   rows[p]  target row of sorted occurrence p (int32), occ[p] its CSR position,
//   bag_of[j] the bag of CSR position j.
__global__ void embedding_bag_bwd_sorted(float* __restrict__ target, int64_t V, int D,
                                         const int* __restrict__ rows, const int64_t* __restrict__ occ,
                                         const int* __restrict__ bag_of, const float* __restrict__ psw,
                                         const float* __restrict__ dout, int64_t N) {
  const int lane = threadIdx.x & 63;
  const int64_t p0 = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64;
  if (p0 >= N) return;
  const int cnt = (int)min((int64_t)64, N - p0);
  const int64_t p = p0 + lane;
  int row = -1, b = 0;
  float w = 0.f;
  if (lane < cnt) {
    const int r = rows[p];
    const int64_t j = occ[p];
    b = bag_of[j];
    if (r >= 0 && r < V) { row = r; w = psw ? psw[j] : 1.f; }
  }
  if (D < 64) {
    // lanes own occurrences: segmented inclusive scan over equal (sorted) rows
    const int nxt = __shfl_down(row, 1, 64);
    const bool tail = row >= 0 && (lane == cnt - 1 || nxt != row);
    for (int d = 0; d < D; ++d) {
      float v = w * dout[(size_t)b * D + d];
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const float vu = __shfl_up(v, off, 64);
        const int ru = __shfl_up(row, off, 64);
        if (lane >= off && ru == row) v += vu;
      }
      if (tail) atomicAdd(&target[(int64_t)row * D + d], v);
    }
    return;
  }
  // lanes own columns (one 64-column slice per blockIdx.y, so wide rows such
  // as BERT's 768-wide token table still spread over many waves): walk the 64
  // occurrences, 8 loads in flight at a time
  {
    const int d = blockIdx.y * 64 + lane;
    const int dc = min(d, D - 1);
    float acc = 0.f;
    for (int q0 = 0; q0 < cnt; q0 += 8) {
      float v[8];
      int r[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int q = min(q0 + u, 63);
        r[u] = q0 + u < cnt ? __shfl(row, q, 64) : -1;
        v[u] = __shfl(w, q, 64) * dout[(size_t)__shfl(b, q, 64) * D + dc];
      }
      const int r_next = q0 + 8 < cnt ? __shfl(row, min(q0 + 8, 63), 64) : -2;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        acc += v[u];
        const int rn = u < 7 ? r[u + 1] : r_next;
        if (rn != r[u]) {
          if (r[u] >= 0 && d < D) atomicAdd(&target[(int64_t)r[u] * D + d], acc);
          acc = 0.f;
        }
      }
    }
  }
}

// rows of [N, C] logits vs int64 labels -> number of argmax hits
__global__ void argmax_correct(const float* __restrict__ x, const int64_t* __restrict__ labels, int Bn,
                               int Cn, int64_t* __restrict__ count) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= Bn) return;
  float m = -3.0e38f;
  int am = 0x7fffffff;
  for (int c = lane; c < Cn; c += 64) {
    const float v = x[(size_t)row * Cn + c];
    if (v > m || (v == m && c < am)) { m = v; am = c; }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float om = __shfl_xor(m, off, 64);
    const int oa = __shfl_xor(am, off, 64);
    if (om > m || (om == m && oa < am)) { m = om; am = oa; }
  }
  if (lane == 0 && am == (int)labels[row]) atomicAdd((unsigned long long*)count, 1ull);
}

// Per-bin positive / negative counts of predictions in [0, 1]; bin k covers
// thresholds [k/(nb-1) ...).  Counts accumulate across calls (streaming).
// streaming_auc's thresholds (TF contrib.metrics): t_0 = -1e-7, t_j = j/(T-1) for
// 0 < j < T-1 (a Python double rounded to fp32), t_{T-1} = 1 + 1e-7.  Bin k of a
// prediction p = #{i : t_i < p} in [0, T]; the confusion counts at threshold i
// (predicted positive <=> p > t_i) are then suffix sums over bins > i.
__device__ __forceinline__ int tf_threshold_bin(float p, int T) {
  if (!(p > -1e-7f)) return 0;          // (also NaN)
  if (p > 1.f + 1e-7f) return T;
  int lo = 1, hi = T - 1;               // first interior j with t_j >= p
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    const float t = (float)((double)mid / (double)(T - 1));
    if (t < p) lo = mid + 1; else hi = mid;
  }
  return lo;                            // 1 (t_0) + (lo - 1) interior thresholds below p
}

// labels: nonzero = positive (TF casts to bool); pos/neg: [T + 1] bins
__global__ void auc_hist(const float* __restrict__ pred, const float* __restrict__ label, int64_t n,
                         int T, unsigned long long* __restrict__ pos, unsigned long long* __restrict__ neg) {
  extern __shared__ unsigned int h[];  // [2][T + 1]
  const int nb = T + 1;
  for (int i = threadIdx.x; i < 2 * nb; i += blockDim.x) h[i] = 0;
  __syncthreads();
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(&h[(label[i] != 0.f ? 0 : nb) + tf_threshold_bin(pred[i], T)], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < nb; i += blockDim.x) {
    if (h[i]) atomicAdd(&pos[i], (unsigned long long)h[i]);
    if (h[nb + i]) atomicAdd(&neg[i], (unsigned long long)h[nb + i]);
  }
}

// ---------------------------------------------------------------- optimizers
// Multi-tensor: `tab` holds per-tensor {param*, grad*, m*, v*, numel}; the grid
// walks (tensor, chunk) pairs from `chunks` (tensor index, start element).
struct TensorRec {
  float* p;
  const void* g;
  float* m;
  float* v;
  int64_t n;
  uint16_t* shadow;   // optional bf16 copy of p refreshed in the same pass (compute weights)
};
constexpr int CHUNK = 4096;

__device__ __forceinline__ float ld_grad(const void* g, int64_t i, int gbf) {
  return gbf ? bf2f(reinterpret_cast<const uint16_t*>(g)[i]) : reinterpret_cast<const float*>(g)[i];
}

// kind 0: sgd, 1: momentum (use_nesterov in flags bit0), 2: adam (TF), 3: adamw,
// 4: adagrad (TF; m = accumulator), 5: rmsprop (TF; m = mean square, v = momentum, b1 = decay)
__global__ void multi_tensor_apply(const TensorRec* __restrict__ tab, const int2* __restrict__ chunks,
                                   int nchunks, int kind, int gbf, const float* __restrict__ lr_ptr,
                                   float lr_scalar, float gscale, float wd, float b1, float b2, float eps,
                                   float momentum, int nesterov, const long long* __restrict__ step_ptr,
                                   const int* __restrict__ skip) {
  const int cidx = blockIdx.x;
  if (cidx >= nchunks) return;
  if (skip != nullptr && *skip != 0) return;   // a voided step (sharded-table overflow): no update at all
  const int2 ch = chunks[cidx];
  const TensorRec t = tab[ch.x];
  const float lr = lr_ptr ? *lr_ptr : lr_scalar;
  float lr_t = lr;
  if (kind == 2 || kind == 3) {
    const double st = (double)(step_ptr ? *step_ptr : 1);
    // TF AdamOptimizer: lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t), eps outside the sqrt
    lr_t = (float)(lr * sqrt(1.0 - pow((double)b2, st)) / (1.0 - pow((double)b1, st)));
  }
  const int64_t s = (int64_t)ch.y, e = min(t.n, s + CHUNK);
  // one element: p, m, v in registers (m / v untouched by the kinds that have none)
  auto upd = [&](float& p, float g, float& m, float& v) {
    const float p0 = p;
    g *= gscale;
    if (kind == 0) {
      if (wd != 0.f) g += wd * p;
      p -= lr * g;
    } else if (kind == 1) {
      if (wd != 0.f) g += wd * p;
      const float mv = momentum * m + g;
      m = mv;
      p -= lr * (nesterov ? g + momentum * mv : mv);
    } else if (kind == 4) {
      // TF ApplyAdagrad: accum += g^2; var -= lr * g / sqrt(accum)
      const float acc = m + g * g;
      m = acc;
      p -= lr * g / sqrtf(acc);
    } else if (kind == 5) {
      // TF ApplyRMSProp: ms = rho ms + (1 - rho) g^2; mom = mu mom + lr g / sqrt(ms + eps); var -= mom
      const float ms = b1 * m + (1.f - b1) * g * g;
      const float mo = momentum * v + lr * g / sqrtf(ms + eps);
      m = ms;
      v = mo;
      p -= mo;
    } else {
      if (kind == 2 && wd != 0.f) g += wd * p;
      const float mv = b1 * m + (1.f - b1) * g;
      const float vv = b2 * v + (1.f - b2) * g * g;
      m = mv;
      v = vv;
      p -= lr_t * mv / (sqrtf(vv) + eps);
      if (kind == 3 && wd != 0.f) p -= lr * wd * p0;
    }
  };
  const bool use_m = kind != 0, use_v = kind == 2 || kind == 3 || kind == 5;
  // 16-byte path (4 elements per access) when every stream of this chunk is aligned:
  // the scalar loop moved 4 B per lane per access (~4.5 TB/s on BERT-base's AdamW)
  const bool vec = (s & 3) == 0 && (reinterpret_cast<uintptr_t>(t.p) & 15) == 0 &&
                   (!use_m || (reinterpret_cast<uintptr_t>(t.m) & 15) == 0) &&
                   (!use_v || (reinterpret_cast<uintptr_t>(t.v) & 15) == 0) &&
                   (reinterpret_cast<uintptr_t>(t.g) & (gbf ? 7 : 15)) == 0 &&
                   (t.shadow == nullptr || (reinterpret_cast<uintptr_t>(t.shadow) & 7) == 0);
  int64_t i0 = s;
  if (vec) {
    const int64_t e4 = s + ((e - s) & ~(int64_t)3);
    for (int64_t i = s + 4 * (int64_t)threadIdx.x; i < e4; i += 4 * (int64_t)blockDim.x) {
      float4 p4 = *reinterpret_cast<const float4*>(t.p + i);
      float4 m4 = use_m ? *reinterpret_cast<const float4*>(t.m + i) : float4{0.f, 0.f, 0.f, 0.f};
      float4 v4 = use_v ? *reinterpret_cast<const float4*>(t.v + i) : float4{0.f, 0.f, 0.f, 0.f};
      float g4[4];
      if (gbf) {
        const uint2 u = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(t.g) + i);
        g4[0] = bf2f(u.x & 0xffff); g4[1] = bf2f(u.x >> 16); g4[2] = bf2f(u.y & 0xffff); g4[3] = bf2f(u.y >> 16);
      } else {
        const float4 f = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(t.g) + i);
        g4[0] = f.x; g4[1] = f.y; g4[2] = f.z; g4[3] = f.w;
      }
      upd(p4.x, g4[0], m4.x, v4.x);
      upd(p4.y, g4[1], m4.y, v4.y);
      upd(p4.z, g4[2], m4.z, v4.z);
      upd(p4.w, g4[3], m4.w, v4.w);
      *reinterpret_cast<float4*>(t.p + i) = p4;
      if (use_m) *reinterpret_cast<float4*>(t.m + i) = m4;
      if (use_v) *reinterpret_cast<float4*>(t.v + i) = v4;
      if (t.shadow)
        *reinterpret_cast<uint2*>(t.shadow + i) = uint2{(uint32_t)f2bf(p4.x) | ((uint32_t)f2bf(p4.y) << 16),
                                                         (uint32_t)f2bf(p4.z) | ((uint32_t)f2bf(p4.w) << 16)};
    }
    i0 = e4;
  }
  for (int64_t i = i0 + threadIdx.x; i < e; i += blockDim.x) {
    float p = t.p[i];
    float m = use_m ? t.m[i] : 0.f, v = use_v ? t.v[i] : 0.f;
    upd(p, ld_grad(t.g, i, gbf), m, v);
    t.p[i] = p;
    if (use_m) t.m[i] = m;
    if (use_v) t.v[i] = v;
    if (t.shadow) t.shadow[i] = f2bf(p);
  }
}

// global-norm of a set of tensors (for clipping / NaN checks): sum of squares
__global__ void multi_tensor_sumsq(const TensorRec* __restrict__ tab, const int2* __restrict__ chunks,
                                   int nchunks, int gbf, float* __restrict__ out) {
  __shared__ float scratch[4];
  const int2 ch = chunks[blockIdx.x];
  const TensorRec t = tab[ch.x];
  const int64_t s = (int64_t)ch.y, e = min(t.n, s + CHUNK);
  float acc = 0.f;
  for (int64_t i = s + threadIdx.x; i < e; i += blockDim.x) {
    const float g = ld_grad(t.g, i, gbf);
    acc += g * g;
  }
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) atomicAdd(out, acc);
}

}  // namespace ops
}  // namespace dtfk

// ---------------------------------------------------------------- launchers
using namespace dtfk::ops;

namespace dtfk {
namespace ops {
// ---------------------------------------------------------------------------
// DDP bucket <-> communication buffer (K16): one pass each way.
//   pack:   comm[i] = half(scale * grad_f32[i])   (the 1/N average folded in)
//   unpack: grad_f32[i]  = scale * f32(comm[i])
// half = bf16 or fp16 (F16).  8 elements per thread (two 16-byte fp32 loads ->
// one 16-byte store); replaces cast + copy-back + mul_ (three full-bucket
// passes) around a 16-bit all-reduce.  Round-to-nearest-even like the cast it
// replaces (fp16 overflow -> inf, as the cast).
template <bool F16>
__device__ __forceinline__ uint32_t pack2h(float lo, float hi) {
  if constexpr (F16) {
    const _Float16 a = static_cast<_Float16>(lo), b = static_cast<_Float16>(hi);
    return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
  } else {
    return pack2bf(lo, hi);
  }
}
template <bool F16>
__device__ __forceinline__ float h2f(uint32_t bits) {
  if constexpr (F16) return static_cast<float>(__builtin_bit_cast(_Float16, (uint16_t)bits));
  else return bf2f((uint16_t)bits);
}

template <bool F16>
__global__ void bucket_pack(const float* __restrict__ g, uint16_t* __restrict__ c, int64_t n, float scale) {
  const int64_t n8 = n >> 3;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 a = reinterpret_cast<const float4*>(g)[2 * i];
    const float4 b = reinterpret_cast<const float4*>(g)[2 * i + 1];
    uint4 o;
    o.x = pack2h<F16>(a.x * scale, a.y * scale);
    o.y = pack2h<F16>(a.z * scale, a.w * scale);
    o.z = pack2h<F16>(b.x * scale, b.y * scale);
    o.w = pack2h<F16>(b.z * scale, b.w * scale);
    reinterpret_cast<uint4*>(c)[i] = o;
  }
  for (int64_t i = (n8 << 3) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    c[i] = (uint16_t)(pack2h<F16>(g[i] * scale, 0.f) & 0xFFFF);
}

template <bool F16>
__global__ void bucket_unpack(const uint16_t* __restrict__ c, float* __restrict__ g, int64_t n, float scale) {
  const int64_t n8 = n >> 3;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const uint4 u = reinterpret_cast<const uint4*>(c)[i];
    float4 a, b;
    a.x = h2f<F16>(u.x & 0xFFFF) * scale; a.y = h2f<F16>(u.x >> 16) * scale;
    a.z = h2f<F16>(u.y & 0xFFFF) * scale; a.w = h2f<F16>(u.y >> 16) * scale;
    b.x = h2f<F16>(u.z & 0xFFFF) * scale; b.y = h2f<F16>(u.z >> 16) * scale;
    b.z = h2f<F16>(u.w & 0xFFFF) * scale; b.w = h2f<F16>(u.w >> 16) * scale;
    reinterpret_cast<float4*>(g)[2 * i] = a;
    reinterpret_cast<float4*>(g)[2 * i + 1] = b;
  }
  for (int64_t i = (n8 << 3) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    g[i] = h2f<F16>(c[i]) * scale;
}
}  // namespace ops
}  // namespace dtfk

static int nblk(int64_t n, int per = 256, int cap = 4096) {
  int64_t b = (n + per - 1) / per;
  return (int)std::max<int64_t>(1, std::min<int64_t>(b, cap));
}

extern "C" {
hipError_t dtfk_bucket_pack(const float* g, uint16_t* c, int64_t n, float scale, int fp16, hipStream_t s) {
  if (fp16) hipLaunchKernelGGL(bucket_pack<true>, dim3(nblk((n + 7) / 8)), dim3(256), 0, s, g, c, n, scale);
  else hipLaunchKernelGGL(bucket_pack<false>, dim3(nblk((n + 7) / 8)), dim3(256), 0, s, g, c, n, scale);
  return hipGetLastError();
}
hipError_t dtfk_bucket_unpack(const uint16_t* c, float* g, int64_t n, float scale, int fp16, hipStream_t s) {
  if (fp16) hipLaunchKernelGGL(bucket_unpack<true>, dim3(nblk((n + 7) / 8)), dim3(256), 0, s, c, g, n, scale);
  else hipLaunchKernelGGL(bucket_unpack<false>, dim3(nblk((n + 7) / 8)), dim3(256), 0, s, c, g, n, scale);
  return hipGetLastError();
}
hipError_t dtfk_act_backward(const float* dy, const float* y, const float* z, float* dz, int64_t n,
                             int act, hipStream_t s) {
  hipLaunchKernelGGL(act_backward, dim3(nblk(n)), dim3(256), 0, s, dy, y, z, dz, n, act);
  return hipGetLastError();
}
// accum: out += the column sums (a gradient sunk into .grad) instead of out =
hipError_t dtfk_col_sum(const float* X, float* out, int M, int N, int accum, hipStream_t s) {
  if (M <= 0 || N <= 0) return hipSuccess;
  const bool vec = N % 4 == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  const int bx = vec ? (N / 4 + 15) / 16 : (N + 63) / 64;
  // ~256 blocks, at most 32 row chunks (atomics per column), >= 64 rows each
  int gy = std::max(1, std::min(std::min(32, (M + 63) / 64), 256 / bx));
  const int rows_per_block = ((M + gy - 1) / gy + 15) / 16 * 16;
  gy = (M + rows_per_block - 1) / rows_per_block;
  if (gy > 1 && !accum) {
    const hipError_t e = dtfk::zero2d_f32(out, N, 1, N, s);   // a kernel: replays from hipGraphs (common.h)
    if (e != hipSuccess) return e;
  }
  if (vec)
    hipLaunchKernelGGL(col_sum4, dim3(bx, gy), dim3(256), 0, s, reinterpret_cast<const float4*>(X), out, M, N / 4,
                       rows_per_block, accum);
  else
    hipLaunchKernelGGL(col_sum, dim3(bx, gy), dim3(256), 0, s, X, out, M, N, rows_per_block, accum);
  return hipGetLastError();
}
hipError_t dtfk_softmax_xent(const float* logits, const int64_t* labels, const float* ydense, float* loss_rows,
                             float* grad, int64_t* correct, int B, int C, float grad_scale, int naive,
                             hipStream_t s) {
  hipLaunchKernelGGL(softmax_xent, dim3((B + 3) / 4), dim3(256), 0, s, logits, labels, ydense, loss_rows,
                     grad, correct, B, C, grad_scale, naive);
  return hipGetLastError();
}
hipError_t dtfk_xent_fwd_bf16(const void* logits, const float* bias, const int64_t* labels, float* lse_rows,
                              float* loss_rows, int B, int C, hipStream_t s) {
  if (C % 2) return hipErrorInvalidValue;
  hipLaunchKernelGGL(xent_fwd_bf16, dim3(B), dim3(256), 0, s, (const uint16_t*)logits, bias, labels, lse_rows,
                     loss_rows, C);
  return hipGetLastError();
}
hipError_t dtfk_xent_bwd_bf16(const void* logits, const float* bias, const int64_t* labels, const float* lse_rows,
                              const float* dloss, void* grad, int B, int C, float scale, hipStream_t s) {
  if (C % 2) return hipErrorInvalidValue;
  hipLaunchKernelGGL(xent_bwd_bf16, dim3(B), dim3(256), 0, s, (const uint16_t*)logits, bias, labels, lse_rows, dloss,
                     (uint16_t*)grad, C, scale);
  return hipGetLastError();
}
hipError_t dtfk_logit3_xent(const float* a, const float* b, const float* bias, const float* t, float* loss,
                            float* dz, int n, hipStream_t s) {
  hipLaunchKernelGGL(logit3_xent, dim3(1), dim3(1024), 0, s, a, b, bias, t, loss, dz, n);
  return hipGetLastError();
}
hipError_t dtfk_logit3_xent_bwd(const float* dz, const float* g, float* d, float* gbias, int accum, int n,
                                hipStream_t s) {
  hipLaunchKernelGGL(logit3_xent_bwd, dim3(1), dim3(1024), 0, s, dz, g, d, gbias, accum, n);
  return hipGetLastError();
}
hipError_t dtfk_bag_index(const int64_t* offsets, int B, int* bag_of, int64_t N, hipStream_t s) {
  if (N <= 0) return hipSuccess;
  const long long blocks = (N + 255) / 256;
  hipLaunchKernelGGL(bag_index, dim3((unsigned)(blocks > 4096 ? 4096 : blocks)), dim3(256), 0, s, offsets, B, bag_of, N);
  return hipGetLastError();
}
hipError_t dtfk_multi_copy(const void* const* src, void* const* dst, const long long* bytes, int n, hipStream_t s) {
  if (n < 1 || n > 8) return hipErrorInvalidValue;
  CopyList c{};
  long long most = 0;
  for (int k = 0; k < n; ++k) {
    c.src[k] = static_cast<const char*>(src[k]);
    c.dst[k] = static_cast<char*>(dst[k]);
    c.bytes[k] = bytes[k];
    most = bytes[k] > most ? bytes[k] : most;
  }
  c.n = n;
  const long long blocks = (most / 16 + 255) / 256;
  hipLaunchKernelGGL(multi_copy, dim3((unsigned)(blocks < 1 ? 1 : (blocks > 1024 ? 1024 : blocks))), dim3(256), 0, s, c);
  return hipGetLastError();
}
hipError_t dtfk_sigmoid_xent(const float* x, const float* t, float* loss, float* grad, int64_t n,
                             float grad_scale, hipStream_t s) {
  hipLaunchKernelGGL(sigmoid_xent, dim3(nblk(n)), dim3(256), 0, s, x, t, loss, grad, n, grad_scale);
  return hipGetLastError();
}
hipError_t dtfk_embedding_bag_fwd(const float* W, int64_t V, int D, const int64_t* ids, const int64_t* offsets,
                                  const float* psw, int B, int mode, float* out, int64_t* bad, const int64_t* remap,
                                  hipStream_t s) {
  hipLaunchKernelGGL(embedding_bag_fwd, dim3((B + 3) / 4, D < 64 ? 1 : (D + 63) / 64), dim3(256), 0, s, W, V, D,
                     ids, offsets, psw, B,
                     mode, out, bad, remap);
  return hipGetLastError();
}
hipError_t dtfk_embedding_bag_bwd(float* target, int64_t V, int D, const int64_t* ids, const int64_t* offsets,
                                  const float* psw, const float* dout, int B, int mode, float lr,
                                  hipStream_t s) {
  hipLaunchKernelGGL(embedding_bag_bwd, dim3((B + 3) / 4), dim3(256), 0, s, target, V, D, ids, offsets, psw,
                     dout, B, mode, lr);
  return hipGetLastError();
}
hipError_t dtfk_embedding_bag_bwd_sorted(float* target, int64_t V, int D, const int* rows, const int64_t* occ,
                                         const int* bag_of, const float* psw, const float* dout, int64_t N,
                                         hipStream_t s) {
  if (N <= 0) return hipSuccess;
  const int64_t waves = (N + 63) / 64;
  const unsigned col_blocks = D < 64 ? 1u : (unsigned)((D + 63) / 64);
  hipLaunchKernelGGL(embedding_bag_bwd_sorted, dim3((unsigned)((waves + 3) / 4), col_blocks), dim3(256), 0, s, target, V, D,
                     rows, occ, bag_of, psw, dout, N);
  return hipGetLastError();
}
hipError_t dtfk_argmax_correct(const float* x, const int64_t* labels, int B, int C, int64_t* count,
                               hipStream_t s) {
  hipLaunchKernelGGL(argmax_correct, dim3((B + 3) / 4), dim3(256), 0, s, x, labels, B, C, count);
  return hipGetLastError();
}
hipError_t dtfk_auc_hist(const float* pred, const float* label, int64_t n, int nbins,
                         unsigned long long* pos, unsigned long long* neg, hipStream_t s) {
  // nbins = T + 1 histogram bins for T thresholds
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(auc_hist, dim3(nblk(n, 256, 1024)), dim3(256), 2 * nbins * sizeof(unsigned int), s, pred,
                     label, n, nbins - 1, pos, neg);
  return hipGetLastError();
}
hipError_t dtfk_multi_tensor_apply(const void* tab, const void* chunks, int nchunks, int kind, int gbf,
                                   const float* lr_ptr, float lr, float gscale, float wd, float b1, float b2,
                                   float eps, float momentum, int nesterov, const long long* step,
                                   const int* skip, hipStream_t s) {
  if (nchunks == 0) return hipSuccess;
  hipLaunchKernelGGL(multi_tensor_apply, dim3(nchunks), dim3(256), 0, s, (const TensorRec*)tab,
                     (const int2*)chunks, nchunks, kind, gbf, lr_ptr, lr, gscale, wd, b1, b2, eps, momentum,
                     nesterov, step, skip);
  return hipGetLastError();
}
hipError_t dtfk_multi_tensor_sumsq(const void* tab, const void* chunks, int nchunks, int gbf, float* out,
                                   hipStream_t s) {
  (void)dtfk::zero2d_f32(out, 1, 1, 1, s);
  if (nchunks == 0) return hipSuccess;
  hipLaunchKernelGGL(multi_tensor_sumsq, dim3(nchunks), dim3(256), 0, s, (const TensorRec*)tab,
                     (const int2*)chunks, nchunks, gbf, out);
  return hipGetLastError();
}
int dtfk_mt_chunk() { return CHUNK; }
int dtfk_tensor_rec_bytes() { return (int)sizeof(TensorRec); }
}
