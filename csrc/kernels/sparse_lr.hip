// lr2.py's training step on ONE GPU as two kernels:
//
//   py_x  = embedding_lookup_sparse(W, ids, vals, 'sum') + b      (lr2.py:383-390)
//   loss  = mean(sigmoid_xent(py_x, y))                          (lr2.py:391)
//   W[id] -= lr * dL/dW[id] ; b -= lr * dL/db                     (lr2.py:394-396)
//
// With one worker every row of W lives on this GPU, so the step needs no
// dedup, no routing and no exchange: the general path (parallel/
// sharded_embedding.py: radix sort + unique + bucketing + bag + xent + bag
// backward + scatter apply, ~40 small kernels, 105 us at B = 500 / 20 k ids)
// collapses into
//
//   slr_fwd    one wave per batch row: z = b + sum_j W[id_j] val_j (lanes stride
//              the row's ids, DPP wave sum), the row's sigmoid cross-entropy and
//              dz = (sigmoid(z) - y) / B;
//   slr_apply  one wave per batch row: W[id_j] -= lr dz val_j by float atomics
//              at the memory side (TF's ScatterSub on the ps: duplicates combine,
//              hot Zipf ids included); workgroup 0 also sums dz and the row losses
//              in a fixed order -> b -= lr sum(dz), the batch's mean loss, and the
//              graph's global_step += 1.
//
// The kernel boundary orders every read of W / b (forward) before any update.
#include "common.h"

namespace dtfk {
namespace slr {

constexpr int THREADS = 256;   // 4 waves = 4 batch rows per workgroup

__device__ __forceinline__ float xent(float v, float y) { return fmaxf(v, 0.f) - v * y + log1pf(__expf(-fabsf(v))); }

__global__ __launch_bounds__(THREADS) void slr_fwd(const float* __restrict__ W, long long F,
                                                   const long long* __restrict__ ids,
                                                   const long long* __restrict__ offsets,
                                                   const float* __restrict__ vals, const float* __restrict__ labels,
                                                   const float* __restrict__ bias, int B, float* __restrict__ dz,
                                                   float* __restrict__ lrow, int* __restrict__ bad) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * (THREADS / 64) + (threadIdx.x >> 6);
  if (b >= B) return;
  const long long s = offsets[b], e = offsets[b + 1];
  float acc = 0.f;
  for (long long j = s + lane; j < e; j += 64) {
    const long long id = ids[j];
    if (id < 0 || id >= F) {   // TF raises on an out-of-range id; counted, skipped
      atomicAdd(bad, 1);
      continue;
    }
    acc += W[id] * (vals != nullptr ? vals[j] : 1.f);
  }
  acc = wave_sum(acc);
  if (lane == 0) {
    const float z = acc + bias[0];
    const float y = labels[b];
    lrow[b] = xent(z, y);
    dz[b] = (1.f / (1.f + __expf(-z)) - y) / (float)B;
  }
}

__global__ __launch_bounds__(THREADS) void slr_apply(float* __restrict__ W, long long F,
                                                     const long long* __restrict__ ids,
                                                     const long long* __restrict__ offsets,
                                                     const float* __restrict__ vals, const float* __restrict__ dz,
                                                     const float* __restrict__ lrow, const float* __restrict__ lr_ptr,
                                                     float lr_val, float* __restrict__ bias, int B,
                                                     float* __restrict__ loss_out, void* gvar, int gkind) {
  const float lr = lr_ptr != nullptr ? *lr_ptr : lr_val;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int b = blockIdx.x * (THREADS / 64) + wv;
  if (b < B) {
    const float g = -lr * dz[b];
    const long long s = offsets[b], e = offsets[b + 1];
    for (long long j = s + lane; j < e; j += 64) {
      const long long id = ids[j];
      const float v = vals != nullptr ? vals[j] : 1.f;
      if (id >= 0 && id < F && v != 0.f) atomicAdd(W + id, g * v);   // padding (val 0) touches nothing
    }
  }
  if (blockIdx.x == 0) {   // fixed-order sums of dz and the row losses
    __shared__ float red[2][THREADS / 64];
    float sd = 0.f, sl = 0.f;
    for (int i = threadIdx.x; i < B; i += THREADS) {
      sd += dz[i];
      sl += lrow[i];
    }
    sd = wave_sum(sd);
    sl = wave_sum(sl);
    if (lane == 0) {
      red[0][wv] = sd;
      red[1][wv] = sl;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      float td = 0.f, tl = 0.f;
      for (int k = 0; k < THREADS / 64; ++k) {
        td += red[0][k];
        tl += red[1][k];
      }
      bias[0] -= lr * td;
      loss_out[0] = tl / (float)B;
      if (gkind == 1) *static_cast<float*>(gvar) += 1.f;
      else if (gkind == 2) *static_cast<long long*>(gvar) += 1;
      else if (gkind == 3) *static_cast<int*>(gvar) += 1;
      else if (gkind == 4) *static_cast<double*>(gvar) += 1.0;
    }
  }
}

}  // namespace slr
}  // namespace dtfk

extern "C" {

// gkind: 0 none, 1 f32, 2 i64, 3 i32, 4 f64 (the graph's global_step variable)
hipError_t dtfk_slr_step(float* W, long long F, const long long* ids, const long long* offsets, const float* vals,
                         const float* labels, float* bias, int B, const float* lr_ptr, float lr_val, float* dz,
                         float* lrow, float* loss_out, int* bad, void* gvar, int gkind, hipStream_t stream) {
  using namespace dtfk::slr;
  if (B < 1 || gkind < 0 || gkind > 4 || (gkind != 0 && gvar == nullptr)) return hipErrorInvalidValue;
  const int grid = (B + THREADS / 64 - 1) / (THREADS / 64);
  hipLaunchKernelGGL(slr_fwd, dim3(grid), dim3(THREADS), 0, stream, W, F, ids, offsets, vals, labels, bias, B, dz,
                     lrow, bad);
  hipLaunchKernelGGL(slr_apply, dim3(grid), dim3(THREADS), 0, stream, W, F, ids, offsets, vals, dz, lrow, lr_ptr,
                     lr_val, bias, B, loss_out, gvar, gkind);
  return hipGetLastError();
}

}  // extern "C"
