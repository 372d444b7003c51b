// Reached by: sharded-table sparse optimizers (Wide&Deep sparse_opt=adagrad/rmsprop/momentum); tests/test_sparse_optim_gpu.py
// Row-sparse optimizer updates of a sharded embedding table, on its owner
// (parallel/sharded_embedding.py: ShardedEmbedding.set_optimizer).
//
// TensorFlow applies an IndexedSlices gradient with its SparseApply* ops:
// duplicate indices are summed first (Optimizer._apply_sparse_duplicate_indices),
// then every touched row is updated on its own -- rows the batch did not touch
// keep their value AND their slots.  The owner has already summed the
// duplicates of a step (every rank that looked a row up sends its gradient);
// this kernel is the per-row update:
//
//   kind 0  GradientDescent  var -= lr g
//   kind 1  Momentum         acc = mu acc + g;  var -= lr acc   (Nesterov: lr (g + mu acc))
//   kind 4  Adagrad          acc += g^2;        var -= lr g / sqrt(acc)
//   kind 5  RMSProp          ms = rho ms + (1-rho) g^2;  mom = mu mom + lr g / sqrt(ms + eps);  var -= mom
//
// (kind numbers = optim.KINDS).  rows[i] < 0 marks an entry with no update
// (exchange padding, the non-first copies of a duplicated row).  Rows with
// rows[i] >= 0 are distinct, so every element has exactly one writer: plain
// loads and stores, no atomics.  One thread per (entry, column), 4 columns
// per thread when D % 4 == 0.  `skip` (device int32, may be null): a voided
// step (sharded-exchange overflow) changes nothing.
#include "common.h"

namespace dtfk {
namespace sparse_optim {

struct Hyper {
  float lr, mu, rho, eps;
  int kind, nesterov;
};

__device__ __forceinline__ void update1(float& var, float& a, float& b, float g, const Hyper& h) {
  switch (h.kind) {
    case 0: var -= h.lr * g; break;
    case 1: {
      const float acc = h.mu * a + g;
      a = acc;
      var -= h.lr * (h.nesterov ? g + h.mu * acc : acc);
      break;
    }
    case 4: {
      const float acc = a + g * g;
      a = acc;
      var -= h.lr * g * rsqrtf(acc);
      break;
    }
    default: {   // 5: RMSProp, a = ms, b = mom
      const float ms = h.rho * a + (1.f - h.rho) * g * g;
      const float mom = h.mu * b + h.lr * g * rsqrtf(ms + h.eps);
      a = ms;
      b = mom;
      var -= mom;
      break;
    }
  }
}

template <int V>
__global__ __launch_bounds__(256) void rows_apply(float* __restrict__ table, float* __restrict__ slot_a,
                                                  float* __restrict__ slot_b, const long long* __restrict__ rows,
                                                  const float* __restrict__ g, long long n, int D, Hyper h,
                                                  const int* __restrict__ skip) {
  if (skip != nullptr && *skip != 0) return;
  const int dv = D / V;
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n * dv) return;
  const long long i = e / dv;
  const int c = (int)(e - i * dv) * V;
  const long long r = rows[i];
  if (r < 0) return;
  const size_t o = (size_t)r * D + c;
  const size_t go = (size_t)i * D + c;
  float var[V], a[V], b[V], gg[V];
#pragma unroll
  for (int k = 0; k < V; ++k) {
    var[k] = table[o + k];
    a[k] = slot_a != nullptr ? slot_a[o + k] : 0.f;
    b[k] = slot_b != nullptr ? slot_b[o + k] : 0.f;
    gg[k] = g[go + k];
  }
#pragma unroll
  for (int k = 0; k < V; ++k) update1(var[k], a[k], b[k], gg[k], h);
#pragma unroll
  for (int k = 0; k < V; ++k) {
    table[o + k] = var[k];
    if (slot_a != nullptr) slot_a[o + k] = a[k];
    if (slot_b != nullptr) slot_b[o + k] = b[k];
  }
}

}  // namespace sparse_optim
}  // namespace dtfk

extern "C" hipError_t dtfk_sparse_rows_apply(float* table, float* slot_a, float* slot_b, const long long* rows,
                                             const float* g, long long n, int D, int kind, float lr, float mu,
                                             int nesterov, float rho, float eps, const int* skip, hipStream_t s) {
  using namespace dtfk::sparse_optim;
  if (n <= 0 || D <= 0) return hipSuccess;
  if (kind != 0 && kind != 1 && kind != 4 && kind != 5) return hipErrorInvalidValue;
  if ((kind == 1 || kind == 4 || kind == 5) && slot_a == nullptr) return hipErrorInvalidValue;
  if (kind == 5 && slot_b == nullptr) return hipErrorInvalidValue;
  const Hyper h{lr, mu, rho, eps, kind, nesterov};
  const bool v4 = D % 4 == 0;
  const long long work = n * (v4 ? D / 4 : D);
  const unsigned grid = (unsigned)((work + 255) / 256);
  if (v4)
    hipLaunchKernelGGL(rows_apply<4>, dim3(grid), dim3(256), 0, s, table, slot_a, slot_b, rows, g, n, D, h, skip);
  else
    hipLaunchKernelGGL(rows_apply<1>, dim3(grid), dim3(256), 0, s, table, slot_a, slot_b, rows, g, n, D, h, skip);
  return hipGetLastError();
}
