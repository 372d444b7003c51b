// Reached by: asynchronous (Hogwild) ps mode (parallel/async_ps.py, --update_mode=async); tests/test_async_ps_gpu.py
// Asynchronous (Hogwild) parameter-server updates: the reference's default
// update rule (example.py:64-118, between-graph replication with a plain
// GradientDescentOptimizer and no SyncReplicasOptimizer: every worker reads the
// ps-held variables, computes its gradient and applies `var -= lr * grad` on the
// ps without waiting for the others; use_locking=False: no lock).
//
// MI355X form: the "ps variables" are ONE flat fp32 buffer in the device memory
// of the hosting rank (hipDeviceMallocUncached, IPC-mapped into every worker:
// csrc/comm/ipc_peer.cpp), followed by a 64-bit global-step counter.  Workers
// on other GPUs reach it over xGMI with system-scope loads/stores; the update
// is applied where the gradient lives (no gradient shipping to a ps process).
//   pull : local[i] <- shared[i]                         (before the forward)
//   step : s = shared[i] - lr g[i]; shared[i] = s; local[i] = s
//          locking = 0: plain read-modify-write (Hogwild: a concurrent update
//          of the same element may be lost, as with TF's use_locking=False);
//          locking = 1: a compare-and-swap loop per element (no lost updates)
//          and global_step += 1 (atomic) -> gstep_out.
#include "common.h"

namespace dtfk {
namespace hogwild {

__device__ __forceinline__ void st_sys_f32(float* p, float v) {
  __hip_atomic_store(reinterpret_cast<uint32_t*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void pull(const float* __restrict__ shared, float* __restrict__ local, long long n) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    local[i] = ld_sys_f32(shared + i);
}

__global__ __launch_bounds__(256) void sgd(float* shared, const float* __restrict__ g, float* __restrict__ local,
                                           float lr, long long n, int locking, unsigned long long* counter,
                                           long long* gstep_out) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float d = lr * g[i];
    float s;
    if (locking) {
      uint32_t* p = reinterpret_cast<uint32_t*>(shared + i);
      uint32_t old = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      for (;;) {
        s = __uint_as_float(old) - d;
        uint32_t want = old;
        if (__hip_atomic_compare_exchange_strong(p, &want, __float_as_uint(s), __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_SYSTEM))
          break;
        old = want;
      }
    } else {
      s = ld_sys_f32(shared + i) - d;
      st_sys_f32(shared + i, s);
    }
    local[i] = s;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && counter != nullptr) {
    const unsigned long long old = __hip_atomic_fetch_add(counter, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (gstep_out != nullptr) *gstep_out = (long long)(old + 1ull);
  }
}

__global__ void read_counter(const unsigned long long* counter, long long* out) {
  *out = (long long)__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void write_counter(unsigned long long* counter, long long v) {
  __hip_atomic_store(counter, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Row-sharded tables (partitioned variables, lr2.py's ps-held W[F, 1]) under the
// asynchronous rule: every rank's shard is IPC-mapped into every rank (row r on
// rank r % W at local row r / W, parallel/sharded_embedding.py); a worker reads
// its batch's unique rows straight from their owners and applies its scatter
// SGD into them, without waiting for anyone (TF's ScatterSub on the ps).
__global__ __launch_bounds__(256) void gather_rows(const long long* __restrict__ ids, int n, int D,
                                                   const float* const* __restrict__ shards, int W,
                                                   float* __restrict__ out) {
  const long long total = (long long)n * D;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const long long u = i / D;
    const int d = (int)(i - u * D);
    const long long id = ids[u];
    const float* sh = shards[(int)(id % W)];
    out[i] = ld_sys_f32(sh + (id / W) * D + d);
  }
}

__global__ __launch_bounds__(256) void scatter_sgd(const long long* __restrict__ ids, const float* __restrict__ g,
                                                   int n, int D, float* const* __restrict__ shards, int W, float lr,
                                                   int locking) {
  const long long total = (long long)n * D;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const long long u = i / D;
    const int d = (int)(i - u * D);
    const long long id = ids[u];
    float* p = shards[(int)(id % W)] + (id / W) * D + d;
    const float dv = lr * g[i];
    if (locking) {
      uint32_t* q = reinterpret_cast<uint32_t*>(p);
      uint32_t old = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      for (;;) {
        uint32_t want = old;
        if (__hip_atomic_compare_exchange_strong(q, &want, __float_as_uint(__uint_as_float(old) - dv),
                                                 __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))
          break;
        old = want;
      }
    } else {
      st_sys_f32(p, ld_sys_f32(p) - dv);    // Hogwild: a concurrent update of the same row may be lost
    }
  }
}

inline int grid_for(long long n) {
  const long long b = (n + 255) / 256;
  return (int)(b < 1024 ? (b < 1 ? 1 : b) : 1024);
}

}  // namespace hogwild
}  // namespace dtfk

extern "C" {

hipError_t dtfk_hogwild_pull(const float* shared, float* local, long long n, hipStream_t s) {
  using namespace dtfk::hogwild;
  hipLaunchKernelGGL(pull, dim3(grid_for(n)), dim3(256), 0, s, shared, local, n);
  return hipGetLastError();
}

hipError_t dtfk_hogwild_sgd(float* shared, const float* g, float* local, float lr, long long n, int locking,
                            unsigned long long* counter, long long* gstep_out, hipStream_t s) {
  using namespace dtfk::hogwild;
  hipLaunchKernelGGL(sgd, dim3(grid_for(n)), dim3(256), 0, s, shared, g, local, lr, n, locking, counter, gstep_out);
  return hipGetLastError();
}

hipError_t dtfk_hogwild_gather_rows(const long long* ids, int n, int D, const float* const* shards, int W, float* out,
                                   hipStream_t s) {
  using namespace dtfk::hogwild;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(gather_rows, dim3(grid_for((long long)n * D)), dim3(256), 0, s, ids, n, D, shards, W, out);
  return hipGetLastError();
}

hipError_t dtfk_hogwild_scatter_sgd(const long long* ids, const float* g, int n, int D, float* const* shards, int W,
                                    float lr, int locking, hipStream_t s) {
  using namespace dtfk::hogwild;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(scatter_sgd, dim3(grid_for((long long)n * D)), dim3(256), 0, s, ids, g, n, D, shards, W, lr,
                     locking);
  return hipGetLastError();
}

hipError_t dtfk_hogwild_counter(unsigned long long* counter, long long* out, long long set, int do_set, hipStream_t s) {
  using namespace dtfk::hogwild;
  if (do_set) hipLaunchKernelGGL(write_counter, dim3(1), dim3(1), 0, s, counter, set);
  else hipLaunchKernelGGL(read_counter, dim3(1), dim3(1), 0, s, counter, out);
  return hipGetLastError();
}

}  // extern "C"
