// Reached by: sharded-table static routing (parallel/sharded_embedding.py _route_static); tests/test_models_gpu.py, test_sharded_ipc_gpu.py
// Device-resident dedup + owner routing for the row-sharded tables
// (parallel/sharded_embedding.py; reference: embedding_lookup_sparse on a
// ps-placed W, lr2.py:383-390 -- the worker sends the batch's unique ids to
// the ps).
//
// From the radix-sorted ids of a batch (sids, perm = torch.sort) it builds
//   inv_sorted[i]  dedup index of sorted occurrence i,
//   inverse[perm[i]] = inv_sorted[i]   (dedup index of each original position),
//   uniq[j]        the j-th distinct id, -1 for j >= U (static length N),
//   dest[j]        W > 1: slot of uniq[j] in the [W][cap] exchange layout
//                  (owner = id % W; positions within an owner in id order),
//   send[W*cap]    W > 1: ids bucketed by owner, -1 padded,
// with every shape static and nothing read back by the host: the exchange is an
// equal-split all-to-all of `cap` slots per peer, the same on every rank, so the
// sparse step can be captured.  `cap` is right-sized to the owners' unique-id
// load (parallel/sharded_embedding.py adapts it), not to the batch: an owner's
// ids beyond `cap` are not sent (dest -1) -- the per-owner unique counts come
// back to the caller, which voids such a step on every rank and replays it
// through the exact exchange.
//
// Fully parallel over the batch: route_flags marks the first occurrence of
// each id (and, W > 1, its owner as a one-hot row), the host-side binding runs
// the prefix sums (rocPRIM scans via at::cumsum: the dedup index and, per
// owner, the position among that owner's ids), route_scatter writes every
// output in one pass (threads i >= U also write the -1 padding of slot i).
#include "common.h"

namespace dtfk {
namespace route {

constexpr int MAXW = 16;

template <typename ID>
__global__ __launch_bounds__(256) void route_flags(const ID* __restrict__ sids, int N, int W,
                                                   int* __restrict__ flag, int* __restrict__ onehot) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const ID v = sids[i];
  const int f = (i == 0 || v != sids[max(i - 1, 0)]) ? 1 : 0;
  flag[i] = f;
  if (W > 1) {   // owner-major rows [W][N] behind the flags: one flat scan covers them all
    const int o = (int)((int64_t)v % W);
    for (int q = 0; q < W; ++q) onehot[(size_t)q * N + i] = (f && q == o) ? 1 : 0;
  }
}

template <typename ID>
__global__ __launch_bounds__(256) void route_scatter(const ID* __restrict__ sids, const int64_t* __restrict__ perm,
                                                     const int* __restrict__ incl, const int* __restrict__ owncum,
                                                     int N, int W, int cap, int* __restrict__ inv_sorted,
                                                     int64_t* __restrict__ inverse, int64_t* __restrict__ uniq,
                                                     int* __restrict__ dest, int64_t* __restrict__ send,
                                                     int* __restrict__ count) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const ID v = sids[i];
  const int k = incl[i] - 1;
  const int U = incl[N - 1];
  inv_sorted[i] = k;
  inverse[perm[i]] = k;
  const bool first = (i == 0) || k != incl[max(i - 1, 0)] - 1;
  if (first) {
    uniq[k] = (int64_t)v;
    if (W > 1) {
      const int o = (int)((int64_t)v % W);
      // rank among owner o's unique ids: the flat inclusive scan of [flags | owner
      // rows] minus the scan's value at the end of the previous row
      const int pos = owncum[(long long)o * N + i] - owncum[(long long)o * N - 1] - 1;
      if (pos < cap) {
        const int d = o * cap + pos;
        dest[k] = d;
        send[d] = (int64_t)v;
      } else {
        dest[k] = -1;                                    // overflow: not exchanged (the step is voided)
      }
    }
  }
  if (i >= U) {            // padding slots of the static-length outputs
    uniq[i] = -1;
    if (W > 1) dest[i] = -1;
  }
  if (i == 0) count[0] = U;
}

__global__ void fill_i64(int64_t* __restrict__ p, long long n, int64_t v) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    p[i] = v;
}

}  // namespace route
}  // namespace dtfk

extern "C" int dtfk_route_max_world() { return dtfk::route::MAXW; }

// Pass 1: first-occurrence flags (+ owner one-hot rows [W][N] when W > 1).
extern "C" hipError_t dtfk_route_flags(const void* sids, int ids32, int N, int W, int* flag, int* onehot,
                                       hipStream_t stream) {
  using namespace dtfk::route;
  if (N <= 0) return hipSuccess;
  if (W > MAXW) return hipErrorInvalidValue;
  const dim3 g((N + 255) / 256), b(256);
  if (ids32)
    hipLaunchKernelGGL(route_flags<int>, g, b, 0, stream, static_cast<const int*>(sids), N, W, flag, onehot);
  else
    hipLaunchKernelGGL(route_flags<int64_t>, g, b, 0, stream, static_cast<const int64_t*>(sids), N, W, flag, onehot);
  return hipGetLastError();
}

// Pass 2 (after ONE flat inclusive scan of [flag (N) | owner rows (W x N)]:
// incl = its first N values, owncum = the scan from the owner rows on -- a
// per-column scan of an [N, W] one-hot (torch's outer-dimension scan) took
// 15 ms at N = 131072, W = 2).
extern "C" hipError_t dtfk_route_scatter(const void* sids, int ids32, const int64_t* perm, const int* incl,
                                         const int* owncum, int N, int W, int cap, int* inv_sorted, int64_t* inverse,
                                         int64_t* uniq, int* dest, int64_t* send, int* count, hipStream_t stream) {
  using namespace dtfk::route;
  if (N <= 0) return hipSuccess;
  if (W > MAXW || (W > 1 && cap < 1)) return hipErrorInvalidValue;
  if (W > 1) {
    const long long n = (long long)W * cap;
    hipLaunchKernelGGL(fill_i64, dim3((unsigned)std::min<long long>((n + 255) / 256, 4096)), dim3(256), 0, stream, send,
                       n, (int64_t)-1);
  }
  const dim3 g((N + 255) / 256), b(256);
  if (ids32)
    hipLaunchKernelGGL(route_scatter<int>, g, b, 0, stream, static_cast<const int*>(sids), perm, incl, owncum, N, W, cap,
                       inv_sorted, inverse, uniq, dest, send, count);
  else
    hipLaunchKernelGGL(route_scatter<int64_t>, g, b, 0, stream, static_cast<const int64_t*>(sids), perm, incl, owncum,
                       N, W, cap, inv_sorted, inverse, uniq, dest, send, count);
  return hipGetLastError();
}
