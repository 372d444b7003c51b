// Device-resident dedup + owner routing for the row-sharded tables
// (parallel/sharded_embedding.py; reference: embedding_lookup_sparse on a
// ps-placed W, lr2.py:383-390 -- the worker sends the batch's unique ids to
// the ps).
//
// One 1024-thread workgroup turns the radix-sorted ids of a batch into
//   inv_sorted[i]  dedup index of sorted occurrence i (block-wide scan of the
//                  "new id" flags),
//   inverse[perm[i]] = inv_sorted[i]   (dedup index of each original position),
//   uniq[j]        the j-th distinct id, -1 for j >= U (static length N),
//   dest[j]        W > 1: slot of uniq[j] in the [W][cap] exchange layout
//                  (owner = id % W; positions within an owner in id order),
//   send[W*cap]    W > 1: ids bucketed by owner, -1 padded,
//   count[0] = U,
// with every shape static and nothing read back by the host: the exchange is an
// equal-split all-to-all of `cap` slots per peer, cap >= N (the ids of this
// rank's batch bound every bucket, so nothing can overflow) and the same on
// every rank (a configured capacity), so the sparse step can be captured.
// Each thread owns a contiguous chunk of <= ceil(N/1024) sorted positions;
// per-owner positions come from a second scan over the threads' owner counts.
#include "common.h"

namespace dtfk {
namespace route {

constexpr int T = 1024;
constexpr int MAXW = 16;

__device__ __forceinline__ int block_excl_scan(int v, int* sh, int& total) {
  // Hillis-Steele over 1024 entries in LDS (two buffers)
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  int* a = sh;
  int* b = sh + T;
  for (int off = 1; off < T; off <<= 1) {
    b[t] = a[t] + (t >= off ? a[t - off] : 0);
    __syncthreads();
    int* tmp = a; a = b; b = tmp;
  }
  const int incl = a[t];
  total = a[T - 1];
  __syncthreads();
  return incl - v;
}

template <typename ID>
__global__ __launch_bounds__(T) void sparse_route(const ID* __restrict__ sids, const int64_t* __restrict__ perm,
                                                  int N, int W, int cap, int* __restrict__ inv_sorted,
                                                  int64_t* __restrict__ inverse, int64_t* __restrict__ uniq,
                                                  int* __restrict__ dest, int64_t* __restrict__ send,
                                                  int* __restrict__ count) {
  __shared__ int sh[2 * T];
  __shared__ int own[T * MAXW];      // per-thread owner counts -> bases
  const int t = threadIdx.x;
  const int chunk = (N + T - 1) / T;
  const int lo = min(N, t * chunk), hi = min(N, lo + chunk);
  // 1. dedup index of each sorted occurrence
  int nnew = 0;
  for (int i = lo; i < hi; ++i) nnew += (i == 0 || sids[i] != sids[i - 1]) ? 1 : 0;
  int U;
  const int base = block_excl_scan(nnew, sh, U);
  int k = base - 1;
  for (int i = lo; i < hi; ++i) {
    const ID v = sids[i];
    if (i == 0 || v != sids[i - 1]) {
      ++k;
      uniq[k] = (int64_t)v;
    }
    inv_sorted[i] = k;
    inverse[perm[i]] = k;
  }
  // uniq / dest positions >= U: -1 (chunking over j; valid entries are < U)
  for (int j = max(lo, U); j < hi; ++j) {
    uniq[j] = -1;
    if (W > 1) dest[j] = -1;
  }
  if (t == 0) count[0] = U;
  if (W <= 1) return;
  // 2. owner buckets.  Thread t re-walks its own sorted chunk: the distinct ids
  // it found are exactly uniq[base .. base + nnew), so no thread reads another
  // thread's global writes.
  int c[MAXW];
#pragma unroll
  for (int o = 0; o < MAXW; ++o) c[o] = 0;
  for (int i = lo; i < hi; ++i) {
    const ID v = sids[i];
    if (i == 0 || v != sids[i - 1]) {
      const int o = (int)((int64_t)v % W);
#pragma unroll
      for (int q = 0; q < MAXW; ++q) c[q] += (q == o) ? 1 : 0;
    }
  }
  // per owner: exclusive scan over threads (thread order == id order)
  for (int o = 0; o < W; ++o) {
    int tot;
    own[t * MAXW + o] = block_excl_scan(c[o], sh, tot);
  }
  int run[MAXW];
#pragma unroll
  for (int o = 0; o < MAXW; ++o) run[o] = o < W ? own[t * MAXW + o] : 0;
  k = base - 1;
  for (int i = lo; i < hi; ++i) {
    const ID v = sids[i];
    if (i == 0 || v != sids[i - 1]) {
      ++k;
      const int o = (int)((int64_t)v % W);
      int p = 0;
#pragma unroll
      for (int q = 0; q < MAXW; ++q)
        if (q == o) { p = run[q]; run[q] = p + 1; }
      const int d = o * cap + p;
      dest[k] = d;
      send[d] = (int64_t)v;
    }
  }
}

__global__ void fill_i64(int64_t* __restrict__ p, long long n, int64_t v) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    p[i] = v;
}

}  // namespace route
}  // namespace dtfk

extern "C" int dtfk_route_max_world() { return dtfk::route::MAXW; }

// sids: sorted ids (int32 if ids32 else int64); perm: torch.sort permutation.
extern "C" hipError_t dtfk_sparse_route(const void* sids, int ids32, const int64_t* perm, int N, int W, int cap,
                                        int* inv_sorted, int64_t* inverse, int64_t* uniq, int* dest, int64_t* send,
                                        int* count, hipStream_t stream) {
  using namespace dtfk::route;
  if (N <= 0) return hipSuccess;
  if (W > MAXW || (W > 1 && cap < N)) return hipErrorInvalidValue;
  if (W > 1) {
    const long long n = (long long)W * cap;
    hipLaunchKernelGGL(fill_i64, dim3((unsigned)std::min<long long>((n + 255) / 256, 4096)), dim3(256), 0, stream, send,
                       n, (int64_t)-1);
  }
  if (ids32)
    hipLaunchKernelGGL(sparse_route<int>, dim3(1), dim3(T), 0, stream, static_cast<const int*>(sids), perm, N, W, cap,
                       inv_sorted, inverse, uniq, dest, send, count);
  else
    hipLaunchKernelGGL(sparse_route<int64_t>, dim3(1), dim3(T), 0, stream, static_cast<const int64_t*>(sids), perm, N,
                       W, cap, inv_sorted, inverse, uniq, dest, send, count);
  return hipGetLastError();
}
