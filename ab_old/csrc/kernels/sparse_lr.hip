// Reached by: one-GPU sparse LR step (csrc/bind_sparse.cpp SparseLRPlan: models/sparse_lr.py, the lr2 compat Session); tests/test_models_gpu.py, test_lowering_gpu.py
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
//   slr_apply  W[id_j] -= lr dz val_j (TF's ScatterSub on the ps: duplicates
//              combine): each workgroup sums its 32 rows' updates per id in an LDS
//              hash table, then one float atomic per distinct id; workgroup 0 also
//              sums dz and the row losses in a fixed order -> b -= lr sum(dz), the
//              batch's mean loss, and the graph's global_step += 1.
//
// The kernel boundary orders every read of W / b (forward) before any update.
#include "common.h"

namespace dtfk {
namespace slr {

constexpr int THREADS = 256;   // 4 waves = 4 batch rows per workgroup

__device__ __forceinline__ float xent(float v, float y) { return fmaxf(v, 0.f) - v * y + log1pf(__expf(-fabsf(v))); }

// COPY: ids / offsets / values / labels are read straight from the packed
// feed in mapped pinned host memory (one pass, no staging copy in front of the
// step) and the ids, offsets and values are written to device buffers for
// slr_apply.
template <typename ID, bool COPY = false>
__global__ __launch_bounds__(THREADS) void slr_fwd(const float* __restrict__ W, long long F,
                                                   const ID* __restrict__ ids,
                                                   const long long* __restrict__ offsets,
                                                   const float* __restrict__ vals, const float* __restrict__ labels,
                                                   const float* __restrict__ bias, int B, float* __restrict__ dz,
                                                   float* __restrict__ lrow, int* __restrict__ bad,
                                                   ID* __restrict__ ids_out = nullptr,
                                                   long long* __restrict__ off_out = nullptr,
                                                   float* __restrict__ vals_out = nullptr) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * (THREADS / 64) + (threadIdx.x >> 6);
  if (b >= B) return;
  const long long s = offsets[b], e = offsets[b + 1];
  if constexpr (COPY) {
    if (lane == 0) off_out[b] = s;
    if (lane == 1 && b == B - 1) off_out[B] = e;
  }
  float acc = 0.f;
  for (long long j = s + lane; j < e; j += 64) {
    const ID idr = ids[j];
    const float v = vals != nullptr ? vals[j] : 1.f;
    if constexpr (COPY) {
      ids_out[j] = idr;
      vals_out[j] = v;
    }
    const long long id = (long long)idr;
    if (id < 0 || id >= F) {   // TF raises on an out-of-range id; counted, skipped
      atomicAdd(bad, 1);
      continue;
    }
    acc += W[id] * v;
  }
  acc = wave_sum(acc);
  if (lane == 0) {
    const float z = acc + bias[0];
    const float y = labels[b];
    lrow[b] = xent(z, y);
    dz[b] = (1.f / (1.f + __expf(-z)) - y) / (float)B;
  }
}

// Scatter-SGD with the updates of a workgroup's rows combined in LDS first:
// Zipf-distributed ids put the same hot rows of W in most bags, and float
// atomics on one address serialize at the memory side (32 us per step at
// B = 500 / 20 k ids with one atomic per entry).  Each workgroup takes RPW
// consecutive batch rows; every entry's update goes into an LDS open-addressing
// table (64-bit key CAS, float add), then each occupied slot makes ONE global
// atomic.  An entry that finds no slot within MAXP probes goes straight to
// memory.  Workgroup 0 also sums dz and the row losses in a fixed order.
// RPW batch rows per workgroup, an LDS table of HS slots (RPW 32: 4096 slots =
// 32 KB keys + 16 KB values); dtfk_slr_set_rows_per_wg picks 8 / 16 / 32
constexpr int MAXP = 16;
constexpr unsigned long long EMPTY = ~0ull;

template <typename ID, int RPW = 32, int HSLOTS = 4096>
__global__ __launch_bounds__(THREADS) void slr_apply(float* __restrict__ W, long long F, const ID* __restrict__ ids,
                                                     const long long* __restrict__ offsets,
                                                     const float* __restrict__ vals, const float* __restrict__ dz,
                                                     const float* __restrict__ lrow, const float* __restrict__ lr_ptr,
                                                     float lr_val, float* __restrict__ bias, int B,
                                                     float* __restrict__ loss_out, void* gvar, int gkind) {
  __shared__ unsigned long long hkey[HSLOTS];
  __shared__ float hval[HSLOTS];
  __shared__ long long soff[RPW + 1];   // the workgroup's row offsets
  __shared__ float sgr[RPW];            // -lr * dz of its rows
  const float lr = lr_ptr != nullptr ? *lr_ptr : lr_val;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r0 = blockIdx.x * RPW;
  const int nr = min(RPW, B - r0);
  if ((int)threadIdx.x <= nr) soff[threadIdx.x] = offsets[r0 + threadIdx.x];
  if ((int)threadIdx.x < nr) sgr[threadIdx.x] = -lr * dz[r0 + threadIdx.x];
  for (int i = threadIdx.x; i < HSLOTS; i += THREADS) {
    hkey[i] = EMPTY;
    hval[i] = 0.f;
  }
  __syncthreads();
  // The rows' entries are one contiguous CSR range: the threads stride it flat,
  // U entries each with every id / value load in flight before the first use
  // (a wave-per-row loop put ~3 dependent memory round trips per row in series:
  // 15 us at B = 500 / 20 k ids), and find an entry's row by a binary search of
  // the LDS offsets.
  constexpr int U = 4;
  const long long s0 = soff[0], e0 = soff[nr];
  for (long long base = s0; base < e0; base += (long long)U * THREADS) {
    long long idv[U];
    float vv[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const long long j = base + threadIdx.x + (long long)k * THREADS;
      const bool in = j < e0;
      idv[k] = in ? (long long)ids[j] : -1;
      vv[k] = in ? (vals != nullptr ? vals[j] : 1.f) : 0.f;
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const long long j = base + threadIdx.x + (long long)k * THREADS;
      const long long id = idv[k];
      const float v = vv[k];
      if (j >= e0 || id < 0 || id >= F || v == 0.f) continue;   // padding (val 0) touches nothing
      int lo = 0, hi = nr;   // the row: largest r with soff[r] <= j (soff[nr] > j)
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (soff[mid] <= j) lo = mid;
        else hi = mid;
      }
      const float u = sgr[lo] * v;
      const unsigned long long key = (unsigned long long)id;
      unsigned h = (unsigned)(key * 0x9E3779B97F4A7C15ull >> 52) & (HSLOTS - 1);
      bool done = false;
      for (int p = 0; p < MAXP; ++p) {
        const unsigned long long cur = atomicCAS(&hkey[h], EMPTY, key);
        if (cur == EMPTY || cur == key) {
          atomicAdd(&hval[h], u);
          done = true;
          break;
        }
        h = (h + 1) & (HSLOTS - 1);
      }
      if (!done) atomicAdd(W + id, u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < HSLOTS; i += THREADS) {
    const unsigned long long k = hkey[i];
    if (k != EMPTY) atomicAdd(W + (long long)k, hval[i]);
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

// The packed Session feed (ids | offsets | values | labels) from mapped, coherent
// pinned host memory into device memory: one 16-byte load + store per thread.  A
// kernel on the step's own queue instead of an SDMA copy -- no copy-engine
// dispatch and no cross-engine wait in front of slr_fwd.
__global__ __launch_bounds__(256) void slr_stage(const uint4* __restrict__ src, uint4* __restrict__ dst, long long n16) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n16; i += (long long)gridDim.x * 256) dst[i] = src[i];
}

}  // namespace slr
}  // namespace dtfk

static int g_rpw = 32;

template <typename ID>
static void launch_apply(int B, hipStream_t stream, float* W, long long F, const ID* ids, const long long* offsets,
                         const float* vals, const float* dz, const float* lrow, const float* lr_ptr, float lr_val,
                         float* bias, float* loss_out, void* gvar, int gkind) {
  using namespace dtfk::slr;
#define DTFK_AP(R, H)                                                                                             \
  hipLaunchKernelGGL((slr_apply<ID, R, H>), dim3((B + R - 1) / R), dim3(THREADS), 0, stream, W, F, ids, offsets, \
                     vals, dz, lrow, lr_ptr, lr_val, bias, B, loss_out, gvar, gkind)
  if (g_rpw == 8) DTFK_AP(8, 1024);
  else if (g_rpw == 16) DTFK_AP(16, 2048);
  else DTFK_AP(32, 4096);
#undef DTFK_AP
}

extern "C" {

// batch rows per slr_apply workgroup (8, 16 or 32; else 32): more workgroups
// vs more cross-workgroup atomics on hot ids
void dtfk_slr_set_rows_per_wg(int rpw) { g_rpw = (rpw == 8 || rpw == 16) ? rpw : 32; }

// The step with its feed read in place from mapped pinned host memory (hids,
// hoffsets, hvals, hlabels: device views): slr_fwd<COPY> copies ids / offsets /
// values into ids_d / off_d / vals_d on the way, slr_apply reads those.
hipError_t dtfk_slr_step_direct(float* W, long long F, const void* hids, int ids32, const long long* hoffsets,
                                const float* hvals, const float* hlabels, void* ids_d, long long* off_d, float* vals_d,
                                float* bias, int B, float lr_val, float* dz, float* lrow, float* loss_out, int* bad,
                                void* gvar, int gkind, hipStream_t stream) {
  using namespace dtfk::slr;
  if (B < 1 || gkind < 0 || gkind > 4 || (gkind != 0 && gvar == nullptr) || hvals == nullptr) return hipErrorInvalidValue;
  const int grid = (B + THREADS / 64 - 1) / (THREADS / 64);
  if (ids32) {
    hipLaunchKernelGGL((slr_fwd<int, true>), dim3(grid), dim3(THREADS), 0, stream, W, F, static_cast<const int*>(hids),
                       hoffsets, hvals, hlabels, bias, B, dz, lrow, bad, static_cast<int*>(ids_d), off_d, vals_d);
    launch_apply<int>(B, stream, W, F, static_cast<const int*>(ids_d), off_d, vals_d, dz, lrow, nullptr, lr_val, bias,
                      loss_out, gvar, gkind);
  } else {
    hipLaunchKernelGGL((slr_fwd<long long, true>), dim3(grid), dim3(THREADS), 0, stream, W, F,
                       static_cast<const long long*>(hids), hoffsets, hvals, hlabels, bias, B, dz, lrow, bad,
                       static_cast<long long*>(ids_d), off_d, vals_d);
    launch_apply<long long>(B, stream, W, F, static_cast<const long long*>(ids_d), off_d, vals_d, dz, lrow, nullptr,
                            lr_val, bias, loss_out, gvar, gkind);
  }
  return hipGetLastError();
}

// bytes: a multiple of 16; src: the device view of mapped pinned host memory
hipError_t dtfk_slr_stage(const void* src, void* dst, long long bytes, hipStream_t stream) {
  if (bytes <= 0 || (bytes & 15)) return hipErrorInvalidValue;
  const long long n16 = bytes / 16;
  long long g = (n16 + 255) / 256;
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(dtfk::slr::slr_stage, dim3((unsigned)g), dim3(256), 0, stream, static_cast<const uint4*>(src),
                     static_cast<uint4*>(dst), n16);
  return hipGetLastError();
}

// gkind: 0 none, 1 f32, 2 i64, 3 i32, 4 f64 (the graph's global_step variable);
// ids32: ids are int32 (the packed Session feed when every id < 2^31), else int64
hipError_t dtfk_slr_step(float* W, long long F, const void* ids, int ids32, const long long* offsets,
                         const float* vals, const float* labels, float* bias, int B, const float* lr_ptr, float lr_val,
                         float* dz, float* lrow, float* loss_out, int* bad, void* gvar, int gkind, hipStream_t stream) {
  using namespace dtfk::slr;
  if (B < 1 || gkind < 0 || gkind > 4 || (gkind != 0 && gvar == nullptr)) return hipErrorInvalidValue;
  const int grid = (B + THREADS / 64 - 1) / (THREADS / 64);
  if (ids32) {
    auto id = static_cast<const int*>(ids);
    hipLaunchKernelGGL(slr_fwd<int>, dim3(grid), dim3(THREADS), 0, stream, W, F, id, offsets, vals, labels, bias, B,
                       dz, lrow, bad);
    launch_apply<int>(B, stream, W, F, id, offsets, vals, dz, lrow, lr_ptr, lr_val, bias, loss_out, gvar, gkind);
  } else {
    auto id = static_cast<const long long*>(ids);
    hipLaunchKernelGGL(slr_fwd<long long>, dim3(grid), dim3(THREADS), 0, stream, W, F, id, offsets, vals, labels,
                       bias, B, dz, lrow, bad);
    launch_apply<long long>(B, stream, W, F, id, offsets, vals, dz, lrow, lr_ptr, lr_val, bias, loss_out, gvar, gkind);
  }
  return hipGetLastError();
}

}  // extern "C"
