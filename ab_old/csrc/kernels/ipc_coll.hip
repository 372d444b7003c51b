// Reached by: parallel/world.py World GPU data plane (every collective on one node), compat N-worker MLP step; tests/test_ipc_coll_gpu.py, test_compat_ipc_gpu.py, test_sharded_ipc_gpu.py
// Collectives over IPC-mapped peer buffers: the node's data plane without RCCL.
//
// Every rank exports ONE uncached (fine-grained) device buffer
// (csrc/comm/ipc_peer.cpp) and maps every peer's; a collective is ONE kernel
// per rank that
//   1. copies this rank's contribution into its own slot (plain stores to
//      uncached memory: a store's completion is its visibility),
//   2. counts its workgroups in (each storing wave drains with
//      `s_waitcnt vmcnt(0)`, then the workgroup's barrier, then one agent-scope
//      add); the LAST workgroup publishes the collective's sequence number in
//      the rank's control block (a system-scope store peers poll),
//   3. waits until every peer published the same sequence number (lane r of
//      every workgroup polls rank r: the W remote polls overlap), and
//   4. reads the peers' slots with system-scope loads (never served from a
//      cache line of this GPU) and writes its output.
// All-reduce sums in RANK ORDER on every rank, so the replicas stay
// bit-identical.  Above a size threshold the all-reduce is two-shot: each rank
// reduces 1/W of the elements from all peers, publishes the reduced chunk
// (second phase), and gathers the other ranks' chunks -- 2(W-1)/W of the
// payload read per rank instead of (W-1)x.
//
// Slots are double-buffered by the parity of the sequence number, which lives
// in DEVICE memory (read at kernel start, bumped by the phase-1 publisher), so
// the kernels replay correctly from captured hipGraphs.  Reuse is safe without
// acknowledgements: rank A rewrites parity p at collective s + 2 only after its
// collective s + 1 saw every peer publish s + 1, and a peer publishes s + 1 only
// in its kernel for s + 1, which its stream starts after its kernel for s --
// the one that read A's parity-p slot -- has completed.  This requires each
// rank to issue its IPC collectives in one stream order (the host driver
// chains streams with events).
//
// Every wait is bounded (s_memrealtime); a timeout raises the device error
// word (later collectives fail fast) and a pinned host word the host checks.
#include "common.h"

#include "comm/ipc_coll.h"

namespace dtfk {
namespace ipcc {

typedef unsigned long long u64;

__device__ __forceinline__ char* slot_in(const Coll& c, int r, u64 s) {
  return static_cast<char*>(c.base[r]) + CTRL + (long long)(s & 1) * 2 * c.cap;
}
__device__ __forceinline__ char* slot_red(const Coll& c, int r, u64 s) { return slot_in(c, r, s) + c.cap; }
__device__ __forceinline__ u64* ctl(const Coll& c, int r, long long off) {
  return reinterpret_cast<u64*>(static_cast<char*>(c.base[r]) + off);
}

// this collective's sequence number: the previous one's + 1 (kernel start is an
// acquire: the previous kernel's bump is visible)
__device__ __forceinline__ u64 seq_of(const Coll& c) {
  return __hip_atomic_load(c.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
}

__device__ __forceinline__ void fail(const Coll& c, int code) {
  atomicOr(c.err, code);
  __hip_atomic_store(c.err_host, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Count this workgroup in for phase `ph` (0: input published, 1: reduced chunk
// published) after every wave's stores drained; the last arriver resets the
// counter, bumps the device sequence word (phase 0) and publishes s.
__device__ void arrive(const Coll& c, int ph, u64 s) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(c.ctr + ph, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {
      __hip_atomic_store(c.ctr + ph, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (ph == 0) __hip_atomic_store(c.seq, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctl(c, c.rank, ph ? RED : PUB), s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// Every peer's phase-`ph` word reached s (bounded).  False: a wait timed out
// here or a previous collective failed (then nothing more is read or written).
__device__ bool wait_peers(const Coll& c, int ph, u64 s) {
  __shared__ int ok;
  if (threadIdx.x == 0) ok = __hip_atomic_load(c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
  __syncthreads();
  const int r = threadIdx.x;
  if (ok && r < c.W && r != c.rank) {
    const u64* f = ctl(c, r, ph ? RED : PUB);
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < s) {
      __builtin_amdgcn_s_sleep(1);
      if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > c.timeout ||
          __hip_atomic_load(c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
        fail(c, 1);
        ok = 0;
        break;
      }
    }
  }
  asm volatile("" ::: "memory");   // no peer-slot load above the flag match
  __syncthreads();
  return ok != 0;
}

// ---------------------------------------------------------------- peer access
// Peer slots are read 16 bytes per lane with system-coherent (sc0 sc1) buffer
// loads -- never served from a cache line of this GPU -- several in flight per
// lane; Coll::wide == 0 (DTF_IPC_NARROW=1, A/B probe) reads 8-byte relaxed
// system-scope atomics instead.
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
constexpr int SYS = 1 | 16;   // sc0 | sc1
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)(bytes < 0x7fffffffLL ? bytes : 0x7fffffffLL),
                                           0x00020000);
}
__device__ __forceinline__ u32x4 ld_peer16(const Coll& c, const char* base, long long off) {
  if (c.wide) return __builtin_amdgcn_raw_buffer_load_b128(rsrc(base, 2 * c.cap), (int)off, 0, SYS);
  const u64 a = ld_sys_u64(base + off), b = ld_sys_u64(base + off + 8);
  return u32x4{(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
}

// ---------------------------------------------------------------- element types
// 16-byte packets of N elements; reductions in A (fp32 for bf16 storage).
template <typename T> struct Ty;
template <> struct Ty<float> {
  typedef float A; static constexpr int N = 4;
  __device__ static void unpack(u32x4 u, A* v) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = __uint_as_float(u[i]);
  }
  __device__ static u32x4 pack(const A* v) {
    return u32x4{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
  }
  __device__ static A ld1(const void* p) { return ld_sys_f32(p); }
  __device__ static A get(float v) { return v; }
  __device__ static float put(A v) { return v; }
};
struct bf16_t { uint16_t b; };
template <> struct Ty<bf16_t> {
  typedef float A; static constexpr int N = 8;
  __device__ static void unpack(u32x4 u, A* v) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = bf2f((uint16_t)(u[i] & 0xFFFFu));
      v[2 * i + 1] = bf2f((uint16_t)(u[i] >> 16));
    }
  }
  __device__ static u32x4 pack(const A* v) {
    return u32x4{pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7])};
  }
  __device__ static A ld1(const void* p) { return bf2f(ld_sys_u16(p)); }
  __device__ static A get(bf16_t v) { return bf2f(v.b); }
  __device__ static bf16_t put(A v) { return bf16_t{f2bf(v)}; }
};
template <> struct Ty<double> {
  typedef double A; static constexpr int N = 2;
  __device__ static void unpack(u32x4 u, A* v) {
    v[0] = __longlong_as_double((long long)((u64)u[0] | ((u64)u[1] << 32)));
    v[1] = __longlong_as_double((long long)((u64)u[2] | ((u64)u[3] << 32)));
  }
  __device__ static u32x4 pack(const A* v) {
    const u64 a = (u64)__double_as_longlong(v[0]), b = (u64)__double_as_longlong(v[1]);
    return u32x4{(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
  }
  __device__ static A ld1(const void* p) { return __longlong_as_double((long long)ld_sys_u64(p)); }
  __device__ static A get(double v) { return v; }
  __device__ static double put(A v) { return v; }
};
template <> struct Ty<int> {
  typedef int A; static constexpr int N = 4;
  __device__ static void unpack(u32x4 u, A* v) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (int)u[i];
  }
  __device__ static u32x4 pack(const A* v) { return u32x4{(uint32_t)v[0], (uint32_t)v[1], (uint32_t)v[2], (uint32_t)v[3]}; }
  __device__ static A ld1(const void* p) { return (int)ld_sys_u32(p); }
  __device__ static A get(int v) { return v; }
  __device__ static int put(A v) { return v; }
};
template <> struct Ty<long long> {
  typedef long long A; static constexpr int N = 2;
  __device__ static void unpack(u32x4 u, A* v) {
    v[0] = (long long)((u64)u[0] | ((u64)u[1] << 32));
    v[1] = (long long)((u64)u[2] | ((u64)u[3] << 32));
  }
  __device__ static u32x4 pack(const A* v) {
    return u32x4{(uint32_t)v[0], (uint32_t)((u64)v[0] >> 32), (uint32_t)v[1], (uint32_t)((u64)v[1] >> 32)};
  }
  __device__ static A ld1(const void* p) { return (long long)ld_sys_u64(p); }
  __device__ static A get(long long v) { return v; }
  __device__ static long long put(A v) { return v; }
};

template <int OP, typename A>
__device__ __forceinline__ A combine(A a, A b) {
  if (OP == 0) return a + b;
  if (OP == 1) return a > b ? a : b;
  return a < b ? a : b;
}

// Copy nbytes (a multiple of 4; pointers 4-byte aligned) grid-stride: 16-byte
// packets where dst, src and nbytes allow, else 8-, else 4-byte words.
// PEER: src is a peer's slot (system-coherent loads, four in flight per lane).
template <bool PEER>
__device__ void copy_bytes(const Coll& c, void* dst, const void* src, long long nbytes, long long tid, long long nth) {
  const uintptr_t al = reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src) | (uintptr_t)nbytes;
  char* d = static_cast<char*>(dst);
  const char* q = static_cast<const char*>(src);
  if ((al & 15) == 0) {
    const long long np = nbytes >> 4;
    long long j = tid;
    if (PEER) {
      for (; j + 3 * nth < np; j += 4 * nth) {
        const u32x4 a = ld_peer16(c, q, 16 * j), b = ld_peer16(c, q, 16 * (j + nth)),
                    e = ld_peer16(c, q, 16 * (j + 2 * nth)), f = ld_peer16(c, q, 16 * (j + 3 * nth));
        reinterpret_cast<u32x4*>(d)[j] = a;
        reinterpret_cast<u32x4*>(d)[j + nth] = b;
        reinterpret_cast<u32x4*>(d)[j + 2 * nth] = e;
        reinterpret_cast<u32x4*>(d)[j + 3 * nth] = f;
      }
      for (; j < np; j += nth) reinterpret_cast<u32x4*>(d)[j] = ld_peer16(c, q, 16 * j);
    } else {
      for (; j < np; j += nth) reinterpret_cast<u32x4*>(d)[j] = reinterpret_cast<const u32x4*>(q)[j];
    }
  } else if ((al & 7) == 0) {
    const long long np = nbytes >> 3;
    for (long long j = tid; j < np; j += nth)
      reinterpret_cast<u64*>(d)[j] = PEER ? ld_sys_u64(q + 8 * j) : reinterpret_cast<const u64*>(q)[j];
  } else {
    const long long np = nbytes >> 2;
    for (long long j = tid; j < np; j += nth)
      reinterpret_cast<uint32_t*>(d)[j] = PEER ? ld_sys_u32(q + 4 * j) : reinterpret_cast<const uint32_t*>(q)[j];
  }
}

// The < N elements past the last whole packet, by one thread (every rank
// computes them from all peers in rank order, also in two-shot mode).
template <typename T, int OP>
__device__ void tail_reduce(const T* in, T* out, long long n, const Coll& c, u64 s, float scale) {
  typedef Ty<T> Y;
  for (long long i = n / Y::N * Y::N; i < n; ++i) {
    typename Y::A acc = 0;
    for (int r = 0; r < c.W; ++r) {
      const typename Y::A v = r == c.rank ? Y::get(in[i]) : Y::ld1(reinterpret_cast<const T*>(slot_in(c, r, s)) + i);
      acc = r == 0 ? v : combine<OP>(acc, v);
    }
    if (OP == 0 && scale != 1.f) acc = (typename Y::A)(acc * scale);
    out[i] = Y::put(acc);
  }
}

// ---------------------------------------------------------------- all-reduce
// in / out 16-byte aligned (elements past the last 16-byte packet go through
// tail_reduce).
template <typename T, int OP>
__global__ __launch_bounds__(256) void allreduce_k(const T* __restrict__ in, T* __restrict__ out, long long n, Coll c,
                                                   float scale, int two_shot) {
  typedef Ty<T> Y;
  typedef typename Y::A A;
  constexpr int N = Y::N;
  const u64 s = seq_of(c);
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x, nth = (long long)gridDim.x * blockDim.x;
  const long long np = n / N;
  const u32x4* inp = reinterpret_cast<const u32x4*>(in);
  u32x4* outp = reinterpret_cast<u32x4*>(out);
  u32x4* mine = reinterpret_cast<u32x4*>(slot_in(c, c.rank, s));
  for (long long j = tid; j < np; j += nth) mine[j] = inp[j];
  if (tid == 0)
    for (long long i = np * N; i < n; ++i) reinterpret_cast<T*>(mine)[i] = in[i];
  arrive(c, 0, s);
  if (!wait_peers(c, 0, s)) return;
  if (tid == 0) tail_reduce<T, OP>(in, out, n, c, s, scale);
  const long long j0 = two_shot ? np * c.rank / c.W : 0, j1 = two_shot ? np * (c.rank + 1) / c.W : np;
  u32x4* red = reinterpret_cast<u32x4*>(slot_red(c, c.rank, s));
  for (long long j = j0 + tid; j < j1; j += nth) {
    u32x4 u[WMAX];
#pragma unroll
    for (int r = 0; r < WMAX; ++r)     // every peer's packet in flight before the combine
      if (r < c.W) u[r] = r == c.rank ? inp[j] : ld_peer16(c, slot_in(c, r, s), 16 * j);
    A acc[N], v[N];
    Y::unpack(u[0], acc);
#pragma unroll
    for (int r = 1; r < WMAX; ++r) {
      if (r < c.W) {
        Y::unpack(u[r], v);
#pragma unroll
        for (int i = 0; i < N; ++i) acc[i] = combine<OP>(acc[i], v[i]);
      }
    }
    if (OP == 0 && scale != 1.f) {
#pragma unroll
      for (int i = 0; i < N; ++i) acc[i] = (A)(acc[i] * scale);
    }
    const u32x4 pk = Y::pack(acc);
    outp[j] = pk;
    if (two_shot) red[j] = pk;
  }
  if (!two_shot) return;
  arrive(c, 1, s);
  if (!wait_peers(c, 1, s)) return;
  for (int r = 0; r < c.W; ++r) {
    if (r == c.rank) continue;
    const long long a0 = np * r / c.W, a1 = np * (r + 1) / c.W;
    copy_bytes<true>(c, outp + a0, slot_red(c, r, s) + 16 * a0, (a1 - a0) * 16, tid, nth);
  }
}

// ---------------------------------------------------------------- all-reduce mean + SGD
// grad: this rank's flat fp32 gradient (n values, 16-byte aligned); every rank
// sums the W gradients in rank order, p -= lr * scale * sum in place, and bumps
// global_step once.
__device__ __forceinline__ void sgd_apply(const SgdArgs& a, long long i, float step, float g) {
  int t = 0;
  while (t < a.np - 1 && i >= a.end[t]) ++t;
  const long long st = t == 0 ? 0 : a.end[t - 1];
  float* p = a.p[t] + (i - st);
  *p = *p - step * g;
}
__global__ __launch_bounds__(256) void reduce_sgd_k(const float* __restrict__ grad, long long n, Coll c, SgdArgs a) {
  const u64 s = seq_of(c);
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x, nth = (long long)gridDim.x * blockDim.x;
  const long long np = n / 4;
  const u32x4* gp = reinterpret_cast<const u32x4*>(grad);
  u32x4* mine = reinterpret_cast<u32x4*>(slot_in(c, c.rank, s));
  for (long long j = tid; j < np; j += nth) mine[j] = gp[j];
  if (tid == 0)
    for (long long i = 4 * np; i < n; ++i) reinterpret_cast<float*>(mine)[i] = grad[i];
  arrive(c, 0, s);
  if (!wait_peers(c, 0, s)) return;
  const float step = (a.lr_ptr != nullptr ? *a.lr_ptr : a.lr_val) * a.scale;
  for (long long j = tid; j < np; j += nth) {
    u32x4 u[WMAX];
#pragma unroll
    for (int r = 0; r < WMAX; ++r)
      if (r < c.W) u[r] = r == c.rank ? gp[j] : ld_peer16(c, slot_in(c, r, s), 16 * j);
    float g[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < WMAX; ++r) {
      if (r < c.W) {
#pragma unroll
        for (int h = 0; h < 4; ++h) g[h] += __uint_as_float(u[r][h]);
      }
    }
#pragma unroll
    for (int h = 0; h < 4; ++h) sgd_apply(a, 4 * j + h, step, g[h]);
  }
  if (tid == 0) {
    for (long long i = 4 * np; i < n; ++i) {
      float g = 0.f;
      for (int r = 0; r < c.W; ++r) g += r == c.rank ? grad[i] : ld_sys_f32(reinterpret_cast<const float*>(slot_in(c, r, s)) + i);
      sgd_apply(a, i, step, g);
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && a.gstep != nullptr) {
    float now;
    switch (a.gkind) {
      case 0: now = (*static_cast<float*>(a.gstep) += 1.f); break;
      case 1: now = (float)(*static_cast<long long*>(a.gstep) += 1); break;
      case 2: now = (float)(*static_cast<int*>(a.gstep) += 1); break;
      default: now = (float)(*static_cast<double*>(a.gstep) += 1.0); break;
    }
    if (a.metrics != nullptr) a.metrics[2] = now;
    if (a.host_metrics != nullptr) {
      __hip_atomic_store(a.host_metrics + 2, now, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
}

// ---------------------------------------------------------------- broadcast / all-gather
__global__ __launch_bounds__(256) void broadcast_k(const void* in, void* out, long long nbytes, int src, Coll c) {
  const u64 s = seq_of(c);
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x, nth = (long long)gridDim.x * blockDim.x;
  if (c.rank == src) {
    copy_bytes<false>(c, slot_in(c, c.rank, s), in, nbytes, tid, nth);
    if (out != in) copy_bytes<false>(c, out, in, nbytes, tid, nth);
  }
  arrive(c, 0, s);
  if (!wait_peers(c, 0, s)) return;
  if (c.rank != src) copy_bytes<true>(c, out, slot_in(c, src, s), nbytes, tid, nth);
}

// out + r * stride receives rank r's nbytes (stride = the whole per-rank size
// when the host chunks a large gather)
__global__ __launch_bounds__(256) void allgather_k(const void* in, void* out, long long nbytes, long long stride,
                                                   Coll c) {
  const u64 s = seq_of(c);
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x, nth = (long long)gridDim.x * blockDim.x;
  copy_bytes<false>(c, slot_in(c, c.rank, s), in, nbytes, tid, nth);
  copy_bytes<false>(c, static_cast<char*>(out) + c.rank * stride, in, nbytes, tid, nth);
  arrive(c, 0, s);
  if (!wait_peers(c, 0, s)) return;
  for (int r = 0; r < c.W; ++r)
    if (r != c.rank) copy_bytes<true>(c, static_cast<char*>(out) + r * stride, slot_in(c, r, s), nbytes, tid, nth);
}

// ---------------------------------------------------------------- all-to-all
// Each rank publishes its whole send buffer plus the table of where each
// destination's rows start; a receiver copies its rows out of every peer's slot.
__global__ __launch_bounds__(256) void alltoall_k(const char* in, char* out, A2A a, Coll c) {
  __shared__ long long src_off[WMAX];
  __shared__ int bad[WMAX];
  const u64 s = seq_of(c);
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x, nth = (long long)gridDim.x * blockDim.x;
  const int par = (int)(s & 1);
  if (!a.overflow) copy_bytes<false>(c, slot_in(c, c.rank, s), in, a.send_total, tid, nth);
  if (blockIdx.x == 0 && threadIdx.x < WMAX) {
    ctl(c, c.rank, OFFS)[par * WMAX + threadIdx.x] = (u64)a.send_off[threadIdx.x];
    if (threadIdx.x == 0) ctl(c, c.rank, STAT)[par] = a.overflow ? 1ull : 0ull;
  }
  arrive(c, 0, s);
  if (!wait_peers(c, 0, s)) return;
  if (threadIdx.x < c.W) {
    const int r = threadIdx.x;
    src_off[r] = r == c.rank ? a.send_off[r] : (long long)ld_sys_u64(ctl(c, r, OFFS) + par * WMAX + c.rank);
    bad[r] = r == c.rank ? a.overflow : (int)ld_sys_u64(ctl(c, r, STAT) + par);
  }
  __syncthreads();
  for (int r = 0; r < c.W; ++r) {
    if (bad[r]) {
      if (tid == 0) fail(c, 2);
      continue;
    }
    if (a.recv_bytes[r] == 0) continue;
    if (r == c.rank)
      copy_bytes<false>(c, out + a.recv_off[r], in + src_off[r], a.recv_bytes[r], tid, nth);
    else
      copy_bytes<true>(c, out + a.recv_off[r], slot_in(c, r, s) + src_off[r], a.recv_bytes[r], tid, nth);
  }
}

}  // namespace ipcc
}  // namespace dtfk

// ---------------------------------------------------------------- launchers
using namespace dtfk::ipcc;

extern "C" hipError_t dtfk_ipcc_allreduce(const void* in, void* out, long long n, int dtype, int op, float scale,
                                          int two_shot, Coll c, int grid, hipStream_t s) {
  if (c.W < 1 || c.W > WMAX || grid < 1) return hipErrorInvalidValue;
#define DTFK_AR(T)                                                                                             \
  switch (op) {                                                                                                \
    case 0: hipLaunchKernelGGL((allreduce_k<T, 0>), dim3(grid), dim3(256), 0, s, (const T*)in, (T*)out, n, c, \
                               scale, two_shot); break;                                                        \
    case 1: hipLaunchKernelGGL((allreduce_k<T, 1>), dim3(grid), dim3(256), 0, s, (const T*)in, (T*)out, n, c, \
                               scale, two_shot); break;                                                        \
    default: hipLaunchKernelGGL((allreduce_k<T, 2>), dim3(grid), dim3(256), 0, s, (const T*)in, (T*)out, n, c, \
                                scale, two_shot); break;                                                       \
  }
  switch (dtype) {
    case 0: DTFK_AR(float); break;
    case 1: DTFK_AR(bf16_t); break;
    case 2: DTFK_AR(double); break;
    case 3: DTFK_AR(int); break;
    case 4: DTFK_AR(long long); break;
    default: return hipErrorInvalidValue;
  }
#undef DTFK_AR
  return hipGetLastError();
}

extern "C" hipError_t dtfk_ipcc_reduce_sgd(const float* grad, long long n, SgdArgs a, Coll c, int grid,
                                           hipStream_t s) {
  if (c.W < 1 || c.W > WMAX || grid < 1 || a.np < 1 || a.np > 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(reduce_sgd_k, dim3(grid), dim3(256), 0, s, grad, n, c, a);
  return hipGetLastError();
}

extern "C" hipError_t dtfk_ipcc_broadcast(const void* in, void* out, long long nbytes, int src, Coll c, int grid,
                                          hipStream_t s) {
  if (c.W < 1 || c.W > WMAX || grid < 1 || (nbytes & 3) || src < 0 || src >= c.W) return hipErrorInvalidValue;
  hipLaunchKernelGGL(broadcast_k, dim3(grid), dim3(256), 0, s, in, out, nbytes, src, c);
  return hipGetLastError();
}

extern "C" hipError_t dtfk_ipcc_allgather(const void* in, void* out, long long nbytes, long long stride, Coll c,
                                          int grid, hipStream_t s) {
  if (c.W < 1 || c.W > WMAX || grid < 1 || (nbytes & 3) || (stride & 3)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(allgather_k, dim3(grid), dim3(256), 0, s, in, out, nbytes, stride, c);
  return hipGetLastError();
}

extern "C" hipError_t dtfk_ipcc_alltoall(const void* in, void* out, A2A a, Coll c, int grid, hipStream_t s) {
  if (c.W < 1 || c.W > WMAX || grid < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(alltoall_k, dim3(grid), dim3(256), 0, s, (const char*)in, (char*)out, a, c);
  return hipGetLastError();
}
