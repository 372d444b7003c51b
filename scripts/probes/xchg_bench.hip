// Microbenchmark: the persistent MLP kernel's per-step all-gather among 7
// workgroups (blockIdx 8j -> one XCD), nothing else running.
//   mode 0: 8-byte {tag,value} granules, plain stores (L2-local), sc1 sweep
//   mode 1: granules, sc1 (write-through) stores, sc1 sweep
//   mode 2: dense fp32 payload (plain stores) + vmcnt(0) + per-wave flag; flag poll then one sc1 payload read
//   mode 3: as 2 with sc1 payload/flag stores
//   mode 4: granules, plain stores, nt loads
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

constexpr int NWG = 7, NBT = 7, NCLS = 10;
constexpr int SLOT = NWG * NBT * NCLS * 16;

__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__global__ __launch_bounds__(512, 1) void xchg(unsigned long long* gran, float* dense, unsigned* flags, int mode,
                                               int nsteps, float* sink, int* err) {
  if (blockIdx.x % 8 != 0 || blockIdx.x / 8 >= NWG) return;
  const int j = blockIdx.x / 8;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, g = lane >> 4;
  float acc = 0.f;
  for (int st = 0; st < nsteps; ++st) {
    const unsigned tag = (unsigned)st + 1u;
    const int par = st & 1;
    if (w < NBT) {
      float pl[4] = {1.f * st, 2.f, 3.f, 4.f};
      if (mode == 0 || mode == 1 || mode == 4) {
        gu64* slot = (gu64*)gran + par * SLOT;
        gu64* mine = slot + (j * NBT + w) * NCLS * 16;
        for (int i = 0; i < 4; ++i) {
          const int c = 4 * g + i;
          const unsigned long long v = ((unsigned long long)tag << 32) | __float_as_uint(pl[i]);
          if (c < NCLS) {
            if (mode == 1) __hip_atomic_store(mine + c * 16 + r, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else __hip_atomic_store(mine + c * 16 + r, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
        }
        const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
        for (;;) {
          bool ok = true;
          float s = 0.f;
          for (int jj = 0; jj < NWG; ++jj) {
            const gu64* src = slot + (jj * NBT + w) * NCLS * 16;
            for (int i = 0; i < 4; ++i) {
              const int c = 4 * g + i;
              if (c < NCLS && jj != j) {
                unsigned long long v;
                if (mode == 4) v = __builtin_nontemporal_load((const unsigned long long*)(src + c * 16 + r));
                else v = __hip_atomic_load(src + c * 16 + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                s += __uint_as_float((unsigned)v);
                ok = ok && (unsigned)(v >> 32) == tag;
              }
            }
          }
          if (__all(ok)) { acc += s; break; }
          if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > 200000000LL) { if (lane == 0) atomicOr(err, 1); break; }
          __builtin_amdgcn_s_sleep(1);
        }
      } else {
        // dense payload: producer (j, w) writes 160 floats at dense[par][j][w][160]
        float* mine = dense + ((par * NWG + j) * NBT + w) * 160;
        if (lane < 40) {
          const float4 v = make_float4(pl[0], pl[1], pl[2], pl[3]);
          if (mode == 3) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                                               __builtin_amdgcn_make_buffer_rsrc(mine, 0, 640, 0x00020000), lane * 16, 0, 16);
          else reinterpret_cast<float4*>(mine)[lane] = v;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        gu32* fl = (gu32*)flags + par * 64;
        if (lane == 0) {
          if (mode == 3) __hip_atomic_store(fl + j * NBT + w, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          else __hip_atomic_store(fl + j * NBT + w, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
        for (;;) {
          bool ok = true;
          if (lane < NWG) ok = __hip_atomic_load(fl + lane * NBT + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == tag;
          if (__all(ok)) break;
          if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > 200000000LL) { if (lane == 0) atomicOr(err, 1); break; }
          __builtin_amdgcn_s_sleep(1);
        }
        // 7 producers x 160 floats = 280 float4; lane reads up to 5
        float s = 0.f;
        for (int q = lane; q < NWG * 40; q += 64) {
          const int jj = q / 40, e = q % 40;
          const float* src = dense + ((par * NWG + jj) * NBT + w) * 160;
          const auto v = __builtin_amdgcn_raw_buffer_load_b128(__builtin_amdgcn_make_buffer_rsrc((void*)src, 0, 640, 0x00020000),
                                                              e * 16, 0, 16);
          s += __uint_as_float(v[0]) + __uint_as_float(v[3]);
        }
        acc += s;
      }
    }
    lds_barrier();
  }
  if (acc == 12345.f) sink[0] = acc;
}

int main() {
  unsigned long long* gran;
  float* dense;
  unsigned* flags;
  float* sink;
  int* err;
  (void)hipMalloc(&gran, 2 * SLOT * 8);
  (void)hipMalloc(&dense, 2 * NWG * NBT * 160 * 4);
  (void)hipMalloc(&flags, 2 * 64 * 4);
  (void)hipMalloc(&sink, 4);
  (void)hipMalloc(&err, 4);
  const char* names[] = {"granules plain-store sc1-load", "granules sc1-store sc1-load", "dense+flag plain",
                         "dense+flag sc1", "granules plain-store nt-load"};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int mode = 0; mode < 5; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipMemset(gran, 0, 2 * SLOT * 8);
      (void)hipMemset(flags, 0, 2 * 64 * 4);
      (void)hipMemset(err, 0, 4);
      const int n = 2000;
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(xchg, dim3(64), dim3(512), 0, 0, gran, dense, flags, mode, n, sink, err);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      int he;
      (void)hipMemcpy(&he, err, 4, hipMemcpyDeviceToHost);
      if (rep) printf("mode %d %-32s %.3f us/step err=%d\n", mode, names[mode], 1000.f * ms / n, he);
    }
  }
  return 0;
}
