// Persistent, weight-stationary training kernel for the reference's
// 784-100-10 MLP (example.py:84-118: x*W1+b1 -> sigmoid -> *W2+b2 -> softmax
// cross-entropy -> GradientDescentOptimizer) -- many SGD steps per launch.
//
// Why: at batch 100 a step is ~32 MFLOP.  The 3-launch path (mlp_step.hip)
// spends ~4.5 of its 13.2 us per step in kernel boundaries and fill/drain.
// Here one launch runs a whole input chunk (e.g. 50 steps):
//
//  * 7 compute workgroups (512 threads), workgroup j OWNS hidden units
//    [16j, 16j+16): its W1 column block (784x16 fp32 master, in VGPRs, in the
//    MFMA accumulator layout of dW1 so the update needs no data movement),
//    its W2 rows and b1 entries (LDS) and a replica of b2.  Weights never
//    leave the CU inside a launch.
//  * per step ONE inter-workgroup edge: every workgroup publishes its partial
//    logits (16 hidden units' contribution, 100x10 fp32) as 8-byte
//    {tag, value} granules with agent-scope (sc1) stores and reads the other
//    six workgroups' granules with sc1 loads until every tag matches (the data
//    is the flag: no fence, no counter).  Every workgroup then computes the
//    same softmax / dz3 in the same order (bit-identical replicas of b2) and
//    its own block's backward and SGD update locally.
//  * x enters MFMA as fp16 "1024 + u" built by ONE v_perm_b32 per two pixels
//    (bytes spliced under the constant exponent byte 0x64); the 1024 offset is
//    removed exactly with the column sums of the fp16 operand it multiplied:
//      sum_f (1024+u_f) w_f = sum_f u_f w_f + 1024 sum_f w_f .
//    The 1/255 pixel scale and the 1/B loss mean are folded into the update.
//  * the forward needs x with features contiguous (K = feature), the weight
//    gradient needs x with batch contiguous (K = batch): the second layout is a
//    feature-major copy xT[800][128] built by the copier workgroups.
//  * the remaining workgroups are COPIERS: while the 7 compute workgroups run
//    chunk c, they pull chunk c+1 from pinned host memory over PCIe into the
//    other device stage and write its transposed copy -- the input stream
//    overlaps compute with no second stream and no cross-queue event.
//
// Placement: compute workgroup j = blockIdx 8j (blocks b and b+8 share an XCD
// under the observed round-robin dispatch -- speed only, never correctness).
//
// Layouts (l = lane, r = l & 15, g = l >> 4; 16x16x32 MFMA maps in common.h):
//  fwd   z^T[hidden][batch] = W1^T . x^T : A = W1 block (lane: hidden r),
//        B = x rows (lane: batch r); k-step s covers features
//        {32s+4g+e} U {32s+16+4g+e}, e<4 -- exactly the features the dW1
//        accumulator tiles 2s, 2s+1 of the same lane hold.
//  head  logits^T partial = W2^T . a2^T, dz3, da2^T = W2 . dz3^T: all in
//        registers (lane: batch r, in-lane 4 hidden units / classes).
//  bwd   dW1 = x^T . dz2 : A = xT rows (lane: feature), B = dz2^T via LDS.
#include "common.h"

namespace dtfk {
namespace mlpp {

typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

constexpr int DIN = 784;
constexpr int NF = 800;        // features padded to 25 k-steps of 32 (xT rows)
constexpr int XR = 832;        // stage row: 13 blocks of 64 features, k-step-pair interleaved (see copier)
constexpr int BPT = 128;       // xT row stride (batch padded)
constexpr int HID = 100, NCLS = 10;
constexpr int NWG = 7;         // hidden blocks of 16 = compute workgroups
constexpr int NBT = 7;         // batch tiles of 16 (B <= 112)
constexpr int NKS = 25;        // k-steps of 32 features
constexpr int NU = 4;          // k-step slots per wave: s = w + 8u for u < 3; wave 7 also owns s = 24
constexpr int NP = 13;         // 16-byte x fetches per forward lane (k-step pairs)
constexpr int OFF_W2 = 78400, OFF_B1 = 79400, OFF_B2 = 79500;
constexpr int THREADS = 512;
constexpr int XCD_STRIDE = 8;  // compute workgroup j runs as blockIdx 8j
constexpr int GRID = 64;       // 7 compute + 57 copier workgroups
constexpr int PAYLOAD = 48 * 4;                        // floats per (producer, tile): lanes g<3 x float4
// exchange buffer (u64 units): [16 header granules][2][64] u32 flags = 64 u64 [2][7][7][PAYLOAD] floats
constexpr int XCH_HDR = 16, XCH_FLAGS = 64, XCH_DENSE = NWG * NBT * PAYLOAD;   // dense: u64 units per parity
constexpr int GRAN_TOTAL = XCH_HDR + XCH_FLAGS + 2 * XCH_DENSE;

struct Args {
  const uint8_t* xs;        // this chunk: stage records of `rec` bytes (B x 832 permuted pixels, B labels)
  const uint8_t* xts;       // this chunk: [nsteps][800][128] feature-major pixels
  long long rec;            // stage record bytes (B*833 rounded up to 16)
  long long rec_h;          // host record bytes (B*785 rounded up to 16)
  int B, nsteps;
  float* params;            // flat fp32 master, TF variable order (read at start, written at end)
  const float* lr;
  float* metrics;
  int ring;
  int act, naive;
  long long* gstep;
  unsigned long long* seq;  // exchange sequence number (monotonic across launches)
  unsigned long long* gran; // placement header granules [16]
  float* dense;             // [2][7 producers][7 tiles][PAYLOAD] partial logits
  unsigned* flags;          // [2][64] (producer, tile) flags = step tag
  int* err;
  long long timeout;        // s_memrealtime ticks (100 MHz)
  // copier: next chunk
  const uint8_t* host_next; // device-visible pointer into pinned host memory
  int next_steps;
  uint8_t* xs_next;
  uint8_t* xts_next;
  long long* ts;            // optional phase stamps (s_memrealtime), see TSP
  // N GPUs: IPC-mapped uncached exchange buffers of every rank (W = 1: none)
  void* const* peer_base;
  int W, rank;
  long long* step_ts;       // optional: s_memrealtime at the start of every global step (ring)
  int ts_ring;
};

// IPC exchange buffer of one rank: [flags: block j at byte 64j][2 parities][7 blocks][slot]
// slot: dW1 block as [tile 49][g 4][r 16] x 4 bf16, then small grads
// (dW2 [g][r] x 4 bf16 = 512 B, db1/db2 bf16 at +512 (lanes 0..25))
constexpr int IPC_FLAGS = 4096;
constexpr int IPC_SMALL = 49 * 4 * 16 * 8;
constexpr int IPC_SLOT = IPC_SMALL + 576;
constexpr int IPC_BYTES = IPC_FLAGS + 2 * NWG * IPC_SLOT;
__device__ __forceinline__ int par_of(int st) { return st & 1; }
__device__ __forceinline__ float bfround(float x) { return bf2f(f2bf(x)); }

// debug stamps: compute workgroup j, wave w, lane 0 -> ts[(step*8 + j)*16 + phase]
__device__ __forceinline__ void lds_barrier() {   // orders LDS only: no vmcnt(0) on in-flight loads
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

#define TSP(ph)                                                                          \
  if (a.ts != nullptr && lane == 0 && st < 64)                                           \
    a.ts[((long long)st * 8 + j) * 16 + (ph)] = (long long)__builtin_amdgcn_s_memrealtime();

// fp16 (1024 + u) pairs from four pixel bytes: one v_perm_b32 per pair
__device__ __forceinline__ uint32_t px_lo(uint32_t w) { return __builtin_amdgcn_perm(0x64646464u, w, 0x04010400u); }
__device__ __forceinline__ uint32_t px_hi(uint32_t w) { return __builtin_amdgcn_perm(0x64646464u, w, 0x04030402u); }
__device__ __forceinline__ f16x8 frag_px(uint32_t w0, uint32_t w1) {
  u32x4 u = {px_lo(w0), px_hi(w0), px_lo(w1), px_hi(w1)};
  return __builtin_bit_cast(f16x8, u);
}
__device__ __forceinline__ f32x4 mfma_h(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f16x8 frag4(float a0, float a1, float a2, float a3) {
  f16x8 v = {(_Float16)a0, (_Float16)a1, (_Float16)a2, (_Float16)a3, (_Float16)0.f, (_Float16)0.f,
             (_Float16)0.f, (_Float16)0.f};
  return v;
}
// lane l <- lane l^16 / l^32 with gfx950's VALU row swaps (no LDS round trip)
__device__ __forceinline__ float xor16(float v) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(((threadIdx.x >> 4) & 1) ? p[0] : p[1]);
}
__device__ __forceinline__ float xor32(float v) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float((threadIdx.x & 32) ? p[0] : p[1]);
}

// ------------------------------------------------------------------ copier
// task = (step of the next chunk, 16-row batch tile): from the pinned host
// records write (1) the stage rows in k-step-pair order -- within each block of
// 64 features, byte 16g + 8sg + 4h + e holds feature 32sg + 16h + 4g + e, so a
// forward lane (g) fetches the B fragments of two k-steps with ONE 16-byte load --
// plus the tile's labels, and (2) the tile's 16 batch columns of the
// feature-major copy xT[800][128] for the weight gradient.
__device__ void copier(const Args& a, int cid, int ncop, uint8_t* smem) {
  if (a.next_steps <= 0) return;
  const int tid = threadIdx.x;
  if (a.ts != nullptr && tid == 0) a.ts[64 * 8 * 16 + 2 * cid] = (long long)__builtin_amdgcn_s_memrealtime();
  constexpr int TS = XR + 16;   // LDS tile row stride (bytes)
  const int ntask = a.next_steps * NBT;
  for (int task = cid; task < ntask; task += ncop) {
    const int st = task / NBT, bt = task % NBT;
    const int nrows = min(16, a.B - 16 * bt);
    const uint8_t* src = a.host_next + (long long)st * a.rec_h + (long long)16 * bt * DIN;
    for (int k = tid; k < 16 * (XR / 16); k += THREADS) {
      const int row = k / (XR / 16), c16 = k % (XR / 16);
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (row < nrows && c16 < DIN / 16) v = reinterpret_cast<const uint4*>(src)[row * (DIN / 16) + c16];
      *reinterpret_cast<uint4*>(smem + row * TS + 16 * c16) = v;
    }
    if (tid < nrows)
      a.xs_next[(long long)st * a.rec + (long long)a.B * XR + 16 * bt + tid] =
          a.host_next[(long long)st * a.rec_h + (long long)a.B * DIN + 16 * bt + tid];
    __syncthreads();
    // (1) permuted stage rows: chunk (row, block p, g) = natural words at 64p + 4g + {0,16,32,48}
    uint8_t* dst = a.xs_next + (long long)st * a.rec + (long long)16 * bt * XR;
    for (int k = tid; k < nrows * (XR / 16); k += THREADS) {
      const int row = k / (XR / 16), c = k % (XR / 16);
      const int p = c >> 2, gg = c & 3;
      const uint8_t* t = smem + row * TS + 64 * p + 4 * gg;
      const uint4 v = make_uint4(*reinterpret_cast<const uint32_t*>(t), *reinterpret_cast<const uint32_t*>(t + 16),
                                 *reinterpret_cast<const uint32_t*>(t + 32), *reinterpret_cast<const uint32_t*>(t + 48));
      *reinterpret_cast<uint4*>(dst + row * XR + 16 * c) = v;
    }
    // (2) feature-major copy
    uint8_t* xt = a.xts_next + (long long)st * NF * BPT + 16 * bt;
    for (int f = tid; f < NF; f += THREADS) {
      uint32_t w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        w[q] = (uint32_t)smem[(4 * q + 0) * TS + f] | ((uint32_t)smem[(4 * q + 1) * TS + f] << 8) |
               ((uint32_t)smem[(4 * q + 2) * TS + f] << 16) | ((uint32_t)smem[(4 * q + 3) * TS + f] << 24);
      }
      *reinterpret_cast<uint4*>(xt + (long long)f * BPT) = make_uint4(w[0], w[1], w[2], w[3]);
    }
    __syncthreads();
  }
  if (a.ts != nullptr && tid == 0) a.ts[64 * 8 * 16 + 2 * cid + 1] = (long long)__builtin_amdgcn_s_memrealtime();
}

// ------------------------------------------------------------------ compute
typedef int v2i __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) v2i lds_v2i;

// LDS carve (dynamic base 16-byte aligned; every offset a multiple of 16)
constexpr int XS = DIN;                          // x image row stride: 784 B -> conflict-free tr_b8 reads
constexpr int L_XIM = 0;                         // [112 rows][784] u8 pixels of the current step
constexpr int L_WFRAG = 112 * XS;                // [25 k-steps][64 lanes] fp16x8 W1^T fragments  25600
constexpr int L_CSUM = L_WFRAG + NKS * 64 * 16;  // [8 waves][16 hidden] fp32 column sums          512
constexpr int L_DZ2T = L_CSUM + 8 * 16 * 4;      // [16 hidden][128 batch] fp16                   4096
constexpr int L_A2T = L_DZ2T + 16 * BPT * 2;     // [16 hidden][128 batch] fp16                   4096
constexpr int L_DZ3T = L_A2T + 16 * BPT * 2;     // [16 class][128 batch] fp16                    4096
constexpr int L_W2 = L_DZ3T + 16 * BPT * 2;      // [16 hidden][16 class] fp32                    1024
constexpr int L_B1 = L_W2 + 1024;                // 16 fp32
constexpr int L_B2 = L_B1 + 64;                  // 16 fp32
constexpr int L_RDB1 = L_B2 + 64;                // [8][16] fp32
constexpr int L_RDB2 = L_RDB1 + 512;             // [8][16] fp32
constexpr int L_RMET = L_RDB2 + 512;             // [8][2] fp32
constexpr int L_FLAG = L_RMET + 64;              // abort flag
constexpr int LDS_BYTES = L_FLAG + 80;

// k-step owned by wave w in slot u (-1: none).  Wave 7 does no forward/head
// work, so it takes the 25th k-step.
__device__ __forceinline__ int kstep_of(int w, int u) { return u < 3 ? w + 8 * u : (w == 7 ? NKS - 1 : -1); }

template <int ACT, bool MULTI>   // ACT 0 sigmoid, 1 relu; MULTI: N-GPU gradient exchange
__device__ void compute(const Args& a, const int j, uint8_t* smem) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int B = a.B;
  uint8_t* xim = smem + L_XIM;
  f16x8* wfrag = reinterpret_cast<f16x8*>(smem + L_WFRAG);
  float* csum = reinterpret_cast<float*>(smem + L_CSUM);
  _Float16* dz2T = reinterpret_cast<_Float16*>(smem + L_DZ2T);
  _Float16* a2T = reinterpret_cast<_Float16*>(smem + L_A2T);
  _Float16* dz3T = reinterpret_cast<_Float16*>(smem + L_DZ3T);
  float* w2s = reinterpret_cast<float*>(smem + L_W2);
  float* b1s = reinterpret_cast<float*>(smem + L_B1);
  float* b2s = reinterpret_cast<float*>(smem + L_B2);
  float* rdb1 = reinterpret_cast<float*>(smem + L_RDB1);
  float* rdb2 = reinterpret_cast<float*>(smem + L_RDB2);
  float* rmet = reinterpret_cast<float*>(smem + L_RMET);
  int* abort_flag = reinterpret_cast<int*>(smem + L_FLAG);
  int* small_done = abort_flag + 1;   // steps whose small-parameter update is complete
  int* wready = abort_flag + 4;       // [8]: steps whose W1 fragments wave v has published
  int* tready = abort_flag + 12;      // [8]: steps whose head outputs batch tile v has published

  // ---- load state
  for (int k = tid; k < 3 * 16 * BPT; k += THREADS) dz2T[k] = (_Float16)0.f;   // also a2T, dz3T
  if (tid < 256) {
    const int n = tid >> 4, c = tid & 15;
    const int hn = 16 * j + n;
    w2s[tid] = (hn < HID && c < NCLS) ? a.params[OFF_W2 + hn * NCLS + c] : 0.f;
  } else if (tid < 272) {
    const int hn = 16 * j + (tid - 256);
    b1s[tid - 256] = hn < HID ? a.params[OFF_B1 + hn] : 0.f;
  } else if (tid < 288) {
    const int c = tid - 272;
    b2s[c] = c < NCLS ? a.params[OFF_B2 + c] : 0.f;
  } else if (tid == 288) {
    *abort_flag = 0;
    *small_done = 0;
    for (int v = 0; v < 8; ++v) wready[v] = tready[v] = 0;
  }
  const int hid = 16 * j + r;       // this lane's hidden unit in the W1^T-fragment / dW1 layouts
  const bool hv = hid < HID;
  float Wm[NU][2][4];               // W1[32s+16h+4g+i][hid], s = w + 8u
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int s = kstep_of(w, u);
        const int f = 32 * s + 16 * h + 4 * g + i;
        Wm[u][h][i] = (s >= 0 && f < DIN && hv) ? a.params[f * HID + hid] : 0.f;
      }
  // publish this wave's fp16 W1^T fragments + their column sums (the fwd's 1024-offset correction)
  auto publish_w1 = [&]() {
    float cp = 0.f;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int s = kstep_of(w, u);
      if (s >= 0) {
        f16x8 A;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          A[i] = (_Float16)Wm[u][0][i];
          A[4 + i] = (_Float16)Wm[u][1][i];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) cp += (float)A[e];
        wfrag[s * 64 + lane] = A;
      }
    }
    cp += xor16(cp);
    cp += xor32(cp);
    if (g == 0) csum[w * 16 + r] = cp;
  };
  publish_w1();
  const unsigned long long seq0 = *a.seq;
  const long long gstep0 = *a.gstep;
  const float lr = *a.lr;
  const float lrB = lr / (float)B;
  const float lrX = lrB * (1.f / 255.f);
  const bool failed_in = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;

  // x fragments of this wave's batch tile (waves 0..6), row 16w + r: fetch p
  // holds k-steps 2p, 2p+1; word 2(s&1)+h = features 32s+16h+4g+(0..3)
  const int xrow = min(16 * w + r, B - 1);
  uint4 xf[NP];
  auto load_x = [&](int st) {
    const uint8_t* xr = a.xs + (long long)st * a.rec + (long long)xrow * XR + 16 * g;
#pragma unroll
    for (int p = 0; p < NP; ++p) xf[p] = *reinterpret_cast<const uint4*>(xr + 64 * p);
  };
  auto xw = [&](int s, int h) -> uint32_t {
    const uint4& v = xf[s >> 1];
    return (s & 1) ? (h ? v.w : v.z) : (h ? v.y : v.x);
  };
  // ---- placement: all 7 compute workgroups on ONE XCD (shared L2) -> the
  // exchange granules are stored plain (they stay in that L2, where the
  // consumers' L1-bypassing sc1 loads hit); otherwise write-through sc1 stores.
  // Decided per launch from HW_REG_XCC_ID, never assumed.
  __shared__ int same_xcd;
  if (tid == 0) {
    const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20) & 15u;
    gu64* hdr = (gu64*)(a.gran);
    const unsigned tag0 = (unsigned)(seq0 + 1ull);
    __hip_atomic_store(hdr + j, ((unsigned long long)tag0 << 32) | xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int same = 1;
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    for (int jj = 0; jj < NWG; ++jj) {
      unsigned long long v;
      while (((v = __hip_atomic_load(hdr + jj, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 32) != tag0) {
        if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) {
          atomicOr(a.err, 1);
          same = -1;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      if (same < 0) break;
      if ((unsigned)v != xcc) same = 0;
    }
    same_xcd = same;
  }
  __syncthreads();
  if (failed_in || same_xcd < 0) return;
  const bool l2_local = same_xcd == 1;
  if (w < NBT) load_x(0);

  bool aborted = false;
  for (int st = 0; st < a.nsteps; ++st) {
    const unsigned long long sq = seq0 + (unsigned long long)st + 1ull;
    const unsigned tag = (unsigned)sq;
    if (j == 0 && tid == 0 && a.step_ts != nullptr)
      a.step_ts[(gstep0 + st) % a.ts_ring] = (long long)__builtin_amdgcn_s_memrealtime();
    if (w == 0) { TSP(0); }

    // ---------------- forward + head (wave w < 7: batch tile w)
    if (w < NBT) {
      const int b = 16 * w + r;
      const bool bv = b < B;
      const int y0 = a.xs[(long long)st * a.rec + (long long)B * XR + xrow];
      const int y = y0 < NCLS ? y0 : 0;
      f32x4 z = {0.f, 0.f, 0.f, 0.f};
      // owner v's fragments as soon as v has published step st's W1 (no block barrier);
      // waves 3 and 7 share SIMD 3 (13 of the 49 weight-gradient tiles) and finish last
#pragma unroll
      for (int vi = 0; vi < 8; ++vi) {
        const int v = vi < 3 ? vi : (vi < 6 ? vi + 1 : (vi == 6 ? 3 : 7));
        while (__hip_atomic_load(wready + v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < st)
          __builtin_amdgcn_s_sleep(1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          const int s = (u < 3) ? v + 8 * u : (v == 7 ? NKS - 1 : -1);
          if (s >= 0) z = mfma_h(wfrag[s * 64 + lane], frag_px(xw(s, 0), xw(s, 1)), z);
        }
      }
      // b1/W2/b2 of step st-1's update (wave 7) before they are read here
      while (__hip_atomic_load(small_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < st)
        __builtin_amdgcn_s_sleep(1);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
      if (w == 0) { TSP(13); }
      // lane (batch r, g): z^T[hidden 16j+4g+i][batch b]
      float a2[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int hl = 4 * g + i;
        float cs = 0.f;
#pragma unroll
        for (int w2 = 0; w2 < 8; ++w2) cs += csum[w2 * 16 + hl];
        const float zt = (z[i] - 1024.f * cs) * (1.f / 255.f) + b1s[hl];
        const float act = ACT == 0 ? sigmoidf_(zt) : fmaxf(zt, 0.f);
        a2[i] = (16 * j + hl < HID) ? act : 0.f;
      }
      // partial logits^T[class][batch] of this hidden block
      const f16x8 Aw2 = frag4(w2s[(4 * g + 0) * 16 + r], w2s[(4 * g + 1) * 16 + r], w2s[(4 * g + 2) * 16 + r],
                              w2s[(4 * g + 3) * 16 + r]);
      const f32x4 pl = mfma_h(Aw2, frag4(a2[0], a2[1], a2[2], a2[3]), f32x4{0.f, 0.f, 0.f, 0.f});
      if (w == 0) { TSP(1); }
      const int par = (int)(sq & 1ull);
      // publish this tile's partial logits: dense fp32 (lane g <= 2: classes
      // 4g..4g+3 of batch row r), drained, then ONE flag word per (workgroup, wave)
      float* mine = a.dense + ((size_t)(par * NWG + j) * NBT + w) * PAYLOAD;
      const f32x4 plv = pl;
      if (g < 3) {
        if (l2_local)   // plain stores: the lines stay in the shared L2
          *reinterpret_cast<f32x4*>(mine + 4 * lane) = plv;
        else            // write-through (sc1): visible to other XCDs' sc1 loads
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, plv),
                                                 __builtin_amdgcn_make_buffer_rsrc(mine, 0, PAYLOAD * 4, 0x00020000),
                                                 16 * lane, 0, 16);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // payload acknowledged before the flag
      gu32* flg = (gu32*)(a.flags) + par * 64;
      if (lane == 0) {
        if (l2_local) __hip_atomic_store(flg + j * NBT + w, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else __hip_atomic_store(flg + j * NBT + w, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      // while the exchange is in flight: x rows -> LDS image (read transposed by the
      // weight-gradient MFMAs), a2 -> LDS (dW2)
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        *reinterpret_cast<uint32_t*>(xim + b * XS + 32 * s + 4 * g) = xw(s, 0);
        if (s < NKS - 1) *reinterpret_cast<uint32_t*>(xim + b * XS + 32 * s + 16 + 4 * g) = xw(s, 1);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) a2T[(4 * g + i) * BPT + b] = (_Float16)a2[i];
      if (w == 0) { TSP(6); }
      // lanes 0..6 poll the 7 producers' flags of this tile (relaxed sc1 loads)
      {
        const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
        int sweeps = 0;
        for (;;) {
          ++sweeps;
          bool ok = true;
          if (lane < NWG && lane != j)
            ok = __hip_atomic_load(flg + lane * NBT + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == tag;
          if (__all(ok)) {
            if (a.ts != nullptr && w == 0 && lane == 0 && st < 64) a.ts[((long long)st * 8 + j) * 16 + 7] = sweeps;
            break;
          }
          if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > a.timeout ||
              __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
            if (lane == 0) {
              atomicOr(a.err, 1);
              *abort_flag = 1;
            }
            break;
          }
        }
      }
      // the other producers' payloads: one sc1 (L1-bypassing) 16-byte load each
      float part[NWG][4];
#pragma unroll
      for (int jj = 0; jj < NWG; ++jj) {
        if (jj == j || g >= 3) {
#pragma unroll
          for (int i = 0; i < 4; ++i) part[jj][i] = pl[i];
        } else {
          const float* src = a.dense + ((size_t)(par * NWG + jj) * NBT + w) * PAYLOAD;
          const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(
              __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, PAYLOAD * 4, 0x00020000), 16 * lane, 0, 16);
#pragma unroll
          for (int i = 0; i < 4; ++i) part[jj][i] = __uint_as_float(v[i]);
        }
      }
      if (w == 0) { TSP(2); }
      // logits, softmax cross-entropy, accuracy -- identical in every workgroup
      float lg[4], e[4];
      float m = -3.0e38f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = b2s[4 * g + i];
#pragma unroll
        for (int jj = 0; jj < NWG; ++jj) v += part[jj][i];
        lg[i] = v;
        if (4 * g + i < NCLS) m = fmaxf(m, v);
      }
      if (w == 0) { TSP(11); }
      m = fmaxf(m, xor16(m));
      m = fmaxf(m, xor32(m));
      float ssum = 0.f, zy = 0.f, am = 1e9f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = 4 * g + i;
        e[i] = c < NCLS ? __expf(lg[i] - m) : 0.f;
        ssum += e[i];
        zy += (c == y) ? lg[i] : 0.f;
        if (c < NCLS && lg[i] == m) am = fminf(am, (float)c);
      }
      ssum += xor16(ssum); ssum += xor32(ssum);
      zy += xor16(zy); zy += xor32(zy);
      am = fminf(am, xor16(am)); am = fminf(am, xor32(am));
      const float inv = 1.f / ssum;
      float dz3[4], py = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = 4 * g + i;
        const float p = e[i] * inv;
        py += (c == y) ? p : 0.f;
        dz3[i] = (bv && c < NCLS) ? p - (c == y ? 1.f : 0.f) : 0.f;   // unscaled: 1/B at the update
      }
      py += xor16(py); py += xor32(py);
      // next step's x: in flight across the rest of the head and the weight gradient
      if (st + 1 < a.nsteps) load_x(st + 1);
      const float loss = a.naive ? -__logf(py) : (m + __logf(ssum) - zy);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float s = row16_sum(dz3[i]);
        if (r == 0) rdb2[w * 16 + 4 * g + i] = s;
      }
      const float ls = row16_sum((g == 0 && bv) ? loss : 0.f);
      const float cr = row16_sum((g == 0 && bv && (int)am == y) ? 1.f : 0.f);
      if (lane == 0) { rmet[2 * w] = ls; rmet[2 * w + 1] = cr; }
      // da2^T = W2 . dz3^T, dz2 = da2 * act'(a2)
      const f16x8 Aw = frag4(w2s[r * 16 + 4 * g + 0], w2s[r * 16 + 4 * g + 1], w2s[r * 16 + 4 * g + 2],
                             w2s[r * 16 + 4 * g + 3]);
      const f32x4 da2 = mfma_h(Aw, frag4(dz3[0], dz3[1], dz3[2], dz3[3]), f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float d = ACT == 0 ? da2[i] * a2[i] * (1.f - a2[i]) : (a2[i] > 0.f ? da2[i] : 0.f);
        dz2T[(4 * g + i) * BPT + b] = (_Float16)d;
        dz3T[(4 * g + i) * BPT + b] = (_Float16)dz3[i];
        const float s = row16_sum(d);
        if (r == 0) rdb1[w * 16 + 4 * g + i] = s;
      }
      // batch tile w's x-image rows, dz2^T / a2^T / dz3^T columns and sums are in LDS
      // (an abort flag set above is ordered before this release)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
      if (lane == 0) __hip_atomic_store(tready + w, st + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (w == 0) { TSP(12); }
    auto wait_tile = [&](int v) {
      while (__hip_atomic_load(tready + v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < st + 1)
        __builtin_amdgcn_s_sleep(1);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    };
    if (w == 0) { TSP(3); }

    // ---------------- small-parameter gradients (wave 7): dW2 on MFMA, db1, db2, metrics.
    // 1 GPU: applied after S_a, overlapping the next forward (the next head waits on
    // small_done).  N GPUs: computed here, exchanged with the block's gradient.
    auto small_grads = [&](float (&gw2)[4], float& gb) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 4; ++q)
        acc = mfma_h(*reinterpret_cast<const f16x8*>(dz3T + r * BPT + 32 * q + 8 * g),
                     *reinterpret_cast<const f16x8*>(a2T + r * BPT + 32 * q + 8 * g), acc);
      // lane (hidden r, g): dW2[16j + r][class 4g + i] (x B: dz3 is unscaled)
#pragma unroll
      for (int i = 0; i < 4; ++i) gw2[i] = (hv && 4 * g + i < NCLS) ? acc[i] : 0.f;
      gb = 0.f;
      if (lane < 16) {
#pragma unroll
        for (int w2 = 0; w2 < NBT; ++w2) gb += rdb1[w2 * 16 + lane];
        if (16 * j + lane >= HID) gb = 0.f;
      } else if (lane < 16 + NCLS) {
#pragma unroll
        for (int w2 = 0; w2 < NBT; ++w2) gb += rdb2[w2 * 16 + lane - 16];
      } else if (lane == 63 && j == 0) {
        float ls = 0.f, cr = 0.f;
#pragma unroll
        for (int w2 = 0; w2 < NBT; ++w2) { ls += rmet[2 * w2]; cr += rmet[2 * w2 + 1]; }
        const int sl = (int)((gstep0 + st) % a.ring);
        a.metrics[2 * sl] = ls / (float)B;
        a.metrics[2 * sl + 1] = cr / (float)B;
      }
    };
    auto small_apply = [&](const float (&gw2)[4], float gb, float scale) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (hv && 4 * g + i < NCLS) w2s[r * 16 + 4 * g + i] -= scale * gw2[i];
      if (lane < 16) b1s[lane] -= scale * gb;
      else if (lane < 16 + NCLS) b2s[lane - 16] -= scale * gb;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
      if (lane == 0) __hip_atomic_store(small_done, st + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    constexpr bool multi = MULTI;
    float sgw2[4] = {0.f, 0.f, 0.f, 0.f};
    float sgb = 0.f;
    char* own_slot = nullptr;
    if constexpr (MULTI) {
      own_slot = static_cast<char*>(a.peer_base[a.rank]) + IPC_FLAGS + (size_t)(par_of(st) * NWG + j) * IPC_SLOT;
      if (w == 7) {   // small gradients (mean over the local batch) -> own slot, bf16
        for (int v = 0; v < NBT; ++v) wait_tile(v);
        small_grads(sgw2, sgb);
#pragma unroll
        for (int i = 0; i < 4; ++i) sgw2[i] = bfround(sgw2[i] * (1.f / (float)B));
        sgb = bfround(sgb * (1.f / (float)B));
        *reinterpret_cast<uint2*>(own_slot + IPC_SMALL + (g * 16 + r) * 8) =
            make_uint2(pack2bf(sgw2[0], sgw2[1]), pack2bf(sgw2[2], sgw2[3]));
        if (lane < 16 + NCLS) *reinterpret_cast<uint16_t*>(own_slot + IPC_SMALL + 512 + 2 * lane) = f2bf(sgb);
      }
    }

    // ---------------- dW1 block (all waves): x^T . dz2, in the accumulator layout.
    // The batch contraction runs in 4 steps of 32 rows (batch tiles 2q, 2q+1), each
    // as soon as those tiles' head outputs are published -- no block barrier.
    uint2 gq[NU][2];   // N GPUs: this rank's bf16 gradient of the wave's tiles
    {
      f32x4 acc[NU][2];
#pragma unroll
      for (int u = 0; u < NU; ++u) acc[u][0] = acc[u][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      float cs2 = 0.f;
      // transposed x fragment: lane 2p'+hh of each 16-lane group addresses batch row
      // 32q + 8g + p' and columns 8hh..8hh+7 of the tile; lane r receives feature
      // column r of those 8 rows (rows >= 112 read row - 16: multiplied by dz2 = 0)
      const int prow = 8 * g + (r >> 1);
      const int pcol = 8 * (r & 1);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        wait_tile(2 * q);
        if (2 * q + 1 < NBT) wait_tile(2 * q + 1);
        const f16x8 bq = *reinterpret_cast<const f16x8*>(dz2T + r * BPT + 32 * q + 8 * g);
#pragma unroll
        for (int e = 0; e < 8; ++e) cs2 += (float)bq[e];
        int row = 32 * q + prow;
        row = row < 112 ? row : row - 16;
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          const int s = kstep_of(w, u);
          if (s >= 0) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int t = 2 * s + h;
              if (t < DIN / 16) {
                const v2i v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)(xim + row * XS + 16 * t + pcol));
                acc[u][h] = mfma_h(frag_px((uint32_t)v.x, (uint32_t)v.y), bq, acc[u][h]);
              }
            }
          }
        }
      }
      cs2 += xor16(cs2);
      cs2 += xor32(cs2);
      const float corr = 1024.f * cs2;
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int s = kstep_of(w, u);
        if (s >= 0) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int t = 2 * s + h;
            if constexpr (!MULTI) {
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const int f = 16 * t + 4 * g + i;
                if (f < DIN && hv) Wm[u][h][i] -= lrX * (acc[u][h][i] - corr);
              }
            } else {
              float gg[4];
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const int f = 16 * t + 4 * g + i;
                gg[i] = (f < DIN && hv) ? (acc[u][h][i] - corr) * (1.f / (255.f * (float)B)) : 0.f;
              }
              gq[u][h] = make_uint2(pack2bf(gg[0], gg[1]), pack2bf(gg[2], gg[3]));
              if (t < DIN / 16) *reinterpret_cast<uint2*>(own_slot + ((t * 4 + g) * 16 + r) * 8) = gq[u][h];
            }
          }
        }
      }
    }
    // every wave has now seen every tile's readiness (and so any abort set before it)
    if (*abort_flag) { aborted = true; break; }
    if constexpr (MULTI) {
      // ---- one-shot exchange of block j with the same workgroup on every peer GPU
      // (IPC-mapped uncached buffers: completion == visibility; rank-order sums keep
      // the replicas bit-identical)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave: its slot stores landed
      lds_barrier();
      if (tid == 0)
        __hip_atomic_store(reinterpret_cast<unsigned*>(static_cast<char*>(a.peer_base[a.rank]) + 64 * j), tag,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (w == 0) {
        const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
        for (;;) {
          bool ok = true;
          if (lane < a.W && lane != a.rank) {
            const unsigned v = __hip_atomic_load(
                reinterpret_cast<const unsigned*>(static_cast<const char*>(a.peer_base[lane]) + 64 * j),
                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            ok = (int)(v - tag) >= 0;
          }
          if (__all(ok)) break;
          if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > a.timeout ||
              __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
            if (lane == 0) {
              atomicOr(a.err, 2);
              *abort_flag = 1;
            }
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      lds_barrier();
      asm volatile("" ::: "memory");   // no peer-slot load hoisted above the flag match
      if (*abort_flag) { aborted = true; break; }
      const float lrW = lr / (float)a.W;
      const size_t soff = IPC_FLAGS + (size_t)(par_of(st) * NWG + j) * IPC_SLOT;
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int s = kstep_of(w, u);
        if (s >= 0) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int t = 2 * s + h;
            if (t < DIN / 16) {
              float sum[4] = {0.f, 0.f, 0.f, 0.f};
              for (int rr = 0; rr < a.W; ++rr) {
                uint2 v = gq[u][h];
                if (rr != a.rank) {
                  const unsigned long long x = ld_sys_u64((
                      static_cast<const char*>(a.peer_base[rr]) + soff + ((t * 4 + g) * 16 + r) * 8));
                  v = make_uint2((unsigned)x, (unsigned)(x >> 32));
                }
                sum[0] += bf2f(v.x & 0xffff); sum[1] += bf2f(v.x >> 16);
                sum[2] += bf2f(v.y & 0xffff); sum[3] += bf2f(v.y >> 16);
              }
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const int f = 16 * t + 4 * g + i;
                if (f < DIN && hv) Wm[u][h][i] -= lrW * sum[i];
              }
            }
          }
        }
      }
      if (w == 7) {
        float sw2[4] = {0.f, 0.f, 0.f, 0.f};
        float sb = 0.f;
        for (int rr = 0; rr < a.W; ++rr) {
          float v2[4] = {sgw2[0], sgw2[1], sgw2[2], sgw2[3]};
          float vb = sgb;
          if (rr != a.rank) {
            const char* ps = static_cast<const char*>(a.peer_base[rr]) + soff + IPC_SMALL;
            const unsigned long long x =
                ld_sys_u64((ps + (g * 16 + r) * 8));
            v2[0] = bf2f((unsigned)x & 0xffff); v2[1] = bf2f(((unsigned)x) >> 16);
            v2[2] = bf2f((unsigned)(x >> 32) & 0xffff); v2[3] = bf2f((unsigned)(x >> 48));
            vb = lane < 16 + NCLS ? bf2f(ld_sys_u16(ps + 512 + 2 * lane))
                                  : 0.f;
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) sw2[i] += v2[i];
          sb += vb;
        }
        small_apply(sw2, sb, lrW);
      }
    }
    if (w == 0 || w == 7) { TSP(w == 0 ? 4 : 10); }
    publish_w1();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    if (lane == 0) __hip_atomic_store(wready + w, st + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (w == 0) { TSP(5); }
    if (!MULTI && w == 7) {   // 1 GPU: small parameters while the next forward runs
      TSP(8);
      float gw2[4], gb;
      small_grads(gw2, gb);
      small_apply(gw2, gb, lrB);
      TSP(9);
    }
  }
  if (aborted) return;
  __syncthreads();   // wave 7's last small-parameter update

  // ---- write back the block (fp32 master), global step and exchange sequence
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int s = kstep_of(w, u);
        const int f = 32 * s + 16 * h + 4 * g + i;
        if (s >= 0 && f < DIN && hv) a.params[f * HID + hid] = Wm[u][h][i];
      }
  if (tid < 256) {
    const int n = tid >> 4, c = tid & 15;
    const int hn = 16 * j + n;
    if (hn < HID && c < NCLS) a.params[OFF_W2 + hn * NCLS + c] = w2s[tid];
  } else if (tid < 272) {
    const int hn = 16 * j + (tid - 256);
    if (hn < HID) a.params[OFF_B1 + hn] = b1s[tid - 256];
  } else if (tid < 282 && j == 0) {
    a.params[OFF_B2 + (tid - 272)] = b2s[tid - 272];
  } else if (tid == 300 && j == 0) {
    *a.gstep = gstep0 + a.nsteps;
    *a.seq = seq0 + (unsigned long long)a.nsteps;
    if (a.step_ts != nullptr)
      a.step_ts[(gstep0 + a.nsteps) % a.ts_ring] = (long long)__builtin_amdgcn_s_memrealtime();
  }
}

template <int ACT, bool MULTI>
__global__ __launch_bounds__(THREADS, 1) void mlp_persist(Args a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int b = blockIdx.x;
  if (b % XCD_STRIDE == 0 && b / XCD_STRIDE < NWG) {
    if (a.nsteps > 0) compute<ACT, MULTI>(a, b / XCD_STRIDE, smem);
    return;
  }
  // copier id among the non-compute blocks
  const int cid = b - min(b / XCD_STRIDE + 1, NWG);
  copier(a, cid, GRID - NWG, smem);
}

}  // namespace mlpp
}  // namespace dtfk

using dtfk::mlpp::Args;

extern "C" {

int dtfk_mlp_persist_gran_count() { return dtfk::mlpp::GRAN_TOTAL; }
int dtfk_mlp_persist_xt_bytes() { return dtfk::mlpp::NF * dtfk::mlpp::BPT; }
int dtfk_mlp_persist_max_batch() { return 16 * dtfk::mlpp::NBT; }

int dtfk_mlp_persist_ipc_bytes() { return dtfk::mlpp::IPC_BYTES; }

int dtfk_mlp_persist_stage_rec(int B) { return ((B * (dtfk::mlpp::XR + 1) + 15) / 16) * 16; }

hipError_t dtfk_mlp_persist(const void* xs, const void* xts, long long rec, long long rec_h, int B, int nsteps, float* params,
                            const float* lr, float* metrics, int ring, int act, int naive, long long* gstep,
                            unsigned long long* seq, unsigned long long* gran, int* err, long long timeout,
                            const void* host_next, int next_steps, void* xs_next, void* xts_next,
                            long long* ts, void* const* peer_base, int W, int rank, long long* step_ts,
                            int ts_ring, hipStream_t stream) {
  Args a;
  a.step_ts = step_ts;
  a.ts_ring = ts_ring > 0 ? ts_ring : 1;
  a.ts = ts;
  a.peer_base = peer_base;
  a.W = W;
  a.rank = rank;
  a.xs = static_cast<const uint8_t*>(xs);
  a.xts = static_cast<const uint8_t*>(xts);
  a.rec = rec;
  a.rec_h = rec_h;
  a.B = B;
  a.nsteps = nsteps;
  a.params = params;
  a.lr = lr;
  a.metrics = metrics;
  a.ring = ring;
  a.act = act;
  a.naive = naive;
  a.gstep = gstep;
  a.seq = seq;
  a.gran = gran;
  a.flags = reinterpret_cast<unsigned*>(gran + dtfk::mlpp::XCH_HDR);
  a.dense = reinterpret_cast<float*>(gran + dtfk::mlpp::XCH_HDR + dtfk::mlpp::XCH_FLAGS);
  a.err = err;
  a.timeout = timeout;
  a.host_next = static_cast<const uint8_t*>(host_next);
  a.next_steps = next_steps;
  a.xs_next = static_cast<uint8_t*>(xs_next);
  a.xts_next = static_cast<uint8_t*>(xts_next);
  constexpr size_t lds = dtfk::mlpp::LDS_BYTES;
  static bool attr_set = false;
  using namespace dtfk::mlpp;
  const void* kerns[4] = {reinterpret_cast<const void*>(mlp_persist<0, false>),
                          reinterpret_cast<const void*>(mlp_persist<1, false>),
                          reinterpret_cast<const void*>(mlp_persist<0, true>),
                          reinterpret_cast<const void*>(mlp_persist<1, true>)};
  if (!attr_set) {
    for (const void* k : kerns) {
      const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
    attr_set = true;
  }
  const int which = (act == 0 ? 0 : 1) + (W > 1 ? 2 : 0);
  switch (which) {
    case 0: hipLaunchKernelGGL((mlp_persist<0, false>), dim3(GRID), dim3(THREADS), lds, stream, a); break;
    case 1: hipLaunchKernelGGL((mlp_persist<1, false>), dim3(GRID), dim3(THREADS), lds, stream, a); break;
    case 2: hipLaunchKernelGGL((mlp_persist<0, true>), dim3(GRID), dim3(THREADS), lds, stream, a); break;
    default: hipLaunchKernelGGL((mlp_persist<1, true>), dim3(GRID), dim3(THREADS), lds, stream, a); break;
  }
  return hipGetLastError();
}

}  // extern "C"
