// Persistent, weight-stationary training kernel for the reference's 784-100-10
// MLP at the reference's precision (example.py:77-118 is fp32 end to end),
// with the two large GEMMs on bf16 MFMA through an EXACT three-way split:
//
//   * every fp32 value v splits as v = hi + mid + lo with hi = bf16(v),
//     mid = bf16(v - hi), lo = bf16(v - hi - mid): both differences are exact in
//     fp32 and lo captures the last bits, so the three bf16 terms sum to v
//     exactly (for |v| > ~1e-33; the weights and gradients here are many orders
//     above that);
//   * uint8 pixels are exact in bf16 (<= 8 significant bits);
//   * so x.W1 = x.hi + x.mid + x.lo and x^T.dz2 likewise are sums of EXACT
//     products accumulated in fp32 by the MFMA -- the numerics of an fp32 GEMM
//     (no rounded operand anywhere), at 3/16 of the f32-input MFMA's cost.
//   The head's small products (a2.W2, dz3.W2^T, a2^T.dz3) use f32-input MFMA.
//
// That makes a whole hidden block's K = 784 cheap enough for ONE workgroup, so
// there is a single inter-workgroup edge per step (the partial logits), as in
// the f16 engine (mlp_persist.hip):
//
//  * 7 compute workgroups (512 threads), workgroup j owns hidden units
//    [16j, 16j+16).  Wave w owns feature k-steps s = w + 8u (u < 3; wave 0 also
//    s = 24) of 32 features: fp32 master W1[32s+16h+4g+i][16j+r] (h < 2, i < 4;
//    r = lane&15, g = lane>>4) in VGPRs -- the C layout of its dW1 tiles 2s+h,
//    so the SGD update is in-register -- and its three bf16 pieces as the
//    forward A fragments (k order within a k-step: element e of lane group g is
//    feature 32s + 16(e>>2) + 4g + (e&3), the same features the C layout holds).
//  * per step:
//      P0  z^T partial of the wave's k-steps for all 7 batch tiles (3 MFMAs per
//          k-step and tile) -> LDS; wave w (batch tile w) sums the 8 partials in
//          wave order: the block's complete z^T, no cross-workgroup reduction.
//      P1  a2 = act(z/255 + b1), partial logits^T of block j (f32 MFMA).
//      E2  partial logits to the 6 other workgroups as tagged 8-byte granules
//          (the data is the flag); logits = b2 + sum_j in block order ->
//          identical in all 7; softmax / cross-entropy / argmax, dz3,
//          da2 = W2 dz3 (f32 MFMA), dz2 = da2 act' -> LDS as three bf16 planes.
//      P2  wave w: dW1 tiles of its k-steps = x^T dz2 (A = x^T bytes of the
//          feature-major stage copy, B = the dz2 planes), W1 -= lr/(255B) dW1,
//          re-split; wave 7 also: dW2 (f32 MFMA), db1, db2, metrics and the LDS
//          copies of W2[block j], b1[block j], b2 -- identical in every
//          workgroup that holds them.
//  * the remaining workgroups are COPIERS pulling the next chunk from pinned
//    host memory over PCIe into the other device stage.
//  * N GPUs (MULTI): after P2 every compute workgroup exchanges its gradient
//    with the same workgroup on every peer through IPC-mapped uncached buffers
//    and sums the ranks in rank order (bit-identical replicas).
//
// Placement: compute workgroup j runs as blockIdx 8j (packed: one XCD under the
// observed round-robin dispatch, so the edge stays in one L2) or j (spread:
// several ranks sharing a GPU in tests).  A per-launch census of HW_REG_XCC_ID
// decides the store flavour; correctness never depends on placement.
#include "common.h"

#include <cstdlib>

namespace dtfk {
namespace mlpx {

typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;
typedef int v2i __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) v2i lds_v2i;

constexpr int DIN = 784, HID = 100, NCLS = 10;
constexpr int NJ = 7;              // hidden blocks of 16 = compute workgroups
constexpr int NKS = 25;            // feature k-steps of 32 (784 padded to 800)
constexpr int NU = 3;              // k-step slots per wave: s = w + 8u (k-steps 0..23 = tiles 0..47)
constexpr int T48 = 768;           // tile 48 (features 768..783, k-step 24): replicated in every wave
constexpr int NBT = 7;             // batch tiles of 16 (B <= 112)
constexpr int BROWS = 16 * NBT;    // 112
constexpr int NF = 32 * NKS;       // 800
constexpr int XTS = 128;           // x^T row stride (batch padded to 4 k-steps of 32)
constexpr int THREADS = 512;
constexpr int NCOP = 24;           // copier workgroups
constexpr int GRID_PACKED = 8 * NJ;           // compute at 0, 8, ..., 48; the rest copy / exit
constexpr int GRID_SPREAD = NJ + NCOP;
constexpr int OFF_W2 = 78400, OFF_B1 = 79400, OFF_B2 = 79500;

// device stage record of one step:
//   xrow [112][800] u8, k-step interleaved: byte 32s + 8g + e of a row is feature
//        32s + 16(e>>2) + 4g + (e&3) (one 8-byte load = one forward B fragment)
//   labels [128]; rows >= B and features >= 784 are zero
// (the weight gradient's x^T fragments come from an LDS image of the step's
// pixels, read transposed with ds_read_b64_tr_b8 -- no feature-major copy)
constexpr long long XROW_BYTES = (long long)BROWS * NF;    // 89600
constexpr long long REC = XROW_BYTES + 128;

// exchange buffer (bytes): E2 [2 parity][NBT][NJ] granule slots (64 lanes x 4 x 8 B)
constexpr int GSLOT = 2048;
constexpr long long E2_OFF = 0;
constexpr long long HDR_OFF = E2_OFF + 2LL * NBT * NJ * GSLOT;   // [64] u64 placement census
constexpr long long XBUF_BYTES = HDR_OFF + 64 * 8;

// IPC buffer of one rank (N GPUs): [flags: workgroup j at byte 64j][2 parities][NJ slots]
// slot: [8 waves][NU][2 halves][64 lanes] x 16 B dW1 (fp32; bf16 payload in the first 8 B)
//       | tile 48 [64 lanes] x 16 B | dW2 64 lanes x 16 B | db1 (16) db2 (16) fp32
constexpr int IPC_FLAGS = 4096;
constexpr int IPC_T48 = 8 * NU * 2 * 64 * 16;
constexpr int IPC_SMALL = IPC_T48 + 64 * 16;
constexpr int IPC_SLOT = IPC_SMALL + 1024 + 128;
constexpr long long IPC_BYTES = IPC_FLAGS + 2LL * NJ * IPC_SLOT;

// LDS carve (compute); the copier reuses the same dynamic allocation
constexpr int LS = BROWS + 4;                          // fp32 [16][LS] images
constexpr int PS = XTS + 8;                            // bf16 plane row stride (elements)
constexpr int XS = DIN;                                // x image row stride: 784 B (conflict-free tr_b8 reads)
constexpr int L_XIM = 0;                               // [112 rows][784] u8 pixels of the step  87808
constexpr int L_ZBUF = L_XIM + BROWS * XS;             // [4 wave pairs][NBT][64] f32x4         28672
constexpr int L_A2T = L_ZBUF + 4 * NBT * 64 * 16;      // [16 hidden][LS] a2 fp32
constexpr int L_DZ3T = L_A2T + 16 * LS * 4;            // [16 class][LS] dz3 fp32
constexpr int L_DZP = L_DZ3T + 16 * LS * 4;            // [3 pieces][16 hidden][PS] dz2 bf16
constexpr int L_W2 = L_DZP + 3 * 16 * PS * 2;          // [16 hidden][16 class] W2 of block j
constexpr int L_B1 = L_W2 + 1024;                      // [16]
constexpr int L_B2 = L_B1 + 64;                        // [16]
constexpr int L_RDB1 = L_B2 + 64;                      // [8][16]
constexpr int L_RDB2 = L_RDB1 + 512;                   // [8][16]
constexpr int L_RMET = L_RDB2 + 512;                   // [8][2]
constexpr int L_FLAG = L_RMET + 64;
constexpr int LDS_COMPUTE = L_FLAG + 64;
constexpr int CROW = NF + 16;                          // copier LDS row stride (816)
static_assert(LDS_COMPUTE <= 160 * 1024, "compute LDS carve exceeds the CU's 160 KB");
constexpr int LDS_COPIER = BROWS * CROW;
constexpr int LDS_BYTES = LDS_COMPUTE > LDS_COPIER ? LDS_COMPUTE : LDS_COPIER;

struct Args {
  const uint8_t* stage;     // this chunk: nsteps records of REC bytes
  long long rec_h;          // host record bytes (B*785 rounded up to 16)
  int B, nsteps;
  float* params;            // flat fp32 master, TF variable order (read at start, written at end)
  const float* lr;
  float* metrics;
  int ring;
  int act, naive;
  long long* gstep;
  unsigned long long* seq;  // exchange sequence number (monotonic across launches)
  uint8_t* xbuf;            // granule exchange buffer (XBUF_BYTES, zeroed once)
  int* err;
  long long timeout;        // s_memrealtime ticks (100 MHz)
  long long* step_ts;       // optional: s_memrealtime at the start of every global step (ring)
  int ts_ring;
  const uint8_t* host_next; // device-visible pointer into pinned host memory
  int next_steps;
  uint8_t* stage_next;
  void* const* peer_base;   // N GPUs: IPC-mapped exchange buffers of every rank
  int W, rank;
  int gbf16;                // N GPUs: dW1 payload in bf16 (BASELINE config #2) instead of fp32
  long long* phase_ts;      // optional phase stamps: [step < 64][workgroup 64][16] (wave 0, lane 0)
  int spread;               // placement: 0 packed on one XCD (default), 1 spread (several ranks per GPU)
  int gmode;                // gather: 0 probe one granule per producer, then load; 1-3 direct loads with
                            // no / short / long s_sleep between passes (DTF_GATHER_MODE, tuning)
};

// phase stamp ph of step st (s_memrealtime, 100 MHz) -- profiling only
#define PH(ph)                                                                                 \
  if (a.phase_ts != nullptr && lane == 0 && st < 64)                                         \
    a.phase_ts[((long long)st * 64 + j) * 16 + (ph)] = (long long)__builtin_amdgcn_s_memrealtime();

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// bf16 bits (RNE) and the exact three-way split v = hi + mid + lo
__device__ __forceinline__ uint32_t bfbits(float v) { return (uint32_t)f2bf(v); }
__device__ __forceinline__ void split3(float v, uint32_t& h, uint32_t& m, uint32_t& l) {
  h = bfbits(v);
  const float r1 = v - bf2f((uint16_t)h);
  m = bfbits(r1);
  l = bfbits(r1 - bf2f((uint16_t)m));
}
// 8 bytes (pixels) -> 8 bf16 (exact: <= 8 significant bits): upper half of the f32
__device__ __forceinline__ bf16x8 px8(u32x2 b) {
  u32x4 o;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t wd = b[k >> 1];
    const int sh = (k & 1) * 16;
    const float f0 = (float)((wd >> sh) & 0xffu), f1 = (float)((wd >> (sh + 8)) & 0xffu);
    o[k] = (__float_as_uint(f0) >> 16) | (__float_as_uint(f1) & 0xffff0000u);
  }
  return __builtin_bit_cast(bf16x8, o);
}

__device__ __forceinline__ void lds_barrier() {   // orders LDS only: no vmcnt(0) on in-flight prefetches
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Granule hand-off through a buffer resource over a wave-uniform region.
// Producer: 4 floats -> 4 granules {value, tag} in two 16-byte stores, plain
// when every consumer shares the producer's XCD (verified at launch; the lines
// stay in that L2, where the consumers' sc1 loads hit) and write-through (sc1)
// otherwise.  Consumer: L1-bypassing (sc1) loads, valid when all four tags match
// (8-byte halves of a 16-byte store are observed untorn on gfx950:
// MI355X_MICROARCH.md "Valid forms", R2).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t region_rsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000);
}
__device__ __forceinline__ void put_gran(__amdgpu_buffer_rsrc_t rs, int voff, f32x4 v, unsigned tag, bool l2_local) {
  const u32x4 lo = {__float_as_uint(v[0]), tag, __float_as_uint(v[1]), tag};
  const u32x4 hi = {__float_as_uint(v[2]), tag, __float_as_uint(v[3]), tag};
  if (l2_local) {
    __builtin_amdgcn_raw_buffer_store_b128(lo, rs, voff, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(hi, rs, voff + 16, 0, 0);
  } else {
    __builtin_amdgcn_raw_buffer_store_b128(lo, rs, voff, 0, 16);
    __builtin_amdgcn_raw_buffer_store_b128(hi, rs, voff + 16, 0, 16);
  }
}
__device__ __forceinline__ bool get_gran(__amdgpu_buffer_rsrc_t rs, int voff, unsigned tag, f32x4& out) {
  const u32x4 lo = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, 16);
  const u32x4 hi = __builtin_amdgcn_raw_buffer_load_b128(rs, voff + 16, 0, 16);
  out = f32x4{__uint_as_float(lo[0]), __uint_as_float(lo[2]), __uint_as_float(hi[0]), __uint_as_float(hi[2])};
  return lo[1] == tag && lo[3] == tag && hi[1] == tag && hi[3] == tag;
}

// lane l <- lane l^16 / l^32 with gfx950's VALU row swaps
__device__ __forceinline__ float xor16(float v) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(((threadIdx.x >> 4) & 1) ? p[0] : p[1]);
}
__device__ __forceinline__ float xor32(float v) {
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float((threadIdx.x & 32) ? p[0] : p[1]);
}

// Gather the N granule slots (slot k at byte k*GSLOT, k != skip) of this lane
// until every tag matches; part[skip] = own (constant-index selects only: a
// runtime index would demote the array to scratch).  need = false: this lane
// takes no data (zeros) but joins the wave-wide exit test.  Each pass re-loads
// only what is still missing.  false on timeout / error.
template <int N>
__device__ __forceinline__ bool gather_gran(__amdgpu_buffer_rsrc_t rs, int skip, bool need, unsigned tag, f32x4 own,
                                            f32x4 (&part)[N], int lane, const Args& a) {
  bool have[N];
#pragma unroll
  for (int k = 0; k < N; ++k) {
    have[k] = (k == skip) || !need;
    part[k] = (k == skip) ? own : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  for (;;) {
    asm volatile("" ::: "memory");   // re-load every pass (no loop-invariant hoisting)
    bool all = true;
#pragma unroll
    for (int k = 0; k < N; ++k) {
      if (!have[k]) have[k] = get_gran(rs, k * GSLOT + 32 * lane, tag, part[k]);
      all = all && have[k];
    }
    if (__all(all)) return true;
    if (a.gmode == 2) __builtin_amdgcn_s_sleep(2);
    else if (a.gmode == 3) __builtin_amdgcn_s_sleep(8);
    if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > a.timeout ||
        __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
      if (lane == 0) atomicOr(a.err, 1);
      return false;
    }
  }
}

// ------------------------------------------------------------------ copier
// task = one step of the next chunk: 112 rows of 784 pixels from the pinned host
// record into LDS (rows >= B and features >= 784 zero), then the k-step
// interleaved rows and the labels into the device stage.
__device__ void copier(const Args& a, int cid, uint8_t* smem) {
  const int tid = threadIdx.x;
  const int B = a.B;
  for (int st = cid; st < a.next_steps; st += NCOP) {
    const uint8_t* src = a.host_next + (long long)st * a.rec_h;
    uint8_t* dst = a.stage_next + (long long)st * REC;
    constexpr int C16 = DIN / 16;   // 49 16-byte chunks of a host row
    for (int k = tid; k < BROWS * (NF / 16); k += THREADS) {
      const int row = k / (NF / 16), c = k % (NF / 16);
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (row < B && c < C16) v = reinterpret_cast<const uint4*>(src)[row * C16 + c];
      *reinterpret_cast<uint4*>(smem + row * CROW + 16 * c) = v;
    }
    if (tid < 128) dst[XROW_BYTES + tid] = tid < B ? src[(long long)B * DIN + tid] : (uint8_t)0;
    __syncthreads();
    // interleaved rows: 8 bytes (row, s, g) = features 32s+4g..+3, 32s+16+4g..+3
    for (int k = tid; k < BROWS * NKS * 4; k += THREADS) {
      const int row = k / (NKS * 4), s = (k / 4) % NKS, g = k & 3;
      const uint8_t* p = smem + row * CROW + 32 * s + 4 * g;
      const uint2 v = make_uint2(*reinterpret_cast<const uint32_t*>(p), *reinterpret_cast<const uint32_t*>(p + 16));
      *reinterpret_cast<uint2*>(dst + (long long)row * NF + 32 * s + 8 * g) = v;
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ compute
template <int ACT, bool MULTI>   // ACT 0 sigmoid, 1 relu; MULTI: N-GPU gradient exchange
__device__ void compute(const Args& a, const int j, uint8_t* smem) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int B = a.B;
  uint8_t* xim = smem + L_XIM;
  f32x4* zbuf = reinterpret_cast<f32x4*>(smem + L_ZBUF);
  float* a2T = reinterpret_cast<float*>(smem + L_A2T);
  float* dz3T = reinterpret_cast<float*>(smem + L_DZ3T);
  uint16_t* dzp = reinterpret_cast<uint16_t*>(smem + L_DZP);
  float* w2s = reinterpret_cast<float*>(smem + L_W2);
  float* b1s = reinterpret_cast<float*>(smem + L_B1);
  float* b2s = reinterpret_cast<float*>(smem + L_B2);
  float* rdb1 = reinterpret_cast<float*>(smem + L_RDB1);
  float* rdb2 = reinterpret_cast<float*>(smem + L_RDB2);
  float* rmet = reinterpret_cast<float*>(smem + L_RMET);
  int* abort_flag = reinterpret_cast<int*>(smem + L_FLAG);
  int* census = abort_flag + 1;

  // ---- load state
  for (int k = tid; k < 2 * 16 * LS; k += THREADS) a2T[k] = 0.f;                // a2T, dz3T (batch pad 0)
  for (int k = tid; k < 3 * 16 * PS; k += THREADS) dzp[k] = (uint16_t)0;        // dz2 planes (batch pad 0)
  if (tid < 256) {
    const int n = tid >> 4, cl = tid & 15;
    const int hn = 16 * j + n;
    w2s[tid] = (hn < HID && cl < NCLS) ? a.params[OFF_W2 + hn * NCLS + cl] : 0.f;
  } else if (tid < 272) {
    const int hn = 16 * j + (tid - 256);
    b1s[tid - 256] = hn < HID ? a.params[OFF_B1 + hn] : 0.f;
  } else if (tid < 288) {
    const int cl = tid - 272;
    b2s[cl] = cl < NCLS ? a.params[OFF_B2 + cl] : 0.f;
  } else if (tid == 288) {
    *abort_flag = 0;
  }
  const int hid = 16 * j + r;       // this lane's hidden unit in the W1 / dW1 layouts
  const bool hv = hid < HID;
  // k-step slot u of wave w: s = w + 8u; half h: tile 2s+h.  Tile 48 (k-step 24,
  // half a k-step) is replicated in EVERY wave (Wx): its forward is done for the
  // wave's own batch tile, its gradient by every wave (identical inputs and order
  // -> identical updates), so all waves carry 3 slots instead of one carrying 4.
  auto ks = [&](int u) { return w + 8 * u; };
  float Wm[NU][2][4];
  float Wx[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) Wx[i] = hv ? a.params[(T48 + 4 * g + i) * HID + hid] : 0.f;
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        Wm[u][h][i] = hv ? a.params[(32 * ks(u) + 16 * h + 4 * g + i) * HID + hid] : 0.f;
  // forward A fragments: the three bf16 pieces of 8 W1^T values (k order as in the
  // header), re-split from the fp32 master at use (not kept: 36 VGPRs)
  auto pieces8 = [&](const float (&v)[8], bf16x8& Ah, bf16x8& Am, bf16x8& Al) {
    u32x4 ph, pm, pl;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint32_t h0, m0, l0, h1, m1, l1;
      split3(v[2 * k], h0, m0, l0);
      split3(v[2 * k + 1], h1, m1, l1);
      ph[k] = h0 | (h1 << 16);
      pm[k] = m0 | (m1 << 16);
      pl[k] = l0 | (l1 << 16);
    }
    Ah = __builtin_bit_cast(bf16x8, ph);
    Am = __builtin_bit_cast(bf16x8, pm);
    Al = __builtin_bit_cast(bf16x8, pl);
  };
  const unsigned long long seq0 = *a.seq;
  const long long gstep0 = *a.gstep;
  const float lr = *a.lr;
  const float lrB = lr / (float)(B * (MULTI ? a.W : 1));
  const float lrX = lrB * (1.f / 255.f);
  const bool failed_in = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;

  // x operands (pixel bytes, converted to bf16 at use):
  //  xf[u][bt]: row 16bt+r, k-step s(u), lane group g (forward B fragment), 8 bytes
  //  xf48: k-step 24 of this wave's batch tile (wave 7: row clamp, unused)
  // After the forward every wave writes its bytes into the LDS x image (natural
  // feature order); the weight gradient reads x^T fragments from it transposed.
  u32x2 xf[NU][NBT], xf48;
  const int brow = 16 * (w < NBT ? w : NBT - 1) + r;
  auto load_xf = [&](int st) {
    const uint8_t* rec = a.stage + (long long)st * REC;
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
      for (int b = 0; b < NBT; ++b)
        xf[u][b] = *reinterpret_cast<const u32x2*>(rec + (16 * b + r) * NF + 32 * ks(u) + 8 * g);
    xf48 = *reinterpret_cast<const u32x2*>(rec + brow * NF + 32 * 24 + 8 * g);
  };
  auto store_image = [&]() {
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
      for (int b = 0; b < NBT; ++b) {
        uint8_t* row = xim + (16 * b + r) * XS + 32 * ks(u) + 4 * g;
        *reinterpret_cast<uint32_t*>(row) = xf[u][b][0];
        *reinterpret_cast<uint32_t*>(row + 16) = xf[u][b][1];
      }
    if (w < NBT) *reinterpret_cast<uint32_t*>(xim + brow * XS + T48 + 4 * g) = xf48[0];
  };
  auto load_lab = [&](int st) -> int {
    return w < NBT ? a.stage[(long long)st * REC + XROW_BYTES + 16 * w + r] : 0;
  };
  __syncthreads();
  if (failed_in) return;
  // ---- placement census: are all 7 compute workgroups on this XCD (edge in one L2)?
  if (tid == 0) {
    const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20) & 15u;
    unsigned long long* hdr = reinterpret_cast<unsigned long long*>(a.xbuf + HDR_OFF);
    const unsigned tag0 = (unsigned)(seq0 + 1ull);
    __hip_atomic_store(hdr + j, ((unsigned long long)tag0 << 32) | xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int same = 1, bad = 0;
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    for (int jj = 0; jj < NJ && !bad; ++jj) {
      unsigned long long v;
      while (((v = __hip_atomic_load(hdr + jj, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 32) != tag0) {
        if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) {
          atomicOr(a.err, 1);
          bad = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      if ((unsigned)v != xcc) same = 0;
    }
    *census = bad ? -1 : same;
  }
  __syncthreads();
  if (*census < 0) return;
  const bool l2_local = *census == 1;
  int lab = 0;
  if (a.nsteps > 0) {
    load_xf(0);
    lab = load_lab(0);
  }

  bool aborted = false;
  for (int st = 0; st < a.nsteps; ++st) {
    const unsigned long long sq = seq0 + (unsigned long long)st + 1ull;
    const unsigned tag = (unsigned)sq;
    const int par = (int)(sq & 1ull);
    if (j == 0 && tid == 0 && a.step_ts != nullptr)
      a.step_ts[(gstep0 + st) % a.ts_ring] = (long long)__builtin_amdgcn_s_memrealtime();
    if (w == 0) { PH(0); }
    if (w == 4) { PH(12); }

    // ---------------- P0: forward partial of the wave's k-steps, all batch tiles
    {
      f32x4 acc[NBT];
#pragma unroll
      for (int b = 0; b < NBT; ++b) acc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const float v8[8] = {Wm[u][0][0], Wm[u][0][1], Wm[u][0][2], Wm[u][0][3],
                             Wm[u][1][0], Wm[u][1][1], Wm[u][1][2], Wm[u][1][3]};
        bf16x8 Ah, Am, Al;
        pieces8(v8, Ah, Am, Al);
        bf16x8 X[NBT];
#pragma unroll
        for (int b = 0; b < NBT; ++b) X[b] = px8(xf[u][b]);
        // piece-major: 7 independent accumulator chains between dependent MFMAs
#pragma unroll
        for (int b = 0; b < NBT; ++b) acc[b] = mfma16x16x32(Al, X[b], acc[b]);
#pragma unroll
        for (int b = 0; b < NBT; ++b) acc[b] = mfma16x16x32(Am, X[b], acc[b]);
#pragma unroll
        for (int b = 0; b < NBT; ++b) acc[b] = mfma16x16x32(Ah, X[b], acc[b]);
      }
      {   // tile 48 for this wave's own batch tile (elements 4..7: zero features 784..799)
        const float v8[8] = {Wx[0], Wx[1], Wx[2], Wx[3], 0.f, 0.f, 0.f, 0.f};
        bf16x8 Ah, Am, Al;
        pieces8(v8, Ah, Am, Al);
        const bf16x8 X = px8(xf48);
#pragma unroll
        for (int b = 0; b < NBT; ++b)
          if (b == w) {   // wave-uniform: a constant-index select, no dynamic indexing
            acc[b] = mfma16x16x32(Al, X, acc[b]);
            acc[b] = mfma16x16x32(Am, X, acc[b]);
            acc[b] = mfma16x16x32(Ah, X, acc[b]);
          }
      }
      if (w == 0) { PH(9); }
      if (w == 4) { PH(10); }
      // wave-pair reduction of the partials (waves w and w+4) into 4 LDS slots
      if (w >= 4) {
#pragma unroll
        for (int b = 0; b < NBT; ++b) zbuf[((w - 4) * NBT + b) * 64 + lane] = acc[b];
      }
      lds_barrier();
      if (w == 0) { PH(11); }
      if (w < 4) {
#pragma unroll
        for (int b = 0; b < NBT; ++b) zbuf[(w * NBT + b) * 64 + lane] += acc[b];
      }
    }
    const int labn = st + 1 < a.nsteps ? load_lab(st + 1) : 0;
    if (w == 0) { PH(1); }
    lds_barrier();
    if (w == 0) { PH(2); }
    // the step's pixels into the LDS image (every wave finished the previous step's
    // weight gradient before the barrier above); then the next step's forward
    // operands are in flight across the head and the weight gradient
    store_image();
    if (st + 1 < a.nsteps) load_xf(st + 1);

    // ---------------- P1 + E2 + head (wave w < 7: batch tile w)
    if (w < NBT) {
      const int bw = 16 * w + r;          // this lane's batch row
      const bool bv = bw < B;
      f32x4 z = zbuf[w * 64 + lane];
#pragma unroll
      for (int v = 1; v < 4; ++v) z += zbuf[(v * NBT + w) * 64 + lane];
      // lane (batch r, g): hidden 16j+4g+i
      float a2[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int hl = 4 * g + i;
        const float zt = z[i] * (1.f / 255.f) + b1s[hl];
        const float av = ACT == 0 ? 1.f / (1.f + expf(-zt)) : fmaxf(zt, 0.f);
        a2[i] = (16 * j + hl < HID) ? av : 0.f;
      }
      // partial logits^T[class][batch] of block j: A = W2^T (lane: class r), B = a2^T
      f32x4 pl = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) pl = mfma4(w2s[(4 * g + e) * 16 + r], a2[e], pl);
      // E2 region of (parity, batch tile w): [block] slots
      const auto r2 = region_rsrc(a.xbuf + E2_OFF + (long long)(par * NBT + w) * NJ * GSLOT, NJ * GSLOT);
      if (g < 3) put_gran(r2, j * GSLOT + 32 * lane, pl, tag, l2_local);
      if (w == 0) { PH(3); }
      // while the logits are in flight: a2 -> LDS (dW2)
#pragma unroll
      for (int i = 0; i < 4; ++i) a2T[(4 * g + i) * LS + bw] = a2[i];
      f32x4 lp[NJ];
      const bool ok = gather_gran<NJ>(r2, j, g < 3, tag, pl, lp, lane, a);
      if (w == 0) { PH(4); }
      if (!ok && lane == 0) *abort_flag = 1;
      // logits, softmax cross-entropy, accuracy -- identical in every workgroup
      float lg[4], ex[4];
      float m = -3.0e38f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = b2s[4 * g + i];
#pragma unroll
        for (int jj = 0; jj < NJ; ++jj) v += lp[jj][i];
        lg[i] = v;
        if (4 * g + i < NCLS) m = fmaxf(m, v);
      }
      m = fmaxf(m, xor16(m));
      m = fmaxf(m, xor32(m));
      const int y = lab < NCLS ? lab : 0;
      float ssum = 0.f, zy = 0.f, am = 1e9f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int cl = 4 * g + i;
        ex[i] = cl < NCLS ? expf(lg[i] - m) : 0.f;
        ssum += ex[i];
        zy += (cl == y) ? lg[i] : 0.f;
        if (cl < NCLS && lg[i] == m) am = fminf(am, (float)cl);
      }
      ssum += xor16(ssum); ssum += xor32(ssum);
      zy += xor16(zy); zy += xor32(zy);
      am = fminf(am, xor16(am)); am = fminf(am, xor32(am));
      const float inv = 1.f / ssum;
      float dz3[4], py = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int cl = 4 * g + i;
        const float p = ex[i] * inv;
        py += (cl == y) ? p : 0.f;
        dz3[i] = (bv && cl < NCLS) ? p - (cl == y ? 1.f : 0.f) : 0.f;   // unscaled: 1/B at the update
      }
      py += xor16(py); py += xor32(py);
      const float loss = a.naive ? -logf(py) : (m + logf(ssum) - zy);
      // da2^T = W2 . dz3^T (A = W2, lane: hidden r), dz2 = da2 * act'(a2)
      f32x4 da = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) da = mfma4(w2s[r * 16 + 4 * g + e], dz3[e], da);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float d = ACT == 0 ? da[i] * a2[i] * (1.f - a2[i]) : (a2[i] > 0.f ? da[i] : 0.f);
        uint32_t ph, pm, plo;
        split3(d, ph, pm, plo);
        const int o = (4 * g + i) * PS + bw;
        dzp[o] = (uint16_t)ph;
        dzp[16 * PS + o] = (uint16_t)pm;
        dzp[32 * PS + o] = (uint16_t)plo;
        dz3T[(4 * g + i) * LS + bw] = dz3[i];
        const float s1 = row16_sum(d);
        const float s2 = row16_sum(dz3[i]);
        if (r == 0) {
          rdb1[w * 16 + 4 * g + i] = s1;
          rdb2[w * 16 + 4 * g + i] = s2;
        }
      }
      const float ls = row16_sum((g == 0 && bv) ? loss : 0.f);
      const float cr = row16_sum((g == 0 && bv && (int)am == y) ? 1.f : 0.f);
      if (lane == 0) { rmet[2 * w] = ls; rmet[2 * w + 1] = cr; }
      if (w == 0) { PH(5); }
    }
    lds_barrier();
    if (w == 0) { PH(6); }
    if (*abort_flag) { aborted = true; break; }

    // ---------------- P2: dW1 tiles of the wave's k-steps = x^T dz2 (batch K = 128)
    f32x4 G[NU][2];                      // dW1[32s+16h+4g+i][16j+r] (x 255 B)
    f32x4 G48 = {0.f, 0.f, 0.f, 0.f};    // dW1[768+4g+i][16j+r], identical in every wave
#pragma unroll
    for (int u = 0; u < NU; ++u) G[u][0] = G[u][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const bf16x8 Bh = *reinterpret_cast<const bf16x8*>(dzp + r * PS + 32 * qq + 8 * g);
      const bf16x8 Bm = *reinterpret_cast<const bf16x8*>(dzp + 16 * PS + r * PS + 32 * qq + 8 * g);
      const bf16x8 Bl = *reinterpret_cast<const bf16x8*>(dzp + 32 * PS + r * PS + 32 * qq + 8 * g);
      // x^T fragment of feature tile t: lane (r, g) addresses image row 32qq + 8g +
      // (r>>1), columns 16t + 8(r&1)..+7 and receives feature column r of those 8
      // rows (rows >= 112 read row - 16: multiplied by dz2 = 0)
      int xrow = 32 * qq + 8 * g + (r >> 1);
      xrow = xrow < BROWS ? xrow : xrow - 16;
      const uint8_t* xr = xim + xrow * XS + 8 * (r & 1);
      auto xtf = [&](int t) -> u32x2 {
        const v2i v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)(xr + 16 * t));
        return u32x2{(uint32_t)v.x, (uint32_t)v.y};
      };
      bf16x8 X[NU][2];
#pragma unroll
      for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int h = 0; h < 2; ++h) X[u][h] = px8(xtf(2 * ks(u) + h));
      const bf16x8 X48 = px8(xtf(48));
      // piece-major: 7 independent accumulator chains between dependent MFMAs
#pragma unroll
      for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int h = 0; h < 2; ++h) G[u][h] = mfma16x16x32(X[u][h], Bl, G[u][h]);
      G48 = mfma16x16x32(X48, Bl, G48);
#pragma unroll
      for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int h = 0; h < 2; ++h) G[u][h] = mfma16x16x32(X[u][h], Bm, G[u][h]);
      G48 = mfma16x16x32(X48, Bm, G48);
#pragma unroll
      for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int h = 0; h < 2; ++h) G[u][h] = mfma16x16x32(X[u][h], Bh, G[u][h]);
      G48 = mfma16x16x32(X48, Bh, G48);
    }
    if (w == 0) { PH(7); }
    f32x4 D = {0.f, 0.f, 0.f, 0.f};      // wave 7: dW2[16j+4g+i][class r] (x B)
    float gb = 0.f;                      // wave 7: db1 (lanes < 16) / db2 (lanes 16..25) (x B)
    if (w == 7) {
      f32x4 d0 = {0.f, 0.f, 0.f, 0.f}, d1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NBT; ++s) {
        const f32x4 av = *reinterpret_cast<const f32x4*>(a2T + r * LS + 16 * s + 4 * g);
        const f32x4 dv = *reinterpret_cast<const f32x4*>(dz3T + r * LS + 16 * s + 4 * g);
        d0 = mfma4(av[0], dv[0], d0);
        d1 = mfma4(av[1], dv[1], d1);
        d0 = mfma4(av[2], dv[2], d0);
        d1 = mfma4(av[3], dv[3], d1);
      }
      D = d0 + d1;
      if (lane < 16) {
#pragma unroll
        for (int v = 0; v < NBT; ++v) gb += rdb1[v * 16 + lane];
      } else if (lane < 16 + NCLS) {
#pragma unroll
        for (int v = 0; v < NBT; ++v) gb += rdb2[v * 16 + lane - 16];
      } else if (lane == 63 && j == 0) {
        float ls = 0.f, cr = 0.f;
#pragma unroll
        for (int v = 0; v < NBT; ++v) { ls += rmet[2 * v]; cr += rmet[2 * v + 1]; }
        const int sl = (int)((gstep0 + st) % a.ring);
        a.metrics[2 * sl] = ls / (float)B;
        a.metrics[2 * sl + 1] = cr / (float)B;
      }
    }
    if constexpr (MULTI) {
      // ---- one-shot exchange of this workgroup's gradient with the same
      // workgroup on every peer GPU (uncached IPC buffers: completion ==
      // visibility); rank-order sums keep the replicas bit-identical
      const size_t soff = IPC_FLAGS + (size_t)(par * NJ + j) * IPC_SLOT;
      char* own = static_cast<char*>(a.peer_base[a.rank]) + soff;
#pragma unroll
      for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          char* p = own + (((w * NU + u) * 2 + h) * 64 + lane) * 16;
          if (a.gbf16) {
            const uint2 v = make_uint2(pack2bf(G[u][h][0], G[u][h][1]), pack2bf(G[u][h][2], G[u][h][3]));
            G[u][h] = f32x4{bf2f(v.x & 0xffff), bf2f(v.x >> 16), bf2f(v.y & 0xffff), bf2f(v.y >> 16)};
            *reinterpret_cast<uint2*>(p) = v;
          } else {
            *reinterpret_cast<f32x4*>(p) = G[u][h];
          }
        }
      {   // tile 48: identical in every wave; wave 0 publishes it
        char* p = own + IPC_T48 + lane * 16;
        if (a.gbf16) {
          const uint2 v = make_uint2(pack2bf(G48[0], G48[1]), pack2bf(G48[2], G48[3]));
          G48 = f32x4{bf2f(v.x & 0xffff), bf2f(v.x >> 16), bf2f(v.y & 0xffff), bf2f(v.y >> 16)};
          if (w == 0) *reinterpret_cast<uint2*>(p) = v;
        } else if (w == 0) {
          *reinterpret_cast<f32x4*>(p) = G48;
        }
      }
      if (w == 7) {
        *reinterpret_cast<f32x4*>(own + IPC_SMALL + lane * 16) = D;
        if (lane < 16 + NCLS) *reinterpret_cast<float*>(own + IPC_SMALL + 1024 + lane * 4) = gb;
      }
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
      f32x4 sum[NU][2];
      f32x4 s48 = {0.f, 0.f, 0.f, 0.f};
      f32x4 sD = {0.f, 0.f, 0.f, 0.f};
      float sb = 0.f;
#pragma unroll
      for (int u = 0; u < NU; ++u) sum[u][0] = sum[u][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int rr = 0; rr < a.W; ++rr) {
        const char* ps = static_cast<const char*>(a.peer_base[rr]) + soff;
#pragma unroll
        for (int u = 0; u < NU; ++u)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            f32x4 v = G[u][h];
            if (rr != a.rank) {
              const char* pk = ps + (((w * NU + u) * 2 + h) * 64 + lane) * 16;
              if (a.gbf16) {
                const unsigned long long x = ld_sys_u64((pk));
                v = f32x4{bf2f((unsigned)x & 0xffff), bf2f(((unsigned)x) >> 16), bf2f((unsigned)(x >> 32) & 0xffff),
                          bf2f((unsigned)(x >> 48))};
              } else {
                v = ld_sys_f32x4((pk));
              }
            }
            sum[u][h] += v;
          }
        {
          f32x4 v = G48;
          if (rr != a.rank) {
            const char* pk = ps + IPC_T48 + lane * 16;
            if (a.gbf16) {
              const unsigned long long x = ld_sys_u64((pk));
              v = f32x4{bf2f((unsigned)x & 0xffff), bf2f(((unsigned)x) >> 16), bf2f((unsigned)(x >> 32) & 0xffff),
                        bf2f((unsigned)(x >> 48))};
            } else {
              v = ld_sys_f32x4((pk));
            }
          }
          s48 += v;
        }
        if (w == 7) {
          f32x4 v = D;
          float vb = gb;
          if (rr != a.rank) {
            v = ld_sys_f32x4((ps + IPC_SMALL + lane * 16));
            vb = lane < 16 + NCLS ? ld_sys_f32(ps + IPC_SMALL + 1024 + 4 * lane)
                                  : 0.f;
          }
          sD += v;
          sb += vb;
        }
      }
#pragma unroll
      for (int u = 0; u < NU; ++u) { G[u][0] = sum[u][0]; G[u][1] = sum[u][1]; }
      G48 = s48;
      if (w == 7) { D = sD; gb = sb; }
    }
    // ---------------- updates (lr / (W B), 1/255 for the pixel scale)
    if (hv) {
#pragma unroll
      for (int u = 0; u < NU; ++u)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int i = 0; i < 4; ++i) Wm[u][h][i] -= lrX * G[u][h][i];
#pragma unroll
      for (int i = 0; i < 4; ++i) Wx[i] -= lrX * G48[i];
    }
    lab = labn;
    if (w == 0) { PH(8); }
    if (w == 7) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (16 * j + 4 * g + i < HID && r < NCLS) w2s[(4 * g + i) * 16 + r] -= lrB * D[i];
      if (lane < 16) {
        if (16 * j + lane < HID) b1s[lane] -= lrB * gb;
      } else if (lane < 16 + NCLS) {
        b2s[lane - 16] -= lrB * gb;
      }
    }
  }
  if (aborted) return;
  __syncthreads();   // wave 7's last small-parameter update

  // ---- write back (fp32 master), global step, exchange sequence, end stamp
  if (hv) {
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i) a.params[(32 * ks(u) + 16 * h + 4 * g + i) * HID + hid] = Wm[u][h][i];
    if (w == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) a.params[(T48 + 4 * g + i) * HID + hid] = Wx[i];
    }
  }
  if (tid < 256) {
    const int n = tid >> 4, cl = tid & 15;
    const int hn = 16 * j + n;
    if (hn < HID && cl < NCLS) a.params[OFF_W2 + hn * NCLS + cl] = w2s[tid];
  } else if (tid < 272) {
    const int hn = 16 * j + (tid - 256);
    if (hn < HID) a.params[OFF_B1 + hn] = b1s[tid - 256];
  }
  if (j == 0) {
    if (tid >= 272 && tid < 272 + NCLS) a.params[OFF_B2 + (tid - 272)] = b2s[tid - 272];
    if (tid == 300) {
      *a.gstep = gstep0 + a.nsteps;
      *a.seq = seq0 + (unsigned long long)a.nsteps;
      if (a.step_ts != nullptr)
        a.step_ts[(gstep0 + a.nsteps) % a.ts_ring] = (long long)__builtin_amdgcn_s_memrealtime();
    }
  }
}

template <int ACT, bool MULTI>
__global__ __launch_bounds__(THREADS, 1) void mlp_persist_x3(Args a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int b = blockIdx.x;
  int j = -1, cid = -1;
  if (a.spread) {
    if (b < NJ) j = b; else cid = b - NJ;
  } else {
    if ((b & 7) == 0) j = b >> 3; else cid = b - (b >> 3) - 1;
  }
  if (j >= 0) {
    if (a.nsteps > 0) compute<ACT, MULTI>(a, j, smem);
    return;
  }
  if (cid < NCOP) copier(a, cid, smem);
}

}  // namespace mlpx
}  // namespace dtfk

extern "C" {

long long dtfk_mlpx_stage_rec() { return dtfk::mlpx::REC; }
long long dtfk_mlpx_xbuf_bytes() { return dtfk::mlpx::XBUF_BYTES; }
long long dtfk_mlpx_ipc_bytes() { return dtfk::mlpx::IPC_BYTES; }

hipError_t dtfk_mlp_persist_x3(const void* stage, long long rec_h, int B, int nsteps, float* params, const float* lr,
                               float* metrics, int ring, int act, int naive, long long* gstep, unsigned long long* seq,
                               void* xbuf, int* err, long long timeout, long long* step_ts, int ts_ring,
                               const void* host_next, int next_steps, void* stage_next, void* const* peer_base, int W,
                               int rank, int gbf16, long long* phase_ts, int spread, int /*xmode: one-shot only*/,
                               hipStream_t stream) {
  using namespace dtfk::mlpx;
  Args a;
  a.stage = static_cast<const uint8_t*>(stage);
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
  a.xbuf = static_cast<uint8_t*>(xbuf);
  a.err = err;
  a.timeout = timeout;
  a.step_ts = step_ts;
  a.ts_ring = ts_ring > 0 ? ts_ring : 1;
  a.host_next = static_cast<const uint8_t*>(host_next);
  a.next_steps = next_steps;
  a.stage_next = static_cast<uint8_t*>(stage_next);
  a.peer_base = peer_base;
  a.W = W;
  a.rank = rank;
  a.gbf16 = gbf16;
  a.phase_ts = phase_ts;
  a.spread = spread;
  {
    const char* gm = getenv("DTF_GATHER_MODE");
    a.gmode = gm ? atoi(gm) : 0;
  }
  constexpr size_t lds = LDS_BYTES;
  static bool attr_set = false;
  const void* kerns[4] = {reinterpret_cast<const void*>(mlp_persist_x3<0, false>),
                          reinterpret_cast<const void*>(mlp_persist_x3<1, false>),
                          reinterpret_cast<const void*>(mlp_persist_x3<0, true>),
                          reinterpret_cast<const void*>(mlp_persist_x3<1, true>)};
  if (!attr_set) {
    for (const void* k : kerns) {
      const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
    attr_set = true;
  }
  const int which = (act == 0 ? 0 : 1) + (W > 1 ? 2 : 0);
  const int grid = spread ? GRID_SPREAD : GRID_PACKED + (NCOP - (GRID_PACKED - NJ) > 0 ? NCOP - (GRID_PACKED - NJ) : 0);
  switch (which) {
    case 0: hipLaunchKernelGGL((mlp_persist_x3<0, false>), dim3(grid), dim3(THREADS), lds, stream, a); break;
    case 1: hipLaunchKernelGGL((mlp_persist_x3<1, false>), dim3(grid), dim3(THREADS), lds, stream, a); break;
    case 2: hipLaunchKernelGGL((mlp_persist_x3<0, true>), dim3(grid), dim3(THREADS), lds, stream, a); break;
    default: hipLaunchKernelGGL((mlp_persist_x3<1, true>), dim3(grid), dim3(THREADS), lds, stream, a); break;
  }
  return hipGetLastError();
}

}  // extern "C"
