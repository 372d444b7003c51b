// Reached by: bench.py headline engine (PersistentMLPRunner), the resident Session engine (compat/resident.py), smoke(); tests/test_mlp_persist_gpu.py, test_resident_gpu.py
// Persistent, weight-stationary training kernel for the reference's 784-100-10
// MLP at the reference's precision: every product is an fp32 x fp32 MFMA
// (v_mfma_f32_16x16x4_f32, bitwise an fmaf chain), fp32 accumulate, fp32
// master weights held in VGPRs for the whole launch (example.py:77-118 is fp32
// end to end: x*W1+b1 -> sigmoid -> *W2+b2 -> softmax cross-entropy -> SGD).
//
// The f32-input MFMA runs at 1/16 of the f16 rate, so where the f16 engine
// (mlp_persist.hip) keeps a hidden block per CU, this one spreads each block's
// weights over 4 CUs:
//
//  * 28 compute workgroups (512 threads) c = (j, q): hidden block j (units
//    16j..16j+15, 7 blocks) x feature slice q (13, 12, 12, 12 tiles of 16
//    features; 49 tiles = 784 exactly).  Wave w owns local tiles w and w + 8 of
//    the slice: 4 fp32 VGPRs per lane and tile hold W1[16t+4g+e][16j+r]
//    (r = lane&15, g = lane>>4), which is at once its forward A operand
//    (k-step e) and the C layout of its weight gradient, so the SGD update is
//    in-register.
//  * per step:
//      P0  forward partial z^T[hidden][batch] of the wave's tiles for all 7
//          batch tiles (7 independent MFMA chains) -> LDS; wave w (batch tile
//          w) sums the 8 waves' partials in a fixed order.
//      E1  the slice partial of (j, batch tile w) goes to the 3 other slices of
//          block j as tagged 8-byte granules (the data is the flag); everyone
//          sums the 4 slices in slice order -> identical z in all 4.
//      P1  a2 = act(z/255 + b1), partial logits^T of block j (4 MFMAs; a2 is
//          the B operand straight from the accumulator layout).
//      E2  partial logits go to the workgroup of the same slice in every other
//          block; logits = b2 + sum_j (block order) -> identical in all 28.
//          softmax / cross-entropy / argmax, dz3, da2 = W2 dz3 (4 MFMAs),
//          dz2 = da2 * act' -> LDS.
//      P2  dW1 tiles = x^T dz2 over the batch (28 MFMAs per tile, x^T bytes from
//          the feature-major stage copy), W1 -= lr/(255 B) dW1 in registers;
//          wave 7 also: dW2 (28 MFMAs), db1, db2, metrics, update of the LDS
//          copies of W2[block j], b1[block j], b2 -- identical in every
//          workgroup that holds them (same inputs, same order).
//      P2 runs without a workgroup barrier: each 32-row batch chunk of the
//          weight gradient starts as soon as the heads of its batch tiles have
//          set their LDS flags; wave 7 signals the next step's stage with a flag.
//    One LDS barrier and two inter-workgroup edges per step; the data of
//    every edge is double-buffered by step parity and tagged with the global
//    exchange sequence number, so buffers are never reset between launches.
//  * x enters the MFMAs as exact integers 0..255 (v_cvt_f32_ubyte); the 1/255
//    pixel scale and the 1/B loss mean are applied to the fp32 sums.
//  * 16 COPIER workgroups pull chunk c+1 from pinned host memory over PCIe into
//    the other device stage (row-major x, feature-major x^T, labels) while the
//    compute workgroups run chunk c.
//  * N GPUs (MULTI, NW = the peer-table width W is unrolled for: 2, 4, 8):
//    after P2 every compute workgroup exchanges its gradient (its dW1 tiles +
//    the block's small gradients) with the same workgroup on every peer through
//    IPC-mapped uncached buffers -- 28 CUs per GPU carry the peer traffic, every
//    peer read a 16-B system-scope buffer load, all NW in flight at once -- and
//    sums the ranks in rank order (bit-identical replicas).  Publication order:
//    the slot bytes go to uncached (MTYPE UC) memory with plain stores, every
//    storing wave waits for them (vmcnt(0)), then a workgroup barrier, then ONE
//    relaxed system-scope flag store; consumers poll the flag with system-scope
//    loads and read the bytes with system-scope (sc0 sc1) loads, never served
//    from a cache of the reading device.
//
// Placement: packed (default) runs workgroup c as blockIdx 8c, so under the
// observed round-robin dispatch all 28 share one XCD and both edges stay in one
// L2 (plain stores); spread (several ranks on one GPU: tests) runs them as
// blocks 0..27.  A per-launch census of HW_REG_XCC_ID picks each edge's store
// flavour (plain if L2-local, write-through otherwise): speed only, never
// correctness.  Measured on MI355X (profiles/mlp_persist_f32_phases_r3_prologue.json,
// BENCH_r04.json): ~8.1 us/step; the per-step critical path is the two hops
// (~1.3 and ~1.9 us after the last producer) plus producer skew, not the MFMA
// phases (~0.5 forward + ~1.1 weight gradient).
//
// RES (the resident Session engine, compat/resident.py): ONE launch serves
// Session.run calls -- per run the copiers wait on a pinned-host doorbell, stage
// the run's record, and the compute workgroups stage it at the top of the step
// (no in-step prefetch: the next run's data does not exist yet); after the step
// the weights are written through to the graph's own variables and workgroup 0
// publishes loss / accuracy / global_step and a done count to pinned memory.
#include "common.h"

#include <atomic>

#include <cstdlib>
#include <cstring>

namespace dtfk {
namespace mlpf {

typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
typedef __attribute__((address_space(1))) unsigned gu32;

constexpr int DIN = 784, HID = 100, NCLS = 10;
constexpr int NJ = 7;              // hidden blocks of 16
constexpr int NQ = 4;              // feature slices: 13, 12, 12, 12 tiles of 16 features (49 = 784 / 16)
constexpr int NTW = 2;             // feature tiles per wave (local tiles w and w + 8)
constexpr int NBT = 7;             // batch tiles of 16 (B <= 112)
constexpr int BROWS = 16 * NBT;    // 112
constexpr int XTS = 128;           // x^T row stride (batch padded)
constexpr int NCOMP = NJ * NQ;     // 28 compute workgroups: one XCD
constexpr int THREADS = 512;
constexpr int NCOP = 16;           // copier workgroups
constexpr int NCOPR = 14;          // RES: copiers of one record (8 batch rows each)
constexpr int RES_LR_BYTE = 124;   // RES: the run's lr rides in the record's label area (B <= 112)
constexpr int GRID_PACKED = 8 * NCOMP;
constexpr int GRID_SPREAD = NCOMP + NCOP;
__host__ __device__ constexpr int tile0(int q) { return q == 0 ? 0 : 13 + 12 * (q - 1); }
__host__ __device__ constexpr int ntile(int q) { return q == 0 ? 13 : 12; }
constexpr int OFF_W2 = 78400, OFF_B1 = 79400, OFF_B2 = 79500;

// device stage record of one step
constexpr long long XROW_BYTES = (long long)BROWS * DIN;   // [112][784] u8, rows >= B zero
constexpr long long XT_BYTES = (long long)DIN * XTS;       // [784][128] u8, batch >= B zero
constexpr long long REC = XROW_BYTES + XT_BYTES + 128;     // + labels [128]

// exchange buffer (bytes): every payload float travels as an 8-byte granule
// {value, tag} (the data is the flag: no separate flag word, no drain before a
// flag, one hop); a slot = 64 lanes x 4 granules = 2 KB.
// E1 [2][NJ][NQ][NBT] slots, E2 [2][NQ][NBT][NJ] slots
constexpr int GSLOT = 2048;
constexpr long long E1_OFF = 0;
constexpr long long E2_OFF = E1_OFF + 2LL * NJ * NQ * NBT * GSLOT;
constexpr long long HDR_OFF = E2_OFF + 2LL * NQ * NBT * NJ * GSLOT;   // [64] u64 placement census
constexpr long long XBUF_BYTES = HDR_OFF + 64 * 8;

// IPC buffer of one rank (N GPUs): [flags: workgroup c at byte 64c][2 parities][28 slots]
// slot: dW1 entries of wave w, lane l at 16 (w 64 + l) (bf16: both tiles' 4 bf16 in
// one 16-B entry, 8 B when the wave has one tile) or 16 ((2 w + k) 64 + l) (fp32:
// one entry per tile k) | dW2 64 lanes x 16 B at IPC_SMALL | db1 / db2 (16 + 10)
// fp32 behind it.  Lanes of padding units and the zero dW2 columns are never
// stored or loaded: the bytes read from a peer are the payload
// (scripts/exchange_cost_model.py, tests/test_exchange_model_cpu.py).
// Two-shot mode adds a reduced area of the same slot layout (the owner's sums:
// bf16 for a bf16 payload, rounded once by the owner) behind the slots, and a
// second flag per workgroup at byte 64c + 8.
constexpr int IPC_FLAGS = 4096;
constexpr int IPC_SMALL = 8 * NTW * 64 * 16;
constexpr int IPC_SLOT = IPC_SMALL + 1024 + 128;
constexpr long long IPC_RED = IPC_FLAGS + 2LL * NCOMP * IPC_SLOT;
constexpr long long IPC_BYTES = IPC_RED + 2LL * NCOMP * IPC_SLOT;

// LDS carve (compute); the copier reuses the same dynamic allocation
constexpr int LS = BROWS + 4;                          // [16][LS] fp32 images (float4-aligned rows)
constexpr int L_ZBUF = 0;                              // [8 waves][NBT][64] f32x4 forward partials  57344
constexpr int L_A2T = L_ZBUF + 8 * NBT * 64 * 16;      // [16 hidden][LS] a2
constexpr int L_DZ2T = L_A2T + 16 * LS * 4;            // [16 hidden][LS] dz2
constexpr int L_DZ3T = L_DZ2T + 16 * LS * 4;           // [16 class][LS] dz3
constexpr int L_W2 = L_DZ3T + 16 * LS * 4;             // [16 hidden][16 class] W2 of block j
constexpr int L_B1 = L_W2 + 1024;                      // [16]
constexpr int L_B2 = L_B1 + 64;                        // [16]
constexpr int L_RDB1 = L_B2 + 64;                      // [8][16]
constexpr int L_RDB2 = L_RDB1 + 512;                   // [8][16]
constexpr int L_RMET = L_RDB2 + 512;                   // [8][2]
constexpr int L_FLAG = L_RMET + 64;
// x operands of one step for this workgroup's feature slice, staged by wave 7
// with LDS-DMA (global_load_lds_dwordx4, lane-linear 1 KiB pieces) instead of
// fragment-shaped global loads in every wave (16 cache lines per instruction:
// those loads were TA-bound, ~2.5 us of every step)
constexpr int XF_ROW = 13 * 16;                        // [112 rows][13 tiles x 16 features] u8
constexpr int L_XF = L_FLAG + 64;
constexpr int XF_CHUNKS = BROWS * 13;                  // 1456 x 16 B
constexpr int L_XT = L_XF + BROWS * XF_ROW;            // [208 features][128 batch] u8, 16-B chunks XOR-swizzled
constexpr int XT_CHUNKS = 13 * 16 * 8;                 // 1664 x 16 B
constexpr int L_LAB = L_XT + 13 * 16 * XTS;            // [128] labels
constexpr int PS = XTS + 8;                            // split mode: bf16 plane row stride (elements)
constexpr int L_DZP = L_LAB + 128;                     // split mode: [3 pieces][16 hidden][PS] dz2 bf16
constexpr int L_HFLAG = L_DZP + 3 * 16 * PS * 2;       // [8] head-done flags (step + 1) of waves 0..6
constexpr int L_DW2P = L_HFLAG + 64;                   // [7 batch tiles][64 lanes] f32x4 dW2 partials
constexpr int L_RLOSS = L_DW2P + NBT * 64 * 16;        // [2][128] per-row loss / correct of the step
constexpr int LDS_COMPUTE = L_RLOSS + 2 * 128 * 4;
static_assert(L_XF % 1024 == 0 && L_XT % 16 == 0 && L_LAB % 16 == 0, "LDS-DMA bases");
static_assert(L_DW2P % 16 == 0, "dW2 partials: 16-B lanes");
constexpr int CROW = DIN + 16;                         // copier LDS row stride (800)
constexpr int LDS_COPIER = BROWS * CROW;               // 89600
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
  int spread;               // placement: 0 packed on one XCD (default), 1 spread (several ranks per GPU)
  long long* phase_ts;      // optional phase stamps: [step < 64][workgroup 64][16] (wave 0 / wave 7, lane 0),
                            // then [64][workgroup 64][16] launch stamps (prologue / epilogue / copier)
  int gmode;                // gather: 0 probe one granule per producer, then load; 1-3 direct loads with
                            // no / short / long s_sleep between passes (DTF_GATHER_MODE, tuning)
  int xmode;                // N GPUs: 0 one-shot (every workgroup reads its slot from every peer),
                            // 1 two-shot (reduce-scatter by wave chunk, then all-gather of the sums)
  long long fault_step;     // fault injection (mlpf_set_fault(rank, step), tests of the bench's fallback):
  int fault_rank;           // that rank stops publishing its exchange flag from that global step on, a dead
                            // peer (-1: off; one skipped flag alone is absorbed: the flags are monotonic)
  // flat master layout: W1 at params[0..78400); W2 / b1 / b2 through their own
  // pointers (params + OFF_* for the flat trainer; a graph's own variables for the
  // resident Session engine)
  float* p_w2;
  float* p_b1;
  float* p_b2;
  // RESIDENT (Session engine, compat/resident.py): one launch serves many
  // Session.run calls.  Host -> device: a doorbell and 2 pinned record slots;
  // device -> host: metrics + a done count in pinned memory.  Exits by itself
  // after `idle` ticks without a doorbell (or on door < 0).
  const long long* door;    // pinned: runs made ready (run k ready when door > k); < 0: stop
  const uint8_t* host_recs; // pinned: 2 slots of rec_h bytes (B x 784 pixels, B labels)
  const float* host_lr;     // pinned: lr of each slot
  float* host_out;          // pinned: [loss, accuracy, global step] of the last run
  long long* host_done;     // pinned: runs completed
  long long* host_state;    // pinned: id of the launch that exited
  long long launch_id, run0, idle;
  unsigned census_tag;      // per-launch placement-census tag from the host (no device load in front of the census)
  void* gvar;               // the graph's global_step variable (kind 0 none, 1 f32, 2 i64, 3 i32, 4 f64)
  int gvar_kind;
  unsigned* dctr;           // device: [0] records staged, [8] runs released, [16] stop, [32] steps done
  long long* res_ts;        // profiling only (DTF_RESIDENT_STAMPS): [run % 64][8] resident per-run stamps
  int dbg;                  // profiling only (DTF_PERSIST_DBG): bit 0 = never stage the next step's x (wrong
                            // numerics; what the per-step LDS-DMA stage costs the hand-offs), bit 1 = head
                            // sub-phase stamps (slots 13-15, wave 0), bits 2 / 3 = stage (half) after the
                            // first head, bit 4 = longer sleeps in the chunk polls (tuning)
};

// resident per-run stamp (s_memrealtime, 100 MHz) -- profiling only: 0 copier 0
// saw the doorbell, 1 copier 0 staged its rows, 2 compute workgroup 0 saw the
// whole record staged, 3 record in LDS / registers, 4 step math done, 5
// variables written through, 6 every workgroup arrived, 7 done count published
#define RTS(k, slot)                                                                             \
  if (a.res_ts != nullptr) a.res_ts[((k) & 63) * 8 + (slot)] = (long long)__builtin_amdgcn_s_memrealtime();
// the same in compute: instrumented instantiations only
#define RTSC(k, slot) \
  if constexpr (INS) { RTS(k, slot); }
// phase stamp ph of step st (s_memrealtime, 100 MHz) -- profiling only: compiled
// into the instrumented instantiations (INS) alone, absent from production code
#define PH(ph)                                                                                   \
  if constexpr (INS) {                                                                           \
    if (a.phase_ts != nullptr && lane == 0 && st < 64)                                           \
      a.phase_ts[((long long)st * 64 + c) * 16 + (ph)] = (long long)__builtin_amdgcn_s_memrealtime(); \
  }
// DTF_PERSIST_DBG bit 1: wave 0 stamps the head's sub-phases into slots 13-15 (wave 7's stamps off)
#define PHX(ph) \
  if ((dbg & 2) != 0) { PH(ph); }
#define PH7(ph) \
  if ((dbg & 2) == 0) { PH(ph); }

// The exact three-way split v = hi + mid + lo by truncation, as fp32 bit
// patterns whose low 16 bits are zero: hi keeps v's top 8 significant bits, the
// remainder r = v - hi is exact (<= 16 bits), mid keeps its top 8, and r - mid
// has <= 8 significant bits, so lo is exact too (normal range).  4 VALU ops.
__device__ __forceinline__ void split3(float v, uint32_t& h, uint32_t& m, uint32_t& l) {
  h = __float_as_uint(v) & 0xffff0000u;
  const float r1 = v - __uint_as_float(h);
  m = __float_as_uint(r1) & 0xffff0000u;
  l = __float_as_uint(r1 - __uint_as_float(m));
}
// two split fp32 patterns -> one packed bf16 pair (upper halves)
__device__ __forceinline__ uint32_t hi2(uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x07060302u); }
// 8 fp32 -> the three bf16x8 pieces
__device__ __forceinline__ void split8(const float (&v)[8], bf16x8& H, bf16x8& M, bf16x8& L) {
  u32x4 ph, pm, pl;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t h0, m0, l0, h1, m1, l1;
    split3(v[2 * k], h0, m0, l0);
    split3(v[2 * k + 1], h1, m1, l1);
    ph[k] = hi2(h0, h1);
    pm[k] = hi2(m0, m1);
    pl[k] = hi2(l0, l1);
  }
  H = __builtin_bit_cast(bf16x8, ph);
  M = __builtin_bit_cast(bf16x8, pm);
  L = __builtin_bit_cast(bf16x8, pl);
}
// 8 pixel bytes (two dwords) -> 8 bf16, exact (<= 8 significant bits): upper half of the f32
__device__ __forceinline__ bf16x8 px8(uint32_t w0, uint32_t w1) {
  u32x4 o;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t wd = k < 2 ? w0 : w1;
    const int sh = (k & 1) * 16;
    const float f0 = (float)((wd >> sh) & 0xffu), f1 = (float)((wd >> (sh + 8)) & 0xffu);
    o[k] = hi2(__float_as_uint(f0), __float_as_uint(f1));
  }
  return __builtin_bit_cast(bf16x8, o);
}

// launch-level stamp k of workgroup slot wg (compute c, copier NCOMP + cid), one lane
#define PRO(wg, k)                                                                             \
  if (a.phase_ts != nullptr)                                                                   \
    a.phase_ts[((long long)64 * 64 + (wg)) * 16 + (k)] = (long long)__builtin_amdgcn_s_memrealtime();
// the same in compute: instrumented instantiations only
#define PROC(wg, k) \
  if constexpr (INS) { PRO(wg, k); }

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float ub(uint32_t w, int e) { return (float)((w >> (8 * e)) & 0xffu); }

__device__ __forceinline__ void lds_barrier() {   // orders LDS only: no vmcnt(0) on in-flight prefetches
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// one lane-linear LDS-DMA piece: lane l's 16 bytes at gsrc land at lds + 16 l
__device__ __forceinline__ void glds16(const void* gsrc, uint8_t* lds) {
  typedef __attribute__((address_space(1))) void gvoid;
  typedef __attribute__((address_space(3))) void lvoid;
  __builtin_amdgcn_global_load_lds((gvoid*)(gsrc), (lvoid*)(lds), 16, 0, 0);
}

// Granule hand-off through a buffer resource over a wave-uniform region (one
// descriptor per edge and step; slot and lane go into the VGPR offset).
// Producer: 4 floats -> 4 granules {value, tag} in two 16-byte write-through
// (sc1) stores; consumer: two L1-bypassing (sc1) 16-byte loads, valid when all
// four tags match (8-byte halves of a 16-byte sc1 store are observed untorn on
// gfx950: MI355X_MICROARCH.md "Valid forms", R2).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t region_rsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000);
}
// l2_local: every consumer shares the producer's XCD (verified at launch) ->
// plain stores, the lines stay in that L2 where the consumers' sc1 loads hit;
// otherwise write-through (sc1) stores, visible to other XCDs' sc1 loads.
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

// Gather the N granule slots slot(k) (k != skip) of this lane until every tag
// matches; part[skip] = own (constant-index selects only: a runtime index would
// demote the array to scratch).  `need` false: this lane takes no data (zeros;
// it still joins the wave-wide exit test).  Polling is cheap: lane k < N watches
// ONE granule of producer k (the last one lane `probe` writes) until it carries
// the tag; only then does every lane load its own granules -- and re-loads the
// few that were not there yet (no order between a producer's lanes).  A sweep
// of every lane over every slot per poll was ~5 MB of L2 traffic per round.
// false on timeout / error.
// (gm: the poll mode -- 1, direct loads without sleeps, in production; the
// instrumented instantiations take DTF_GATHER_MODE)
template <int N, bool INS, typename SlotOff>
__device__ __forceinline__ bool gather_gran(__amdgpu_buffer_rsrc_t rs, SlotOff slot, int skip, bool need, int probe,
                                            unsigned tag, f32x4 own, f32x4 (&part)[N], int lane, const Args& a) {
  const int gm = INS ? a.gmode : 1;
  bool have[N];
#pragma unroll
  for (int k = 0; k < N; ++k) {
    have[k] = (k == skip) || !need;
    part[k] = (k == skip) ? own : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  bool seen = lane >= N || lane == skip || gm != 0;
  for (;;) {
    asm volatile("" ::: "memory");   // re-load every pass (no loop-invariant hoisting)
    if (!seen) {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, slot(lane) + 32 * probe + 16, 0, 16);
      seen = v[1] == tag && v[3] == tag;
    }
    if (__all(seen)) break;
    if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > a.timeout ||
        __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
      if (lane == 0) atomicOr(a.err, 1);
      return false;
    }
  }
  // the clock and the error word are checked every 8th pass only: a pass is one
  // L2 round trip, and the consumer CU's memory queue is what a hand-off waits on
  for (int it = 1;; ++it) {
    asm volatile("" ::: "memory");
    bool all = true;
#pragma unroll
    for (int k = 0; k < N; ++k) {
      if (!have[k]) have[k] = get_gran(rs, slot(k) + 32 * lane, tag, part[k]);
      all = all && have[k];
    }
    if (__all(all)) return true;
    if (gm == 2) __builtin_amdgcn_s_sleep(2);
    else if (gm == 3) __builtin_amdgcn_s_sleep(8);
    if ((it & 7) == 0 && ((long long)__builtin_amdgcn_s_memrealtime() - t0 > a.timeout ||
                          __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)) {
      if (lane == 0) atomicOr(a.err, 1);
      return false;
    }
  }
}

// ------------------------------------------------------------------ N-GPU exchange loads
// Peer IPC buffers are read with 16-B (8-B / 4-B) system-scope loads (sc0 sc1:
// never served from a cache of this device) through a wave-uniform buffer
// resource per rank.  Loads of ranks outside `sel`, of ranks >= W and of
// masked lanes use an offset past the buffer's range: the buffer unit returns
// zero without touching memory, so the NW loads of a lane stay unconditional
// (no branch, no wait between them: all in flight at once) and only payload
// crosses the fabric.
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;
constexpr int SYS = 1 | 16;            // sc0 | sc1
constexpr int OOB_OFF = 0x7ffffff0;
// one resource per rank, built once per launch in SGPRs (the table entry is read
// by one lane and broadcast: a per-use vector load of the pointer would turn
// every peer load into a waterfall loop behind a vmcnt(0))
template <int NW>
struct PeerRs {
  __amdgpu_buffer_rsrc_t r[NW];
};
template <int NW>
__device__ __forceinline__ PeerRs<NW> peer_rsrcs(void* const* peers, int W) {
  PeerRs<NW> o;
#pragma unroll
  for (int r = 0; r < NW; ++r) {
    const unsigned long long u = reinterpret_cast<unsigned long long>(peers[r < W ? r : 0]);
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
    void* pp = reinterpret_cast<void*>(((unsigned long long)hi << 32) | lo);
    o.r[r] = __builtin_amdgcn_make_buffer_rsrc(pp, 0, (int)IPC_BYTES, 0x00020000);
  }
  return o;
}
__device__ __forceinline__ f32x4 unbf4(uint32_t lo, uint32_t hi) {
  return f32x4{__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u), __uint_as_float(hi << 16),
               __uint_as_float(hi & 0xffff0000u)};
}
__device__ __forceinline__ f32x4 round_bf16x4(f32x4 v) {
  const uint32_t lo = pack2bf(v[0], v[1]), hi = pack2bf(v[2], v[3]);
  return unbf4(lo, hi);
}
// Rank-order sum of this lane's dW1 entries over the W ranks (this rank's own
// term G0 / G1 from registers), GRP peer loads in flight per group.  BF: both
// tiles' bf16 in ONE 16-B entry at e0 (TWO false: the wave has one tile, 8 B);
// fp32: one 16-B entry per tile at e0 / e1.
template <int NW, int GRP, bool BF, bool TWO>
__device__ __forceinline__ void sum_entries(const PeerRs<NW>& prs, int W, int rank, int so, bool hv, int e0, int e1,
                                            f32x4& G0, f32x4& G1) {
  f32x4 S0 = {0.f, 0.f, 0.f, 0.f}, S1 = S0;
#pragma unroll
  for (int r0 = 0; r0 < NW; r0 += GRP) {
    if (r0 >= W) break;   // wave-uniform
    u32x4 v0[GRP], v1[GRP];
#pragma unroll
    for (int i = 0; i < GRP; ++i) {
      const int r = r0 + i;
      const bool on = r < W && r != rank && hv;
      const auto rs = prs.r[r];
      if constexpr (BF) {
        if constexpr (TWO) {
          v0[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, on ? so + e0 : OOB_OFF, 0, SYS);
        } else {
          const u32x2 h = __builtin_amdgcn_raw_buffer_load_b64(rs, on ? so + e0 : OOB_OFF, 0, SYS);
          v0[i] = u32x4{h[0], h[1], 0u, 0u};
        }
      } else {
        v0[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, on ? so + e0 : OOB_OFF, 0, SYS);
        if constexpr (TWO) v1[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, on ? so + e1 : OOB_OFF, 0, SYS);
      }
    }
#pragma unroll
    for (int i = 0; i < GRP; ++i) {
      const int r = r0 + i;
      if (r >= W) break;
      const bool me = r == rank;
      f32x4 P0, P1 = {0.f, 0.f, 0.f, 0.f};
      if constexpr (BF) {
        P0 = unbf4(v0[i][0], v0[i][1]);
        if constexpr (TWO) P1 = unbf4(v0[i][2], v0[i][3]);
      } else {
        P0 = __builtin_bit_cast(f32x4, v0[i]);
        if constexpr (TWO) P1 = __builtin_bit_cast(f32x4, v1[i]);
      }
      S0 += me ? G0 : P0;
      S1 += me ? G1 : P1;
    }
  }
  G0 = S0;
  G1 = S1;
}
// wave 7's small part: rank-order sums of the dW2 entry (16 B, lanes with data)
// and db1 / db2 (4 B)
template <int NW>
__device__ __forceinline__ void sum_small(const PeerRs<NW>& prs, int W, int rank, int so, bool dlane, bool blane,
                                          int lane, f32x4& D, float& gb) {
  u32x4 d[NW];
  uint32_t b[NW];
#pragma unroll
  for (int r = 0; r < NW; ++r) {
    const bool on = r < W && r != rank;
    const auto rs = prs.r[r];
    d[r] = __builtin_amdgcn_raw_buffer_load_b128(rs, (on && dlane) ? so + lane * 16 : OOB_OFF, 0, SYS);
    b[r] = __builtin_amdgcn_raw_buffer_load_b32(rs, (on && blane) ? so + 1024 + lane * 4 : OOB_OFF, 0, SYS);
  }
  f32x4 SD = {0.f, 0.f, 0.f, 0.f};
  float SB = 0.f;
#pragma unroll
  for (int r = 0; r < NW; ++r) {
    if (r >= W) break;
    const bool me = r == rank;
    SD += me ? D : __builtin_bit_cast(f32x4, d[r]);
    SB += me ? gb : __uint_as_float(b[r]);
  }
  D = SD;
  gb = SB;
}

// ------------------------------------------------------------------ copier
// task = one step of the next chunk: 112 rows of 784 pixels from the pinned host
// record into LDS (rows >= B zero), then the row-major image, the feature-major
// copy (4x4 byte transposes with v_perm) and the labels into the device stage.
__device__ void copier(const Args& a, int cid, uint8_t* smem) {
  const int tid = threadIdx.x;
  const int B = a.B;
  if (tid == 0) { PRO(NCOMP + cid, 0); }
  for (int st = cid; st < a.next_steps; st += NCOP) {
    const uint8_t* src = a.host_next + (long long)st * a.rec_h;
    uint8_t* dst = a.stage_next + (long long)st * REC;
    constexpr int C16 = DIN / 16;   // 49
    for (int k = tid; k < BROWS * C16; k += THREADS) {
      const int row = k / C16, c = k % C16;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (row < B) v = reinterpret_cast<const uint4*>(src)[row * C16 + c];
      *reinterpret_cast<uint4*>(smem + row * CROW + 16 * c) = v;
    }
    if (tid < 128) dst[XROW_BYTES + XT_BYTES + tid] = tid < B ? src[(long long)B * DIN + tid] : (uint8_t)0;
    __syncthreads();
    for (int k = tid; k < BROWS * C16; k += THREADS) {
      const int row = k / C16, c = k % C16;
      reinterpret_cast<uint4*>(dst)[row * C16 + c] = *reinterpret_cast<const uint4*>(smem + row * CROW + 16 * c);
    }
    uint8_t* xt = dst + XROW_BYTES;
    for (int k = tid; k < (DIN / 4) * (BROWS / 4); k += THREADS) {
      const int fq = k / (BROWS / 4), rq = k % (BROWS / 4);
      const uint8_t* p = smem + 4 * rq * CROW + 4 * fq;
      const uint32_t r0 = *reinterpret_cast<const uint32_t*>(p);
      const uint32_t r1 = *reinterpret_cast<const uint32_t*>(p + CROW);
      const uint32_t r2 = *reinterpret_cast<const uint32_t*>(p + 2 * CROW);
      const uint32_t r3 = *reinterpret_cast<const uint32_t*>(p + 3 * CROW);
      // t01 = [r0.b0 r1.b0 r0.b1 r1.b1], u01 = [r0.b2 r1.b2 r0.b3 r1.b3] (likewise r2/r3)
      const uint32_t t01 = __builtin_amdgcn_perm(r1, r0, 0x05010400u);
      const uint32_t t23 = __builtin_amdgcn_perm(r3, r2, 0x05010400u);
      const uint32_t u01 = __builtin_amdgcn_perm(r1, r0, 0x07030602u);
      const uint32_t u23 = __builtin_amdgcn_perm(r3, r2, 0x07030602u);
      uint32_t* o = reinterpret_cast<uint32_t*>(xt + (long long)(4 * fq) * XTS + 4 * rq);
      o[0] = __builtin_amdgcn_perm(t23, t01, 0x05040100u);             // feature 4fq+0, batch 4rq..4rq+3
      o[XTS / 4] = __builtin_amdgcn_perm(t23, t01, 0x07060302u);       // 4fq+1
      o[2 * XTS / 4] = __builtin_amdgcn_perm(u23, u01, 0x05040100u);   // 4fq+2
      o[3 * XTS / 4] = __builtin_amdgcn_perm(u23, u01, 0x07060302u);   // 4fq+3
    }
    __syncthreads();
  }
  if (tid == 0) { PRO(NCOMP + cid, 1); }
}

// RES copier: copier 0 watches the doorbell (system-scope loads of pinned host
// memory) and releases run k to the others, or stops the launch after `idle`
// ticks without one (or on door < 0) and reports that to the host; copiers
// 0..13 each move 8 batch rows of the run's pinned record into device stage
// slot (st & 1): row-major image, the x^T bytes of those rows (4x4 v_perm
// transposes), labels + lr (copier 0); every store write-through (sc1), then
// every wave's vmcnt(0), the barrier and one agent add to the staged count.
__device__ void copier_res(const Args& a, int cid, uint8_t* smem) {
  if (cid >= NCOPR) return;
  const int tid = threadIdx.x;
  constexpr int RR = 8;                                   // rows per copier
  int* dec = reinterpret_cast<int*>(smem + RR * CROW);
  const int B = a.B;
  const int hb = (int)(2 * a.rec_h);
  const auto hrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.host_recs), 0, hb, 0x00020000);
  for (int st = 0;; ++st) {
    const long long k = a.run0 + st;
    if (tid == 0) {
      // every copier watches the doorbell (no second hop through a device flag);
      // copier 0 alone may stop the launch: its rows complete every record, so a
      // run it did not take never reaches the compute workgroups' staged count
      int d = 1;
      const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
      const long long lim = cid == 0 ? a.idle : a.idle + a.timeout;
      for (;;) {
        const long long v = __hip_atomic_load(a.door, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (v < 0) { d = 0; break; }
        if (v > k) break;
        if (cid != 0 && __hip_atomic_load(a.dctr + 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) { d = 0; break; }
        if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > lim) { d = 0; break; }
        __builtin_amdgcn_s_sleep(1);
      }
      if (cid == 0 && !d) __hip_atomic_store(a.dctr + 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cid == 0 && d) { RTS(k, 0); }
      *dec = d;
    }
    __syncthreads();
    if (*dec == 0) break;
    const int slot = (int)(k & 1);
    const int hbase = slot * (int)a.rec_h;
    const int r0 = RR * cid;
    uint8_t* dst = const_cast<uint8_t*>(a.stage) + (long long)(st & 1) * REC;
    constexpr int C16 = DIN / 16;   // 49
    // pinned rows -> LDS (rows >= B zero): 16-B system-scope loads, a thread's
    // NLD loads all issued before the first LDS store (one host-memory round
    // trip, not NLD of them in series)
    constexpr int NLD = (RR * C16 + THREADS - 1) / THREADS;
    u32x4 hv[NLD];
    uint32_t lv = 0;   // copier 0, threads < 32: a label dword or the run's lr
    if (cid == 0 && tid < 32) {
      if (4 * tid == RES_LR_BYTE)
        lv = __float_as_uint(__hip_atomic_load(a.host_lr + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
      else
        lv = __builtin_amdgcn_raw_buffer_load_b32(hrs, 4 * tid < B ? hbase + B * DIN + 4 * tid : OOB_OFF, 0, SYS);
    }
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int t = tid + i * THREADS;
      const int rr = t / C16, cc = t % C16;
      const int row = r0 + rr;
      hv[i] = __builtin_amdgcn_raw_buffer_load_b128(hrs, (t < RR * C16 && row < B) ? hbase + row * DIN + 16 * cc : OOB_OFF,
                                                    0, SYS);
    }
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int t = tid + i * THREADS;
      if (t < RR * C16) *reinterpret_cast<u32x4*>(smem + (t / C16) * CROW + 16 * (t % C16)) = hv[i];
    }
    __syncthreads();
    for (int t = tid; t < RR * C16; t += THREADS) {
      const int rr = t / C16, cc = t % C16;
      const u32x4 v = *reinterpret_cast<const u32x4*>(smem + rr * CROW + 16 * cc);
      __builtin_amdgcn_raw_buffer_store_b128(v, region_rsrc(dst, (int)REC), (r0 + rr) * DIN + 16 * cc, 0, 16);
    }
    // x^T: feature quad fq x row quad rq (2 per copier) -> 4 dwords of 4 batch bytes
    for (int t = tid; t < (DIN / 4) * (RR / 4); t += THREADS) {
      const int fq = t >> 1, rq = t & 1;
      const uint8_t* p = smem + 4 * rq * CROW + 4 * fq;
      const uint32_t q0 = *reinterpret_cast<const uint32_t*>(p);
      const uint32_t q1 = *reinterpret_cast<const uint32_t*>(p + CROW);
      const uint32_t q2 = *reinterpret_cast<const uint32_t*>(p + 2 * CROW);
      const uint32_t q3 = *reinterpret_cast<const uint32_t*>(p + 3 * CROW);
      const uint32_t t01 = __builtin_amdgcn_perm(q1, q0, 0x05010400u);
      const uint32_t t23 = __builtin_amdgcn_perm(q3, q2, 0x05010400u);
      const uint32_t u01 = __builtin_amdgcn_perm(q1, q0, 0x07030602u);
      const uint32_t u23 = __builtin_amdgcn_perm(q3, q2, 0x07030602u);
      const auto rs = region_rsrc(dst, (int)REC);
      const int o = (int)XROW_BYTES + (4 * fq) * XTS + r0 + 4 * rq;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_amdgcn_perm(t23, t01, 0x05040100u), rs, o, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_amdgcn_perm(t23, t01, 0x07060302u), rs, o + XTS, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_amdgcn_perm(u23, u01, 0x05040100u), rs, o + 2 * XTS, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_amdgcn_perm(u23, u01, 0x07060302u), rs, o + 3 * XTS, 0, 16);
    }
    if (cid == 0 && tid < 32) {   // labels (dwords 0..27) and the run's lr (byte RES_LR_BYTE), loaded with the rows
      uint32_t v = lv;
      if (4 * tid != RES_LR_BYTE) {
        const int nv = B - 4 * tid;   // valid label bytes in this dword
        if (nv < 4) v = nv <= 0 ? 0u : (v & ((1u << (8 * nv)) - 1u));
      }
      __builtin_amdgcn_raw_buffer_store_b32(v, region_rsrc(dst, (int)REC), (int)(XROW_BYTES + XT_BYTES) + 4 * tid, 0,
                                            16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __hip_atomic_fetch_add(a.dctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cid == 0) { RTS(k, 1); }
    }
  }
  if (cid == 0 && tid == 0)   // no further run is taken by this launch
    __hip_atomic_store(a.host_state, a.launch_id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ------------------------------------------------------------------ compute
// ACT 0 sigmoid, 1 relu; MULTI: N-GPU gradient exchange; SPLIT: the two big
// GEMMs (forward x W1, weight gradient x^T dz2) on bf16 MFMA through the exact
// three-way split of their fp32 operand (pixels are exact in bf16), so every
// product is exact and accumulates in fp32 -- 16x16x32 bf16 MFMAs at 8x the
// f32-MFMA rate; the head stays on f32-input MFMA
// EXP (timing experiment only, never the production instantiations; DTF_PERSIST_EXP,
// scripts/probes/decomposition_sim.sh): the per-workgroup work of the 14- (EXP 2)
// and 7-workgroup (EXP 4) decompositions on this 28-workgroup engine -- every
// forward / weight-gradient MFMA chain and the next-step stage DMA run EXP times
// (a 2x / 4x wider feature slice), E1 gathers 2 slices (EXP 2) or disappears
// (EXP 4).  The sums are rescaled, so training still runs, but the numerics are
// not the reference's: stamps and step times only.
// INS: the instrumented build (phase stamps, DTF_PERSIST_DBG / DTF_GATHER_MODE
// knobs) -- production instantiations carry none of that code
template <int ACT, int NW, bool SPLIT, bool RES, int EXP = 0, bool INS = false>
__device__ void compute(const Args& a, const int j, const int q, uint8_t* smem) {
  constexpr int XR = EXP > 1 ? EXP : 1;
  const int dbg = INS ? a.dbg : 0;
  constexpr bool MULTI = NW > 1;
  // w through readfirstlane: the compiler then knows it is wave-uniform, so the
  // per-wave conditions (w == 7, w < NBT, the tile-valid flags) are scalar
  // branches, not 64-bit lane masks hoisted out of the step loop
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int c = j * NQ + q;
  const int B = a.B;
  f32x4* zbuf = reinterpret_cast<f32x4*>(smem + L_ZBUF);
  float* a2T = reinterpret_cast<float*>(smem + L_A2T);
  float* dz2T = reinterpret_cast<float*>(smem + L_DZ2T);
  float* dz3T = reinterpret_cast<float*>(smem + L_DZ3T);
  float* w2s = reinterpret_cast<float*>(smem + L_W2);
  float* b1s = reinterpret_cast<float*>(smem + L_B1);
  float* b2s = reinterpret_cast<float*>(smem + L_B2);
  float* rdb2 = reinterpret_cast<float*>(smem + L_RDB2);
  int* abort_flag = reinterpret_cast<int*>(smem + L_FLAG);
  int* census = abort_flag + 1;
  uint16_t* dzp = reinterpret_cast<uint16_t*>(smem + L_DZP);
  if (tid == 0) { PROC(c, 0); }

  // ---- load state: every global load of the prologue is issued first (the
  // master weights, the small parameters into registers, the step / sequence /
  // lr scalars); the LDS stores that consume them come after the LDS clears, so
  // no store waits on a load before the next load is even issued (~2 us of every
  // launch when the W2 / b loads fed LDS stores ahead of the W1 loads)
  const int hid = 16 * j + r;       // this lane's hidden unit in the W1 / dW1 layouts
  const bool hv = hid < HID;
  // wave w owns local feature tiles w and w + 8 of the slice (global tile ft[k])
  const int nt = ntile(q);
  // (constant-index scalars, not arrays a lambda captures: those would live in scratch)
  const bool tv0 = w < nt, tv1 = w + 8 < nt;
  const int ft0 = tile0(q) + w, ft1 = tile0(q) + (tv1 ? w + 8 : 0);
  auto tvk = [=](int k) { return k ? tv1 : tv0; };
  auto ftk = [=](int k) { return k ? ft1 : ft0; };
  // W1 slice: 16-byte loads of 4 consecutive hidden units of one feature row
  // (the 16 lanes of a lane group cover a 4-row x 16-unit block: 4 cache lines
  // per load), transposed across those lanes after the prologue's drain so lane
  // (r, g) holds unit 16j + r of rows 4g..4g+3 -- the accumulator layout of dW1.
  // (4-byte column loads touched 64 lines per wave instruction: ~2 us of issue
  // at the top of every launch.)
  // (RES keeps the column loads: the transposes' registers spill there, and its
  // prologue runs once per idle period, not once per timed launch)
  float Wt[NTW][4];
  f32x4 wld[NTW];
  if constexpr (RES) {
#pragma unroll
    for (int k = 0; k < NTW; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        Wt[k][e] = (tvk(k) && hv) ? a.params[(16 * ftk(k) + 4 * g + e) * HID + hid] : 0.f;
  } else if constexpr (MULTI) {   // (N GPUs: the branchy loads -- the unconditional ones below spill there)
    const int u0 = 16 * j + 4 * (r & 3);
#pragma unroll
    for (int k = 0; k < NTW; ++k)
      wld[k] = (tvk(k) && u0 < HID)
                   ? *reinterpret_cast<const f32x4*>(a.params + (16 * ftk(k) + 4 * g + (r >> 2)) * HID + u0)
                   : f32x4{0.f, 0.f, 0.f, 0.f};
  } else {
    // unconditional buffer loads (an absent tile / padding unit reads past the
    // range: zero, no branch) -- a conditional load's result merged at the branch
    // end cost a vmcnt(0) right behind it, one serial HBM round trip per launch
    const int u0 = 16 * j + 4 * (r & 3);           // units 4(r&3)..+3 of block j, row 4g + (r >> 2)
    const auto rw1 = __builtin_amdgcn_make_buffer_rsrc(a.params, 0, DIN * HID * 4, 0x00020000);
#pragma unroll
    for (int k = 0; k < NTW; ++k)
      wld[k] = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                     rw1, (tvk(k) && u0 < HID) ? ((16 * ftk(k) + 4 * g + (r >> 2)) * HID + u0) * 4 : OOB_OFF, 0, 0));
  }
  // this thread's W2 / b1 / b2 entry (threads < 288): three unconditional loads,
  // at most one in range, OR-ed (the others read zero)
  float pv = 0.f;
  if constexpr (MULTI) {
    if (tid < 256) {
      const int n = tid >> 4, cl = tid & 15;
      const int hn = 16 * j + n;
      pv = (hn < HID && cl < NCLS) ? a.p_w2[hn * NCLS + cl] : 0.f;
    } else if (tid < 272) {
      const int hn = 16 * j + (tid - 256);
      pv = hn < HID ? a.p_b1[hn] : 0.f;
    } else if (tid < 288) {
      const int cl = tid - 272;
      pv = cl < NCLS ? a.p_b2[cl] : 0.f;
    }
  } else {
    const int n = tid >> 4, cl = tid & 15, hn = 16 * j + n, hb = 16 * j + (tid - 256), c2 = tid - 272;
    const auto rw2 = __builtin_amdgcn_make_buffer_rsrc(a.p_w2, 0, HID * NCLS * 4, 0x00020000);
    const auto rb1 = __builtin_amdgcn_make_buffer_rsrc(a.p_b1, 0, HID * 4, 0x00020000);
    const auto rb2 = __builtin_amdgcn_make_buffer_rsrc(a.p_b2, 0, NCLS * 4, 0x00020000);
    const uint32_t v0 =
        __builtin_amdgcn_raw_buffer_load_b32(rw2, (tid < 256 && hn < HID && cl < NCLS) ? (hn * NCLS + cl) * 4 : OOB_OFF, 0, 0);
    const uint32_t v1 =
        __builtin_amdgcn_raw_buffer_load_b32(rb1, (tid >= 256 && tid < 272 && hb < HID) ? hb * 4 : OOB_OFF, 0, 0);
    const uint32_t v2 =
        __builtin_amdgcn_raw_buffer_load_b32(rb2, (tid >= 272 && tid < 288 && c2 < NCLS) ? c2 * 4 : OOB_OFF, 0, 0);
    pv = __uint_as_float(v0 | v1 | v2);
  }
  // the step / sequence / lr scalars stay in VGPRs until the prologue's drain
  // (converted to SGPRs there): a readfirstlane right behind each load waited
  // for it, another serial round trip in front of the stage and census
  unsigned long long seq0 = *a.seq;
  long long gstep0 = *a.gstep;
  float lr = *a.lr;
  // the placement-census entry goes out before anything waits on a load: its
  // tag is the host's per-launch tag, not the device sequence counter (whose
  // load, with the lr / parameter waits ahead of the LDS stores, held every
  // workgroup's entry back ~2 us per launch)
  const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20) & 15u;
  unsigned long long* hdr = reinterpret_cast<unsigned long long*>(a.xbuf + HDR_OFF);
  const unsigned tag0 = a.census_tag;
  if (tid == 0)
    __hip_atomic_store(hdr + c, ((unsigned long long)tag0 << 32) | xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int k = tid; k < 3 * 16 * LS; k += THREADS) a2T[k] = 0.f;   // a2T, dz2T, dz3T (batch pad stays 0)
  if constexpr (SPLIT)
    for (int k = tid; k < 3 * 16 * PS; k += THREADS) dzp[k] = (uint16_t)0;   // dz2 planes (batch pad 0)
  const bool failed_in = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;

  // x operands of the wave's feature tiles (registers, read from the LDS stage):
  //  xf[k][bt]: row 16bt+r, features 16ft+4g..+3 (forward B operand)
  //  xt[k][s] : feature 16ft+r, batch 16s+4g..+3 (weight-gradient A operand);
  //             SPLIT: dwords 2c, 2c+1 = batch 32c+8g..+7 (c < 4, batch >= 112 zero)
  //  lab      : label of batch row 16w+r (head, waves < 7)
  constexpr int XTN = SPLIT ? 8 : NBT;
  uint32_t xf[NTW][NBT], xt[NTW][XTN];
  int lab = 0;
  // local tile of k (an absent second tile reads local tile 0: staged, never used)
  auto tlk = [=](int k) { return k ? (tv1 ? w + 8 : 0) : w; };
  // wave 7: step st's slice -> LDS.  x rows: lane-linear [row][13 tiles] (rows of
  // 208 B, conflict-free reads); x^T rows of the slice's features are contiguous
  // in the stage, their 16-B batch chunks XOR-swizzled by (feature >> 1) & 7 on the
  // source address so the fragment reads below are conflict-free
  auto stage_x = [&](int st, int n0, int dn) {   // pieces n0, n0 + dn, ... of each part
    const uint8_t* rec = a.stage + (long long)st * REC;
    const uint8_t* xr = rec + 16 * tile0(q);
#pragma unroll 1   // a rolled loop: unrolled, the 49 pieces' addresses get hoisted out of the step loop
    for (int n = n0; n < (XF_CHUNKS + 63) / 64; n += dn) {
      const int k = 64 * n + lane;
      // q = 3's 13th tile reads the next row's first 16 B (inside the record): unused
      if (k < XF_CHUNKS) glds16(xr + (k / 13) * DIN + 16 * (k % 13), smem + L_XF + 1024 * n);
    }
    const uint8_t* xtb = rec + XROW_BYTES + (long long)(16 * tile0(q)) * XTS;
#pragma unroll 1
    for (int n = n0; n < XT_CHUNKS / 64; n += dn) {
      const int f = 8 * n + (lane >> 3);
      const int s = (lane & 7) ^ ((f >> 1) & 7);
      if (f < 16 * nt) glds16(xtb + f * XTS + 16 * s, smem + L_XT + 1024 * n);
    }
    if (n0 == 0 && lane < 8) glds16(rec + XROW_BYTES + XT_BYTES + 16 * lane, smem + L_LAB);
  };
  auto read_xf = [&]() {
#pragma unroll
    for (int k = 0; k < NTW; ++k)
#pragma unroll
      for (int b = 0; b < NBT; ++b)
        xf[k][b] = *reinterpret_cast<const uint32_t*>(smem + L_XF + (16 * b + r) * XF_ROW + 16 * tlk(k) + 4 * g);
    lab = smem[L_LAB + 16 * (w < NBT ? w : NBT - 1) + r];
  };
  auto read_xt = [&]() {
#pragma unroll
    for (int k = 0; k < NTW; ++k) {
      const int f = 16 * tlk(k) + r;
      if constexpr (SPLIT) {
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
          const uint2 v = *reinterpret_cast<const uint2*>(
              smem + L_XT + f * XTS + 16 * ((2 * cc + (g >> 1)) ^ ((f >> 1) & 7)) + 8 * (g & 1));
          xt[k][2 * cc] = v.x;
          xt[k][2 * cc + 1] = v.y;
        }
      } else {
#pragma unroll
        for (int s = 0; s < NBT; ++s)
          xt[k][s] = *reinterpret_cast<const uint32_t*>(smem + L_XT + f * XTS + 16 * (s ^ ((f >> 1) & 7)) + 4 * g);
      }
    }
  };
  // Prologue, all latency overlapped (it was three serial phases, ~6 us per
  // launch): the census entry goes out first, the first step's x stage is
  // issued (LDS-DMA) while the parameter loads above are still in flight, and
  // wave 0 polls the census meanwhile; one drain + barrier then covers all three.
  if (tid == 0) { PROC(c, 4); }
  // ---- placement census: E1 group (the NQ slices of block j) and E2 group (the
  // NJ blocks of slice q) each on this workgroup's XCD -> that edge stays in one
  // L2 (plain stores).  Decided per launch from HW_REG_XCC_ID, never assumed.
  // (this workgroup's entry was stored above, right after the loads were issued)
  if constexpr (!RES) stage_x(0, w, 8);   // the first step's stage: every wave a share (RES: per run)
  if (w == 0) {   // lane cc watches workgroup cc's entry: all 28 polls in flight at once
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    unsigned long long v = 0;
    bool seen = lane >= NCOMP, bad = false;
    for (;;) {
      if (!seen) {
        v = __hip_atomic_load(hdr + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        seen = (unsigned)(v >> 32) == tag0;
      }
      if (__all(seen)) break;
      if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) {
        if (lane == 0) atomicOr(a.err, 1);
        bad = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    const bool off = lane < NCOMP && (unsigned)v != xcc;   // workgroup `lane` on another XCD
    const bool e1 = !__any(off && lane / NQ == j);
    const bool e2 = !__any(off && lane % NQ == q);
    if (lane == 0) *census = bad ? -1 : ((e1 ? 1 : 0) | (e2 ? 2 : 0));
  }
  // the small parameters' LDS stores wait for their loads: placed after the
  // census entry and the stage DMA are out
  if (tid < 256) {
    w2s[tid] = pv;
  } else if (tid < 272) {
    b1s[tid - 256] = pv;
  } else if (tid < 288) {
    b2s[tid - 272] = pv;
  } else if (tid == 288) {
    *abort_flag = 0;
  } else if (tid >= 296 && tid < 304) {
    reinterpret_cast<int*>(smem + L_HFLAG)[tid - 296] = 0;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // parameter loads + the first stage landed
  if constexpr (!MULTI) {
    asm volatile("" : "+v"(seq0), "+v"(gstep0), "+v"(lr));
    seq0 = ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(seq0 >> 32)) << 32) |
           __builtin_amdgcn_readfirstlane((unsigned)seq0);
    gstep0 = (long long)(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)((unsigned long long)gstep0 >> 32))
                          << 32) |
                         __builtin_amdgcn_readfirstlane((unsigned)gstep0));
  }
  double gvar0 = 0.0;   // RES: the graph's global_step at launch
  if constexpr (RES) {
    if (a.gvar_kind == 1) gvar0 = *static_cast<const float*>(a.gvar);
    else if (a.gvar_kind == 2) gvar0 = (double)*static_cast<const long long*>(a.gvar);
    else if (a.gvar_kind == 3) gvar0 = *static_cast<const int*>(a.gvar);
    else if (a.gvar_kind == 4) gvar0 = *static_cast<const double*>(a.gvar);
    else gvar0 = (double)gstep0;
  }
  // the 4x4 transposes of the W1 blocks in 4 rounds of one lane permute:
  // in round t the lane that loaded row e_s offers component (e_s + t) & 3, and
  // lane r (unit 4b + m) takes row (m - t) & 3 from lane 4((m - t) & 3) + b --
  // which offers exactly component m
#pragma unroll
  for (int k = 0; k < NTW && !RES; ++k) {
    const int m = r & 3, b = r >> 2;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int cs = (b + t) & 3;          // as a source: this lane loaded row b (= r >> 2)
      const float v = cs == 0 ? wld[k][0] : (cs == 1 ? wld[k][1] : (cs == 2 ? wld[k][2] : wld[k][3]));
      const int e = (m - t) & 3;
      const float got = __shfl(v, 16 * g + 4 * e + b);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (q == e) Wt[k][q] = got;
    }
  }
  __syncthreads();
  float lrB = lr / (float)(B * (MULTI ? a.W : 1));   // RES: per run (the record's lr)
  float lrX = lrB * (1.f / 255.f);
  // an earlier launch failed (err set): nothing runs.  Checked only here, so the
  // wait for that load does not serialize the parameter loads behind it
  if (failed_in || *census < 0) return;
  const bool l2_e1 = (*census & 1) != 0;
  const bool l2_e2 = (*census & 2) != 0;
  if (tid == 0) { PROC(c, 1); }
  if constexpr (!RES) {
    read_xf();
    read_xt();
  }
  if (tid == 0) { PROC(c, 2); }

  // RES: the run's record -> LDS at the top of every step.  The copiers stored it
  // write-through (sc1) and each added to the staged count after its waves'
  // vmcnt(0) + barrier; one lane polls that count with sc1 loads, the workgroup
  // barrier follows, and every load of the record is an sc1 load to registers
  // (MI355X_MICROARCH.md "Valid forms", first table row) -> the LDS layout of
  // stage_x (x^T chunks XOR-swizzled).  false: stop (idle / door < 0 / error).
  auto res_stage = [&](int st) -> bool {
    int* rflag = abort_flag + 2;
    if (tid == 0) {
      const unsigned need = (unsigned)NCOPR * (unsigned)(st + 1);
      const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
      int v = 1;
      for (;;) {
        if (__hip_atomic_load(a.dctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= need) break;
        if (__hip_atomic_load(a.dctr + 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) { v = 0; break; }
        if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > a.idle + a.timeout) {   // copiers gone: bounded
          atomicOr(a.err, 4);
          v = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      *rflag = v;
    }
    __syncthreads();
    if (*rflag == 0) return false;
    if (c == 0 && tid == 0) { RTSC(a.run0 + st, 2); }
    const auto rs = region_rsrc(a.stage + (long long)(st & 1) * REC, (int)REC);
    const int xr0 = 16 * tile0(q);
#pragma unroll 4
    for (int k = tid; k < XF_CHUNKS; k += THREADS) {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (k / 13) * DIN + 16 * (k % 13) + xr0, 0, 16);
      *reinterpret_cast<u32x4*>(smem + L_XF + 16 * k) = v;
    }
    const int xt0 = (int)XROW_BYTES + 16 * tile0(q) * XTS;
#pragma unroll 4
    for (int k = tid; k < XT_CHUNKS; k += THREADS) {
      const int f = k >> 3;
      if (f < 16 * nt) {
        const int sw = (k & 7) ^ ((f >> 1) & 7);
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, xt0 + f * XTS + 16 * sw, 0, 16);
        *reinterpret_cast<u32x4*>(smem + L_XT + 16 * k) = v;
      }
    }
    if (tid < 8) {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(XROW_BYTES + XT_BYTES) + 16 * tid, 0, 16);
      *reinterpret_cast<u32x4*>(smem + L_LAB + 16 * tid) = v;
    }
    __syncthreads();
    read_xf();
    read_xt();
    if (c == 0 && tid == 0) { RTSC(a.run0 + st, 3); }
    const float lr_run = *reinterpret_cast<const float*>(smem + L_LAB + RES_LR_BYTE);
    lrB = lr_run / (float)B;
    lrX = lrB * (1.f / 255.f);
    return true;
  };
  int st_done = 0;
  // fp32 master -> memory: W1 entries of this lane; W2 / b1 / b2 of block j from
  // the q == 0 workgroups, b2 from workgroup 0.  wt: write-through (sc1) stores
  // (RES: every step, read by torch kernels / copies between runs)
  auto write_params = [&](bool wt) {
    auto put = [wt](float* p, float v) {
      if (wt) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else *p = v;
    };
    if (hv) {
#pragma unroll
      for (int k = 0; k < NTW; ++k)
        if (tvk(k)) {
#pragma unroll
          for (int e = 0; e < 4; ++e) put(a.params + (16 * ftk(k) + 4 * g + e) * HID + hid, Wt[k][e]);
        }
    }
    if (q == 0) {
      if (tid < 256) {
        const int n = tid >> 4, cl = tid & 15;
        const int hn = 16 * j + n;
        if (hn < HID && cl < NCLS) put(a.p_w2 + hn * NCLS + cl, w2s[tid]);
      } else if (tid < 272) {
        const int hn = 16 * j + (tid - 256);
        if (hn < HID) put(a.p_b1 + hn, b1s[tid - 256]);
      }
    }
    if (c == 0 && tid >= 272 && tid < 272 + NCLS) put(a.p_b2 + (tid - 272), b2s[tid - 272]);
  };

  const PeerRs<NW> prs = peer_rsrcs<NW>(a.peer_base, MULTI ? a.W : 1);
  bool aborted = false;
  for (int st = 0; st < a.nsteps; ++st) {
    if constexpr (RES) {
      if (!res_stage(st)) break;
    }
    // this workgroup's block / slice as opaque values per step: the gathers'
    // slot selects (k == skip) would otherwise be hoisted out of the step loop as
    // ten 64-bit lane masks held across it (SGPR spills, a v_readlane per use)
    int jq[2] = {j, q};
    asm volatile("" : "+s"(jq[0]), "+s"(jq[1]));
    const unsigned long long sq = seq0 + (unsigned long long)st + 1ull;
    const unsigned tag = (unsigned)sq;
    const int par = (int)(sq & 1ull);
    if (c == 0 && tid == 0 && a.step_ts != nullptr)
      a.step_ts[(gstep0 + st) % a.ts_ring] = (long long)__builtin_amdgcn_s_memrealtime();
    if (w == 0) { PH(0); }
    if (w == 7) { PH7(14); }

    // ---------------- P0: forward partial of the wave's tiles, all batch tiles
    {
      f32x4 acc[NBT];
#pragma unroll
      for (int b = 0; b < NBT; ++b) acc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (SPLIT) {
        // K = 32: k = 8g + i -> tile i >> 2, feature 4g + (i & 3) -- the A piece is this
        // lane's 8 master weights, the B operand its two x dwords (an absent second
        // tile has zero weights); pieces lo, mid, hi (small terms first)
        float wv[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) wv[i] = Wt[i >> 2][i & 3];
        bf16x8 Ah, Am, Al;
        split8(wv, Ah, Am, Al);
        bf16x8 X[NBT];
#pragma unroll
        for (int b = 0; b < NBT; ++b) X[b] = px8(xf[0][b], xf[1][b]);
#pragma unroll
        for (int xr = 0; xr < XR; ++xr) {
#pragma unroll
          for (int b = 0; b < NBT; ++b) acc[b] = mfma16x16x32(Al, X[b], acc[b]);
#pragma unroll
          for (int b = 0; b < NBT; ++b) acc[b] = mfma16x16x32(Am, X[b], acc[b]);
#pragma unroll
          for (int b = 0; b < NBT; ++b) acc[b] = mfma16x16x32(Ah, X[b], acc[b]);
        }
        if constexpr (XR > 1) {
#pragma unroll
          for (int b = 0; b < NBT; ++b) acc[b] *= 1.f / (float)XR;
        }
      } else {
#pragma unroll
        for (int k = 0; k < NTW; ++k) {
          if (tvk(k)) {
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
              for (int b = 0; b < NBT; ++b) acc[b] = mfma4(Wt[k][e], ub(xf[k][b], e), acc[b]);
          }
        }
      }
#pragma unroll
      for (int b = 0; b < NBT; ++b) zbuf[(w * NBT + b) * 64 + lane] = acc[b];
    }
    if (w == 0) { PH(1); }
    lds_barrier();
    if (w == 0) { PH(2); }
    const bool more = !RES && st + 1 < a.nsteps;   // RES: the next run's record is staged at its top
    // everyone's reads of this step's stage retired at barrier A: wave 7 (idle
    // until P2) stages the next step while the others run the edges and the head
    int* hflag = reinterpret_cast<int*>(smem + L_HFLAG);   // [0..6] head of batch tile v done; [7] stage landed
    auto heads_done = [&]() -> unsigned {   // bit v: head of batch tile v finished this step
      const bool ok = lane < NBT && __hip_atomic_load(hflag + (lane < NBT ? lane : 0), __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_WORKGROUP) >= st + 1;
      return (unsigned)__ballot(ok) & ((1u << NBT) - 1u);
    };
    if (w == 7 && more && !(dbg & 1)) {
      // DTF_PERSIST_DBG bits 2 / 3 (tuning): the whole stage / its second half only
      // once the first head is done (its DMA then does not queue in front of this
      // CU's E1 / E2 gather loads)
      if (dbg & 8) stage_x(st + 1, 0, 2);
      if (dbg & 12) {
        while (heads_done() == 0u) __builtin_amdgcn_s_sleep(1);
      }
      if (dbg & 8) stage_x(st + 1, 1, 2);
      else
        for (int xr = 0; xr < XR; ++xr) stage_x(st + 1, 0, 1);
      // idle until the first head is done anyway: wait for the DMA here and tell the
      // other waves the next step's operands are in LDS
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
      if (lane == 0) __hip_atomic_store(hflag + 7, st + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if (w == 7 && more && lane == 0) {
      __hip_atomic_store(hflag + 7, st + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }

    // ---------------- E1 + P1 + E2 + head (wave w < 7: batch tile w)
    if (w < NBT) {
      const int bw = 16 * w + r;          // this lane's batch row
      const bool bv = bw < B;
      f32x4 zs = zbuf[w * 64 + lane];
#pragma unroll
      for (int v = 1; v < 8; ++v) zs += zbuf[(v * NBT + w) * 64 + lane];
      // publish the slice partial of (j, batch tile w) as granules; gather the others
      // E1 region of (parity, block j): [slice][batch tile] slots
      const auto r1 = region_rsrc(a.xbuf + E1_OFF + (long long)(par * NJ + j) * NQ * NBT * GSLOT, NQ * NBT * GSLOT);
      if constexpr (EXP != 4) put_gran(r1, (q * NBT + w) * GSLOT + 32 * lane, zs, tag, l2_e1);
      if (w == 0) { PH(3); }
      // this step's W2 / b1 / b2 operands of the lane, read from LDS while the
      // partial is in flight (their LDS latency off the E1 -> P1 -> E2 -> head chain)
      float w2p[4], w2d[4], b1v[4], b2v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        w2p[e] = w2s[(4 * g + e) * 16 + r];
        w2d[e] = w2s[r * 16 + 4 * g + e];
        b1v[e] = b1s[4 * g + e];
        b2v[e] = b2s[4 * g + e];
      }
      f32x4 z;
      bool ok = true;
      if constexpr (EXP == 4) {
        z = zs * 4.f;
      } else if constexpr (EXP == 2) {
        f32x4 part[2];
        ok = gather_gran<2, INS>(r1, [&](int k) { return (((q & 2) + k) * NBT + w) * GSLOT; }, q & 1, true, 63, tag, zs, part,
                            lane, a);
        z = (part[0] + part[1]) * 2.f;
      } else {
        f32x4 part[NQ];
        ok = gather_gran<NQ, INS>(r1, [&](int k) { return (k * NBT + w) * GSLOT; }, jq[1], true, 63, tag, zs, part, lane,
                                  a);
        z = part[0];
#pragma unroll
        for (int qq = 1; qq < NQ; ++qq) z += part[qq];
      }
      if (w == 0) { PH(4); }
      if (w == 0) { PH(5); }
      // lane (batch r, g): hidden 16j+4g+i
      float a2[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int hl = 4 * g + i;
        const float zt = z[i] * (1.f / 255.f) + b1v[i];
        // v_exp_f32 / v_rcp_f32 (<= 2 ulp each, 1e-7 relative): ~20 instructions per
        // element less than IEEE expf + division on this single-wave critical path
        const float av = ACT == 0 ? __builtin_amdgcn_rcpf(1.f + __expf(-zt)) : fmaxf(zt, 0.f);
        a2[i] = (16 * j + hl < HID) ? av : 0.f;
      }
      // partial logits^T[class][batch] of block j: A = W2^T (lane: class r), B = a2^T
      f32x4 pl = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) pl = mfma4(w2p[e], a2[e], pl);
      // E2 region of (parity, slice q, batch tile w): [block] slots
      const auto r2 = region_rsrc(a.xbuf + E2_OFF + (long long)((par * NQ + q) * NBT + w) * NJ * GSLOT, NJ * GSLOT);
      if (g < 3) put_gran(r2, j * GSLOT + 32 * lane, pl, tag, l2_e2);
      if (w == 0) { PH(6); }
      // while the logits are in flight: a2 -> LDS (dW2)
#pragma unroll
      for (int i = 0; i < 4; ++i) a2T[(4 * g + i) * LS + bw] = a2[i];
      f32x4 lp[NJ];
      ok = gather_gran<NJ, INS>(r2, [&](int k) { return k * GSLOT; }, jq[0], g < 3, 47, tag, pl, lp, lane, a) && ok;
      if (w == 0) { PH(7); }
      if (!ok && lane == 0) *abort_flag = 1;
      // logits, softmax cross-entropy, accuracy -- identical in every workgroup
      float lg[4], ex[4];
      float m = -3.0e38f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = b2v[i];
#pragma unroll
        for (int jj = 0; jj < NJ; ++jj) v += lp[jj][i];
        lg[i] = v;
        if (4 * g + i < NCLS) m = fmaxf(m, v);
      }
      if (w == 0) { PH(8); }
      m = fmaxf(m, xor16(m));
      m = fmaxf(m, xor32(m));
      const int y = lab < NCLS ? lab : 0;
      float ssum = 0.f, zy = 0.f, am = 1e9f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int cl = 4 * g + i;
        ex[i] = cl < NCLS ? __expf(lg[i] - m) : 0.f;
        ssum += ex[i];
        zy += (cl == y) ? lg[i] : 0.f;
        if (cl < NCLS && lg[i] == m) am = fminf(am, (float)cl);
      }
      ssum += xor16(ssum); ssum += xor32(ssum);
      zy += xor16(zy); zy += xor32(zy);
      am = fminf(am, xor16(am)); am = fminf(am, xor32(am));
      const float inv = __builtin_amdgcn_rcpf(ssum);
      if (w == 0) { PHX(13); }
      float dz3[4], py = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int cl = 4 * g + i;
        const float p = ex[i] * inv;
        py += (cl == y) ? p : 0.f;
        dz3[i] = (bv && cl < NCLS) ? p - (cl == y ? 1.f : 0.f) : 0.f;   // unscaled: 1/B at the update
      }
      py += xor16(py); py += xor32(py);
      const float loss = a.naive ? -__logf(py) : (m + __logf(ssum) - zy);
      // da2^T = W2 . dz3^T (A = W2, lane: hidden r), dz2 = da2 * act'(a2)
      f32x4 da = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) da = mfma4(w2d[e], dz3[e], da);
      if (w == 0) { PHX(14); }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float d = ACT == 0 ? da[i] * a2[i] * (1.f - a2[i]) : (a2[i] > 0.f ? da[i] : 0.f);
        if constexpr (SPLIT) {
          uint32_t ph, pm, pl;
          split3(d, ph, pm, pl);
          const int o = (4 * g + i) * PS + bw;
          dzp[o] = (uint16_t)(ph >> 16);
          dzp[16 * PS + o] = (uint16_t)(pm >> 16);
          dzp[32 * PS + o] = (uint16_t)(pl >> 16);
        } else {
          dz2T[(4 * g + i) * LS + bw] = d;
        }
        dz3T[(4 * g + i) * LS + bw] = dz3[i];
      }
      if (w == 0) { PHX(15); }
      // per-row loss / hit, summed by wave 7 (no row reductions on the head's path)
      if (g == 0) {
        float* rl = reinterpret_cast<float*>(smem + L_RLOSS);
        rl[bw] = bv ? loss : 0.f;
        rl[128 + bw] = (bv && (int)am == y) ? 1.f : 0.f;
      }
      // this tile's dW2 = a2^T dz3 and db2 = 1^T dz3 partials over its 16 rows (two
      // independent f32 MFMA chains; k = batch 4g + e, from the rows this wave just
      // wrote: LDS ops of one wave complete in order).  db1 rides along with wave
      // 7's weight-gradient MFMAs as a ones "feature" tile.
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      {
        const f32x4 av = *reinterpret_cast<const f32x4*>(a2T + r * LS + 16 * w + 4 * g);
        const f32x4 dv = *reinterpret_cast<const f32x4*>(dz3T + r * LS + 16 * w + 4 * g);
        const float one = r == 0 ? 1.f : 0.f;   // A = rows of ones at row 0
        f32x4 dp = {0.f, 0.f, 0.f, 0.f}, p2 = dp;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          dp = mfma4(av[e], dv[e], dp);
          p2 = mfma4(one, dv[e], p2);
        }
        reinterpret_cast<f32x4*>(smem + L_DW2P)[w * 64 + lane] = dp;
        if (g == 0) rdb2[w * 16 + r] = p2[0];   // D[0][class r]
      }
      // head of batch tile w done (dz2 / dz3 / a2 rows and the row metrics are in LDS,
      // its reads of W2 / b1 / b2 are over)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
      if (lane == 0)
        __hip_atomic_store(reinterpret_cast<int*>(smem + L_HFLAG) + w, st + 1, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
      if (w == 0) { PH(9); }
    }
    // ---------------- P2 without a workgroup barrier: a wave multiplies the weight-
    // gradient chunk of batch rows 32cc..32cc+31 (one batch tile without SPLIT) as
    // soon as the heads of its batch tiles are done (LDS flags), chunks in order
    // (one accumulator chain: deterministic).  Barrier B used to wait for the LAST
    // head before any chunk started.  Reuse of everything the heads wrote is still
    // fenced by barrier A of the next step.
    f32x4 G[NTW];                        // dW1[16ft+4g+i][16j+r] (x 255 B)
    f32x4 G1[NTW];                       // !SPLIT: second accumulator chain
#pragma unroll
    for (int k = 0; k < NTW; ++k) G[k] = G1[k] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int NCH = SPLIT ? 4 : NBT;
    auto need_of = [](int ch) -> unsigned {
      return SPLIT ? ((1u << (2 * ch)) | (2 * ch + 1 < NBT ? 1u << (2 * ch + 1) : 0u)) : (1u << ch);
    };
    auto chunk = [&](int ch) {   // ch is a constant after unrolling (register operands)
      if constexpr (SPLIT) {
        // dW1 tile = x^T dz2 over K = 128 batch rows in 4 chunks: A = x^T bytes (exact),
        // B = the dz2 pieces; an absent second tile computes a zero-weight copy (unused)
        const uint16_t* bp = dzp + r * PS + 32 * ch + 8 * g;
        const bf16x8 Bh = *reinterpret_cast<const bf16x8*>(bp);
        const bf16x8 Bm = *reinterpret_cast<const bf16x8*>(bp + 16 * PS);
        const bf16x8 Bl = *reinterpret_cast<const bf16x8*>(bp + 32 * PS);
        const bf16x8 X0 = px8(xt[0][2 * ch], xt[0][2 * ch + 1]);
        if (tv1 || w == 7) {   // wave-uniform: waves without a second tile skip its MFMAs
          // wave 7 (always one tile) multiplies a tile of ones instead: G[1] = db1
          // (lane (r, g): hidden 16j + r, every i), exact like the rest
          const bf16x8 X1 = tv1 ? px8(xt[1][2 * ch], xt[1][2 * ch + 1]) : px8(0x01010101u, 0x01010101u);
          G[0] = mfma16x16x32(X0, Bl, G[0]);
          G[1] = mfma16x16x32(X1, Bl, G[1]);
          G[0] = mfma16x16x32(X0, Bm, G[0]);
          G[1] = mfma16x16x32(X1, Bm, G[1]);
          G[0] = mfma16x16x32(X0, Bh, G[0]);
          G[1] = mfma16x16x32(X1, Bh, G[1]);
        } else {
          G[0] = mfma16x16x32(X0, Bl, G[0]);
          G[0] = mfma16x16x32(X0, Bm, G[0]);
          G[0] = mfma16x16x32(X0, Bh, G[0]);
        }
      } else {
        const f32x4 bz = *reinterpret_cast<const f32x4*>(dz2T + r * LS + 16 * ch + 4 * g);
#pragma unroll
        for (int k = 0; k < NTW; ++k) {
          if (tvk(k)) {
            G[k] = mfma4(ub(xt[k][ch], 0), bz[0], G[k]);
            G1[k] = mfma4(ub(xt[k][ch], 1), bz[1], G1[k]);
            G[k] = mfma4(ub(xt[k][ch], 2), bz[2], G[k]);
            G1[k] = mfma4(ub(xt[k][ch], 3), bz[3], G1[k]);
          }
        }
        if (w == 7) {   // one tile: a ones tile in the second slot gives db1
          G[1] = mfma4(1.f, bz[0], G[1]);
          G1[1] = mfma4(1.f, bz[1], G1[1]);
          G[1] = mfma4(1.f, bz[2], G[1]);
          G1[1] = mfma4(1.f, bz[3], G1[1]);
        }
      }
    };
    {
      int cc = 0;   // next chunk
      for (;;) {
        const unsigned hm = heads_done();
        bool did = false;
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
          if (ch == cc && (hm & need_of(ch)) == need_of(ch)) {   // wave-uniform
            if (!did) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
            if (cc == 0 && w == 0) { PH(10); }
#pragma unroll
            for (int xr = 0; xr < XR; ++xr) chunk(ch);
            ++cc;
            did = true;
          }
        }
        if (cc == NCH) break;
        if (!did) {
          if (dbg & 16) __builtin_amdgcn_s_sleep(2);
          else __builtin_amdgcn_s_sleep(0);
        }
      }
    }
    if constexpr (!SPLIT) {
#pragma unroll
      for (int k = 0; k < NTW; ++k) G[k] = G[k] + G1[k];
    }
    if constexpr (XR > 1) {
#pragma unroll
      for (int k = 0; k < NTW; ++k) G[k] *= 1.f / (float)XR;
    }
    // every head is done here.  Wave 7 sums the 7 head waves' dW2 / db2 partials
    // and the per-row metrics in fixed order (all loads in flight at once); one
    // GPU: the W2 / b1 / b2 updates too (their readers, this step's heads, are done;
    // the next step's read them after barrier A)
    f32x4 D = {0.f, 0.f, 0.f, 0.f};      // wave 7: dW2[16j+4g+i][class r] (x B)
    float gb = 0.f;                      // wave 7: db1 (lanes < 16) / db2 (lanes 16..25) (x B)
    if (w == 7) {
      // lanes 16..25: db2 column lane - 16 (lanes < 16 take db1 from the ones tile)
      const float* gsrc = rdb2 + (lane >= 16 && lane < 16 + NCLS ? lane - 16 : 0);
      const f32x4* dw2p = reinterpret_cast<const f32x4*>(smem + L_DW2P);
#pragma unroll
      for (int v = 0; v < NBT; ++v) {
        D += dw2p[v * 64 + lane];
        gb += gsrc[v * 16];
      }
      if (lane < 16) gb = G[1][0];   // db1 of hidden 16j + lane from the ones tile
      if (lane >= 16 + NCLS) gb = 0.f;
      PH7(13);
      PH7(15);
      if (c == 0) {   // loss / accuracy of the batch: per-row values, fixed reduction order
        const float* rl = reinterpret_cast<const float*>(smem + L_RLOSS);
        const bool hi = lane + 64 < BROWS;
        const float ls = wave_sum(rl[lane] + (hi ? rl[lane + 64] : 0.f));
        const float cr = wave_sum(rl[128 + lane] + (hi ? rl[128 + lane + 64] : 0.f));
        if (lane == 63) {
          const int sl = (int)((gstep0 + st) % a.ring);
          if constexpr (RES) {   // workgroup 0 publishes them (LDS), the ring keeps them too
            reinterpret_cast<float*>(abort_flag)[4] = ls / (float)B;
            reinterpret_cast<float*>(abort_flag)[5] = cr / (float)B;
            __hip_atomic_store(a.metrics + 2 * sl, ls / (float)B, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.metrics + 2 * sl + 1, cr / (float)B, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          } else {
            a.metrics[2 * sl] = ls / (float)B;
            a.metrics[2 * sl + 1] = cr / (float)B;
          }
        }
      }
      if constexpr (!MULTI) {
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
    if (*abort_flag) { aborted = true; break; }   // final for this step: every head has reported
    if (more) {
      // next step's operands (this step's are consumed): x rows + label once wave 7
      // saw the stage land, x^T
      while (__hip_atomic_load(hflag + 7, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < st + 1)
        __builtin_amdgcn_s_sleep(1);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
      read_xf();
      read_xt();
    }
    if (w == 0) { PH(11); }
    if constexpr (MULTI) {
      // ---- exchange of this workgroup's gradient with the same workgroup on
      // every peer GPU (uncached IPC buffers: completion == visibility); sums in
      // rank order keep the replicas bit-identical.  Only payload crosses the
      // fabric: bf16 packs a lane's two tiles into ONE 16-B entry (8 B when the
      // wave has one tile), hidden-padding lanes (unit >= 100) and the zero
      // columns of dW2 (class >= 10) neither store nor load, and every peer is
      // read with single 16-B system-scope loads, all NW of them in flight
      // (absent peers / masked lanes read out of the buffer's range: zero, no
      // memory traffic).
      const bool pk = a.gbf16 != 0;
      const size_t soff = IPC_FLAGS + (size_t)(par * NCOMP + c) * IPC_SLOT;
      char* own = static_cast<char*>(a.peer_base[a.rank]) + soff;
      const int eb = (w * 64 + lane) * 16;                       // bf16: both tiles
      const int ef0 = ((w * NTW + 0) * 64 + lane) * 16;          // fp32: tile 0
      const int ef1 = ((w * NTW + 1) * 64 + lane) * 16;          // fp32: tile 1
      const bool dlane = r < NCLS && 16 * j + 4 * g < HID;       // wave 7: dW2 entry carries data
      const bool blane = lane < 16 ? 16 * j + lane < HID : lane < 16 + NCLS;   // wave 7: db1 / db2
      if (hv) {
        if (pk) {
          const uint32_t p0 = pack2bf(G[0][0], G[0][1]), p1 = pack2bf(G[0][2], G[0][3]);
          const uint32_t p2 = pack2bf(G[1][0], G[1][1]), p3 = pack2bf(G[1][2], G[1][3]);
          if (tv1) *reinterpret_cast<uint4*>(own + eb) = make_uint4(p0, p1, p2, p3);
          else if (tv0) *reinterpret_cast<uint2*>(own + eb) = make_uint2(p0, p1);
        } else {
          if (tv0) *reinterpret_cast<f32x4*>(own + ef0) = G[0];
          if (tv1) *reinterpret_cast<f32x4*>(own + ef1) = G[1];
        }
      }
      if (pk) {   // this rank's own term, as every peer sees it
        G[0] = round_bf16x4(G[0]);
        G[1] = round_bf16x4(G[1]);
      }
      if (w == 7) {
        if (dlane) *reinterpret_cast<f32x4*>(own + IPC_SMALL + lane * 16) = D;
        if (blane) *reinterpret_cast<float*>(own + IPC_SMALL + 1024 + lane * 4) = gb;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave: its slot stores landed
      lds_barrier();
      char* flags = static_cast<char*>(a.peer_base[a.rank]);
      // wave 0 waits until every peer's flag word `fo` of this workgroup reached `tag`
      auto wait_peers = [&](int fo) {
        if (w == 0) {
          const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
          for (;;) {
            bool ok = true;
            if (lane < a.W && lane != a.rank) {
              const unsigned v = __hip_atomic_load(
                  reinterpret_cast<const unsigned*>(static_cast<const char*>(a.peer_base[lane]) + 64 * c + fo),
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
      };
      if (tid == 0 && !(a.rank == a.fault_rank && gstep0 + st >= a.fault_step))
        __hip_atomic_store(reinterpret_cast<unsigned*>(flags + 64 * c), tag, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      wait_peers(0);
      if (*abort_flag) { aborted = true; break; }
      // rank-order sums of this lane's entries at slot offset `so` over all ranks
      auto sum_ranks = [&](size_t so) {
        constexpr int GF = NW < 4 ? NW : 4;   // fp32 payload: 4 peers in flight per group (registers)
        if (pk) {
          if (tv1) sum_entries<NW, NW, true, true>(prs, a.W, a.rank, (int)so, hv, eb, eb, G[0], G[1]);
          else sum_entries<NW, NW, true, false>(prs, a.W, a.rank, (int)so, hv, eb, eb, G[0], G[1]);
        } else {
          if (tv1) sum_entries<NW, GF, false, true>(prs, a.W, a.rank, (int)so, hv, ef0, ef1, G[0], G[1]);
          else sum_entries<NW, GF, false, false>(prs, a.W, a.rank, (int)so, hv, ef0, ef1, G[0], G[1]);
        }
        if (w == 7) sum_small<NW>(prs, a.W, a.rank, (int)so + IPC_SMALL, dlane, blane, lane, D, gb);
      };
      if (a.xmode == 0) {
        // one-shot: every wave sums its entries over all ranks
        sum_ranks(soff);
      } else {
        // two-shot: wave w's entries form chunk w % W, reduced (rank order) by
        // that rank only, then every rank reads each chunk's sums from its owner:
        // 2 (W-1)/W of a slot crosses the fabric per GPU instead of (W-1) slots.
        // bf16 payload: the owner rounds the sum to bf16 once and uses the rounded
        // value itself, so the all-gather moves bf16 too and replicas stay identical
        const int own_chunk = w % a.W;
        const size_t roff = IPC_RED + (size_t)(par * NCOMP + c) * IPC_SLOT;
        char* ored = static_cast<char*>(a.peer_base[a.rank]) + roff;
        if (own_chunk == a.rank) {
          sum_ranks(soff);
          if (hv) {
            if (pk) {
              const uint32_t p0 = pack2bf(G[0][0], G[0][1]), p1 = pack2bf(G[0][2], G[0][3]);
              const uint32_t p2 = pack2bf(G[1][0], G[1][1]), p3 = pack2bf(G[1][2], G[1][3]);
              if (tv1) *reinterpret_cast<uint4*>(ored + eb) = make_uint4(p0, p1, p2, p3);
              else if (tv0) *reinterpret_cast<uint2*>(ored + eb) = make_uint2(p0, p1);
              G[0] = round_bf16x4(G[0]);
              G[1] = round_bf16x4(G[1]);
            } else {
              if (tv0) *reinterpret_cast<f32x4*>(ored + ef0) = G[0];
              if (tv1) *reinterpret_cast<f32x4*>(ored + ef1) = G[1];
            }
          }
          if (w == 7) {
            if (dlane) *reinterpret_cast<f32x4*>(ored + IPC_SMALL + lane * 16) = D;
            if (blane) *reinterpret_cast<float*>(ored + IPC_SMALL + 1024 + lane * 4) = gb;
          }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the reduced chunk landed
        lds_barrier();
        if (tid == 0)
          __hip_atomic_store(reinterpret_cast<unsigned*>(flags + 64 * c + 8), tag, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
        wait_peers(8);
        if (*abort_flag) { aborted = true; break; }
        if (own_chunk != a.rank) {
          // all-gather: this wave's chunk sums from their owner
          __amdgpu_buffer_rsrc_t rs = prs.r[0];
#pragma unroll
          for (int rr = 1; rr < NW; ++rr)
            if (rr == own_chunk) rs = prs.r[rr];   // wave-uniform
          const int ro = (int)roff;
          if (pk) {
            if (tv1) {
              const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, hv ? ro + eb : OOB_OFF, 0, SYS);
              G[0] = unbf4(v[0], v[1]);
              G[1] = unbf4(v[2], v[3]);
            } else {
              const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, hv ? ro + eb : OOB_OFF, 0, SYS);
              G[0] = unbf4(v[0], v[1]);
            }
          } else {
            G[0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, hv ? ro + ef0 : OOB_OFF, 0, SYS));
            if (tv1)
              G[1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, hv ? ro + ef1 : OOB_OFF, 0, SYS));
          }
          if (w == 7) {
            D = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, dlane ? ro + IPC_SMALL + lane * 16 : OOB_OFF, 0, SYS));
            gb = __uint_as_float(
                __builtin_amdgcn_raw_buffer_load_b32(rs, blane ? ro + IPC_SMALL + 1024 + lane * 4 : OOB_OFF, 0, SYS));
          }
        }
      }
    }
    // ---------------- updates (lr / (W B), 1/255 for the pixel scale)
    if (hv) {   // an absent second tile keeps its zero weights (wave 7's G[1] is db1)
#pragma unroll
      for (int k = 0; k < NTW; ++k)
#pragma unroll
        for (int i = 0; i < 4; ++i) Wt[k][i] -= (k == 0 || tv1) ? lrX * G[k][i] : 0.f;
    }
    if (w == 0) { PH(12); }
    if (MULTI && w == 7) {   // N GPUs: with the rank sums of dW2 / db1 / db2
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (16 * j + 4 * g + i < HID && r < NCLS) w2s[(4 * g + i) * 16 + r] -= lrB * D[i];
      if (lane < 16) {
        if (16 * j + lane < HID) b1s[lane] -= lrB * gb;
      } else if (lane < 16 + NCLS) {
        b2s[lane - 16] -= lrB * gb;
      }
    }
    st_done = st + 1;
    if constexpr (RES) {
      // the run is complete once every compute workgroup's parameters are in
      // memory: write-through stores, every wave's vmcnt(0), barrier, one agent add;
      // the last arriver (its add's return value says so) publishes the metrics,
      // global_step and the done count to pinned host memory
      __syncthreads();   // wave 7's LDS updates of W2 / b1 / b2 (and workgroup 0's metrics)
      if (c == 0 && tid == 0) { RTSC(a.run0 + st, 4); }
      write_params(true);
      // the graph's global_step: counted here (anything else that writes it stops
      // the engine first), stored write-through by workgroup 0
      const double gsv = gvar0 + (double)(st + 1);
      if (c == 0 && tid == 0) {
        if (a.gvar_kind == 1) __hip_atomic_store(static_cast<float*>(a.gvar), (float)gsv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else if (a.gvar_kind == 2) __hip_atomic_store(static_cast<long long*>(a.gvar), (long long)gsv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else if (a.gvar_kind == 3) __hip_atomic_store(static_cast<int*>(a.gvar), (int)gsv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else if (a.gvar_kind == 4) __hip_atomic_store(static_cast<double*>(a.gvar), gsv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        if (c == 0) { RTSC(a.run0 + st, 5); }
        __hip_atomic_fetch_add(a.dctr + 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (c == 0) {
          // workgroup 0 (it holds the metrics) publishes once all 28 have arrived
          const unsigned need = (unsigned)NCOMP * (unsigned)(st + 1);
          const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
          while (__hip_atomic_load(a.dctr + 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
            if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) {
              atomicOr(a.err, 8);
              break;
            }
          }
          RTSC(a.run0 + st, 6);
          const float* mf = reinterpret_cast<const float*>(abort_flag);
          __hip_atomic_store(a.host_out, mf[4], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(a.host_out + 1, mf[5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(a.host_out + 2, (float)gsv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __hip_atomic_store(a.host_done, a.run0 + st + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          RTSC(a.run0 + st, 7);
        }
      }
    }
  }
  if (aborted) return;
  __syncthreads();   // wave 7's last small-parameter update
  if (tid == 0) { PROC(c, 3); }

  // ---- write back (fp32 master), global step, exchange sequence, end stamp
  // (RES: the steps that ran -- the sequence never falls behind the tags in use)
  write_params(false);
  if (c == 0 && tid == 300) {
    *a.gstep = gstep0 + st_done;
    *a.seq = seq0 + (unsigned long long)st_done;
    if (a.step_ts != nullptr)
      a.step_ts[(gstep0 + st_done) % a.ts_ring] = (long long)__builtin_amdgcn_s_memrealtime();
  }
  if (tid == 0) { PROC(c, 5); }
}

// packed placement (a.spread == 0): compute workgroup c runs as blockIdx 8c, so
// under the observed round-robin dispatch all 28 share ONE XCD (both edges in one
// L2); the first NCOP other blocks copy, the rest exit.  spread (several ranks on
// one GPU, tests): compute = blocks 0..27, copiers = 28..43.  Placement is speed
// only: the census above decides each edge's store flavour.
template <int ACT, int NW, bool SPLIT, bool RES = false, int EXP = 0, bool INS = false>
__global__ __launch_bounds__(THREADS, 1) void mlp_persist_f32(Args a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int b = blockIdx.x;
  int c = -1, cid = -1;
  if (a.spread) {
    if (b < NCOMP) c = b; else cid = b - NCOMP;
  } else {
    if ((b & 7) == 0) c = b >> 3; else cid = b - (b >> 3) - 1;
  }
  if (c >= 0) {
    if (a.nsteps > 0) compute<ACT, NW, SPLIT, RES, EXP, INS>(a, c / NQ, c % NQ, smem);
    return;
  }
  if constexpr (RES) copier_res(a, cid, smem);
  else if (cid < NCOP) copier(a, cid, smem);
}

}  // namespace mlpf
}  // namespace dtfk

// fault injection (tests of the bench's in-process fallback): rank `rank` stops
// publishing its exchange flag from global step `step` on; rank -1 = off
static int g_fault_rank = -1;
static long long g_fault_step = -1;

// Placement-census tags: unique per launch within the process (the census
// buffer lives in a runner's exchange buffer, zeroed once; tag 0 never matches)
static unsigned next_census_tag() {
  static std::atomic<unsigned> ctr{0};
  unsigned t = ctr.fetch_add(1u, std::memory_order_relaxed) + 1u;
  return t == 0u ? ctr.fetch_add(1u, std::memory_order_relaxed) + 1u : t;
}

extern "C" {

void dtfk_mlpf_set_fault(int rank, long long step) {
  g_fault_rank = rank;
  g_fault_step = step;
}

// profiling only: the resident launches' per-run stamp ring (nullptr: off)
static long long* g_res_ts = nullptr;
void dtfk_mlpf_set_res_ts(long long* p) { g_res_ts = p; }

long long dtfk_mlpf_stage_rec() { return dtfk::mlpf::REC; }
long long dtfk_mlpf_xbuf_bytes() { return dtfk::mlpf::XBUF_BYTES; }
long long dtfk_mlpf_ipc_bytes() { return dtfk::mlpf::IPC_BYTES; }
int dtfk_mlpf_max_batch() { return dtfk::mlpf::BROWS; }

typedef void (*Kern2)(dtfk::mlpf::Args);
hipError_t dtfk_mlp_persist_f32(const void* stage, long long rec_h, int B, int nsteps, float* params, const float* lr,
                                float* metrics, int ring, int act, int naive, long long* gstep, unsigned long long* seq,
                                void* xbuf, int* err, long long timeout, long long* step_ts, int ts_ring,
                                const void* host_next, int next_steps, void* stage_next, void* const* peer_base, int W,
                                int rank, int gbf16, long long* phase_ts, int spread, int xmode, int split,
                                hipStream_t stream) {
  using namespace dtfk::mlpf;
  Args a;
  a.phase_ts = phase_ts;
  a.res_ts = nullptr;
  a.stage = static_cast<const uint8_t*>(stage);
  a.rec_h = rec_h;
  a.B = B;
  a.nsteps = nsteps;
  a.params = params;
  a.p_w2 = params + OFF_W2;
  a.p_b1 = params + OFF_B1;
  a.p_b2 = params + OFF_B2;
  a.door = nullptr;
  a.host_recs = nullptr;
  a.host_lr = nullptr;
  a.host_out = nullptr;
  a.host_done = nullptr;
  a.host_state = nullptr;
  a.launch_id = a.run0 = a.idle = 0;
  a.census_tag = next_census_tag();
  a.gvar = nullptr;
  a.gvar_kind = 0;
  a.dctr = nullptr;
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
  a.spread = spread;
  a.xmode = xmode;
  {
    // read once per process (a getenv per launch is host time inside a short timed run)
    static const int gmode = [] {
      const char* gm = getenv("DTF_GATHER_MODE");   // r3: direct loads, no sleep 8.68 / long sleep 8.72 / probe 9.56 us
      return gm ? atoi(gm) : 1;
    }();
    static const int dbg = [] {
      const char* db = getenv("DTF_PERSIST_DBG");
      return db ? atoi(db) : 0;
    }();
    a.gmode = gmode;
    a.dbg = dbg;
    // timing experiment only (see compute's EXP): 2 / 4 = the 14- / 7-workgroup
    // decompositions' per-workgroup work, sigmoid one-GPU split engine only
    static const int exper = [] {
      const char* e = getenv("DTF_PERSIST_EXP");
      return e ? atoi(e) : 0;
    }();
    if (exper == 2 || exper == 4) {
      if (act != 0 || W != 1 || !split || spread) return hipErrorInvalidValue;
      static const Kern2 xk[2] = {mlp_persist_f32<0, 1, true, false, 2, true>,
                                  mlp_persist_f32<0, 1, true, false, 4, true>};
      const Kern2 k = xk[exper == 2 ? 0 : 1];
      static bool xattr = false;
      if (!xattr) {
        for (Kern2 kk : xk) {
          const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kk),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_BYTES);
          if (e != hipSuccess) return e;
        }
        xattr = true;
      }
      hipLaunchKernelGGL(k, dim3(GRID_PACKED), dim3(THREADS), LDS_BYTES, stream, a);
      return hipGetLastError();
    }
    a.fault_rank = g_fault_rank;
    a.fault_step = g_fault_step;
  }
  constexpr size_t lds = LDS_BYTES;
  typedef void (*Kern)(Args);
  // NW: peer-table width the exchange is unrolled for (W rounded up to 2 / 4 / 8)
  static const Kern kerns[16] = {
      mlp_persist_f32<0, 1, false>, mlp_persist_f32<1, 1, false>, mlp_persist_f32<0, 2, false>,
      mlp_persist_f32<1, 2, false>, mlp_persist_f32<0, 4, false>, mlp_persist_f32<1, 4, false>,
      mlp_persist_f32<0, 8, false>, mlp_persist_f32<1, 8, false>, mlp_persist_f32<0, 1, true>,
      mlp_persist_f32<1, 1, true>,  mlp_persist_f32<0, 2, true>,  mlp_persist_f32<1, 2, true>,
      mlp_persist_f32<0, 4, true>,  mlp_persist_f32<1, 4, true>,  mlp_persist_f32<0, 8, true>,
      mlp_persist_f32<1, 8, true>};
  static bool attr_set = false;
  if (!attr_set) {
    for (Kern k : kerns) {
      const hipError_t e =
          hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
    attr_set = true;
  }
  if (W < 1 || W > 8 || rank < 0 || rank >= W) return hipErrorInvalidValue;
  const int nwi = W <= 1 ? 0 : (W <= 2 ? 1 : (W <= 4 ? 2 : 3));
  const int which = (act == 0 ? 0 : 1) + 2 * nwi + (split ? 8 : 0);
  const int grid = spread ? GRID_SPREAD : GRID_PACKED;
  if (phase_ts != nullptr || a.dbg != 0 || a.gmode != 1) {
    // profiling / tuning: the instrumented build (one GPU only)
    if (W != 1) return hipErrorInvalidValue;
    static const Kern ik[4] = {mlp_persist_f32<0, 1, false, false, 0, true>, mlp_persist_f32<1, 1, false, false, 0, true>,
                               mlp_persist_f32<0, 1, true, false, 0, true>, mlp_persist_f32<1, 1, true, false, 0, true>};
    static bool iattr = false;
    if (!iattr) {
      for (Kern k : ik) {
        const hipError_t e =
            hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
      }
      iattr = true;
    }
    hipLaunchKernelGGL(ik[(act == 0 ? 0 : 1) + (split ? 2 : 0)], dim3(grid), dim3(THREADS), lds, stream, a);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(kerns[which], dim3(grid), dim3(THREADS), lds, stream, a);
  return hipGetLastError();
}

// The resident Session engine (compat/resident.py, csrc/bind_mlp.cpp
// ResidentMLPPlan): ONE launch serves Session.run calls until `idle` ticks pass
// without a doorbell or the host writes door < 0.  One GPU, the reference's
// precision (SPLIT), packed placement; the graph's own W1 / W2 / b1 / b2 tensors
// and global_step variable are read at launch and written through every step.
hipError_t dtfk_mlp_persist_f32_resident(void* stage, int B, float* W1, float* W2, float* b1, float* b2, const float* lr,
                                         float* metrics, int ring, int act, int naive, long long* gstep,
                                         unsigned long long* seq, void* xbuf, int* err, long long timeout,
                                         const long long* door, const void* host_recs, long long rec_h,
                                         const float* host_lr, float* host_out, long long* host_done,
                                         long long* host_state, long long launch_id, long long run0, long long idle,
                                         void* gvar, int gvar_kind, unsigned* dctr, hipStream_t stream) {
  using namespace dtfk::mlpf;
  if (B < 1 || B > BROWS || rec_h < (long long)B * (DIN + 1) || gvar_kind < 0 || gvar_kind > 4 ||
      (gvar_kind != 0 && gvar == nullptr))
    return hipErrorInvalidValue;
  Args a;
  std::memset(&a, 0, sizeof(a));
  a.stage = static_cast<const uint8_t*>(stage);
  a.rec_h = rec_h;
  a.B = B;
  a.nsteps = 0x7fffffff;   // bounded by the doorbell / idle exit
  a.params = W1;
  a.p_w2 = W2;
  a.p_b1 = b1;
  a.p_b2 = b2;
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
  a.ts_ring = 1;
  a.W = 1;
  a.gmode = 1;
  a.fault_rank = -1;
  a.fault_step = -1;
  a.door = door;
  a.host_recs = static_cast<const uint8_t*>(host_recs);
  a.host_lr = host_lr;
  a.host_out = host_out;
  a.host_done = host_done;
  a.host_state = host_state;
  a.launch_id = launch_id;
  a.census_tag = next_census_tag();
  a.run0 = run0;
  a.idle = idle;
  a.gvar = gvar;
  a.gvar_kind = gvar_kind;
  a.dctr = dctr;
  a.res_ts = g_res_ts;
  constexpr size_t lds = LDS_BYTES;
  typedef void (*Kern)(Args);
  // per-run stamps (DTF_RESIDENT_STAMPS): the instrumented build
  static const Kern kerns[4] = {mlp_persist_f32<0, 1, true, true>, mlp_persist_f32<1, 1, true, true>,
                                mlp_persist_f32<0, 1, true, true, 0, true>, mlp_persist_f32<1, 1, true, true, 0, true>};
  static bool attr_set = false;
  if (!attr_set) {
    for (Kern k : kerns) {
      const hipError_t e =
          hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
    attr_set = true;
  }
  hipLaunchKernelGGL(kerns[(act == 0 ? 0 : 1) + (a.res_ts != nullptr ? 2 : 0)], dim3(GRID_PACKED), dim3(THREADS), lds,
                     stream, a);
  return hipGetLastError();
}

}  // extern "C"
