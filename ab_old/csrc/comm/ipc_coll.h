// Shared between the IPC collective kernels (csrc/kernels/ipc_coll.hip) and
// their host driver (csrc/comm/ipc_coll.cpp): the per-rank buffer layout and
// the POD argument blocks the launchers take.
#pragma once
#include <hip/hip_runtime.h>

namespace dtfk {
namespace ipcc {

constexpr int WMAX = 16;               // ranks of one node (8 GPUs; 16 for same-GPU rehearsals)
constexpr long long CTRL = 4096;       // control block at the front of every rank's exported buffer
// control block words (u64, written by the owner, read by peers with system-scope loads)
constexpr long long PUB = 0;           // seq of the last collective whose phase-1 data is in the slot
constexpr long long RED = 64;          // seq of the last collective whose reduced chunk is in the slot
constexpr long long OFFS = 128;        // [2 parities][WMAX]: all_to_all byte offset of destination d's rows
constexpr long long STAT = OFFS + 2 * WMAX * 8;   // [2 parities]: 1 = this rank's all_to_all overflowed (no data)

// Bytes of one rank's exported buffer for an input-region capacity `cap`:
// [control][parity 0: input cap | reduced cap][parity 1: input cap | reduced cap]
inline long long buffer_bytes(long long cap) { return CTRL + 4 * cap; }

struct Coll {
  void* const* base;             // device table of the W exported buffers (own + mapped peers)
  int W, rank;
  long long cap;                 // input-region bytes per parity slot
  unsigned long long* seq;       // device word: seq of this rank's last collective (each bumps it)
  unsigned* ctr;                 // device words: per-phase workgroup arrival counters (reset by the last)
  int* err;                      // device error word: later collectives fail fast
  int* err_host;                 // pinned host error word: the host raises on its next call
  long long timeout;             // s_memrealtime ticks (100 MHz) a wait may take before it reports
  int wide;                      // 1: 16-byte system-coherent buffer loads of peer slots; 0: 8-byte atomics (A/B)
};

struct SgdArgs {                 // fused all-reduce-mean + SGD over up to 8 fp32 parameters (flat order)
  float* p[8];
  long long end[8];              // exclusive prefix ends of the parameters in the flat gradient
  int np;
  const float* lr_ptr;           // device learning rate, or null: lr_val
  float lr_val;
  float scale;                   // 1 / W (mean)
  void* gstep;                   // global_step storage (+1 once per step) or null
  int gkind;                     // 0 f32, 1 i64, 2 i32, 3 f64
  float* metrics;                // [2] <- global_step after the update (or null)
  float* host_metrics;           // pinned [2] <- the same (or null)
};

struct A2A {                     // all_to_all byte layout of one rank
  long long send_off[WMAX];      // where destination d's rows start in the send buffer
  long long recv_off[WMAX];      // where source r's rows go in the receive buffer
  long long recv_bytes[WMAX];    // how many bytes come from source r
  long long send_total;          // bytes of the whole send buffer
  int overflow;                  // send_total > cap: publish the overflow status instead of data
};

}  // namespace ipcc
}  // namespace dtfk

extern "C" {
// dtype: 0 f32, 1 bf16, 2 f64, 3 i32, 4 i64; op: 0 sum, 1 max, 2 min
hipError_t dtfk_ipcc_allreduce(const void* in, void* out, long long n, int dtype, int op, float scale, int two_shot,
                               dtfk::ipcc::Coll c, int grid, hipStream_t s);
hipError_t dtfk_ipcc_reduce_sgd(const float* grad, long long n, dtfk::ipcc::SgdArgs a, dtfk::ipcc::Coll c, int grid,
                                hipStream_t s);
hipError_t dtfk_ipcc_broadcast(const void* in, void* out, long long nbytes, int src, dtfk::ipcc::Coll c, int grid,
                               hipStream_t s);
hipError_t dtfk_ipcc_allgather(const void* in, void* out, long long nbytes, long long stride, dtfk::ipcc::Coll c,
                               int grid, hipStream_t s);
hipError_t dtfk_ipcc_alltoall(const void* in, void* out, dtfk::ipcc::A2A a, dtfk::ipcc::Coll c, int grid,
                              hipStream_t s);
}
