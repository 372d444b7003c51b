// Host driver of the IPC collectives (csrc/kernels/ipc_coll.hip): one object
// per rank over its IpcPeerBuffers (csrc/comm/ipc_peer.cpp, sized
// ipcc::buffer_bytes(cap)).  Header-only so other bindings (the compat
// Session's MLP step plan, csrc/bind_mlp.cpp) can fuse a collective into their
// own launch sequence.
//
// * The collective's sequence number lives on the device (a captured hipGraph
//   replays correctly); the host keeps none.
// * One stream order per rank: when a collective is issued on a different
//   stream than the previous one, the new stream first waits for an event
//   recorded on the old one (the kernels' slot-reuse argument needs it).
// * Sizes above the slot capacity are chunked (all-reduce, broadcast,
//   all-gather: every rank chunks the same way); an all-to-all whose send
//   buffer exceeds it still runs (so no peer hangs), publishes an overflow
//   status every receiver sees, and raises here.
// * Errors (a bounded wait timed out, a peer's overflow) land in a pinned host
//   word the kernels write; every call checks it first and raises.
#pragma once
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "comm/ipc_coll.h"

namespace dtf {

class IpcColl {
 public:
  IpcColl(py::object buffers, int64_t table_ptr, int W, int rank, int64_t cap, double timeout_s,
          int64_t two_shot_bytes, int max_grid)
      : keep_(std::move(buffers)), W_(W), rank_(rank), cap_(cap), two_shot_(two_shot_bytes),
        max_grid_(std::max(1, max_grid)) {
    if (W < 1 || W > dtfk::ipcc::WMAX || rank < 0 || rank >= W) throw std::runtime_error("IpcColl: bad world/rank");
    if (cap < 4096 || (cap & 255)) throw std::runtime_error("IpcColl: capacity must be a multiple of 256 >= 4096");
    table_ = reinterpret_cast<void* const*>(table_ptr);
    auto dev = at::TensorOptions().device(at::kCUDA, c10::hip::current_device());
    words_ = at::zeros({4}, dev.dtype(at::kLong));          // [seq u64][ctr0 u32, ctr1 u32][..]
    err_ = at::zeros({1}, dev.dtype(at::kInt));
    err_host_ = at::zeros({2}, at::TensorOptions().dtype(at::kInt).pinned_memory(true));
    timeout_ = (long long)(std::max(0.001, timeout_s) * 1e8);   // s_memrealtime: 100 MHz
    const char* nw = std::getenv("DTF_IPC_NARROW");                // A/B probe: 8-byte peer loads
    wide_ = (nw != nullptr && nw[0] == '1') ? 0 : 1;
    ck(hipEventCreateWithFlags(&ev_, hipEventDisableTiming), "hipEventCreate");
  }
  ~IpcColl() {
    if (ev_) (void)hipEventDestroy(ev_);
  }

  int world_size() const { return W_; }
  int rank() const { return rank_; }
  int64_t capacity() const { return cap_; }
  int64_t calls() const { return calls_; }
  int error() const { return *reinterpret_cast<volatile int*>(err_host_.data_ptr<int>()); }

  dtfk::ipcc::Coll coll() const {
    dtfk::ipcc::Coll c;
    c.base = table_;
    c.W = W_;
    c.rank = rank_;
    c.cap = cap_;
    char* w = static_cast<char*>(words_.data_ptr());
    c.seq = reinterpret_cast<unsigned long long*>(w);
    c.ctr = reinterpret_cast<unsigned*>(w + 8);
    c.err = err_.data_ptr<int>();
    c.err_host = err_host_.data_ptr<int>();
    c.timeout = timeout_;
    c.wide = wide_;
    return c;
  }

  int grid_for(int64_t bytes) const {
    const int64_t g = (bytes / 8 + 1023) / 1024;      // ~4 packets per thread
    return (int)std::max<int64_t>(1, std::min<int64_t>(max_grid_, g));
  }

  // -------------------------------------------------------------- stream order
  hipStream_t begin() {
    check();
    hipStream_t s = c10::hip::getCurrentHIPStream().stream();
    if (last_ != nullptr && last_ != s) {       // chain: everything queued on the old stream first
      ck(hipEventRecord(ev_, last_), "IpcColl: event");
      ck(hipStreamWaitEvent(s, ev_, 0), "IpcColl: wait");
    }
    last_ = s;
    ++calls_;
    return s;
  }
  void check() const {
    const int e = error();
    if (e != 0)
      throw std::runtime_error(std::string("IPC collective failed on this rank (code ") + std::to_string(e) +
                               (e & 2 ? ": a peer's all_to_all send buffer exceeded the IPC slot capacity"
                                      : ": a wait for a peer timed out -- a peer died or stopped issuing "
                                        "collectives in the same order") + ")");
  }

  // -------------------------------------------------------------- raw collectives
  // dtype: 0 f32, 1 bf16, 2 f64, 3 i32, 4 i64; op 0 sum, 1 max, 2 min
  void all_reduce_raw(const void* in, void* out, int64_t n, int dtype, int op, float scale, hipStream_t s) {
    const int es = dtype == 1 ? 2 : (dtype == 0 || dtype == 3) ? 4 : 8;
    if ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15)
      throw std::runtime_error("IpcColl.all_reduce: 16-byte aligned buffers expected");
    const int64_t chunk = cap_ / 16 * 16 / es;       // whole 16-byte packets per chunk
    for (int64_t off = 0; off < n; off += chunk) {
      const int64_t m = std::min(chunk, n - off);
      const int two = (W_ > 2 && m * es >= two_shot_) ? 1 : 0;
      ck(dtfk_ipcc_allreduce(static_cast<const char*>(in) + off * es, static_cast<char*>(out) + off * es, m, dtype,
                             op, scale, two, coll(), grid_for(m * es), s),
         "IpcColl: all_reduce launch");
    }
  }

  // fused all-reduce mean + SGD: grad (fp32, n values, 16-byte aligned)
  void reduce_sgd_raw(const float* grad, int64_t n, const std::vector<float*>& params,
                      const std::vector<int64_t>& numels, const float* lr_ptr, float lr_val, float scale, void* gstep,
                      int gkind, float* metrics, float* host_metrics, hipStream_t s) {
    if (params.empty() || params.size() > 8 || params.size() != numels.size())
      throw std::runtime_error("IpcColl.reduce_sgd: 1..8 parameters expected");
    if (n * 4 > cap_) throw std::runtime_error("IpcColl.reduce_sgd: gradient larger than the IPC slot");
    if (reinterpret_cast<uintptr_t>(grad) & 15)
      throw std::runtime_error("IpcColl.reduce_sgd: 16-byte aligned gradient");
    dtfk::ipcc::SgdArgs a{};
    int64_t e = 0;
    for (size_t i = 0; i < params.size(); ++i) {
      a.p[i] = params[i];
      e += numels[i];
      a.end[i] = e;
    }
    if (e != n) throw std::runtime_error("IpcColl.reduce_sgd: parameter sizes do not add up to the gradient");
    a.np = (int)params.size();
    a.lr_ptr = lr_ptr;
    a.lr_val = lr_val;
    a.scale = scale;
    a.gstep = gstep;
    a.gkind = gkind;
    a.metrics = metrics;
    a.host_metrics = host_metrics;
    ck(dtfk_ipcc_reduce_sgd(grad, n, a, coll(), grid_for(n * 4), s), "IpcColl: reduce_sgd launch");
  }

  void broadcast_raw(void* buf, int64_t nbytes, int src, hipStream_t s) {
    if ((reinterpret_cast<uintptr_t>(buf) & 3) || (nbytes & 3))
      throw std::runtime_error("IpcColl.broadcast: 4-byte aligned buffer and size expected");
    const int64_t chunk = cap_ / 16 * 16;
    for (int64_t off = 0; off < nbytes; off += chunk) {
      const int64_t m = std::min(chunk, nbytes - off);
      char* p = static_cast<char*>(buf) + off;
      ck(dtfk_ipcc_broadcast(p, p, m, src, coll(), grid_for(m), s), "IpcColl: broadcast launch");
    }
  }

  void all_gather_raw(const void* in, void* out, int64_t nbytes, hipStream_t s) {
    if (((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 3) || (nbytes & 3))
      throw std::runtime_error("IpcColl.all_gather: 4-byte aligned buffers and size expected");
    const int64_t chunk = cap_ / 16 * 16;
    for (int64_t off = 0; off < nbytes; off += chunk) {
      const int64_t m = std::min(chunk, nbytes - off);
      ck(dtfk_ipcc_allgather(static_cast<const char*>(in) + off, static_cast<char*>(out) + off, m, nbytes, coll(),
                             grid_for(m * W_), s),
         "IpcColl: all_gather launch");
    }
  }

  // counts in bytes per peer
  void all_to_all_raw(const void* in, const std::vector<int64_t>& send_bytes, void* out,
                      const std::vector<int64_t>& recv_bytes, hipStream_t s) {
    if ((int)send_bytes.size() != W_ || (int)recv_bytes.size() != W_)
      throw std::runtime_error("IpcColl.all_to_all: one count per rank expected");
    dtfk::ipcc::A2A a{};
    int64_t so = 0, ro = 0;
    for (int r = 0; r < W_; ++r) {
      if ((send_bytes[r] | recv_bytes[r]) & 3)
        throw std::runtime_error("IpcColl.all_to_all: counts must be whole 4-byte words");
      a.send_off[r] = so;
      a.recv_off[r] = ro;
      a.recv_bytes[r] = recv_bytes[r];
      so += send_bytes[r];
      ro += recv_bytes[r];
    }
    if ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 3)
      throw std::runtime_error("IpcColl.all_to_all: 4-byte aligned buffers expected");
    a.send_total = so;
    a.overflow = so > cap_ ? 1 : 0;
    ck(dtfk_ipcc_alltoall(in, out, a, coll(), grid_for(std::max(so, ro)), s), "IpcColl: all_to_all launch");
    if (a.overflow)
      throw std::runtime_error("IpcColl.all_to_all: this rank's send buffer (" + std::to_string(so) +
                               " bytes) exceeds the IPC slot capacity (" + std::to_string(cap_) +
                               " bytes; raise DTF_IPC_SLOT_MB)");
  }

 private:
  static void ck(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
  }

  py::object keep_;                 // the IpcPeerBuffers whose memory the table points into
  void* const* table_ = nullptr;
  int W_, rank_;
  int64_t cap_, two_shot_;
  int max_grid_;
  long long timeout_ = 0;
  int wide_ = 1;
  at::Tensor words_, err_, err_host_;
  hipEvent_t ev_ = nullptr;
  hipStream_t last_ = nullptr;
  int64_t calls_ = 0;
};

}  // namespace dtf
