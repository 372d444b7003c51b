// Python bindings for the fused MLP step kernels (csrc/kernels/mlp_step.hip)
// and the pinned-host -> device batch copy used by the input pipeline.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <pybind11/numpy.h>
#include <hip/hip_runtime.h>

#include "comm/ipc_coll_host.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <cstring>
#include <stdexcept>
#include <string>

extern "C" {
int dtfk_mlp_ksplit();
hipError_t dtfk_mlp_l1_fwd(const void* x, int x_kind, int B, const void* W1T, float* z2p,
                           long long* ts, hipStream_t stream);
hipError_t dtfk_mlp_head_bwd(const float* a2, const void* labels, int B, const void* W2T,
                             const void* W2N, const float* params, void* dz2T, int BP, float* partials,
                             float inv_batch, int act, int naive_loss, long long* gstep, long long* ts,
                             hipStream_t stream);
hipError_t dtfk_mlp_wgrad(const void* x, int x_kind, const void* dz2T, int BP, int B,
                          const float* partials, float* params, void* W1T, void* W2T, void* W2N,
                          void* grads, int grad_kind, const float* lr, float* metrics,
                          long long* gstep, int ring, long long* ts, void* const* ipc_table, int ipc_W,
                          int ipc_rank, int ipc_parity, long long ipc_slot_bytes, int* ipc_err,
                          long long ipc_timeout, hipStream_t stream);
hipError_t dtfk_mlp_apply_flat(float* params, const void* grads, int grad_kind, const float* lr,
                               float scale, void* W1T, void* W2T, void* W2N, hipStream_t stream);
int dtfk_mlp_ipc_flag_bytes();
int dtfk_mlpg_p1_floats();
hipError_t dtfk_mlpg_fwd(const void* x, const void* labels, int B, int BP, const void* W1F, const float* params,
                         float* a2g, float* P1, void* dz2F, int act, int naive, float gscale, hipStream_t s);
hipError_t dtfk_mlpg_wgrad(const void* x, int B, const void* dz2F, float* P2, int nchunk, hipStream_t s);
int dtfk_mlpg_wchunk(int B);
int dtfk_mlpg_p2_floats();
hipError_t dtfk_mlpg_apply(float* params, const float* P1, int n1, const float* P2, int n2, const float* gin,
                           float* gout, const float* lr, float scale, void* W1S, float* metrics, int ring,
                           long long* gstep, int B, int mode, hipStream_t s);
hipError_t dtfk_mlp_ipc_reduce_apply(float* params, void* const* peer_table, int W, int rank, int parity,
                                     long long slot_bytes, const long long* gstep, const float* lr, float scale,
                                     void* W1T, void* W2T, void* W2N, int* err, long long timeout_ticks,
                                     hipStream_t stream);
long long dtfk_mlpf_stage_rec();
void dtfk_mlpf_set_fault(int rank, long long step);
void dtfk_mlpf_set_res_ts(long long* p);
long long dtfk_mlpf_xbuf_bytes();
long long dtfk_mlpf_ipc_bytes();
int dtfk_mlpf_max_batch();
hipError_t dtfk_mlp_persist_f32(const void* stage, long long rec_h, int B, int nsteps, float* params, const float* lr,
                                float* metrics, int ring, int act, int naive, long long* gstep, unsigned long long* seq,
                                void* xbuf, int* err, long long timeout, long long* step_ts, int ts_ring,
                                const void* host_next, int next_steps, void* stage_next, void* const* peer_base, int W,
                                int rank, int gbf16, long long* phase_ts, int spread, int xmode, int split,
                                hipStream_t stream);
hipError_t dtfk_mlp_persist_f32_resident(void* stage, int B, float* W1, float* W2, float* b1, float* b2, const float* lr,
                                         float* metrics, int ring, int act, int naive, long long* gstep,
                                         unsigned long long* seq, void* xbuf, int* err, long long timeout,
                                         const long long* door, const void* host_recs, long long rec_h,
                                         const float* host_lr, float* host_out, long long* host_done,
                                         long long* host_state, long long launch_id, long long run0, long long idle,
                                         void* gvar, int gvar_kind, unsigned* dctr, hipStream_t stream);
long long dtfk_graph_mlp_part_floats(int B, int H);
hipError_t dtfk_graph_feed_ingest(const void* host, void* dev, long long bytes, hipStream_t stream);
hipError_t dtfk_graph_mlp_step(const float* x, const uint8_t* xu, const float* ylab, float* W1, float* b1, float* W2,
                               float* b2,
                               float* a2buf, float* dz2buf, float* part, float* gW1, float* gb1, float* gW2,
                               float* gb2, float* metrics, float* host_metrics, void* gstep, int gstep_kind,
                               const float* lr_ptr, int B, int K, int H, int C, int act, int naive, int sgd,
                               hipStream_t stream);
hipError_t dtfk_mlp_fwd_head(const void* x, int x_kind, int B, const void* W1T, float* z2p, const void* labels,
                             const void* W2T, const void* W2N, const float* params, void* dz2T, int BP,
                             float* partials, float inv_batch, int act, int naive_loss, int* counters,
                             long long* gstep, hipStream_t stream);
}

namespace dtf {

static hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

static void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

static void need(const at::Tensor& t, at::ScalarType dt, int64_t numel, const char* name) {
  if (!t.is_cuda()) throw std::runtime_error(std::string(name) + " must be a GPU tensor");
  if (!t.is_contiguous()) throw std::runtime_error(std::string(name) + " must be contiguous");
  if (t.scalar_type() != dt) throw std::runtime_error(std::string(name) + " has wrong dtype");
  if (numel >= 0 && t.numel() < numel)
    throw std::runtime_error(std::string(name) + " too small: " + std::to_string(t.numel()) +
                             " < " + std::to_string(numel));
}

constexpr int kNParam = 79510;

static long long* ts_ptr(const c10::optional<at::Tensor>& ts, int64_t need_numel) {
  if (!ts.has_value()) return nullptr;
  need(*ts, at::kLong, need_numel, "ts");
  return reinterpret_cast<long long*>(ts->data_ptr<int64_t>());
}

// optional per-step s_memrealtime ring (int64)
static long long* step_ts_ptr(const c10::optional<at::Tensor>& t, int* ring) {
  *ring = 1;
  if (!t.has_value()) return nullptr;
  need(*t, at::kLong, 2, "step_ts");
  *ring = (int)t->numel();
  return reinterpret_cast<long long*>(t->data_ptr<int64_t>());
}

// device-visible address of `nbytes` of pinned host memory at `off`
static const void* pinned_device_ptr(const c10::optional<at::Tensor>& host, int64_t off, int64_t nbytes) {
  if (!host.has_value()) throw std::runtime_error("next chunk needs the pinned host epoch");
  const at::Tensor& h = *host;
  if (h.is_cuda() || !h.is_pinned()) throw std::runtime_error("host must be pinned host memory");
  if (off < 0 || off % 16 != 0 || off + nbytes > (int64_t)(h.numel() * h.element_size()))
    throw std::runtime_error("host range out of bounds");
  void* dp = nullptr;
  char* hp = reinterpret_cast<char*>(h.data_ptr()) + off;
  if (hipHostGetDevicePointer(&dp, hp, 0) != hipSuccess || dp == nullptr) {
    (void)hipGetLastError();
    dp = hp;   // unified addressing: the host address is device-visible
  }
  if (reinterpret_cast<uintptr_t>(dp) % 16 != 0) throw std::runtime_error("pinned host pointer not aligned");
  return dp;
}

static int bp_of(int B) { return ((B + 31) / 32) * 32; }

// x_kind: 0 u8 pixels (/255), 1 fp32, 2 bf16; rows of 784 features.
static const char* x_ptr(const at::Tensor& x, int64_t off, int x_kind, int B) {
  const int64_t esz = x_kind == 0 ? 1 : (x_kind == 1 ? 4 : 2);
  if (x_kind < 0 || x_kind > 2) throw std::runtime_error("bad x_kind");
  if (!x.is_cuda() || !x.is_contiguous()) throw std::runtime_error("x must be a contiguous GPU tensor");
  if ((int64_t)x.numel() * x.element_size() < off + (int64_t)B * 784 * esz)
    throw std::runtime_error("x buffer too small");
  if (off % 16 != 0 || (reinterpret_cast<uintptr_t>(x.data_ptr()) % 16) != 0)
    throw std::runtime_error("x must be 16-byte aligned");
  return reinterpret_cast<const char*>(x.data_ptr()) + off;
}

// z2p: per-K-half partial pre-activations [ksplit][nb*16][112] fp32
void mlp_l1_fwd(at::Tensor x, int64_t x_off, int x_kind, int B, at::Tensor W1T, at::Tensor z2p,
                c10::optional<at::Tensor> ts) {
  if (B <= 0) throw std::runtime_error("B must be positive");
  const int nb = (B + 15) / 16;
  const char* xb = x_ptr(x, x_off, x_kind, B);
  need(W1T, at::kBFloat16, 112 * 800, "W1T");
  need(z2p, at::kFloat, (int64_t)dtfk_mlp_ksplit() * nb * 16 * 112, "z2p");
  hip_check(dtfk_mlp_l1_fwd(xb, x_kind, B, W1T.data_ptr(), z2p.data_ptr<float>(),
                            ts_ptr(ts, (int64_t)nb * 7 * dtfk_mlp_ksplit() * 16), cur_stream()),
            "mlp_l1_fwd");
}

// A1 + A2 in one launch (last-arriver row-block handoff); counters: int32[nb], zero at rest
void mlp_fwd_head(at::Tensor x, int64_t x_off, int x_kind, int B, at::Tensor W1T, at::Tensor z2p, at::Tensor labels,
                  int64_t labels_off, at::Tensor W2T, at::Tensor W2N, at::Tensor params, at::Tensor dz2T,
                  at::Tensor partials, double inv_batch, int act, bool naive_loss, at::Tensor counters,
                  at::Tensor gstep) {
  if (B <= 0) throw std::runtime_error("B must be positive");
  const int nb = (B + 15) / 16, BP = bp_of(B);
  const char* xb = x_ptr(x, x_off, x_kind, B);
  need(W1T, at::kBFloat16, 112 * 800, "W1T");
  need(z2p, at::kFloat, (int64_t)dtfk_mlp_ksplit() * nb * 16 * 112, "z2p");
  if (!labels.is_cuda() || labels.scalar_type() != at::kByte)
    throw std::runtime_error("labels must be a uint8 GPU tensor");
  if (labels.numel() < labels_off + B) throw std::runtime_error("labels buffer too small");
  need(W2T, at::kBFloat16, 16 * 128, "W2T");
  need(W2N, at::kBFloat16, 112 * 32, "W2N");
  need(params, at::kFloat, kNParam, "params");
  need(dz2T, at::kBFloat16, (int64_t)112 * BP, "dz2T");
  need(partials, at::kFloat, (int64_t)nb * 1112, "partials");
  need(counters, at::kInt, nb, "counters");
  hip_check(dtfk_mlp_fwd_head(xb, x_kind, B, W1T.data_ptr(), z2p.data_ptr<float>(),
                              reinterpret_cast<const uint8_t*>(labels.data_ptr()) + labels_off, W2T.data_ptr(),
                              W2N.data_ptr(), params.data_ptr<float>(), dz2T.data_ptr(), BP,
                              partials.data_ptr<float>(), (float)inv_batch, act, naive_loss ? 1 : 0,
                              counters.data_ptr<int>(), reinterpret_cast<long long*>(gstep.data_ptr<int64_t>()),
                              cur_stream()),
            "mlp_fwd_head");
}

void mlp_head_bwd(at::Tensor z2p, at::Tensor labels, int64_t labels_off, int B, at::Tensor W2T,
                  at::Tensor W2N, at::Tensor params, at::Tensor dz2T, at::Tensor partials, double inv_batch, int act,
                  bool naive_loss, at::Tensor gstep, c10::optional<at::Tensor> ts) {
  const int nb = (B + 15) / 16, BP = bp_of(B);
  need(z2p, at::kFloat, (int64_t)dtfk_mlp_ksplit() * nb * 16 * 112, "z2p");
  if (!labels.is_cuda() || labels.scalar_type() != at::kByte)
    throw std::runtime_error("labels must be a uint8 GPU tensor");
  if (labels.numel() < labels_off + B) throw std::runtime_error("labels buffer too small");
  need(W2T, at::kBFloat16, 16 * 128, "W2T");
  need(W2N, at::kBFloat16, 112 * 32, "W2N");
  need(params, at::kFloat, kNParam, "params");
  need(dz2T, at::kBFloat16, (int64_t)112 * BP, "dz2T");
  need(partials, at::kFloat, (int64_t)nb * 1112, "partials");
  hip_check(dtfk_mlp_head_bwd(z2p.data_ptr<float>(),
                              reinterpret_cast<const uint8_t*>(labels.data_ptr()) + labels_off, B,
                              W2T.data_ptr(), W2N.data_ptr(), params.data_ptr<float>(), dz2T.data_ptr(), BP,
                              partials.data_ptr<float>(), (float)inv_batch, act, naive_loss ? 1 : 0,
                              reinterpret_cast<long long*>(gstep.data_ptr<int64_t>()),
                              ts_ptr(ts, (int64_t)nb * 16), cur_stream()),
            "mlp_head_bwd");
}

// grad_kind: 0 fused SGD (grads ignored), 1 fp32 grads, 2 bf16 grads
void mlp_wgrad(at::Tensor x, int64_t x_off, int x_kind, at::Tensor dz2T, int B,
               at::Tensor partials, at::Tensor params, at::Tensor W1T, at::Tensor W2T,
               at::Tensor W2N, c10::optional<at::Tensor> grads, int grad_kind, at::Tensor lr, at::Tensor metrics,
               at::Tensor gstep, c10::optional<at::Tensor> ts, int64_t ipc_table, int ipc_W, int ipc_rank,
               int ipc_parity, int64_t ipc_slot_bytes, c10::optional<at::Tensor> ipc_err, double ipc_timeout_s) {
  const int nb = (B + 15) / 16, BP = bp_of(B);
  if (BP > 4096) throw std::runtime_error("per-GPU batch > 4096 not supported by mlp_wgrad");
  const char* xb = x_ptr(x, x_off, x_kind, B);
  need(dz2T, at::kBFloat16, (int64_t)112 * BP, "dz2T");
  need(partials, at::kFloat, (int64_t)nb * 1112, "partials");
  need(params, at::kFloat, kNParam, "params");
  need(W1T, at::kBFloat16, 112 * 800, "W1T");
  need(W2T, at::kBFloat16, 16 * 128, "W2T");
  need(W2N, at::kBFloat16, 112 * 32, "W2N");
  need(lr, at::kFloat, 1, "lr");
  need(metrics, at::kFloat, 2, "metrics");
  need(gstep, at::kLong, 1, "global_step");
  void* g = nullptr;
  int* errp = nullptr;
  if (grad_kind == 3) {
    if (ipc_table == 0 || ipc_W < 2 || ipc_rank < 0 || ipc_rank >= ipc_W || ipc_W > 64 || (ipc_parity & ~1) ||
        ipc_slot_bytes < kNParam * 2 || !ipc_err.has_value())
      throw std::runtime_error("mlp_wgrad: bad IPC arguments");
    if (!ipc_err->is_cuda() || ipc_err->scalar_type() != at::kInt) throw std::runtime_error("ipc_err: GPU int32");
    errp = ipc_err->data_ptr<int>();
  } else if (grad_kind != 0) {
    if (!grads.has_value()) throw std::runtime_error("grads required");
    need(*grads, grad_kind == 1 ? at::kFloat : at::kBFloat16, kNParam, "grads");
    g = grads->data_ptr();
  }
  const int ring = (int)(metrics.numel() / 2);
  hip_check(dtfk_mlp_wgrad(xb, x_kind, dz2T.data_ptr(), BP, B, partials.data_ptr<float>(),
                           params.data_ptr<float>(), W1T.data_ptr(), W2T.data_ptr(),
                           W2N.data_ptr(), g, grad_kind,
                           lr.data_ptr<float>(), metrics.data_ptr<float>(),
                           reinterpret_cast<long long*>(gstep.data_ptr<int64_t>()), ring,
                           ts_ptr(ts, (int64_t)(49 * 7 + 4) * 16), reinterpret_cast<void* const*>(ipc_table),
                           grad_kind == 3 ? ipc_W : 0, ipc_rank, ipc_parity, ipc_slot_bytes, errp,
                           (long long)(ipc_timeout_s * 1.0e8), cur_stream()),
            "mlp_wgrad");
}

// one-shot IPC all-reduce fused with SGD apply (see mlp_step.hip); peer_table is the
// device address of IpcPeerBuffers.table_ptr(); err: int32[1] device flag
void mlp_ipc_reduce_apply(at::Tensor params, int64_t peer_table, int W, int rank, int parity, int64_t slot_bytes,
                          at::Tensor gstep, at::Tensor lr, double scale, at::Tensor W1T, at::Tensor W2T,
                          at::Tensor W2N, at::Tensor err, double timeout_s) {
  need(params, at::kFloat, kNParam, "params");
  need(W1T, at::kBFloat16, 112 * 800, "W1T");
  need(W2T, at::kBFloat16, 16 * 128, "W2T");
  need(W2N, at::kBFloat16, 112 * 32, "W2N");
  if (!err.is_cuda() || err.scalar_type() != at::kInt) throw std::runtime_error("err must be a GPU int32 tensor");
  if (peer_table == 0 || W < 2 || rank < 0 || rank >= W || (parity & ~1) || slot_bytes < kNParam * 2)
    throw std::runtime_error("mlp_ipc_reduce_apply: bad arguments");
  const long long ticks = (long long)(timeout_s * 1.0e8);  // s_memrealtime runs at 100 MHz
  hip_check(dtfk_mlp_ipc_reduce_apply(params.data_ptr<float>(), reinterpret_cast<void* const*>(peer_table), W, rank, parity,
                               slot_bytes, reinterpret_cast<const long long*>(gstep.data_ptr<int64_t>()), lr.data_ptr<float>(), (float)scale,
                               W1T.data_ptr(), W2T.data_ptr(), W2N.data_ptr(), err.data_ptr<int>(), ticks, cur_stream()),
     "mlp_ipc_reduce_apply");
}

void mlp_apply_flat(at::Tensor params, c10::optional<at::Tensor> grads, at::Tensor lr,
                    double scale, at::Tensor W1T, at::Tensor W2T, at::Tensor W2N) {
  need(W2N, at::kBFloat16, 112 * 32, "W2N");
  need(params, at::kFloat, kNParam, "params");
  need(lr, at::kFloat, 1, "lr");
  need(W1T, at::kBFloat16, 112 * 800, "W1T");
  need(W2T, at::kBFloat16, 16 * 128, "W2T");
  const void* g = nullptr;
  int kind = 1;
  if (grads.has_value()) {
    if (grads->scalar_type() == at::kFloat) kind = 1;
    else if (grads->scalar_type() == at::kBFloat16) kind = 2;
    else throw std::runtime_error("grads must be fp32 or bf16");
    need(*grads, grads->scalar_type(), kNParam, "grads");
    g = grads->data_ptr();
  }
  hip_check(dtfk_mlp_apply_flat(params.data_ptr<float>(), g, kind, lr.data_ptr<float>(),
                                (float)scale, W1T.data_ptr(), W2T.data_ptr(), W2N.data_ptr(),
                                cur_stream()),
            "mlp_apply_flat");
}

// ---- large-batch GEMM step (kernels/mlp_gemm.hip); x / labels: u8 stage at a byte offset
static const uint8_t* stage_ptr(const at::Tensor& st, int64_t off, int64_t nbytes, const char* name) {
  need(st, at::kByte, -1, name);
  if (off < 0 || off + nbytes > st.numel()) throw std::runtime_error(std::string(name) + ": offset out of range");
  return st.data_ptr<uint8_t>() + off;
}

static int64_t mlpg_bp(int B) { return ((int64_t)B + 63) / 64 * 64; }
static int64_t mlpg_bp2(int B) {
  const int64_t c = dtfk_mlpg_wchunk(B);
  return ((int64_t)B + c - 1) / c * c;
}


void mlpg_fwd(at::Tensor x, int64_t x_off, at::Tensor labels, int64_t labels_off, int B, at::Tensor W1F,
              at::Tensor params, at::Tensor a2, at::Tensor P1, at::Tensor dz2F, int act, bool naive, double gscale) {
  const int64_t BP = mlpg_bp(B);
  if (B < 1) throw std::runtime_error("mlpg_fwd: B >= 1");
  const uint8_t* px = stage_ptr(x, x_off, (int64_t)B * 784, "x");
  if (reinterpret_cast<uintptr_t>(px) & 15) throw std::runtime_error("mlpg_fwd: x must be 16-byte aligned");
  const uint8_t* pl = stage_ptr(labels, labels_off, B, "labels");
  need(W1F, at::kBFloat16, 3 * 112 * 800, "W1F");
  need(params, at::kFloat, kNParam, "params");
  need(a2, at::kFloat, BP * 112, "a2");
  need(P1, at::kFloat, BP / 16 * dtfk_mlpg_p1_floats(), "P1");
  need(dz2F, at::kBFloat16, 3 * 112 * mlpg_bp2(B), "dz2F");
  hip_check(dtfk_mlpg_fwd(px, pl, B, (int)BP, W1F.data_ptr(), params.data_ptr<float>(), a2.data_ptr<float>(),
                          P1.data_ptr<float>(), dz2F.data_ptr(), act, naive ? 1 : 0, (float)gscale, cur_stream()),
            "mlpg_fwd");
}

void mlpg_wgrad(at::Tensor x, int64_t x_off, int B, at::Tensor dz2F, at::Tensor P2, int nchunk) {
  const int64_t BP2 = mlpg_bp2(B);
  const uint8_t* px = stage_ptr(x, x_off, (int64_t)B * 784, "x");
  if (reinterpret_cast<uintptr_t>(px) & 15) throw std::runtime_error("mlpg_wgrad: x must be 16-byte aligned");
  if (nchunk != BP2 / dtfk_mlpg_wchunk(B)) throw std::runtime_error("mlpg_wgrad: nchunk must be ceil(B / chunk)");
  need(dz2F, at::kBFloat16, 3 * 112 * BP2, "dz2F");
  need(P2, at::kFloat, (int64_t)nchunk * dtfk_mlpg_p2_floats(), "P2");
  hip_check(dtfk_mlpg_wgrad(px, B, dz2F.data_ptr(), P2.data_ptr<float>(), nchunk, cur_stream()), "mlpg_wgrad");
}

void mlpg_apply(at::Tensor params, at::Tensor P1, at::Tensor P2, int nchunk, c10::optional<at::Tensor> gin,
                c10::optional<at::Tensor> gout, at::Tensor lr, double scale, at::Tensor W1S, at::Tensor metrics,
                at::Tensor gstep, int B, int mode) {
  const int64_t BP = mlpg_bp(B);
  if (mode < 0 || mode > 3) throw std::runtime_error("mlpg_apply: mode 0..3");
  need(params, at::kFloat, kNParam, "params");
  need(P1, at::kFloat, BP / 16 * dtfk_mlpg_p1_floats(), "P1");
  need(P2, at::kFloat, (int64_t)nchunk * dtfk_mlpg_p2_floats(), "P2");
  if (mode == 2 && !gin.has_value()) throw std::runtime_error("mlpg_apply: mode 2 needs gin");
  if (mode == 1 && !gout.has_value()) throw std::runtime_error("mlpg_apply: mode 1 needs gout");
  if (gin.has_value()) need(*gin, at::kFloat, kNParam, "gin");
  if (gout.has_value()) need(*gout, at::kFloat, kNParam, "gout");
  need(lr, at::kFloat, 1, "lr");
  need(W1S, at::kBFloat16, 3 * 112 * 800, "W1S");
  need(metrics, at::kFloat, 2, "metrics");
  need(gstep, at::kLong, 1, "gstep");
  hip_check(dtfk_mlpg_apply(params.data_ptr<float>(), P1.data_ptr<float>(), (int)(BP / 16), P2.data_ptr<float>(),
                            nchunk, gin.has_value() ? gin->data_ptr<float>() : nullptr,
                            gout.has_value() ? gout->data_ptr<float>() : nullptr, lr.data_ptr<float>(), (float)scale,
                            W1S.data_ptr(), metrics.data_ptr<float>(), (int)(metrics.numel() / 2),
                            reinterpret_cast<long long*>(gstep.data_ptr<int64_t>()), B, mode, cur_stream()),
            "mlpg_apply");
}

// hipMemcpyAsync host(pinned) -> device on the *current* stream (graph-capturable).
void memcpy_h2d_async(at::Tensor dst, int64_t dst_offset, at::Tensor src, int64_t src_offset,
                      int64_t nbytes) {
  if (!dst.is_cuda()) throw std::runtime_error("dst must be a GPU tensor");
  if (src.is_cuda()) throw std::runtime_error("src must be a host tensor");
  if (!src.is_pinned()) throw std::runtime_error("src must be pinned host memory");
  if (dst_offset + nbytes > (int64_t)(dst.numel() * dst.element_size()) ||
      src_offset + nbytes > (int64_t)(src.numel() * src.element_size()))
    throw std::runtime_error("memcpy_h2d_async out of range");
  hip_check(hipMemcpyAsync(reinterpret_cast<char*>(dst.data_ptr()) + dst_offset,
                           reinterpret_cast<const char*>(src.data_ptr()) + src_offset, nbytes,
                           hipMemcpyHostToDevice, cur_stream()),
            "hipMemcpyAsync");
}

// The fp32 persistent engine (csrc/kernels/mlp_persist_f32.hip; mfma_split: the big
// GEMMs as exact 3-way bf16 splits, else f32-input MFMA): `nsteps` SGD steps of
// the chunk staged in `stage` (records of mlpf_stage_rec() bytes) and, in the same
// launch, `next_steps` host records from byte `host_off` of the pinned epoch into
// `stage_next`.  nsteps = 0: copy only.  xbuf: exchange buffer (zeroed once).
void mlp_persist_f32(at::Tensor stage, int64_t rec_h, int B, int nsteps, at::Tensor params, at::Tensor lr,
                     at::Tensor metrics, at::Tensor gstep, at::Tensor seq, at::Tensor xbuf, at::Tensor err,
                     double timeout_s, int act, int naive, c10::optional<at::Tensor> host, int64_t host_off,
                     int next_steps, c10::optional<at::Tensor> stage_next, c10::optional<at::Tensor> step_ts,
                     int64_t ipc_table, int ipc_W, int ipc_rank, bool grad_bf16,
                     c10::optional<at::Tensor> phase_ts, bool spread, bool two_shot, bool mfma_split) {
  if (ipc_W > 1 && (ipc_table == 0 || ipc_rank < 0 || ipc_rank >= ipc_W || ipc_W > 64))
    throw std::runtime_error("mlp_persist_f32: N-GPU exchange needs the IPC peer table");
  if (B <= 0 || B > dtfk_mlpf_max_batch()) throw std::runtime_error("mlp_persist_f32: B out of range");
  if (rec_h < (int64_t)B * 785 || rec_h % 16 != 0) throw std::runtime_error("mlp_persist_f32: bad host record size");
  if (nsteps < 0 || next_steps < 0) throw std::runtime_error("mlp_persist_f32: negative step count");
  const int64_t rec_s = dtfk_mlpf_stage_rec();
  need(stage, at::kByte, (int64_t)std::max(nsteps, 1) * rec_s, "stage");
  need(params, at::kFloat, kNParam, "params");
  need(lr, at::kFloat, 1, "lr");
  need(metrics, at::kFloat, 2, "metrics");
  need(gstep, at::kLong, 1, "gstep");
  need(seq, at::kLong, 1, "seq");
  need(xbuf, at::kByte, dtfk_mlpf_xbuf_bytes(), "xbuf");
  need(err, at::kInt, 1, "err");
  if (((uintptr_t)stage.data_ptr() | (uintptr_t)xbuf.data_ptr()) % 16 != 0)
    throw std::runtime_error("mlp_persist_f32: stage / xbuf must be 16-byte aligned");
  const void* hn = nullptr;
  void* sn = nullptr;
  if (next_steps > 0) {
    if (!stage_next.has_value()) throw std::runtime_error("mlp_persist_f32: next chunk needs stage_next");
    need(*stage_next, at::kByte, (int64_t)next_steps * rec_s, "stage_next");
    if ((uintptr_t)stage_next->data_ptr() % 16 != 0) throw std::runtime_error("stage_next must be 16-byte aligned");
    if (stage_next->data_ptr() == stage.data_ptr() && nsteps > 0)
      throw std::runtime_error("mlp_persist_f32: stage_next must not alias the running stage");
    hn = pinned_device_ptr(host, host_off, (int64_t)next_steps * rec_h);
    sn = stage_next->data_ptr();
  }
  int ts_ring = 1;
  long long* sts = step_ts_ptr(step_ts, &ts_ring);
  const long long ticks = (long long)(timeout_s * 1e8);   // s_memrealtime: 100 MHz
  const hipError_t e =
      dtfk_mlp_persist_f32(stage.data_ptr(), rec_h, B, nsteps, params.data_ptr<float>(), lr.data_ptr<float>(),
                             metrics.data_ptr<float>(), (int)(metrics.numel() / 2), act, naive,
                             reinterpret_cast<long long*>(gstep.data_ptr<int64_t>()),
                             reinterpret_cast<unsigned long long*>(seq.data_ptr<int64_t>()), xbuf.data_ptr(),
                             err.data_ptr<int>(), ticks, sts, ts_ring, hn, next_steps, sn,
                             reinterpret_cast<void* const*>(ipc_table), ipc_W > 1 ? ipc_W : 1,
                             ipc_W > 1 ? ipc_rank : 0, grad_bf16 ? 1 : 0, ts_ptr(phase_ts, 65 * 64 * 16),
                             spread ? 1 : 0, two_shot ? 1 : 0, mfma_split ? 1 : 0, cur_stream());
  hip_check(e,
            "mlp_persist_f32");
}

// A prepared launcher for the fp32 persistent engine: every tensor checked and
// every pointer resolved once, so a launch from Python is a call with 6 ints
// (the generic binding's ~27 keyword arguments and per-call checks cost ~10 us
// of host time on a 20-step run: scripts/probes/launch_overhead.py).
struct PersistF32Plan {
  at::Tensor stage0, stage1, params, lr, metrics, gstep, seq, xbuf, err, step_ts, host;
  void* st[2];
  const char* host_dev = nullptr;
  int64_t host_bytes = 0, rec_h = 0, rec_s = 0;
  int B, act, naive, ring, ts_ring = 1, W, rank, gbf16, spread, two_shot, split;
  long long ticks;
  int64_t ipc_table;

  PersistF32Plan(at::Tensor s0, at::Tensor s1, int64_t rec_h_, int B_, at::Tensor params_, at::Tensor lr_,
                 at::Tensor metrics_, at::Tensor gstep_, at::Tensor seq_, at::Tensor xbuf_, at::Tensor err_,
                 double timeout_s, int act_, int naive_, at::Tensor host_, at::Tensor step_ts_, int64_t ipc_table_,
                 int ipc_W, int ipc_rank, bool grad_bf16, bool spread_, bool two_shot_, bool mfma_split)
      : stage0(s0), stage1(s1), params(params_), lr(lr_), metrics(metrics_), gstep(gstep_), seq(seq_), xbuf(xbuf_),
        err(err_), step_ts(step_ts_), host(host_) {
    if (ipc_W > 1 && (ipc_table_ == 0 || ipc_rank < 0 || ipc_rank >= ipc_W || ipc_W > 64))
      throw std::runtime_error("PersistF32Plan: N-GPU exchange needs the IPC peer table");
    if (B_ <= 0 || B_ > dtfk_mlpf_max_batch()) throw std::runtime_error("PersistF32Plan: B out of range");
    if (rec_h_ < (int64_t)B_ * 785 || rec_h_ % 16 != 0) throw std::runtime_error("PersistF32Plan: bad record size");
    rec_s = dtfk_mlpf_stage_rec();
    need(stage0, at::kByte, rec_s, "stage0");
    need(stage1, at::kByte, rec_s, "stage1");
    need(params, at::kFloat, kNParam, "params");
    need(lr, at::kFloat, 1, "lr");
    need(metrics, at::kFloat, 2, "metrics");
    need(gstep, at::kLong, 1, "gstep");
    need(seq, at::kLong, 1, "seq");
    need(xbuf, at::kByte, dtfk_mlpf_xbuf_bytes(), "xbuf");
    need(err, at::kInt, 1, "err");
    need(step_ts, at::kLong, 2, "step_ts");
    st[0] = stage0.data_ptr();
    st[1] = stage1.data_ptr();
    if ((((uintptr_t)st[0]) | ((uintptr_t)st[1]) | (uintptr_t)xbuf.data_ptr()) % 16 != 0)
      throw std::runtime_error("PersistF32Plan: stage / xbuf must be 16-byte aligned");
    host_bytes = host.numel() * host.element_size();
    host_dev = static_cast<const char*>(pinned_device_ptr(host, 0, host_bytes));
    rec_h = rec_h_;
    B = B_;
    act = act_;
    naive = naive_;
    ring = (int)(metrics.numel() / 2);
    ts_ring = (int)step_ts.numel();
    ticks = (long long)(timeout_s * 1e8);
    ipc_table = ipc_table_;
    W = ipc_W > 1 ? ipc_W : 1;
    rank = ipc_W > 1 ? ipc_rank : 0;
    gbf16 = grad_bf16 ? 1 : 0;
    spread = spread_ ? 1 : 0;
    two_shot = two_shot_ ? 1 : 0;
    split = mfma_split ? 1 : 0;
  }

  // nsteps steps from stage `par` at step offset `off`; next_steps host records from
  // byte host_off into stage par ^ 1 (same contract as mlp_persist_f32 above)
  void launch(int par, int64_t off, int nsteps, int64_t host_off, int next_steps) {
    if ((par & ~1) != 0 || nsteps < 0 || next_steps < 0 || off < 0) throw std::runtime_error("PersistF32Plan: args");
    const at::Tensor& cur = par ? stage1 : stage0;
    const at::Tensor& nxt = par ? stage0 : stage1;
    if ((off + std::max(nsteps, 1)) * rec_s > cur.numel()) throw std::runtime_error("PersistF32Plan: stage overrun");
    const void* hn = nullptr;
    void* sn = nullptr;
    if (next_steps > 0) {
      if ((int64_t)next_steps * rec_s > nxt.numel()) throw std::runtime_error("PersistF32Plan: next stage too small");
      if (host_off < 0 || host_off % 16 != 0 || host_off + (int64_t)next_steps * rec_h > host_bytes)
        throw std::runtime_error("PersistF32Plan: host range out of bounds");
      hn = host_dev + host_off;
      sn = st[par ^ 1];
    }
    hip_check(dtfk_mlp_persist_f32(static_cast<const char*>(st[par]) + off * rec_s, rec_h, B, nsteps,
                                   params.data_ptr<float>(), lr.data_ptr<float>(), metrics.data_ptr<float>(), ring,
                                   act, naive, reinterpret_cast<long long*>(gstep.data_ptr<int64_t>()),
                                   reinterpret_cast<unsigned long long*>(seq.data_ptr<int64_t>()), xbuf.data_ptr(),
                                   err.data_ptr<int>(), ticks,
                                   reinterpret_cast<long long*>(step_ts.data_ptr<int64_t>()), ts_ring, hn,
                                   next_steps, sn, reinterpret_cast<void* const*>(ipc_table), W, rank, gbf16,
                                   nullptr, spread, two_shot, split, cur_stream()),
              "PersistF32Plan.launch");
  }
};

static int gstep_kind_of(const at::Tensor& g) {
  TORCH_CHECK(g.is_cuda() && g.numel() == 1, "graph_mlp_step: device scalar global_step");
  switch (g.scalar_type()) {
    case at::kFloat: return 0;
    case at::kLong: return 1;
    case at::kInt: return 2;
    case at::kDouble: return 3;
    default: TORCH_CHECK(false, "graph_mlp_step: unsupported global_step dtype");
  }
  return 0;
}

// The compat graph's matched MLP training step (csrc/kernels/graph_mlp.hip).
// sgd: W/b updated in place with lr; else gradients into g* (same shapes).
void graph_mlp_step(at::Tensor x, at::Tensor ylab, at::Tensor W1, at::Tensor b1, at::Tensor W2, at::Tensor b2,
                    at::Tensor a2buf, at::Tensor dz2buf, c10::optional<std::vector<at::Tensor>> grads,
                    at::Tensor metrics,
                    c10::optional<at::Tensor> gstep, double lr, int act, bool naive, bool sgd) {
  for (const at::Tensor* t : {&x, &ylab, &W1, &b1, &W2, &b2, &a2buf, &dz2buf, &metrics}) {
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous(),
                "graph_mlp_step: fp32 contiguous device tensors expected");
  }
  TORCH_CHECK(x.dim() == 2 && W1.dim() == 2 && W2.dim() == 2, "graph_mlp_step: 2-D x, W1, W2");
  const int B = (int)x.size(0), K = (int)x.size(1), H = (int)W1.size(1), C = (int)W2.size(1);
  TORCH_CHECK(W1.size(0) == K && W2.size(0) == H && b1.numel() == H && b2.numel() == C &&
                  ylab.numel() == (int64_t)B * C,
              "graph_mlp_step: shape mismatch");
  const int HP = (H + 16) & ~15, BP = (B + 15) & ~15;
  TORCH_CHECK(a2buf.numel() >= (int64_t)BP * HP && dz2buf.numel() >= (int64_t)BP * HP && metrics.numel() >= 3,
              "graph_mlp_step: scratch too small");
  float *gW1 = nullptr, *gb1 = nullptr, *gW2 = nullptr, *gb2 = nullptr;
  if (!sgd) {
    TORCH_CHECK(grads.has_value() && grads->size() == 4, "graph_mlp_step: gradients [dW1, db1, dW2, db2] expected");
    const int64_t n[4] = {(int64_t)K * H, H, (int64_t)H * C, C};
    float** dst[4] = {&gW1, &gb1, &gW2, &gb2};
    for (int i = 0; i < 4; ++i) {
      const at::Tensor& g = (*grads)[i];
      TORCH_CHECK(g.is_cuda() && g.scalar_type() == at::kFloat && g.is_contiguous() && g.numel() == n[i],
                  "graph_mlp_step: bad gradient tensor ", i);
      *dst[i] = g.data_ptr<float>();
    }
  }
  void* gp = nullptr;
  int kind = 0;
  if (gstep.has_value()) {
    kind = gstep_kind_of(*gstep);
    gp = gstep->data_ptr();
  }
  // L2's partials + the learning rate on the device (scratch from the caching allocator)
  at::Tensor part = at::zeros({dtfk_graph_mlp_part_floats(B, H) + 1}, x.options());
  part.narrow(0, 0, 1).fill_(lr);
  hip_check(dtfk_graph_mlp_step(x.data_ptr<float>(), nullptr, ylab.data_ptr<float>(), W1.data_ptr<float>(),
                                b1.data_ptr<float>(), W2.data_ptr<float>(), b2.data_ptr<float>(),
                                a2buf.data_ptr<float>(), dz2buf.data_ptr<float>(), part.data_ptr<float>() + 1, gW1,
                                gb1, gW2, gb2, metrics.data_ptr<float>(), nullptr, gp, kind, part.data_ptr<float>(), B, K, H, C,
                                act, naive ? 1 : 0, sgd ? 1 : 0, cur_stream()),
            "graph_mlp_step");
}

// The lowered Session.run of the reference's training graph as ONE host call
// (compat/lowering.py, in-kernel SGD): the numpy feeds x [B,K] / y_ [B,C] and the
// learning rate go into a pinned staging slot (one memcpy, GIL released), ONE
// host-to-device copy, then L1 / L2 / L3 and the loss / accuracy / global_step
// device-to-host copy replayed from a captured hipGraph; with `sync` the call
// returns after the step (the reference fetches the loss every step).
class GraphStepPlan {
 public:
  GraphStepPlan(at::Tensor W1, at::Tensor b1, at::Tensor W2, at::Tensor b2, c10::optional<at::Tensor> gstep, int B,
                int act, bool naive, bool use_graph)
      : W1_(W1), b1_(b1), W2_(W2), b2_(b2), B_(B), act_(act), naive_(naive), use_graph_(use_graph) {
    const char* df = getenv("DTF_GRAPH_STEP_DIRECT_FEED");
    direct_feed_ = df != nullptr && df[0] == '1';
    const char* hs = getenv("DTF_GRAPH_STEP_METRICS_COPY");   // 1: copy the metrics back with a D2H op
    host_store_ = !(hs != nullptr && hs[0] == '1');
    // 1: the feed read over PCIe by an ingest kernel instead of the copy engine
    // (system-scope 8-byte loads: 17 us for the 0.3 MB feed vs ~15 us by DMA -- kept off)
    const char* fk = getenv("DTF_GRAPH_STEP_FEED_KERNEL");
    kernel_feed_ = fk != nullptr && fk[0] == '1';
    for (const at::Tensor* t : {&W1, &b1, &W2, &b2})
      TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous(),
                  "GraphStepPlan: fp32 contiguous device parameters expected");
    K_ = (int)W1.size(0);
    H_ = (int)W1.size(1);
    C_ = (int)W2.size(1);
    TORCH_CHECK(W2.size(0) == H_ && b1.numel() == H_ && b2.numel() == C_, "GraphStepPlan: shape mismatch");
    HP_ = (H_ + 16) & ~15;
    const int BP = (B_ + 15) & ~15;
    if (gstep.has_value()) {
      gkind_ = gstep_kind_of(*gstep);
      gstep_ = *gstep;
    }
    nfeed_ = ((int64_t)B_ * K_ + (int64_t)B_ * C_ + 1 + 3) / 4 * 4;   // x | y | lr, padded to 16 bytes
    feed_bytes_ = nfeed_ * (int64_t)sizeof(float);
    auto fo = W1.options();
    dev_ = at::empty({nfeed_}, fo);
    a2_ = at::empty({(int64_t)BP * HP_}, fo);
    dz2_ = at::empty({(int64_t)BP * HP_}, fo);
    part_ = at::zeros({dtfk_graph_mlp_part_floats(B_, H_)}, fo);
    metrics_ = at::zeros({4}, fo);
    auto ho = at::TensorOptions().dtype(at::kFloat).pinned_memory(true);
    for (int i = 0; i < 2; ++i) stage_[i] = at::empty({nfeed_}, ho);
    host_metrics_ = at::zeros({4}, ho);
    for (int i = 0; i < 2; ++i) hip_check(hipEventCreateWithFlags(&ev_[i], hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventCreateWithFlags(&in_ev_, hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventCreateWithFlags(&out_ev_, hipEventDisableTiming), "hipEventCreate");
    // its own stream: graph capture needs one that is not the legacy default stream
    hip_check(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking), "hipStreamCreate");
  }
  ~GraphStepPlan() {
    if (exec_) (void)hipGraphExecDestroy(exec_);
    if (graph_) (void)hipGraphDestroy(graph_);
    for (auto& e : ev_)
      if (e) (void)hipEventDestroy(e);
    if (in_ev_) (void)hipEventDestroy(in_ev_);
    if (out_ev_) (void)hipEventDestroy(out_ev_);
    if (st_) (void)hipStreamDestroy(st_);
  }

  at::Tensor host_metrics() const { return host_metrics_; }

  // Synchronous data parallelism over the node's IPC data plane: the step's
  // kernels write this worker's gradients (flat [W1 | b1 | W2 | b2], fp32) and
  // ONE more kernel all-reduces them with every worker's in rank order, applies
  // p -= lr / W * sum on the graph's variables and bumps global_step
  // (csrc/kernels/ipc_coll.hip reduce_sgd_k) -- no RCCL, no host round trip.
  // Direct launches only (the collective's sequence number lives on the device,
  // but the plan's own graph capture is single-worker).
  void attach_ipc(py::object coll) {
    TORCH_CHECK(!use_graph_, "GraphStepPlan.attach_ipc: direct-launch plans only");
    ipc_obj_ = coll;
    ipc_ = coll.cast<IpcColl*>();
    const int64_t n = (int64_t)K_ * H_ + H_ + (int64_t)H_ * C_ + C_;
    grad_ = at::zeros({(n + 1) & ~1LL}, W1_.options());
  }
  bool has_ipc() const { return ipc_ != nullptr; }

  // One training step.  x, y: C-contiguous float32 numpy arrays of the plan's
  // shapes.  Returns after the step when `sync` (host_metrics() then holds
  // loss, accuracy, global_step after the step).
  void run(py::array x, py::array y, double lr, bool sync) {
    const int64_t nx = (int64_t)B_ * K_, ny = (int64_t)B_ * C_;
    TORCH_CHECK(x.dtype().is(py::dtype::of<float>()) && y.dtype().is(py::dtype::of<float>()),
                "GraphStepPlan.run: float32 feeds expected");
    TORCH_CHECK((x.flags() & py::array::c_style) && (y.flags() & py::array::c_style),
                "GraphStepPlan.run: C-contiguous feeds expected");
    TORCH_CHECK(x.size() == nx && y.size() == ny, "GraphStepPlan.run: feed shapes differ from the plan's");
    const float* xp = static_cast<const float*>(x.data());
    const float* yp = static_cast<const float*>(y.data());
    hipStream_t cur = cur_stream(), st = use_graph_ ? st_ : cur;
    const int slot = slot_ ^= 1;
    {
      py::gil_scoped_release nogil;
      if (!use_graph_) {   // direct launches on the caller's stream: no cross-stream events, no replay floor
        using clk = std::chrono::steady_clock;
        const auto t0 = clk::now();
        // the copy that last read this staging slot: only an unsynchronized call
        // leaves one in flight (a synchronizing call needs no event at all)
        if (pending_[slot]) hip_check(hipEventSynchronize(ev_[slot]), "GraphStepPlan: staging slot");
        pending_[slot] = false;
        float* h = stage_[slot].data_ptr<float>();
        float* d = dev_.data_ptr<float>();
        if (direct_feed_) {
          // x / y_ straight from the caller's memory (zero-copy DMA when it is
          // pinned; HIP's own pipelined staging when pageable); lr via the slot
          h[nx + ny] = (float)lr;
          hip_check(hipMemcpyAsync(d, xp, sizeof(float) * nx, hipMemcpyHostToDevice, st), "GraphStepPlan: x copy");
          hip_check(hipMemcpyAsync(d + nx, yp, sizeof(float) * ny, hipMemcpyHostToDevice, st), "GraphStepPlan: y copy");
          hip_check(hipMemcpyAsync(d + nx + ny, h + nx + ny, sizeof(float), hipMemcpyHostToDevice, st),
                    "GraphStepPlan: lr copy");
        } else {
          std::memcpy(h, xp, sizeof(float) * nx);
          std::memcpy(h + nx, yp, sizeof(float) * ny);
          h[nx + ny] = (float)lr;
          t_[0] += std::chrono::duration<double, std::micro>(clk::now() - t0).count();
          if (kernel_feed_)   // workgroups read the pinned slot over PCIe (no copy-engine op)
            hip_check(dtfk_graph_feed_ingest(h, d, feed_bytes_, st), "GraphStepPlan: feed ingest");
          else
            hip_check(hipMemcpyAsync(d, h, sizeof(float) * (nx + ny + 1), hipMemcpyHostToDevice, st),
                      "GraphStepPlan: feed copy");
        }
        if (!sync) {
          hip_check(hipEventRecord(ev_[slot], st), "GraphStepPlan: event");
          pending_[slot] = true;
        }
        hip_check(launch_step(st, host_store_), "GraphStepPlan: launch");
        const auto t2 = clk::now();
        t_[1] += std::chrono::duration<double, std::micro>(t2 - t0).count();
        if (sync) {
          hip_check(hipStreamSynchronize(st), "GraphStepPlan: sync");
          pending_[0] = pending_[1] = false;
        }
        t_[2] += std::chrono::duration<double, std::micro>(clk::now() - t2).count();
        ++steps_;
        return;
      }
      hip_check(hipEventSynchronize(ev_[slot]), "GraphStepPlan: staging slot");   // its last copy is done
      pending_[slot] = false;
      float* h = stage_[slot].data_ptr<float>();
      std::memcpy(h, xp, sizeof(float) * nx);
      std::memcpy(h + nx, yp, sizeof(float) * ny);
      h[nx + ny] = (float)lr;
      // after whatever the caller's stream queued (variable init, eager updates)
      hip_check(hipEventRecord(in_ev_, cur), "GraphStepPlan: event");
      hip_check(hipStreamWaitEvent(st, in_ev_, 0), "GraphStepPlan: wait");
      hip_check(hipMemcpyAsync(dev_.data_ptr<float>(), h, sizeof(float) * (nx + ny + 1), hipMemcpyHostToDevice, st),
                "GraphStepPlan: feed copy");
      hip_check(hipEventRecord(ev_[slot], st), "GraphStepPlan: event");
      if (exec_ == nullptr) capture(st);
      hip_check(hipGraphLaunch(exec_, st), "GraphStepPlan: graph launch");
      if (sync) {
        hip_check(hipStreamSynchronize(st), "GraphStepPlan: sync");
      } else {   // later work on the caller's stream sees the updated variables
        hip_check(hipEventRecord(out_ev_, st), "GraphStepPlan: event");
        hip_check(hipStreamWaitEvent(cur, out_ev_, 0), "GraphStepPlan: wait");
      }
    }
    ++steps_;
  }
  // The same step fed uint8 pixels (the MNIST loader's source bytes of a float
  // batch x = u8 / 255, data/mnist.py): a 4x smaller staging copy and transfer;
  // the kernels convert with the loader's exact float32 division, so the step is
  // bit-identical to run() with that float batch.  Direct launches only.
  void run_u8(py::array xu8, py::array y, double lr, bool sync) {
    const int64_t nx = (int64_t)B_ * K_, ny = (int64_t)B_ * C_;
    TORCH_CHECK(!use_graph_, "GraphStepPlan.run_u8: direct-launch plans only");
    TORCH_CHECK(xu8.dtype().is(py::dtype::of<uint8_t>()) && y.dtype().is(py::dtype::of<float>()),
                "GraphStepPlan.run_u8: uint8 x and float32 y_ expected");
    TORCH_CHECK((xu8.flags() & py::array::c_style) && (y.flags() & py::array::c_style),
                "GraphStepPlan.run_u8: C-contiguous feeds expected");
    TORCH_CHECK(xu8.size() == nx && y.size() == ny, "GraphStepPlan.run_u8: feed shapes differ from the plan's");
    TORCH_CHECK(K_ % 4 == 0, "GraphStepPlan.run_u8: K % 4 == 0 expected");
    const uint8_t* xp = static_cast<const uint8_t*>(xu8.data());
    const float* yp = static_cast<const float*>(y.data());
    hipStream_t st = cur_stream();
    const int slot = slot_ ^= 1;
    const int64_t xf = u8_x_floats();
    {
      py::gil_scoped_release nogil;
      using clk = std::chrono::steady_clock;
      const auto t0 = clk::now();
      if (pending_[slot]) hip_check(hipEventSynchronize(ev_[slot]), "GraphStepPlan: staging slot");
      pending_[slot] = false;
      float* h = stage_[slot].data_ptr<float>();
      std::memcpy(h, xp, (size_t)nx);
      std::memcpy(h + xf, yp, sizeof(float) * ny);
      h[xf + ny] = (float)lr;
      t_[0] += std::chrono::duration<double, std::micro>(clk::now() - t0).count();
      hip_check(hipMemcpyAsync(dev_.data_ptr<float>(), h, sizeof(float) * (xf + ny + 1), hipMemcpyHostToDevice, st),
                "GraphStepPlan: feed copy");
      if (!sync) {
        hip_check(hipEventRecord(ev_[slot], st), "GraphStepPlan: event");
        pending_[slot] = true;
      }
      hip_check(launch_step(st, host_store_, true), "GraphStepPlan: launch");
      const auto t2 = clk::now();
      t_[1] += std::chrono::duration<double, std::micro>(t2 - t0).count();
      if (sync) {
        hip_check(hipStreamSynchronize(st), "GraphStepPlan: sync");
        pending_[0] = pending_[1] = false;
      }
      t_[2] += std::chrono::duration<double, std::micro>(clk::now() - t2).count();
      ++steps_;
    }
  }
  int64_t steps() const { return steps_; }
  bool use_graph() const { return use_graph_; }
  // host-side split of the direct-launch calls so far, us per call: feed copy
  // into the staging slot, everything up to the last enqueue, the final wait
  py::dict timing() const {
    py::dict d;
    const double n = steps_ > 0 ? (double)steps_ : 1.0;
    d["feed_memcpy_us"] = t_[0] / n;
    d["enqueue_us"] = t_[1] / n;
    d["sync_us"] = t_[2] / n;
    d["calls"] = steps_;
    return d;
  }

 private:
  // the step's three kernels on stream st; the metrics reach host_metrics_
  // either from the last kernel itself (system-scope stores into the pinned
  // buffer: direct launches) or by a copy back (captured graphs)
  hipError_t launch_step(hipStream_t st, bool host_store, bool u8 = false) {
    const int64_t nx = (int64_t)B_ * K_, ny = (int64_t)B_ * C_;
    float* d = dev_.data_ptr<float>();
    // uint8 feed: [x bytes padded to 16 | y_ | lr] in the same device buffer
    const uint8_t* xu = u8 ? reinterpret_cast<const uint8_t*>(d) : nullptr;
    float* yd = u8 ? d + u8_x_floats() : d + nx;
    float* gW1 = nullptr, *gb1 = nullptr, *gW2 = nullptr, *gb2 = nullptr;
    if (ipc_ != nullptr) {     // gradients out (flat, variable order), then the IPC reduce + SGD
      gW1 = grad_.data_ptr<float>();
      gb1 = gW1 + (int64_t)K_ * H_;
      gW2 = gb1 + H_;
      gb2 = gW2 + (int64_t)H_ * C_;
    }
    hipError_t e = dtfk_graph_mlp_step(u8 ? nullptr : d, xu, yd, W1_.data_ptr<float>(), b1_.data_ptr<float>(), W2_.data_ptr<float>(),
                                       b2_.data_ptr<float>(), a2_.data_ptr<float>(), dz2_.data_ptr<float>(),
                                       part_.data_ptr<float>(), gW1, gb1, gW2, gb2,
                                       metrics_.data_ptr<float>(), host_store ? host_metrics_.data_ptr<float>() : nullptr,
                                       ipc_ == nullptr && gstep_.defined() ? gstep_.data_ptr() : nullptr, gkind_,
                                       yd + ny, B_, K_, H_, C_, act_, naive_ ? 1 : 0, ipc_ == nullptr ? 1 : 0, st);
    if (e == hipSuccess && ipc_ != nullptr) {
      {   // (throws on a failed earlier collective; chains streams like every IPC call)
        (void)ipc_->begin();
        ipc_->reduce_sgd_raw(grad_.data_ptr<float>(), (int64_t)K_ * H_ + H_ + (int64_t)H_ * C_ + C_,
                             {W1_.data_ptr<float>(), b1_.data_ptr<float>(), W2_.data_ptr<float>(), b2_.data_ptr<float>()},
                             {(int64_t)K_ * H_, (int64_t)H_, (int64_t)H_ * C_, (int64_t)C_}, yd + ny, 0.f,
                             1.f / (float)ipc_->world_size(), gstep_.defined() ? gstep_.data_ptr() : nullptr, gkind_,
                             metrics_.data_ptr<float>(), host_store ? host_metrics_.data_ptr<float>() : nullptr, st);
      }
    }
    if (e == hipSuccess && !host_store)
      e = hipMemcpyAsync(host_metrics_.data_ptr<float>(), metrics_.data_ptr<float>(), 3 * sizeof(float),
                         hipMemcpyDeviceToHost, st);
    return e;
  }

  void capture(hipStream_t st) {
    if (exec_) { (void)hipGraphExecDestroy(exec_); exec_ = nullptr; }
    if (graph_) { (void)hipGraphDestroy(graph_); graph_ = nullptr; }
    hip_check(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal), "GraphStepPlan: begin capture");
    const hipError_t e = launch_step(st, false);
    hipGraph_t g = nullptr;
    const hipError_t e2 = hipStreamEndCapture(st, &g);
    hip_check(e, "GraphStepPlan: captured launches");
    hip_check(e2, "GraphStepPlan: end capture");
    graph_ = g;
    hip_check(hipGraphInstantiate(&exec_, graph_, nullptr, nullptr, 0), "GraphStepPlan: instantiate");
  }

  // floats the uint8 x occupies at the front of the feed buffer (16-byte padded)
  int64_t u8_x_floats() const { return ((int64_t)B_ * K_ + 15) / 16 * 4; }

  at::Tensor W1_, b1_, W2_, b2_, gstep_, dev_, a2_, dz2_, part_, metrics_, host_metrics_, grad_;
  at::Tensor stage_[2];
  py::object ipc_obj_;
  IpcColl* ipc_ = nullptr;
  hipEvent_t ev_[2] = {nullptr, nullptr};
  hipEvent_t in_ev_ = nullptr, out_ev_ = nullptr;
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t exec_ = nullptr;
  hipStream_t st_ = nullptr;
  int B_, K_ = 0, H_ = 0, C_ = 0, HP_ = 0, act_, gkind_ = 0, slot_ = 0;
  bool naive_, use_graph_, direct_feed_ = false;
  int64_t nfeed_ = 0, steps_ = 0;
  bool host_store_ = true, kernel_feed_ = false;
  bool pending_[2] = {false, false};   // an event on the staging slot's copy may still be in flight
  int64_t feed_bytes_ = 0;
  double t_[3] = {0, 0, 0};
};

// The resident Session engine (compat/resident.py): the persistent fp32 kernel
// (csrc/kernels/mlp_persist_f32.hip, RES) stays launched across Session.run
// calls of the reference's training graph and is driven through pinned host
// memory -- per run the host writes the uint8 batch, its labels and lr into a
// record slot and bumps a doorbell; the kernel stages, trains one step on the
// graph's own W1 / b1 / W2 / b2 (written through every step, so other readers
// see current values), bumps global_step and stores loss / accuracy /
// global_step and a done count back into pinned memory.  No launch, no
// completion, no copy-engine op per run.  The launch exits by itself after
// `idle_s` without a doorbell (relaunched on the next run) or when stop() rings
// door = -1; either way every wave reaches the exit.
class ResidentMLPPlan {
 public:
  ResidentMLPPlan(at::Tensor W1, at::Tensor b1, at::Tensor W2, at::Tensor b2, c10::optional<at::Tensor> gstep, int B,
                  int act, bool naive, double idle_s, double timeout_s)
      : W1_(W1), b1_(b1), W2_(W2), b2_(b2), B_(B), act_(act), naive_(naive) {
    for (const at::Tensor* t : {&W1, &b1, &W2, &b2})
      TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous(),
                  "ResidentMLPPlan: fp32 contiguous device parameters expected");
    TORCH_CHECK(W1.dim() == 2 && W1.size(0) == 784 && W1.size(1) == 100 && b1.numel() == 100 && W2.dim() == 2 &&
                    W2.size(0) == 100 && W2.size(1) == 10 && b2.numel() == 10,
                "ResidentMLPPlan: the reference's 784-100-10 shapes expected");
    TORCH_CHECK(B >= 1 && B <= dtfk_mlpf_max_batch(), "ResidentMLPPlan: batch must be in [1, ",
                dtfk_mlpf_max_batch(), "]");
    if (gstep.has_value()) {
      const int k = gstep_kind_of(*gstep);   // 0 f32, 1 i64, 2 i32, 3 f64
      gkind_ = k + 1;
      gstep_ = *gstep;
    }
    rec_h_ = ((int64_t)B * 785 + 15) / 16 * 16;
    const size_t bytes = 512 + 2 * (size_t)rec_h_;
    hip_check(hipHostMalloc(&mail_, bytes, hipHostMallocMapped | hipHostMallocCoherent), "ResidentMLPPlan: mailbox");
    std::memset(mail_, 0, bytes);
    char* m = static_cast<char*>(mail_);
    door_ = reinterpret_cast<long long*>(m);
    done_ = reinterpret_cast<long long*>(m + 64);
    state_ = reinterpret_cast<long long*>(m + 128);
    out_ = reinterpret_cast<float*>(m + 192);
    lr_ = reinterpret_cast<float*>(m + 256);
    recs_ = reinterpret_cast<uint8_t*>(m + 512);
    void* dp = nullptr;   // device-visible alias of the mailbox (unified addressing: the same address)
    if (hipHostGetDevicePointer(&dp, mail_, 0) != hipSuccess || dp == nullptr) {
      (void)hipGetLastError();
      dp = mail_;
    }
    dmail_ = static_cast<char*>(dp);
    auto o8 = W1.options().dtype(at::kByte);
    stage_ = at::zeros({2 * dtfk_mlpf_stage_rec()}, o8);
    xbuf_ = at::zeros({dtfk_mlpf_xbuf_bytes()}, o8);
    seq_ = at::zeros({1}, W1.options().dtype(at::kLong));
    kgstep_ = at::zeros({1}, W1.options().dtype(at::kLong));
    err_ = at::zeros({1}, W1.options().dtype(at::kInt));
    lrdev_ = at::zeros({1}, W1.options());
    metrics_ = at::zeros({2 * kRing}, W1.options());
    dctr_ = at::zeros({64}, W1.options().dtype(at::kInt));
    const char* rs = std::getenv("DTF_RESIDENT_STAMPS");   // profiling: per-run device stamps
    if (rs != nullptr && rs[0] == '1') res_ts_ = at::zeros({64 * 8}, W1.options().dtype(at::kLong));
    idle_ = (long long)(idle_s * 1e8);            // s_memrealtime: 100 MHz
    timeout_ = (long long)(timeout_s * 1e8);
    wait_s_ = std::max(5.0, 4.0 * idle_s + timeout_s);
    // The launch stays resident between runs, so no other work may queue behind
    // it: HIP maps streams onto GPU_MAX_HW_QUEUES (4) hardware queues round-robin,
    // and a stream sharing the resident kernel's queue (e.g. torch's, reading a
    // variable) waits until the idle exit.  DTF_RESIDENT_STREAM: "priority"
    // (default: a non-blocking high-priority stream -- its own queue as long as no
    // other high-priority stream exists), "cumask" (a CU-masked stream: its own
    // queue, but BLOCKING -- legacy-default-stream work waits for it; measured:
    // every variable read waited out the idle bound,
    // scripts/probes/resident_relaunch.py) or "plain".
    const char* sk = std::getenv("DTF_RESIDENT_STREAM");
    const std::string want = sk != nullptr ? sk : "priority";
    bool made = false;
    if (want == "cumask") {
      int ncu = 0;
      (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, W1.get_device());
      std::vector<uint32_t> mask((size_t)std::max(1, (ncu + 31) / 32), 0xffffffffu);
      made = ncu > 0 && hipExtStreamCreateWithCUMask(&st_, (uint32_t)mask.size(), mask.data()) == hipSuccess;
      if (made) stream_kind_ = "CU-masked (blocking) stream";
    } else if (want != "plain") {
      int lo = 0, hi = 0;
      made = hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess &&
             hipStreamCreateWithPriority(&st_, hipStreamNonBlocking, hi) == hipSuccess;
      if (made) stream_kind_ = "high-priority non-blocking stream";
    }
    if (!made) {
      (void)hipGetLastError();
      hip_check(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking), "hipStreamCreate");
      stream_kind_ = "plain non-blocking stream";
    }
    hip_check(hipEventCreateWithFlags(&ev_, hipEventDisableTiming), "hipEventCreate");
  }
  ~ResidentMLPPlan() {
    try {
      stop();
    } catch (...) {
    }
    if (ev_) (void)hipEventDestroy(ev_);
    if (st_) (void)hipStreamDestroy(st_);
    if (mail_) (void)hipHostFree(mail_);
  }

  // One training step from the MNIST loader's uint8 batch [B, 784] and one-hot
  // float32 labels [B, 10].  False (nothing ran) when y_ is not exactly one-hot:
  // the caller takes the general plan.  Returns after the step; host_metrics()
  // then holds loss, accuracy, global_step (pre-update loss / accuracy, as the
  // graph evaluates them in the same run).
  bool run_u8(py::array xu8, py::array y, double lr) {
    TORCH_CHECK(xu8.dtype().is(py::dtype::of<uint8_t>()) && y.dtype().is(py::dtype::of<float>()),
                "ResidentMLPPlan.run_u8: uint8 x and float32 y_ expected");
    TORCH_CHECK((xu8.flags() & py::array::c_style) && (y.flags() & py::array::c_style),
                "ResidentMLPPlan.run_u8: C-contiguous feeds expected");
    TORCH_CHECK(xu8.size() == (int64_t)B_ * 784 && y.size() == (int64_t)B_ * 10,
                "ResidentMLPPlan.run_u8: feed shapes differ from the plan's");
    const uint8_t* xp = static_cast<const uint8_t*>(xu8.data());
    const float* yp = static_cast<const float*>(y.data());
    uint8_t lab[128];
    for (int b = 0; b < B_; ++b) {   // class ids; anything but an exact one-hot row -> general plan
      int hot = -1;
      for (int c = 0; c < 10; ++c) {
        const float v = yp[b * 10 + c];
        if (v == 1.0f && hot < 0) hot = c;
        else if (v != 0.0f) return false;
      }
      if (hot < 0) return false;
      lab[b] = (uint8_t)hot;
    }
    {
      py::gil_scoped_release nogil;
      using clk = std::chrono::steady_clock;
      const auto t0 = clk::now();
      if (alive_ && __atomic_load_n(state_, __ATOMIC_ACQUIRE) == launch_id_) {   // exited while idle
        reap();
        ++idle_exits_;
      }
      if (!alive_) launch();
      const int slot = (int)(runs_ & 1);
      uint8_t* rec = recs_ + slot * rec_h_;
      std::memcpy(rec, xp, (size_t)B_ * 784);
      std::memcpy(rec + (size_t)B_ * 784, lab, (size_t)B_);
      lr_[slot] = (float)lr;
      std::atomic_thread_fence(std::memory_order_seq_cst);
      __atomic_store_n(door_, runs_ + 1, __ATOMIC_RELEASE);
      const auto t1 = clk::now();
      t_[0] += std::chrono::duration<double, std::micro>(t1 - t0).count();
      long long spins = 0;
      while (__atomic_load_n(done_, __ATOMIC_ACQUIRE) < runs_ + 1) {
        if ((++spins & 1023) == 0) {
          if (__atomic_load_n(state_, __ATOMIC_ACQUIRE) == launch_id_ &&
              __atomic_load_n(done_, __ATOMIC_ACQUIRE) < runs_ + 1) {
            // the launch stopped (idle) without taking this run: start another
            reap();
            ++idle_exits_;
            launch();
          }
          if (std::chrono::duration<double>(clk::now() - t1).count() > wait_s_) {
            dead_ = true;
            throw std::runtime_error("ResidentMLPPlan: no completion within the wait bound");
          }
        }
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
      }
      const double waited = std::chrono::duration<double, std::micro>(clk::now() - t1).count();
      host_wait_[runs_ & 63] = waited;
      ++runs_;
      t_[1] += waited;
    }
    return true;
  }

  // door = -1, then wait for the launch to finish (the variables hold the
  // trained values either way: every step writes them through)
  void stop() {
    if (!alive_) return;
    ++stops_;
    __atomic_store_n(door_, -1LL, __ATOMIC_RELEASE);
    reap();
  }

  bool alive() const { return alive_; }
  int64_t runs() const { return runs_; }
  int64_t launches() const { return launch_id_; }
  // profiling (DTF_RESIDENT_STAMPS=1): device stamps [run % 64][8] and the host's
  // door -> done wait of the same runs (us)
  py::object stamps() const {
    if (!res_ts_.defined()) return py::none();
    return py::make_tuple(res_ts_.cpu(), at::from_blob(const_cast<double*>(host_wait_), {64},
                                                       at::TensorOptions().dtype(at::kDouble)).clone());
  }
  at::Tensor host_metrics() const {
    return at::from_blob(out_, {3}, at::TensorOptions().dtype(at::kFloat));
  }
  py::dict timing() const {
    py::dict d;
    const double n = runs_ > 0 ? (double)runs_ : 1.0;
    d["feed_us"] = t_[0] / n;
    d["wait_us"] = t_[1] / n;
    d["runs"] = runs_;
    d["launches"] = launch_id_;
    d["stream"] = stream_kind_;
    d["stops"] = stops_;             // host-requested (quiesce / close)
    d["idle_exits"] = idle_exits_;   // the launch left by itself (idle bound)
    return d;
  }

 private:
  static constexpr int kRing = 64;

  void reap() {
    const hipError_t e = hipStreamSynchronize(st_);
    alive_ = false;
    hip_check(e, "ResidentMLPPlan: launch");
    int err = 0;
    hip_check(hipMemcpy(&err, err_.data_ptr(), sizeof(int), hipMemcpyDeviceToHost), "ResidentMLPPlan: err");
    if (err != 0) {
      dead_ = true;
      throw std::runtime_error("ResidentMLPPlan: the resident kernel reported error " + std::to_string(err));
    }
  }

  void launch() {
    TORCH_CHECK(!dead_, "ResidentMLPPlan: failed earlier");
    // whatever the caller's stream queued (initialisation, restores) lands first
    hip_check(hipEventRecord(ev_, cur_stream()), "ResidentMLPPlan: event");
    hip_check(hipStreamWaitEvent(st_, ev_, 0), "ResidentMLPPlan: wait");
    hip_check(hipMemsetAsync(dctr_.data_ptr(), 0, dctr_.numel() * sizeof(int), st_), "ResidentMLPPlan: counters");
    if (__atomic_load_n(door_, __ATOMIC_ACQUIRE) < 0) __atomic_store_n(door_, runs_, __ATOMIC_RELEASE);   // after stop()
    ++launch_id_;
    dtfk_mlpf_set_res_ts(res_ts_.defined() ? reinterpret_cast<long long*>(res_ts_.data_ptr<int64_t>()) : nullptr);
    hip_check(dtfk_mlp_persist_f32_resident(
                  stage_.data_ptr(), B_, W1_.data_ptr<float>(), W2_.data_ptr<float>(), b1_.data_ptr<float>(),
                  b2_.data_ptr<float>(), lrdev_.data_ptr<float>(), metrics_.data_ptr<float>(), kRing, act_,
                  naive_ ? 1 : 0, reinterpret_cast<long long*>(kgstep_.data_ptr<int64_t>()),
                  reinterpret_cast<unsigned long long*>(seq_.data_ptr<int64_t>()), xbuf_.data_ptr(),
                  err_.data_ptr<int>(), timeout_, reinterpret_cast<const long long*>(dmail_),
                  dmail_ + 512, rec_h_, reinterpret_cast<const float*>(dmail_ + 256),
                  reinterpret_cast<float*>(dmail_ + 192), reinterpret_cast<long long*>(dmail_ + 64),
                  reinterpret_cast<long long*>(dmail_ + 128), launch_id_, runs_, idle_,
                  gkind_ ? gstep_.data_ptr() : nullptr, gkind_, reinterpret_cast<unsigned*>(dctr_.data_ptr<int>()),
                  st_),
              "ResidentMLPPlan: launch");
    alive_ = true;
  }

  at::Tensor W1_, b1_, W2_, b2_, gstep_, stage_, xbuf_, seq_, kgstep_, err_, lrdev_, metrics_, dctr_, res_ts_;
  double host_wait_[64] = {0};
  int B_, act_, gkind_ = 0;
  bool naive_;
  int64_t rec_h_ = 0;
  const char* stream_kind_ = "";
  int64_t stops_ = 0, idle_exits_ = 0;
  void* mail_ = nullptr;
  char* dmail_ = nullptr;
  long long* door_ = nullptr;
  long long* done_ = nullptr;
  long long* state_ = nullptr;
  float* out_ = nullptr;
  float* lr_ = nullptr;
  uint8_t* recs_ = nullptr;
  long long idle_ = 0, timeout_ = 0;
  double wait_s_ = 5.0;
  hipStream_t st_ = nullptr;
  hipEvent_t ev_ = nullptr;
  bool alive_ = false, dead_ = false;
  long long runs_ = 0, launch_id_ = 0;
  double t_[2] = {0, 0};
};

void init_mlp(py::module& m) {
  py::class_<ResidentMLPPlan>(m, "ResidentMLPPlan")
      .def(py::init<at::Tensor, at::Tensor, at::Tensor, at::Tensor, c10::optional<at::Tensor>, int, int, bool, double,
                    double>(),
           py::arg("W1"), py::arg("b1"), py::arg("W2"), py::arg("b2"), py::arg("gstep"), py::arg("B"), py::arg("act"),
           py::arg("naive"), py::arg("idle_s") = 0.002, py::arg("timeout_s") = 10.0)
      .def("run_u8", &ResidentMLPPlan::run_u8, py::arg("xu8"), py::arg("y"), py::arg("lr"))
      .def("stop", &ResidentMLPPlan::stop)
      .def("alive", &ResidentMLPPlan::alive)
      .def("runs", &ResidentMLPPlan::runs)
      .def("launches", &ResidentMLPPlan::launches)
      .def("host_metrics", &ResidentMLPPlan::host_metrics)
      .def("timing", &ResidentMLPPlan::timing)
      .def("stamps", &ResidentMLPPlan::stamps);
  py::class_<GraphStepPlan>(m, "GraphStepPlan")
      .def(py::init<at::Tensor, at::Tensor, at::Tensor, at::Tensor, c10::optional<at::Tensor>, int, int, bool, bool>(),
           py::arg("W1"), py::arg("b1"), py::arg("W2"), py::arg("b2"), py::arg("gstep"), py::arg("B"), py::arg("act"),
           py::arg("naive"), py::arg("use_graph") = false)
      .def("use_graph", &GraphStepPlan::use_graph)
      .def("run", &GraphStepPlan::run, py::arg("x"), py::arg("y"), py::arg("lr"), py::arg("sync"))
      .def("run_u8", &GraphStepPlan::run_u8, py::arg("xu8"), py::arg("y"), py::arg("lr"), py::arg("sync"))
      .def("host_metrics", &GraphStepPlan::host_metrics)
      .def("attach_ipc", &GraphStepPlan::attach_ipc)
      .def("has_ipc", &GraphStepPlan::has_ipc)
      .def("steps", &GraphStepPlan::steps)
      .def("timing", &GraphStepPlan::timing);
  m.def("graph_mlp_step", &graph_mlp_step, py::arg("x"), py::arg("ylab"), py::arg("W1"), py::arg("b1"),
        py::arg("W2"), py::arg("b2"), py::arg("a2buf"), py::arg("dz2buf"), py::arg("grads"), py::arg("metrics"),
        py::arg("gstep"), py::arg("lr"), py::arg("act"), py::arg("naive"), py::arg("sgd"));
  m.def("mlp_persist_f32", &mlp_persist_f32, py::arg("stage"), py::arg("rec_h"), py::arg("B"), py::arg("nsteps"),
        py::arg("params"), py::arg("lr"), py::arg("metrics"), py::arg("gstep"), py::arg("seq"), py::arg("xbuf"),
        py::arg("err"), py::arg("timeout_s"), py::arg("act"), py::arg("naive"), py::arg("host") = py::none(),
        py::arg("host_offset") = 0, py::arg("next_steps") = 0, py::arg("stage_next") = py::none(),
        py::arg("step_ts") = py::none(), py::arg("ipc_table") = 0, py::arg("ipc_W") = 1, py::arg("ipc_rank") = 0,
        py::arg("grad_bf16") = true, py::arg("phase_ts") = py::none(), py::arg("spread") = false,
        py::arg("two_shot") = false, py::arg("mfma_split") = false);
  py::class_<PersistF32Plan>(m, "PersistF32Plan")
      .def(py::init<at::Tensor, at::Tensor, int64_t, int, at::Tensor, at::Tensor, at::Tensor, at::Tensor,
                    at::Tensor, at::Tensor, at::Tensor, double, int, int, at::Tensor, at::Tensor, int64_t, int, int,
                    bool, bool, bool, bool>())
      .def("launch", &PersistF32Plan::launch);
  m.def("mlpf_stage_rec", &dtfk_mlpf_stage_rec);
  m.def("mlpf_set_fault", &dtfk_mlpf_set_fault, py::arg("rank"), py::arg("step"));
  m.def("mlpf_xbuf_bytes", &dtfk_mlpf_xbuf_bytes);
  m.def("mlpf_ipc_bytes", &dtfk_mlpf_ipc_bytes);
  m.def("mlpf_max_batch", &dtfk_mlpf_max_batch);
  m.def("mlp_ksplit", &dtfk_mlp_ksplit);
  m.def("mlp_l1_fwd", &mlp_l1_fwd, py::arg("x"), py::arg("x_offset"), py::arg("x_kind"),
        py::arg("B"), py::arg("W1T"), py::arg("z2p"), py::arg("ts") = py::none());
  m.def("mlp_head_bwd", &mlp_head_bwd, py::arg("z2p"), py::arg("labels"), py::arg("labels_offset"),
        py::arg("B"), py::arg("W2T"), py::arg("W2N"), py::arg("params"), py::arg("dz2T"),
        py::arg("partials"),
        py::arg("inv_batch"), py::arg("act"), py::arg("naive_loss"), py::arg("gstep"), py::arg("ts") = py::none());
  m.def("mlp_wgrad", &mlp_wgrad, py::arg("x"), py::arg("x_offset"), py::arg("x_kind"),
        py::arg("dz2T"), py::arg("B"), py::arg("partials"), py::arg("params"), py::arg("W1T"),
        py::arg("W2T"), py::arg("W2N"), py::arg("grads"), py::arg("grad_kind"), py::arg("lr"),
        py::arg("metrics"),
        py::arg("gstep"), py::arg("ts") = py::none(), py::arg("ipc_table") = 0, py::arg("ipc_W") = 0,
        py::arg("ipc_rank") = 0, py::arg("ipc_parity") = 0, py::arg("ipc_slot_bytes") = 0,
        py::arg("ipc_err") = py::none(), py::arg("ipc_timeout_s") = 5.0);
  m.def("mlp_apply_flat", &mlp_apply_flat);
  m.def("mlp_fwd_head", &mlp_fwd_head);
  m.def("mlp_ipc_reduce_apply", &mlp_ipc_reduce_apply);
  m.def("mlp_ipc_flag_bytes", &dtfk_mlp_ipc_flag_bytes);
  m.def("memcpy_h2d_async", &memcpy_h2d_async);
  m.def("mlpg_fwd", &mlpg_fwd, py::arg("x"), py::arg("x_offset"), py::arg("labels"), py::arg("labels_offset"),
        py::arg("B"), py::arg("W1F"), py::arg("params"), py::arg("a2"), py::arg("P1"), py::arg("dz2F"), py::arg("act"),
        py::arg("naive"), py::arg("gscale"));
  m.def("mlpg_wgrad", &mlpg_wgrad, py::arg("x"), py::arg("x_offset"), py::arg("B"), py::arg("dz2S"), py::arg("P2"),
        py::arg("nchunk"));
  m.def("mlpg_apply", &mlpg_apply, py::arg("params"), py::arg("P1"), py::arg("P2"), py::arg("nchunk"),
        py::arg("gin"), py::arg("gout"), py::arg("lr"), py::arg("scale"), py::arg("W1S"), py::arg("metrics"),
        py::arg("gstep"), py::arg("B"), py::arg("mode"));
  m.def("mlpg_p1_floats", &dtfk_mlpg_p1_floats);
  m.def("mlpg_wchunk", &dtfk_mlpg_wchunk);
  m.def("mlpg_p2_floats", &dtfk_mlpg_p2_floats);
}

}  // namespace dtf
