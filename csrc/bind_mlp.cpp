// Python bindings for the fused MLP step kernels (csrc/kernels/mlp_step.hip)
// and the pinned-host -> device batch copy used by the input pipeline.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

extern "C" {
hipError_t dtfk_mlp_fwd_bwd(const void* x, int x_kind, const void* labels, int B, const void* W1T,
                            const void* W2T, const float* params, void* xT, void* dz2T, int BP,
                            float* partials, float inv_batch, int act, int naive_loss,
                            hipStream_t stream);
hipError_t dtfk_mlp_wgrad(const void* xT, const void* dz2T, int BP, int B, const float* partials,
                          float* params, void* W1T, void* W2T, void* grads, int grad_kind,
                          const float* lr, float* metrics, long long* gstep, int ring,
                          hipStream_t stream);
hipError_t dtfk_mlp_apply_flat(float* params, const void* grads, int grad_kind, const float* lr,
                               float scale, void* W1T, void* W2T, hipStream_t stream);
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

// x_kind: 0 u8 pixels, 1 fp32, 2 bf16.  labels: uint8 class ids.
void mlp_fwd_bwd(at::Tensor x, int64_t x_offset, int x_kind, at::Tensor labels,
                 int64_t labels_offset, int B, at::Tensor W1T, at::Tensor W2T, at::Tensor params,
                 at::Tensor xT, at::Tensor dz2T, int BP, at::Tensor partials, double inv_batch,
                 int act, bool naive_loss) {
  const int nb = (B + 15) / 16;
  if (BP < nb * 16 || BP % 32) throw std::runtime_error("bad BP");
  const int64_t esz = x_kind == 0 ? 1 : (x_kind == 1 ? 4 : 2);
  if (!x.is_cuda() || !labels.is_cuda()) throw std::runtime_error("x/labels must be on GPU");
  if ((int64_t)x.numel() * x.element_size() < x_offset + (int64_t)B * 784 * esz)
    throw std::runtime_error("x buffer too small");
  if ((int64_t)labels.numel() * labels.element_size() < labels_offset + B)
    throw std::runtime_error("labels buffer too small");
  if ((x_offset % 16) != 0) throw std::runtime_error("x offset must be 16-byte aligned");
  need(W1T, at::kBFloat16, 112 * 800, "W1T");
  need(W2T, at::kBFloat16, 16 * 128, "W2T");
  need(params, at::kFloat, kNParam, "params");
  need(xT, at::kBFloat16, (int64_t)800 * BP, "xT");
  need(dz2T, at::kBFloat16, (int64_t)112 * BP, "dz2T");
  need(partials, at::kFloat, (int64_t)nb * 1112, "partials");
  const char* xb = reinterpret_cast<const char*>(x.data_ptr()) + x_offset;
  const char* lb = reinterpret_cast<const char*>(labels.data_ptr()) + labels_offset;
  hip_check(dtfk_mlp_fwd_bwd(xb, x_kind, lb, B, W1T.data_ptr(), W2T.data_ptr(),
                             params.data_ptr<float>(), xT.data_ptr(), dz2T.data_ptr(), BP,
                             partials.data_ptr<float>(), (float)inv_batch, act, naive_loss ? 1 : 0,
                             cur_stream()),
            "mlp_fwd_bwd");
}

// grad_kind: 0 fused SGD (grads ignored), 1 fp32 grads, 2 bf16 grads
void mlp_wgrad(at::Tensor xT, at::Tensor dz2T, int BP, int B, at::Tensor partials,
               at::Tensor params, at::Tensor W1T, at::Tensor W2T, c10::optional<at::Tensor> grads,
               int grad_kind, at::Tensor lr, at::Tensor metrics, at::Tensor gstep) {
  const int nb = (B + 15) / 16;
  need(xT, at::kBFloat16, (int64_t)800 * BP, "xT");
  need(dz2T, at::kBFloat16, (int64_t)112 * BP, "dz2T");
  need(partials, at::kFloat, (int64_t)nb * 1112, "partials");
  need(params, at::kFloat, kNParam, "params");
  need(W1T, at::kBFloat16, 112 * 800, "W1T");
  need(W2T, at::kBFloat16, 16 * 128, "W2T");
  need(lr, at::kFloat, 1, "lr");
  need(metrics, at::kFloat, 2, "metrics");
  need(gstep, at::kLong, 1, "global_step");
  void* g = nullptr;
  if (grad_kind != 0) {
    if (!grads.has_value()) throw std::runtime_error("grads required");
    need(*grads, grad_kind == 1 ? at::kFloat : at::kBFloat16, kNParam, "grads");
    g = grads->data_ptr();
  }
  const int ring = (int)(metrics.numel() / 2);
  hip_check(dtfk_mlp_wgrad(xT.data_ptr(), dz2T.data_ptr(), BP, B, partials.data_ptr<float>(),
                           params.data_ptr<float>(), W1T.data_ptr(), W2T.data_ptr(), g, grad_kind,
                           lr.data_ptr<float>(), metrics.data_ptr<float>(),
                           reinterpret_cast<long long*>(gstep.data_ptr<int64_t>()), ring,
                           cur_stream()),
            "mlp_wgrad");
}

void mlp_apply_flat(at::Tensor params, c10::optional<at::Tensor> grads, at::Tensor lr,
                    double scale, at::Tensor W1T, at::Tensor W2T) {
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
                                (float)scale, W1T.data_ptr(), W2T.data_ptr(), cur_stream()),
            "mlp_apply_flat");
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

void init_mlp(py::module& m) {
  m.def("mlp_fwd_bwd", &mlp_fwd_bwd);
  m.def("mlp_wgrad", &mlp_wgrad);
  m.def("mlp_apply_flat", &mlp_apply_flat);
  m.def("memcpy_h2d_async", &memcpy_h2d_async);
}

}  // namespace dtf
