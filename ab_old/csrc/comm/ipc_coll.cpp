// Python bindings of the IPC collectives (the node's RCCL-free data plane):
// tensor-level all_reduce / broadcast / all_gather / all_to_all and the fused
// all-reduce-mean + SGD step (csrc/comm/ipc_coll_host.h, kernels in
// csrc/kernels/ipc_coll.hip).  parallel/world.py routes World's GPU
// collectives here.
#include "comm/ipc_coll_host.h"

namespace dtf {
namespace {

int dtype_code(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return 0;
    case at::kBFloat16: return 1;
    case at::kDouble: return 2;
    case at::kInt: return 3;
    case at::kLong: return 4;
    default: throw std::runtime_error("IpcColl: dtype not supported (float32 / bfloat16 / float64 / int32 / int64)");
  }
}

void need_cuda_contig(const at::Tensor& t, const char* what) {
  if (!t.is_cuda() || !t.is_contiguous()) throw std::runtime_error(std::string(what) + ": contiguous GPU tensor expected");
}

int op_code(const std::string& op) {
  if (op == "sum" || op == "avg") return 0;
  if (op == "max") return 1;
  if (op == "min") return 2;
  throw std::runtime_error("IpcColl: op must be sum / avg / max / min");
}

void all_reduce(IpcColl& c, at::Tensor t, const std::string& op, c10::optional<at::Tensor> out) {
  need_cuda_contig(t, "IpcColl.all_reduce");
  at::Tensor o = out.has_value() ? *out : t;
  need_cuda_contig(o, "IpcColl.all_reduce out");
  if (o.numel() != t.numel() || o.scalar_type() != t.scalar_type())
    throw std::runtime_error("IpcColl.all_reduce: out must match the input");
  const int dt = dtype_code(t);
  float scale = 1.f;
  if (op == "avg") {
    if (dt >= 3) throw std::runtime_error("IpcColl.all_reduce: avg of an integer tensor");
    scale = 1.f / (float)c.world_size();
  }
  if (t.numel() == 0) return;
  hipStream_t s = c.begin();
  c.all_reduce_raw(t.data_ptr(), o.data_ptr(), t.numel(), dt, op_code(op), scale, s);
}

void broadcast(IpcColl& c, at::Tensor t, int src) {
  need_cuda_contig(t, "IpcColl.broadcast");
  if (t.numel() == 0) return;
  hipStream_t s = c.begin();
  c.broadcast_raw(t.data_ptr(), t.numel() * t.element_size(), src, s);
}

void all_gather(IpcColl& c, at::Tensor src, at::Tensor dst) {
  need_cuda_contig(src, "IpcColl.all_gather src");
  need_cuda_contig(dst, "IpcColl.all_gather dst");
  const int64_t nb = src.numel() * src.element_size();
  if (dst.numel() * dst.element_size() != nb * c.world_size())
    throw std::runtime_error("IpcColl.all_gather: dst must hold world_size x src");
  if (nb == 0) return;
  hipStream_t s = c.begin();
  c.all_gather_raw(src.data_ptr(), dst.data_ptr(), nb, s);
}

// counts in rows of the first dimension
void all_to_all(IpcColl& c, at::Tensor src, std::vector<int64_t> send_counts, at::Tensor dst,
                std::vector<int64_t> recv_counts) {
  need_cuda_contig(src, "IpcColl.all_to_all src");
  need_cuda_contig(dst, "IpcColl.all_to_all dst");
  const int64_t rs = src.dim() > 0 && src.size(0) > 0 ? src.numel() / src.size(0) * src.element_size()
                                                      : (src.dim() > 1 ? src.numel() * src.element_size() : src.element_size());
  const int64_t rd = dst.dim() > 0 && dst.size(0) > 0 ? dst.numel() / dst.size(0) * dst.element_size() : rs;
  if (rs != rd) throw std::runtime_error("IpcColl.all_to_all: src and dst rows differ in size");
  std::vector<int64_t> sb(send_counts.size()), rb(recv_counts.size());
  int64_t ts = 0, tr = 0;
  for (size_t i = 0; i < sb.size(); ++i) { sb[i] = send_counts[i] * rs; ts += sb[i]; }
  for (size_t i = 0; i < rb.size(); ++i) { rb[i] = recv_counts[i] * rs; tr += rb[i]; }
  if (ts > src.numel() * src.element_size() || tr > dst.numel() * dst.element_size())
    throw std::runtime_error("IpcColl.all_to_all: counts exceed the buffers");
  hipStream_t s = c.begin();
  c.all_to_all_raw(src.data_ptr(), sb, dst.data_ptr(), rb, s);
}

// grad: flat fp32 gradient of `params` (in order, 16-byte aligned);
// every rank applies p -= lr / W * sum of the W gradients, global_step += 1
void reduce_sgd(IpcColl& c, at::Tensor grad, std::vector<at::Tensor> params, c10::optional<at::Tensor> lr,
                double lr_val, c10::optional<at::Tensor> gstep, c10::optional<at::Tensor> host_metrics) {
  need_cuda_contig(grad, "IpcColl.reduce_sgd grad");
  if (grad.scalar_type() != at::kFloat) throw std::runtime_error("IpcColl.reduce_sgd: fp32 gradient expected");
  std::vector<float*> ps;
  std::vector<int64_t> ns;
  int64_t n = 0;
  for (auto& p : params) {
    need_cuda_contig(p, "IpcColl.reduce_sgd param");
    if (p.scalar_type() != at::kFloat) throw std::runtime_error("IpcColl.reduce_sgd: fp32 parameters expected");
    ps.push_back(p.data_ptr<float>());
    ns.push_back(p.numel());
    n += p.numel();
  }
  if (grad.numel() < n) throw std::runtime_error("IpcColl.reduce_sgd: gradient smaller than the parameters");
  void* gs = nullptr;
  int gk = 0;
  if (gstep.has_value()) {
    need_cuda_contig(*gstep, "IpcColl.reduce_sgd global_step");
    switch (gstep->scalar_type()) {
      case at::kFloat: gk = 0; break;
      case at::kLong: gk = 1; break;
      case at::kInt: gk = 2; break;
      case at::kDouble: gk = 3; break;
      default: throw std::runtime_error("IpcColl.reduce_sgd: global_step dtype");
    }
    gs = gstep->data_ptr();
  }
  const float* lp = nullptr;
  if (lr.has_value()) {
    need_cuda_contig(*lr, "IpcColl.reduce_sgd lr");
    lp = lr->data_ptr<float>();
  }
  float* hm = host_metrics.has_value() ? host_metrics->data_ptr<float>() : nullptr;
  hipStream_t s = c.begin();
  c.reduce_sgd_raw(grad.data_ptr<float>(), n, ps, ns, lp, (float)lr_val, 1.f / (float)c.world_size(), gs, gk, nullptr,
                   hm, s);
}

}  // namespace

void init_ipc_coll(py::module& m) {
  m.def("ipc_coll_buffer_bytes", [](int64_t cap) { return (int64_t)dtfk::ipcc::buffer_bytes(cap); });
  m.attr("IPC_COLL_WMAX") = dtfk::ipcc::WMAX;
  py::class_<IpcColl>(m, "IpcColl")
      .def(py::init<py::object, int64_t, int, int, int64_t, double, int64_t, int>(), py::arg("buffers"),
           py::arg("table_ptr"), py::arg("world_size"), py::arg("rank"), py::arg("cap"), py::arg("timeout_s"),
           py::arg("two_shot_bytes"), py::arg("max_grid"))
      .def("all_reduce", &all_reduce, py::arg("t"), py::arg("op") = "sum", py::arg("out") = py::none())
      .def("broadcast", &broadcast, py::arg("t"), py::arg("src") = 0)
      .def("all_gather", &all_gather)
      .def("all_to_all", &all_to_all)
      .def("reduce_sgd", &reduce_sgd, py::arg("grad"), py::arg("params"), py::arg("lr") = py::none(),
           py::arg("lr_val") = 0.0, py::arg("gstep") = py::none(), py::arg("host_metrics") = py::none())
      .def("error", &IpcColl::error)
      .def("check", &IpcColl::check)
      .def("calls", &IpcColl::calls)
      .def("capacity", &IpcColl::capacity)
      .def("world_size", &IpcColl::world_size)
      .def("rank", &IpcColl::rank);
}

}  // namespace dtf
