// IPC-mapped peer buffers for one-shot intra-node reductions over xGMI.
//
// Each rank allocates ONE uncached (fine-grained, coherent across xGMI)
// device buffer with hipExtMallocWithFlags(hipDeviceMallocUncached) -- the
// same kind RCCL uses for its own peer buffers -- exports it with
// hipIpcGetMemHandle, and maps every peer's buffer with hipIpcOpenMemHandle.
// The handles travel through the control plane (gloo / native store), so
// this class only deals with bytes.  Kernels then address peer memory
// directly: a device table holds the W base pointers (own + mapped).
//
// Layout of a rank's buffer is decided by the user (the MLP uses
// [flags 256 B][grad parity 0][grad parity 1]); tensor(offset, numel, dtype)
// exposes a region of the OWN buffer as a non-owning torch tensor.
#include <torch/extension.h>
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>
#include <vector>

namespace dtf {
namespace {
void hck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
}  // namespace

class IpcPeerBuffers {
 public:
  IpcPeerBuffers(int64_t nbytes, int world_size, int rank)
      : nbytes_(nbytes), world_(world_size), rank_(rank), peers_(world_size, nullptr) {
    if (world_size < 1 || rank < 0 || rank >= world_size) throw std::runtime_error("bad world/rank");
    hck(hipGetDevice(&device_), "hipGetDevice");
    hck(hipExtMallocWithFlags(&own_, (size_t)nbytes, hipDeviceMallocUncached), "hipExtMallocWithFlags(uncached)");
    hck(hipMemset(own_, 0, (size_t)nbytes), "hipMemset");
    peers_[rank] = own_;
    hck(hipMalloc(&table_, sizeof(void*) * world_size), "hipMalloc(table)");
  }
  ~IpcPeerBuffers() { close(); }

  py::bytes handle() const {
    hipIpcMemHandle_t h;
    hck(hipIpcGetMemHandle(&h, own_), "hipIpcGetMemHandle");
    return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
  }

  // handles[r] for every rank (own entry ignored); maps all peers.
  void open(std::vector<std::string> handles) {
    if ((int)handles.size() != world_) throw std::runtime_error("open: need one handle per rank");
    for (int r = 0; r < world_; ++r) {
      if (r == rank_) continue;
      if (handles[r].size() != sizeof(hipIpcMemHandle_t)) throw std::runtime_error("open: bad handle size");
      hipIpcMemHandle_t h;
      memcpy(&h, handles[r].data(), sizeof(h));
      void* p = nullptr;
      hck(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
      peers_[r] = p;
      opened_.push_back(p);
    }
    hck(hipMemcpy(table_, peers_.data(), sizeof(void*) * world_, hipMemcpyHostToDevice), "hipMemcpy(table)");
    ready_ = true;
  }

  // kind: 0 float32, 1 bfloat16, 2 uint8, 3 int64
  at::Tensor tensor(int64_t offset, int64_t numel, int kind) {
    const at::ScalarType st = kind == 0 ? at::kFloat : kind == 1 ? at::kBFloat16 : kind == 2 ? at::kByte : at::kLong;
    const int64_t es = c10::elementSize(st);
    if (offset < 0 || offset + numel * es > nbytes_) throw std::runtime_error("tensor: region out of range");
    auto opts = at::TensorOptions().dtype(st).device(at::kCUDA, device_);
    return torch::from_blob(static_cast<char*>(own_) + offset, {numel}, opts);
  }

  int64_t table_ptr() const { return reinterpret_cast<int64_t>(table_); }
  int64_t own_ptr() const { return reinterpret_cast<int64_t>(own_); }
  int64_t peer_ptr(int r) const { return reinterpret_cast<int64_t>(peers_.at(r)); }
  bool ready() const { return ready_; }
  int64_t nbytes() const { return nbytes_; }

  void close() {
    for (void* p : opened_) hipIpcCloseMemHandle(p);
    opened_.clear();
    if (table_) hipFree(table_);
    table_ = nullptr;
    if (own_) hipFree(own_);
    own_ = nullptr;
    ready_ = false;
  }

 private:
  int64_t nbytes_;
  int world_, rank_, device_ = 0;
  void* own_ = nullptr;
  void** table_ = nullptr;
  std::vector<void*> peers_;
  std::vector<void*> opened_;
  bool ready_ = false;
};

void init_ipc(py::module& m) {
  py::class_<IpcPeerBuffers>(m, "IpcPeerBuffers")
      .def(py::init<int64_t, int, int>(), py::arg("nbytes"), py::arg("world_size"), py::arg("rank"))
      .def("handle", &IpcPeerBuffers::handle)
      .def("open", &IpcPeerBuffers::open)
      .def("tensor", &IpcPeerBuffers::tensor)
      .def("table_ptr", &IpcPeerBuffers::table_ptr)
      .def("own_ptr", &IpcPeerBuffers::own_ptr)
      .def("peer_ptr", &IpcPeerBuffers::peer_ptr)
      .def("ready", &IpcPeerBuffers::ready)
      .def("nbytes", &IpcPeerBuffers::nbytes)
      .def("close", &IpcPeerBuffers::close);
}

}  // namespace dtf
