// Single Python extension module `_C` for the framework's native code:
// HIP kernels (bound per area), the RCCL communicator and the C++ runtime
// (TCP store, blocking queue, libsvm parser, CRC32C, TF bundle, tfevents).
#include <torch/extension.h>

namespace dtf {
void init_mlp(py::module& m);
void init_comm(py::module& m);
void init_tfrecord(py::module& m);
void init_bundle(py::module& m);
void init_store(py::module& m);
void init_queue(py::module& m);
void init_libsvm(py::module& m);
void init_ops(py::module& m);
void init_transformer(py::module& m);
void init_ipc(py::module& m);
void init_roctx(py::module& m);
void init_bn(py::module& m);
}  // namespace dtf

PYBIND11_MODULE(_C, m) {
  m.doc() = "MI355X-native kernels and runtime for distributed_tensorflow_example_amd";
  m.attr("ARCH") = "gfx950";
  dtf::init_mlp(m);
  dtf::init_comm(m);
  dtf::init_tfrecord(m);
  dtf::init_bundle(m);
  dtf::init_store(m);
  dtf::init_queue(m);
  dtf::init_libsvm(m);
  dtf::init_ops(m);
  dtf::init_transformer(m);
  dtf::init_ipc(m);
  dtf::init_roctx(m);
  dtf::init_bn(m);
}
