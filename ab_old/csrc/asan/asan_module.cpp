// Host-only build of the C++ runtime (TF bundle, tfevents/TFRecord, TCP store,
// blocking queue, libsvm parser) as its own module `_rt_asan`, compiled with
// -fsanitize=address,undefined by scripts/asan_runtime.py and exercised under
// the sanitizers (race / memory-error detection for the native
// runtime; GPU sanitizers are not available on the MI355X pool).
#include <torch/extension.h>

namespace dtf {
void init_tfrecord(py::module& m);
void init_bundle(py::module& m);
void init_store(py::module& m);
void init_queue(py::module& m);
void init_libsvm(py::module& m);
}  // namespace dtf

PYBIND11_MODULE(_rt_asan, m) {
  m.doc() = "sanitizer build of the distributed_tensorflow_example_amd C++ runtime";
  dtf::init_tfrecord(m);
  dtf::init_bundle(m);
  dtf::init_store(m);
  dtf::init_queue(m);
  dtf::init_libsvm(m);
}
