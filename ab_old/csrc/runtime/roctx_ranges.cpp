// roctx ranges/markers for rocprofv3 --marker-trace (rocprofiler-sdk-roctx):
// the Python `utils.profiling.range()` wraps fwd / bwd / all-reduce /
// optimizer phases so they show up next to the kernels in a trace.
#include <pybind11/pybind11.h>
#include <rocprofiler-sdk-roctx/roctx.h>

namespace py = pybind11;

namespace dtf {

void init_roctx(py::module& m) {
  m.def("roctx_push", [](const std::string& name) { return (int)roctxRangePushA(name.c_str()); });
  m.def("roctx_pop", []() { return (int)roctxRangePop(); });
  m.def("roctx_mark", [](const std::string& name) { roctxMarkA(name.c_str()); });
}

}  // namespace dtf
