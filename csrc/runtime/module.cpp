// butterfly_amd._native: host-side C++ runtime (no torch / HIP dependency).
#include <pybind11/pybind11.h>

namespace py = pybind11;

namespace bfly_rt {
void register_kv_manager(py::module_& m);
void register_partition(py::module_& m);
void register_scheduler(py::module_& m);
void register_program_sim(py::module_& m);
}  // namespace bfly_rt

PYBIND11_MODULE(_native, m) {
  m.doc() = "butterfly_amd host runtime: paged-KV block manager, pipeline cut search, scheduler core, rank-program simulator";
  bfly_rt::register_kv_manager(m);
  bfly_rt::register_partition(m);
  bfly_rt::register_scheduler(m);
  bfly_rt::register_program_sim(m);
}
