// pybind11 registration of the continuous-batching scheduler (scheduler.h).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "scheduler.h"

namespace py = pybind11;

namespace bfly_rt {

void register_scheduler(py::module_& m) {
  py::class_<StepPlan>(m, "StepPlan")
      .def_readonly("kind", &StepPlan::kind)
      .def_readonly("seq_ids", &StepPlan::seq_ids)
      .def_readonly("num_decode", &StepPlan::num_decode)
      .def_readonly("prefill_slots", &StepPlan::prefill_slots)
      .def_readonly("prefill_lens", &StepPlan::prefill_lens)
      .def_readonly("prefill_starts", &StepPlan::prefill_starts)
      .def_readonly("prefill_final", &StepPlan::prefill_final)
      .def_readonly("decode_slots", &StepPlan::decode_slots)
      .def_readonly("decode_positions", &StepPlan::decode_positions)
      .def_readonly("cow", &StepPlan::cow)
      .def_readonly("preempted", &StepPlan::preempted);
  py::class_<Scheduler>(m, "Scheduler")
      .def(py::init<KVBlockManager&, int, int64_t, bool, bool>(), py::arg("kv"), py::arg("max_batch"),
           py::arg("max_prefill_tokens"), py::arg("mixed") = false, py::arg("prefix_cache") = false,
           py::keep_alive<1, 2>())
      .def("add", &Scheduler::add, py::arg("sid"), py::arg("prompt_len"), py::arg("max_new_tokens"),
           py::arg("tokens") = std::vector<int32_t>{})
      .def("admit_prefilled", &Scheduler::admit_prefilled, py::arg("sid"), py::arg("prompt_len"),
           py::arg("max_new_tokens"))
      .def("can_admit_prefilled", &Scheduler::can_admit_prefilled)
      .def_property_readonly("prefix_hit_tokens", &Scheduler::prefix_hit_tokens)
      .def("on_token", &Scheduler::on_token)
      .def("finish", &Scheduler::finish)
      .def("schedule", &Scheduler::schedule)
      .def_property_readonly("num_waiting", &Scheduler::num_waiting)
      .def_property_readonly("num_running", &Scheduler::num_running)
      .def("running", &Scheduler::running)
      .def("waiting", &Scheduler::waiting);
}

}  // namespace bfly_rt
