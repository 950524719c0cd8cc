// Python binding of the rank-program simulator (program_sim.h).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>

#include "program_sim.h"

namespace py = pybind11;

namespace bfly_rt {

void register_program_sim(py::module_& m) {
  m.def(
      "simulate_programs",
      [](const std::vector<std::vector<std::tuple<std::string, std::vector<int>, int64_t, std::string>>>& progs,
         bool rendezvous) {
        std::vector<std::vector<SimOp>> ps(progs.size());
        for (size_t r = 0; r < progs.size(); ++r)
          for (const auto& t : progs[r]) {
            SimOp o;
            o.op = std::get<0>(t);
            o.group = std::get<1>(t);
            o.nbytes = std::get<2>(t);
            o.nonblocking = std::get<3>(t) == "send";
            o.kind = o.op == "send" ? kSimSend : o.op == "recv" ? kSimRecv : kSimCollective;
            if (o.kind == kSimCollective) std::sort(o.group.begin(), o.group.end());
            ps[r].push_back(std::move(o));
          }
        SimResult res;
        {
          py::gil_scoped_release release;
          res = simulate_programs(ps, rendezvous);
        }
        py::list blocked;
        for (const auto& b : res.blocked) blocked.append(py::make_tuple(b.rank, b.index, b.what));
        py::dict d;
        d["ok"] = res.ok;
        d["error"] = res.error;
        d["blocked"] = blocked;
        d["completed"] = res.completed;
        return d;
      },
      py::arg("programs"), py::arg("rendezvous") = false,
      "Run every rank's communication program against the others under blocking semantics "
      "(collectives meet all members, recvs wait for their message, sends buffer or rendezvous); "
      "returns {ok, error, blocked: [(rank, index, instruction)], completed}.");
}

}  // namespace bfly_rt
