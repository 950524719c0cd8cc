// Pipeline cut-point search (host runtime, C++): the O(P * L^2) dynamic program behind
// butterfly_amd.partition.search ("DP over cut points ... hot loop").
//
// Given per-layer time t[i] and bytes m[i], fixed extra time/bytes on the first stage
// (embedding) and on the last stage (final norm + LM head), a per-boundary transfer time,
// and a per-stage memory capacity, split layers [0, L) into exactly P contiguous non-empty
// stages minimising  max_s (stage_time_s + boundary_time)  (throughput objective; the
// pipeline's steady-state step is bound by its slowest stage), subject to stage memory <= cap.
// Returns the P+1 cut offsets, or an empty vector if infeasible.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <limits>
#include <vector>

namespace py = pybind11;

namespace bfly_rt {

std::vector<int> pipeline_cuts(const std::vector<double>& t, const std::vector<double>& m, int P,
                               double first_t, double first_m, double last_t, double last_m,
                               double boundary_t, double cap) {
  const int L = (int)t.size();
  if (P <= 0 || P > L || (int)m.size() != L) return {};
  std::vector<double> pt(L + 1, 0.0), pm(L + 1, 0.0);
  for (int i = 0; i < L; ++i) {
    pt[i + 1] = pt[i] + t[i];
    pm[i + 1] = pm[i] + m[i];
  }
  const double INF = std::numeric_limits<double>::infinity();
  auto stage_cost = [&](int s, int i, int j) -> double {  // stage s holds layers [i, j)
    double tm = pt[j] - pt[i], mm = pm[j] - pm[i];
    if (s == 0) { tm += first_t; mm += first_m; }
    if (s == P - 1) { tm += last_t; mm += last_m; }
    if (mm > cap) return INF;
    if (s != P - 1) tm += boundary_t;
    return tm;
  };
  // best[s][j]: min over cuts of the max stage cost for layers [0, j) in stages 0..s
  std::vector<std::vector<double>> best(P, std::vector<double>(L + 1, INF));
  std::vector<std::vector<int>> arg(P, std::vector<int>(L + 1, -1));
  for (int j = 1; j <= L; ++j) best[0][j] = stage_cost(0, 0, j);
  for (int s = 1; s < P; ++s) {
    for (int j = s + 1; j <= L; ++j) {
      double b = INF;
      int a = -1;
      for (int i = s; i < j; ++i) {
        if (best[s - 1][i] == INF) continue;
        const double c = std::max(best[s - 1][i], stage_cost(s, i, j));
        if (c < b) { b = c; a = i; }
      }
      best[s][j] = b;
      arg[s][j] = a;
    }
  }
  if (best[P - 1][L] == INF) return {};
  std::vector<int> cuts(P + 1);
  cuts[P] = L;
  int j = L;
  for (int s = P - 1; s >= 1; --s) {
    j = arg[s][j];
    cuts[s] = j;
  }
  cuts[0] = 0;
  return cuts;
}

void register_partition(py::module_& m) {
  m.def("pipeline_cuts", &pipeline_cuts, py::arg("layer_time"), py::arg("layer_bytes"),
        py::arg("num_stages"), py::arg("first_time") = 0.0, py::arg("first_bytes") = 0.0,
        py::arg("last_time") = 0.0, py::arg("last_bytes") = 0.0, py::arg("boundary_time") = 0.0,
        py::arg("capacity") = std::numeric_limits<double>::infinity(),
        "Min-max contiguous pipeline split; returns P+1 cut offsets (empty if infeasible).");
}

}  // namespace bfly_rt
