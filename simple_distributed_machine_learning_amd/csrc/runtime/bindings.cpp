// pybind11 bindings of the host runtime (_runtime module).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <thread>
#include <vector>

#include "schedule.h"
#include "synth_fill.h"
#include "synth_hash.h"

namespace py = pybind11;
using sdml::Instr;
using sdml::ScheduleSpec;
using sdml::SimStats;

namespace {

ScheduleSpec make_spec(const std::string& kind, int P, int M, int R, double cf, double cb, bool fo) {
  ScheduleSpec s;
  s.kind = kind;
  s.num_stages = P;
  s.num_microbatches = M;
  s.num_ranks = R;
  s.cost_f = cf;
  s.cost_b = cb;
  s.forward_only = fo;
  return s;
}

using PyInstr = std::tuple<int, int, int, int, int, int>;

std::vector<std::vector<PyInstr>> to_py(const std::vector<std::vector<Instr>>& prog) {
  std::vector<std::vector<PyInstr>> out(prog.size());
  for (size_t r = 0; r < prog.size(); ++r)
    for (const Instr& i : prog[r]) out[r].emplace_back(i.op, i.pipe, i.stage, i.mb, i.peer, i.payload);
  return out;
}

std::vector<std::vector<Instr>> from_py(const std::vector<std::vector<PyInstr>>& prog) {
  std::vector<std::vector<Instr>> out(prog.size());
  for (size_t r = 0; r < prog.size(); ++r)
    for (auto& t : prog[r]) {
      Instr i;
      std::tie(i.op, i.pipe, i.stage, i.mb, i.peer, i.payload) = t;
      out[r].push_back(i);
    }
  return out;
}

py::dict stats_dict(const SimStats& s) {
  py::dict d;
  d["makespan"] = s.makespan;
  d["busy"] = s.busy;
  d["max_inflight"] = s.max_inflight;
  d["num_messages"] = s.num_messages;
  return d;
}

// Fill a float32 [n, H*W] image block and int64 [n] label block for samples
// [start, start+n) — host twin of the HIP generator (bit-identical).
void synth_fill(uint64_t seed, int64_t start, int64_t n, int H, int W, int mode, uintptr_t x_ptr,
                uintptr_t y_ptr) {
  unsigned nt = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
  if (n < 4096) nt = 1;
  py::gil_scoped_release nogil;
  sdml::synth_fill_host(seed, start, n, H, W, mode, reinterpret_cast<float*>(x_ptr), reinterpret_cast<int64_t*>(y_ptr),
                        nt);
}

}  // namespace

PYBIND11_MODULE(_runtime, m) {
  m.doc() = "sdml host runtime: pipeline schedules, validator, synthetic data";
  m.attr("OP_FWD") = (int)sdml::OP_FWD;
  m.attr("OP_BWD") = (int)sdml::OP_BWD;
  m.attr("OP_SEND") = (int)sdml::OP_SEND;
  m.attr("OP_RECV") = (int)sdml::OP_RECV;
  m.attr("PL_ACT") = (int)sdml::PL_ACT;
  m.attr("PL_GRAD") = (int)sdml::PL_GRAD;

  m.def(
      "build_schedule",
      [](const std::string& kind, int P, int M, int R, double cf, double cb, bool fo) {
        auto spec = make_spec(kind, P, M, R, cf, cb, fo);
        SimStats st;
        auto prog = sdml::build_schedule(spec, &st);
        return py::make_tuple(to_py(prog), stats_dict(st));
      },
      py::arg("kind"), py::arg("num_stages"), py::arg("num_microbatches"), py::arg("num_ranks"),
      py::arg("cost_f") = 1.0, py::arg("cost_b") = 2.0, py::arg("forward_only") = false,
      "Generate per-rank instruction lists: [(op, pipe, stage, mb, peer, payload), ...] per rank, plus "
      "simulated stats.");
  m.def(
      "validate_schedule",
      [](const std::string& kind, int P, int M, int R, const std::vector<std::vector<PyInstr>>& prog, double cf,
         double cb, bool fo) {
        auto spec = make_spec(kind, P, M, R, cf, cb, fo);
        try {
          return stats_dict(sdml::validate_schedule(spec, from_py(prog)));
        } catch (const std::runtime_error& e) {
          throw py::value_error(e.what());
        }
      },
      py::arg("kind"), py::arg("num_stages"), py::arg("num_microbatches"), py::arg("num_ranks"), py::arg("program"),
      py::arg("cost_f") = 1.0, py::arg("cost_b") = 2.0, py::arg("forward_only") = false,
      "Replay a program under per-channel FIFO + compute-stream semantics; raises ValueError on "
      "mismatch or deadlock.");
  m.def("stage_rank", [](const std::string& kind, int P, int M, int R, int pipe, int stage) {
    return sdml::stage_rank(make_spec(kind, P, M, R, 1, 2, false), pipe, stage);
  });
  m.def("task_rank", [](const std::string& kind, int P, int M, int R, int mb, int stage) {
    return sdml::task_rank(make_spec(kind, P, M, R, 1, 2, false), mb, stage);
  });
  m.def("mb_pipe", [](const std::string& kind, int P, int M, int R, int mb) {
    return sdml::mb_pipe(make_spec(kind, P, M, R, 1, 2, false), mb);
  });
  m.def("synth_fill", &synth_fill, py::arg("seed"), py::arg("start"), py::arg("n"), py::arg("H"), py::arg("W"),
        py::arg("mode"), py::arg("x_ptr"), py::arg("y_ptr"),
        "Fill host buffers with the counter-based synthetic MNIST-shape data (0 pointers skip).");
}
