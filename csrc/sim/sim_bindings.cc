// pybind11 glue for the simulator (part of flexmi._native).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cmath>
#include <limits>

#include "simulator.h"

namespace py = pybind11;
using namespace flexmi::sim;

namespace {

LayoutD to_layout(const py::handle& h) {
  LayoutD lay;
  for (auto item : h) {
    auto tup = item.cast<py::tuple>();
    auto lo = tup[0].cast<std::vector<int64_t>>();
    auto hi = tup[1].cast<std::vector<int64_t>>();
    if (lo.size() != hi.size() || lo.size() > (size_t)kMaxDims) throw std::runtime_error("bad box rank");
    Part p;
    p.box.nd = (int)lo.size();
    for (size_t i = 0; i < lo.size(); ++i) {
      p.box.lo[i] = lo[i];
      p.box.hi[i] = hi[i];
    }
    p.holders = tup[2].cast<std::vector<int>>();
    if (p.holders.empty()) throw std::runtime_error("part without holders");
    lay.push_back(std::move(p));
  }
  return lay;
}

Candidate to_cand(const py::dict& d, int ndev) {
  Candidate c;
  c.part_dev = d["part_dev"].cast<std::vector<int>>();
  c.fwd_us = d["fwd_us"].cast<std::vector<double>>();
  c.bwd_us = d["bwd_us"].cast<std::vector<double>>();
  if (c.fwd_us.size() != c.part_dev.size() || c.bwd_us.size() != c.part_dev.size())
    throw std::runtime_error("per-part cost arrays must match part_dev");
  for (int dv : c.part_dev)
    if (dv < 0 || dv >= ndev) throw std::runtime_error("device id out of range");
  for (auto l : d["out"]) c.out.push_back(to_layout(l));
  for (auto l : d["inp"]) c.in.push_back(to_layout(l));
  if (d.contains("wsync"))
    for (auto w : d["wsync"]) {
      auto t = w.cast<py::tuple>();
      WeightSync ws;
      ws.bytes = t[0].cast<double>();
      ws.group = t[1].cast<std::vector<int>>();
      c.wsync.push_back(ws);
    }
  if (d.contains("mem")) c.mem = d["mem"].cast<std::vector<std::pair<int, double>>>();
  if (d.contains("upd")) c.upd_us = d["upd"].cast<std::vector<std::pair<int, double>>>();
  if (d.contains("label")) c.label = d["label"].cast<std::string>();
  if (d.contains("sample_only")) c.sample_only = d["sample_only"].cast<bool>();
  return c;
}

Machine to_machine(const py::dict& d) {
  Machine m;
  auto get = [&](const char* k, double& v) {
    if (d.contains(k)) v = d[k].cast<double>();
  };
  if (d.contains("ndev")) m.ndev = d["ndev"].cast<int>();
  if (d.contains("gpus_per_node")) m.gpus_per_node = d["gpus_per_node"].cast<int>();
  get("link_GBps", m.link_GBps);
  get("link_lat_us", m.link_lat_us);
  get("nic_GBps", m.nic_GBps);
  get("nic_lat_us", m.nic_lat_us);
  get("ar_busbw_GBps", m.ar_busbw_GBps);
  get("ar_lat_us", m.ar_lat_us);
  get("hbm_bytes", m.hbm_bytes);
  get("bucket_bytes", m.bucket_bytes);
  if (d.contains("overlap")) m.overlap = d["overlap"].cast<bool>();
  if (d.contains("xchg_chunks")) m.xchg_chunks = std::max(1, d["xchg_chunks"].cast<int>());
  get("chunk_us", m.chunk_us);
  if (m.ndev < 1 || m.gpus_per_node < 1) throw std::runtime_error("bad machine");
  return m;
}

}  // namespace

void register_sim(py::module_& m) {
  py::class_<Simulator>(m, "Simulator")
      .def(py::init([](const py::dict& machine) { return new Simulator(to_machine(machine)); }))
      .def("add_tensor",
           [](Simulator& s, int elem_bytes, int producer, int producer_out, bool needs_grad) {
             TensorD t;
             t.elem_bytes = elem_bytes;
             t.producer = producer;
             t.producer_out = producer_out;
             t.needs_grad = needs_grad;
             return s.add_tensor(t);
           })
      .def("add_op",
           [](Simulator& s, const std::string& name, const std::vector<int>& in_t, const std::vector<int>& out_t,
              const py::list& cands, int ndev, bool rowwise) {
             OpD op;
             op.name = name;
             op.rowwise = rowwise;
             op.in_t = in_t;
             op.out_t = out_t;
             for (auto c : cands) {
               op.cands.push_back(to_cand(c.cast<py::dict>(), ndev));
               if (op.cands.back().in.size() != in_t.size() || op.cands.back().out.size() != out_t.size())
                 throw std::runtime_error("candidate layouts do not match op arity: " + name);
             }
             if (op.cands.empty()) throw std::runtime_error("op without candidates: " + name);
             return s.add_op(std::move(op));
           },
           py::arg("name"), py::arg("in_t"), py::arg("out_t"), py::arg("cands"), py::arg("ndev"), py::arg("rowwise") = false)
      .def("num_ops", &Simulator::num_ops)
      .def("num_cands", [](const Simulator& s, int i) { return (int)s.op(i).cands.size(); })
      .def("simulate",
           [](Simulator& s, const std::vector<int>& a) {
             if (a.size() != s.num_ops()) throw std::runtime_error("assignment size mismatch");
             py::gil_scoped_release nogil;
             return s.simulate(a);
           })
      .def("memory", &Simulator::memory)
      .def("trace",
           [](Simulator& s, const std::vector<int>& a) {
             std::vector<TraceEvent> tr;
             s.simulate(a, &tr);
             py::list out;
             for (auto& e : tr) out.append(py::make_tuple(e.name, e.kind, e.resource, e.start, e.end));
             return out;
           })
      .def("search",
           [](Simulator& s, const std::vector<int>& init, long budget, double alpha, uint64_t seed, bool verbose,
              const std::vector<char>& frozen, int greedy_passes) {
             if (init.size() != s.num_ops()) throw std::runtime_error("assignment size mismatch");
             SearchResult r;
             {
               py::gil_scoped_release nogil;
               r = s.search(init, budget, alpha, seed, verbose, frozen, greedy_passes);
             }
             return py::make_tuple(r.best, r.best_us, r.init_us, r.history, r.accepted);
           },
           py::arg("init"), py::arg("budget"), py::arg("alpha") = 1.0, py::arg("seed") = 0,
           py::arg("verbose") = false, py::arg("frozen") = std::vector<char>(), py::arg("greedy_passes") = 2);
}
