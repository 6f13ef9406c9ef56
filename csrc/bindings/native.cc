// pybind11 module flexmi._native: the C++ runtime components (no GPU dependency).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "strategy_pb.h"

namespace py = pybind11;
using flexmi::OpStrategy;

void register_sim(py::module_& m);  // simulator.cc

namespace {

using OpTuple = std::tuple<std::string, int, std::vector<int>, std::vector<int>, std::vector<int>>;

std::vector<OpTuple> to_tuples(const std::vector<OpStrategy>& ops) {
  std::vector<OpTuple> out;
  for (auto& o : ops) out.emplace_back(o.name, o.device_type, o.dims, o.device_ids, o.memory_types);
  return out;
}

std::vector<OpStrategy> from_tuples(const std::vector<OpTuple>& t) {
  std::vector<OpStrategy> ops;
  for (auto& x : t) {
    OpStrategy o;
    o.name = std::get<0>(x);
    o.device_type = std::get<1>(x);
    o.dims = std::get<2>(x);
    o.device_ids = std::get<3>(x);
    o.memory_types = std::get<4>(x);
    ops.push_back(o);
  }
  return ops;
}

}  // namespace

PYBIND11_MODULE(_native, m) {
  m.doc() = "flexmi native runtime: strategy codec, MI355X simulator and MCMC search";
  m.def("load_strategy", [](const std::string& path) {
    std::vector<OpStrategy> ops;
    std::string err;
    if (!flexmi::load_strategy_file(path, ops, err)) throw std::runtime_error("load_strategy: " + err);
    return to_tuples(ops);
  });
  m.def("save_strategy", [](const std::string& path, const std::vector<OpTuple>& t) {
    std::string err;
    if (!flexmi::save_strategy_file(path, from_tuples(t), err)) throw std::runtime_error("save_strategy: " + err);
    return true;
  });
  m.def("encode_strategy", [](const std::vector<OpTuple>& t) { return py::bytes(flexmi::encode_strategy(from_tuples(t))); });
  m.def("decode_strategy", [](const py::bytes& b) {
    std::vector<OpStrategy> ops;
    std::string err;
    if (!flexmi::decode_strategy(std::string(b), ops, err)) throw std::runtime_error("decode_strategy: " + err);
    return to_tuples(ops);
  });
  register_sim(m);
}
