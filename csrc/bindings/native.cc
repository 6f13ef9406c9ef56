// pybind11 module flexmi._native: the C++ runtime components (no GPU dependency).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <optional>

#include "hdf5_lite.h"
#include "loader.h"
#include "native_model.h"
#include "planner.h"
#include "shard.h"
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

using PyBox = std::vector<std::pair<int64_t, int64_t>>;
// (shape, degrees, holders, boxes | None, partial)
using PyLayout = std::tuple<std::vector<int64_t>, std::vector<int64_t>, std::vector<std::vector<int>>,
                            std::optional<std::vector<PyBox>>, bool>;

flexmi::ShardLayout to_layout(const PyLayout& t) {
  flexmi::ShardLayout l;
  l.shape = std::get<0>(t);
  l.degrees = std::get<1>(t);
  l.holders = std::get<2>(t);
  if (std::get<3>(t)) l.boxes = *std::get<3>(t);
  l.partial = std::get<4>(t);
  return l;
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

  // sharding algebra (csrc/runtime/shard.h): layouts are (shape, degrees, holders, boxes|None, partial)
  m.def("split_extent", &flexmi::split_extent);
  m.def("part_box", [](const PyLayout& l, int64_t p) { return to_layout(l).part_box(p); });
  m.def("reshard_transfers", [](const PyLayout& src, const PyLayout& dst) {
    std::vector<std::tuple<int, int, PyBox, int64_t, int64_t>> out;
    for (auto& t : flexmi::reshard_transfers(to_layout(src), to_layout(dst)))
      out.emplace_back(t.src, t.dst, t.box, t.src_part, t.dst_part);
    return out;
  });
  m.def("split_launches", [](const std::vector<int64_t>& dst, const std::vector<std::optional<PyBox>>& boxes,
                             int max_per_launch) {
    std::vector<flexmi::Box> b;
    b.reserve(boxes.size());
    for (auto& x : boxes) b.push_back(x ? *x : flexmi::Box{});
    return flexmi::split_launches(dst, b, max_per_launch);
  });

  // graph planner (csrc/runtime/planner.h): op = (guid, [input], [output guid]) with
  // input = (tensor, producer, dtype, need, is_float, needs_grad, reshard, remote);
  // returns (order, fwd, bwd_live, grad_needed, bwd) with steps (kind, op guid, [input idx])
  using PyIn = std::tuple<int64_t, int64_t, int, int64_t, bool, bool, bool, bool>;
  using PyOp = std::tuple<int64_t, std::vector<PyIn>, std::vector<int64_t>>;
  // flat weight buffer + gradient all-reduce buckets (native_model.cc): offsets, numel, buckets
  // [begin, end, entry ids...] -- shared by the Python executor and the native model
  m.def("plan_weights", [](const std::vector<int64_t>& numels, int64_t cap) {
    const flexmi::WeightPlan p = flexmi::plan_weights(numels, cap);
    return py::make_tuple(p.offset, p.numel, p.buckets);
  });
  m.def("plan_graph", [](const std::vector<PyOp>& ops, int world, bool input_grads) {
    std::vector<flexmi::PlanOp> v;
    v.reserve(ops.size());
    for (auto& o : ops) {
      flexmi::PlanOp op;
      op.guid = std::get<0>(o);
      for (auto& t : std::get<1>(o)) {
        flexmi::PlanInput in;
        std::tie(in.tensor, in.producer, in.dtype, in.need, in.is_float, in.needs_grad, in.reshard, in.remote) = t;
        op.inputs.push_back(in);
      }
      op.outputs = std::get<2>(o);
      v.push_back(std::move(op));
    }
    flexmi::GraphPlan p;
    {
      py::gil_scoped_release nogil;
      p = flexmi::plan_graph(v, world, input_grads);
    }
    auto steps = [](const std::vector<flexmi::PlanStep>& s) {
      std::vector<std::tuple<int, int64_t, std::vector<int>>> out;
      for (auto& x : s) out.emplace_back(x.kind, x.op, x.inputs);
      return out;
    };
    return py::make_tuple(p.order, steps(p.fwd), p.bwd_live, p.grad_needed, steps(p.bwd));
  }, py::arg("ops"), py::arg("world"), py::arg("input_grads") = false);

  // minimal HDF5 reader (csrc/runtime/hdf5_lite.h): datasets with their dtype, shape and the byte
  // offset of their contiguous data (memory-mapped by flexmi.utils.hdf5)
  m.def("h5_datasets", [](const std::string& path) {
    std::vector<flexmi::H5Dataset> ds;
    std::string err;
    if (!flexmi::h5_list_datasets(path, ds, err)) throw std::runtime_error("h5_datasets: " + err);
    std::vector<std::tuple<std::string, std::string, std::vector<int64_t>, int64_t, int64_t>> out;
    for (auto& d : ds) out.emplace_back(d.name, d.dtype, d.shape, d.offset, d.nbytes);
    return out;
  });

  // data-loader ring (csrc/runtime/loader.h); pointers are raw addresses of host buffers
  py::class_<flexmi::BatchRing>(m, "BatchRing")
      .def(py::init<int64_t, int64_t, int, int, bool, uint64_t>(), py::arg("batch"), py::arg("num_samples"),
           py::arg("depth") = 3, py::arg("threads") = 2, py::arg("shuffle") = false, py::arg("seed") = 0)
      .def("add_source",
           [](flexmi::BatchRing& r, uintptr_t base, int64_t rows, int64_t row_bytes, int64_t col_off,
              int64_t col_bytes, int64_t row_lo, int64_t row_hi, int64_t dst_pitch) {
             return r.add_source((const void*)base, rows, row_bytes, col_off, col_bytes, row_lo, row_hi, dst_pitch);
           },
           py::arg("base"), py::arg("rows"), py::arg("row_bytes"), py::arg("col_off"), py::arg("col_bytes"),
           py::arg("row_lo"), py::arg("row_hi"), py::arg("dst_pitch") = -1)
      .def("set_slot", [](flexmi::BatchRing& r, int src, int slot, uintptr_t p) { r.set_slot(src, slot, (void*)p); })
      .def("start", &flexmi::BatchRing::start)
      .def("stop", &flexmi::BatchRing::stop, py::call_guard<py::gil_scoped_release>())
      .def("acquire", &flexmi::BatchRing::acquire, py::call_guard<py::gil_scoped_release>())
      .def("release", &flexmi::BatchRing::release)
      .def("batch_ids", &flexmi::BatchRing::batch_ids)
      .def_property_readonly("batches_per_epoch", &flexmi::BatchRing::batches_per_epoch)
      .def_property_readonly("consumed", &flexmi::BatchRing::consumed)
      .def_property_readonly("depth", &flexmi::BatchRing::depth);
}
