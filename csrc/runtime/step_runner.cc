// flexmi native step runner (module flexmi._rt): replays a compiled per-rank program.
//
// The plan compiler (flexmi/runtime/executor.py) turns (graph, strategy, rank) into flat item
// lists; this runner executes them without a Python loop: hipGraph segments are launched with
// hipGraphLaunch on the current HIP stream, collectives go straight to the rank's c10d process
// group (RCCL over xGMI on MI355X, gloo in CPU tests) and their Work handles live in numbered
// slots so a collective started in one program (e.g. a gradient bucket all-reduce in backward)
// is waited on in another (the update).  Items that are not natively expressible stay Python
// callables.  Replaces the reference's Legion runtime loop -- per-op index launches
// (src/runtime/model.cc:948-993) replayed through Legion tracing (examples/cpp/DLRM/dlrm.cc:178-185)
// with DMA copies inserted by the dependence analysis.
#include <hip/hip_runtime_api.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>
#include <torch/csrc/distributed/c10d/Work.hpp>
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <map>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;
using PG = c10::intrusive_ptr<c10d::ProcessGroup>;
using WorkPtr = c10::intrusive_ptr<c10d::Work>;

namespace {

enum Kind : int {
  CALL = 0,        // Python callable
  GRAPH = 1,       // hipGraphLaunch(exec, current stream)
  A2A_START = 2,   // alltoall_base(recv, send, recv_splits, send_splits) -> slot
  AR_START = 3,    // allreduce([t]) -> slot
  WAIT = 4,        // wait(slot) (no-op when the slot is empty)
  AR_SYNC = 5,     // wait(slot) if a work is pending, else allreduce([t]) + wait
  RS_START = 6,    // _reduce_scatter_base(out, in) -> slot       (ZeRO-1 gradient shard sync)
  RS_SYNC = 7,     // wait(slot) if pending, else reduce-scatter + wait
  AG_SYNC = 8,     // _allgather_base(out, in) + wait             (ZeRO-1 parameter gather)
  P2P_START = 9,   // grouped send/recv with the peers of non-zero splits only -> slot
};

const char* kind_name(int k) {
  static const char* n[] = {"call", "graph", "all_to_all", "all_reduce", "wait", "all_reduce_sync",
                            "reduce_scatter", "reduce_scatter_sync", "all_gather_sync", "p2p"};
  return (k >= 0 && k <= 9) ? n[k] : "?";
}

struct Step {
  int kind = CALL;
  std::string name;
  py::object fn;
  uintptr_t graph = 0;
  int slot = -1;
  PG pg;
  at::Tensor a, b;                 // A2A: recv, send; AR: tensor
  std::vector<int64_t> sa, sb;     // A2A: recv splits, send splits (elements along dim 0)
};

#define HIP_OK(x)                                                                              \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("flexmi._rt: ") + #x + ": " + \
                                                   hipGetErrorString(e_));                     \
  } while (0)

// A C++-owned alias (new TensorImpl over the same storage, no Python object attached) of a
// tensor handed in from Python.  The collectives' works capture these, so the backend threads
// that drop the last reference to a finished work never need the GIL -- which they cannot take
// once the interpreter is shutting down.
at::Tensor c_alias(const at::Tensor& t) { return at::alias(t); }

class StepRunner {
 public:
  int new_program() {
    progs_.emplace_back();
    return (int)progs_.size() - 1;
  }
  int new_slot() {
    slots_.emplace_back();
    extra_.emplace_back();
    drops_.emplace_back();
    pending_.push_back(false);
    return (int)slots_.size() - 1;
  }
  int num_programs() const { return (int)progs_.size(); }
  int program_size(int p) const { return (int)prog(p).size(); }

  void add_call(int p, py::object fn, const std::string& name) {
    Step s;
    s.kind = CALL;
    s.fn = std::move(fn);
    s.name = name;
    prog(p).push_back(std::move(s));
  }
  void add_graph(int p, uintptr_t exec, const std::string& name) {
    if (!exec) throw std::invalid_argument("add_graph: null hipGraphExec_t");
    Step s;
    s.kind = GRAPH;
    s.graph = exec;
    s.name = name;
    prog(p).push_back(std::move(s));
  }
  void add_all_to_all(int p, int slot, PG pg, at::Tensor recv, at::Tensor send, std::vector<int64_t> recv_splits,
                      std::vector<int64_t> send_splits, const std::string& name) {
    check_slot(slot);
    int64_t nr = 0, ns = 0;
    for (auto v : recv_splits) nr += v;
    for (auto v : send_splits) ns += v;
    if (recv.dim() != 1 || send.dim() != 1 || nr != recv.numel() || ns != send.numel())
      throw std::invalid_argument("add_all_to_all: 1-D buffers whose sizes equal the split sums expected");
    if ((int64_t)recv_splits.size() != pg->getSize() || (int64_t)send_splits.size() != pg->getSize())
      throw std::invalid_argument("add_all_to_all: one split per rank of the group expected");
    Step s;
    s.kind = A2A_START;
    s.slot = slot;
    s.pg = std::move(pg);
    s.a = c_alias(recv);
    s.b = c_alias(send);
    s.sa = std::move(recv_splits);
    s.sb = std::move(send_splits);
    s.name = name;
    prog(p).push_back(std::move(s));
  }
  // Sparse exchange (halos, pipeline hand-offs, placement-local reshards): same buffers and
  // per-group-rank splits as add_all_to_all, but only the peers with a non-zero split are posted,
  // as ONE grouped launch on RCCL (start/endCoalescing) -- point-to-point xGMI transfers instead
  // of an all-to-all over the whole group.
  void add_p2p(int p, int slot, PG pg, at::Tensor recv, at::Tensor send, std::vector<int64_t> recv_splits,
               std::vector<int64_t> send_splits, const std::string& name) {
    add_all_to_all(p, slot, std::move(pg), recv, send, std::move(recv_splits), std::move(send_splits), name);
    prog(p).back().kind = P2P_START;
  }
  void add_all_reduce(int p, int slot, PG pg, at::Tensor t, bool sync, const std::string& name) {
    check_slot(slot);
    Step s;
    s.kind = sync ? AR_SYNC : AR_START;
    s.slot = slot;
    s.pg = std::move(pg);
    s.a = c_alias(t);
    s.name = name;
    prog(p).push_back(std::move(s));
  }
  // out = this rank's 1/n of the element-wise sum of every rank's `in` (in.numel() == n * out.numel())
  void add_reduce_scatter(int p, int slot, PG pg, at::Tensor out, at::Tensor in, bool sync, const std::string& name) {
    check_slot(slot);
    if (in.numel() != out.numel() * pg->getSize())
      throw std::invalid_argument("add_reduce_scatter: in.numel() must be group size x out.numel()");
    Step s;
    s.kind = sync ? RS_SYNC : RS_START;
    s.slot = slot;
    s.pg = std::move(pg);
    s.a = c_alias(out);
    s.b = c_alias(in);
    s.name = name;
    prog(p).push_back(std::move(s));
  }
  // out = concat over ranks of `in` (out.numel() == n * in.numel()), waited on before returning
  void add_all_gather(int p, int slot, PG pg, at::Tensor out, at::Tensor in, const std::string& name) {
    check_slot(slot);
    if (out.numel() != in.numel() * pg->getSize())
      throw std::invalid_argument("add_all_gather: out.numel() must be group size x in.numel()");
    Step s;
    s.kind = AG_SYNC;
    s.slot = slot;
    s.pg = std::move(pg);
    s.a = c_alias(out);
    s.b = c_alias(in);
    s.name = name;
    prog(p).push_back(std::move(s));
  }
  void add_wait(int p, int slot, const std::string& name) {
    check_slot(slot);
    Step s;
    s.kind = WAIT;
    s.slot = slot;
    s.name = name;
    prog(p).push_back(std::move(s));
  }

  // Execute program p in order.  The GIL is held only while a Python callable runs.  Optional
  // hooks (debug / watchdog modes): pre(i, name) before and post(i, name) after
  // every step -- heartbeats and per-item NaN/Inf guards without leaving the native runner.
  void run(int p, py::object pre = py::none(), py::object post = py::none()) {
    if (released_) throw std::runtime_error("StepRunner: released (process group torn down)");
    auto& steps = prog(p);
    const bool hooks = !pre.is_none() || !post.is_none();
    for (size_t i = 0; i < steps.size(); ++i) {
      Step& s = steps[i];
      current_ = (int)i;
      if (!pre.is_none()) pre((int)i, s.name);
      if (s.kind == CALL) {
        s.fn();
      } else {
        py::gil_scoped_release nogil;
        exec_native(s);
      }
      if (hooks && !post.is_none()) post((int)i, s.name);
    }
    current_ = -1;
    ++runs_;
  }

  // Fault injection into the collectives this runner issues (the native form of
  // flexmi.runtime.health.FaultyComm): {ordinal of the collective: (kind, arg)} with kind
  // "delay" (sleep arg seconds first), "drop" (the collective runs on a scratch copy, so this
  // rank loses its result), "corrupt" (NaN written into the first payload element) or "kill"
  // (the process exits with code 3).
  void set_faults(const std::map<int64_t, std::pair<std::string, double>>& f) {
    faults_.clear();
    for (auto& kv : f) {
      const std::string& k = kv.second.first;
      int kind = k == "delay" ? 0 : k == "drop" ? 1 : k == "corrupt" ? 2 : k == "kill" ? 3 : -1;
      if (kind < 0) throw std::invalid_argument("set_faults: unknown fault kind " + k);
      faults_[kv.first] = {kind, kv.second.second};
    }
    fault_n_ = 0;
  }
  int64_t fault_calls() const { return fault_n_; }

  // drop every pending Work handle (after an error / before tear-down)
  void reset_slots() {
    for (auto& w : slots_) w.reset();
    for (auto& v : extra_) v.clear();
    for (auto& d : drops_) d = {};
    std::fill(pending_.begin(), pending_.end(), false);
  }

  // drop every reference the programs hold (process groups, tensors, callables): a c10d process
  // group must not outlive the interpreter state it was created in
  void release() {
    reset_slots();
    for (auto& p : progs_) p.clear();
    released_ = true;
  }
  bool released() const { return released_; }

  py::dict stats() const {
    py::dict d;
    d["runs"] = runs_;
    d["collectives"] = collectives_;
    d["bytes_sent"] = bytes_sent_;
    d["graph_launches"] = graph_launches_;
    d["waits"] = waits_;
    return d;
  }
  std::string current_name(int p) const {
    if (current_ < 0 || p < 0 || p >= (int)progs_.size() || current_ >= (int)progs_[p].size()) return "";
    return progs_[p][current_].name;
  }
  std::vector<std::pair<std::string, std::string>> describe(int p) const {
    std::vector<std::pair<std::string, std::string>> out;
    for (auto& s : prog(p)) out.emplace_back(kind_name(s.kind), s.name);
    return out;
  }
  int64_t collectives() const { return collectives_; }
  int64_t bytes_sent() const { return bytes_sent_; }

 private:
  std::vector<Step>& prog(int p) {
    if (p < 0 || p >= (int)progs_.size()) throw std::out_of_range("StepRunner: bad program id");
    return progs_[p];
  }
  const std::vector<Step>& prog(int p) const {
    if (p < 0 || p >= (int)progs_.size()) throw std::out_of_range("StepRunner: bad program id");
    return progs_[p];
  }
  void check_slot(int slot) const {
    if (slot < 0 || slot >= (int)slots_.size()) throw std::out_of_range("StepRunner: bad slot id");
  }

  // A finished Work stays in its slot until the slot is reused (or released): the backend's
  // worker thread drops its own reference right after completing the work, so the LAST reference
  // -- and with it the tensors the work captured -- is released on this thread, never on a
  // backend thread racing interpreter shutdown.
  struct Fault {
    int kind;
    double arg;
  };
  // next collective: apply its injected fault (if any); returns the tensor the collective should
  // write into (a scratch copy when the result is dropped)
  // A dropped result: the collective writes into a scratch copy that stays alive (drops_) until
  // the slot's works have finished; an out-of-place result buffer is then zeroed and an in-place
  // one (all-reduce) keeps this rank's local values -- the outcomes of the Python FaultyComm.
  at::Tensor inject(at::Tensor payload, at::Tensor result) {
    auto it = faults_.find(fault_n_++);
    if (it == faults_.end()) return result;
    const Fault f = it->second;
    if (f.kind == 0) std::this_thread::sleep_for(std::chrono::duration<double>(f.arg));
    if (f.kind == 3) std::_Exit(3);
    if (f.kind == 2 && payload.numel() > 0) payload.reshape({-1}).narrow(0, 0, 1).fill_(NAN);
    if (f.kind == 1) {   // in-place collectives (all-reduce) keep this rank's local data instead
      pending_drop_ = {result.clone(), payload.is_same(result) ? at::Tensor() : result};
      return pending_drop_.first;
    }
    return result;
  }

  void start(int slot, WorkPtr w, std::vector<WorkPtr> more = {}) {
    if (pending_[slot]) finish(slot);
    slots_[slot] = std::move(w);
    extra_[slot] = std::move(more);
    drops_[slot] = std::move(pending_drop_);
    pending_drop_ = {};
    pending_[slot] = true;
    ++collectives_;
  }
  void finish(int slot) {
    if (!pending_[slot]) return;
    if (slots_[slot]) slots_[slot]->wait();
    for (auto& w : extra_[slot])
      if (w) w->wait();
    if (drops_[slot].first.defined()) {
      if (drops_[slot].second.defined()) drops_[slot].second.zero_();
      drops_[slot] = {};
    }
    pending_[slot] = false;
    ++waits_;
  }

  void exec_native(Step& s) {
    switch (s.kind) {
      case GRAPH: {
        hipStream_t st = c10::hip::getCurrentHIPStream().stream();
        HIP_OK(hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(s.graph), st));
        ++graph_launches_;
        break;
      }
      case A2A_START: {
        if (pending_[s.slot]) finish(s.slot);
        c10d::AllToAllOptions o;
        at::Tensor recv = faults_.empty() ? s.a : inject(s.b, s.a);
        start(s.slot, s.pg->alltoall_base(recv, s.b, s.sa, s.sb, o));
        bytes_sent_ += s.b.numel() * s.b.element_size();
        break;
      }
      case P2P_START: {
        if (pending_[s.slot]) finish(s.slot);
        at::Tensor recv = faults_.empty() ? s.a : inject(s.b, s.a);
        const bool coalesce = s.pg->getBackendType() == c10d::ProcessGroup::BackendType::NCCL;
        if (coalesce) s.pg->startCoalescing(recv.device().type());
        std::vector<WorkPtr> works;
        int64_t ro = 0, so = 0;
        for (size_t q = 0; q < s.sa.size(); ++q) {
          if (s.sb[q] > 0) {
            std::vector<at::Tensor> t{s.b.narrow(0, so, s.sb[q])};
            works.push_back(s.pg->send(t, (int)q, 0));
          }
          if (s.sa[q] > 0) {
            std::vector<at::Tensor> t{recv.narrow(0, ro, s.sa[q])};
            works.push_back(s.pg->recv(t, (int)q, 0));
          }
          so += s.sb[q];
          ro += s.sa[q];
        }
        if (coalesce) start(s.slot, s.pg->endCoalescing(recv.device().type()));
        else start(s.slot, WorkPtr(), std::move(works));
        bytes_sent_ += s.b.numel() * s.b.element_size();
        break;
      }
      case AR_START: {
        if (pending_[s.slot]) finish(s.slot);
        std::vector<at::Tensor> v{faults_.empty() ? s.a : inject(s.a, s.a)};
        start(s.slot, s.pg->allreduce(v));
        bytes_sent_ += s.a.numel() * s.a.element_size();
        break;
      }
      case AR_SYNC: {
        if (!pending_[s.slot]) {
          std::vector<at::Tensor> v{faults_.empty() ? s.a : inject(s.a, s.a)};
          start(s.slot, s.pg->allreduce(v));
          bytes_sent_ += s.a.numel() * s.a.element_size();
        }
        finish(s.slot);
        break;
      }
      case RS_START:
      case RS_SYNC: {
        if (s.kind == RS_START && pending_[s.slot]) finish(s.slot);
        if (s.kind == RS_START || !pending_[s.slot]) {
          c10d::ReduceScatterOptions o;
          at::Tensor out = faults_.empty() ? s.a : inject(s.b, s.a);
          start(s.slot, s.pg->_reduce_scatter_base(out, s.b, o));
          bytes_sent_ += s.b.numel() * s.b.element_size();
        }
        if (s.kind == RS_SYNC) finish(s.slot);
        break;
      }
      case AG_SYNC: {
        if (pending_[s.slot]) finish(s.slot);
        c10d::AllgatherOptions o;
        at::Tensor out = faults_.empty() ? s.a : inject(s.b, s.a);
        start(s.slot, s.pg->_allgather_base(out, s.b, o));
        bytes_sent_ += s.b.numel() * s.b.element_size();
        finish(s.slot);
        break;
      }
      case WAIT:
        finish(s.slot);
        break;
      default:
        throw std::logic_error("StepRunner: unknown step kind");
    }
  }

  std::vector<std::vector<Step>> progs_;
  std::map<int64_t, Fault> faults_;
  int64_t fault_n_ = 0;
  std::vector<WorkPtr> slots_;
  std::vector<std::vector<WorkPtr>> extra_;   // further works of a slot (uncoalesced p2p)
  std::vector<std::pair<at::Tensor, at::Tensor>> drops_;   // (scratch, real result) of a dropped collective
  std::pair<at::Tensor, at::Tensor> pending_drop_;
  std::vector<bool> pending_;
  int current_ = -1;
  bool released_ = false;
  int64_t runs_ = 0, collectives_ = 0, bytes_sent_ = 0, graph_launches_ = 0, waits_ = 0;
};

}  // namespace

PYBIND11_MODULE(_rt, m) {
  m.doc() = "flexmi native step runner: hipGraph segments + c10d (RCCL) collectives without a Python loop";
  py::class_<StepRunner>(m, "StepRunner")
      .def(py::init<>())
      .def("new_program", &StepRunner::new_program)
      .def("new_slot", &StepRunner::new_slot)
      .def("num_programs", &StepRunner::num_programs)
      .def("program_size", &StepRunner::program_size)
      .def("add_call", &StepRunner::add_call, py::arg("program"), py::arg("fn"), py::arg("name") = "")
      .def("add_graph", &StepRunner::add_graph, py::arg("program"), py::arg("exec"), py::arg("name") = "")
      .def("add_all_to_all", &StepRunner::add_all_to_all, py::arg("program"), py::arg("slot"), py::arg("pg"),
           py::arg("recv"), py::arg("send"), py::arg("recv_splits"), py::arg("send_splits"), py::arg("name") = "")
      .def("add_p2p", &StepRunner::add_p2p, py::arg("program"), py::arg("slot"), py::arg("pg"), py::arg("recv"),
           py::arg("send"), py::arg("recv_splits"), py::arg("send_splits"), py::arg("name") = "")
      .def("add_all_reduce", &StepRunner::add_all_reduce, py::arg("program"), py::arg("slot"), py::arg("pg"),
           py::arg("tensor"), py::arg("sync") = false, py::arg("name") = "")
      .def("add_reduce_scatter", &StepRunner::add_reduce_scatter, py::arg("program"), py::arg("slot"), py::arg("pg"),
           py::arg("out"), py::arg("input"), py::arg("sync") = false, py::arg("name") = "")
      .def("add_all_gather", &StepRunner::add_all_gather, py::arg("program"), py::arg("slot"), py::arg("pg"),
           py::arg("out"), py::arg("input"), py::arg("name") = "")
      .def("add_wait", &StepRunner::add_wait, py::arg("program"), py::arg("slot"), py::arg("name") = "")
      .def("run", &StepRunner::run, py::arg("program"), py::arg("pre") = py::none(), py::arg("post") = py::none())
      .def("set_faults", &StepRunner::set_faults)
      .def_property_readonly("fault_calls", &StepRunner::fault_calls)
      .def("reset_slots", &StepRunner::reset_slots)
      .def("release", &StepRunner::release)
      .def_property_readonly("released", &StepRunner::released)
      .def("stats", &StepRunner::stats)
      .def("current_name", &StepRunner::current_name)
      .def("describe", &StepRunner::describe)
      .def_property_readonly("collectives", &StepRunner::collectives)
      .def_property_readonly("bytes_sent", &StepRunner::bytes_sent);
}
