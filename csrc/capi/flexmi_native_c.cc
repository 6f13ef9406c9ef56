// flexmi native C API (flexmi_native_c.h): thin C handles over the C++ runtime -- strategy
// codec, sharding algebra, simulator + search, HDF5 reader, batch loader ring, CPU embedding
// kernels.  No Python anywhere: libflexmi_native_c.so links only these sources.
#include "flexmi_native_c.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <exception>
#include <limits>
#include <memory>
#include <string>
#include <vector>

#include "../cpu/emb_kernels.h"
#include "../runtime/hdf5_lite.h"
#include "../runtime/loader.h"
#include "../runtime/planner.h"
#include "../runtime/shard.h"
#include "../runtime/strategy_pb.h"
#include "../sim/simulator.h"
#include "../runtime/native_model.h"

namespace {

thread_local std::string g_err;

int fail(const std::string& m) {
  g_err = m;
  return -1;
}

template <typename F>
auto guarded(F&& f, decltype(f()) bad) -> decltype(f()) {
  try {
    return f();
  } catch (const std::exception& e) {
    g_err = e.what();
  } catch (...) {
    g_err = "unknown C++ exception";
  }
  return bad;
}

int itemsize(const std::string& dtype) {
  // numpy-style "<f4", "<i8", "|u1": trailing digits are the byte size
  size_t i = dtype.size();
  while (i > 0 && isdigit((unsigned char)dtype[i - 1])) --i;
  return i < dtype.size() ? atoi(dtype.c_str() + i) : 0;
}

}  // namespace

struct fmn_strategy_s {
  std::vector<flexmi::OpStrategy> ops;
};
struct fmn_layout_s {
  flexmi::ShardLayout l;
};
struct fmn_sim_s {
  flexmi::sim::Machine m;
  std::vector<flexmi::sim::TensorD> tensors;
  std::vector<flexmi::sim::OpD> ops;
  std::unique_ptr<flexmi::sim::Simulator> sim;   // built on first simulate / search
  flexmi::sim::Simulator& get() {
    if (!sim) {
      sim.reset(new flexmi::sim::Simulator(m));
      for (auto& t : tensors) sim->add_tensor(t);
      for (auto& o : ops) sim->add_op(o);
    }
    return *sim;
  }
};
struct fmn_h5_s {
  std::string path;
  std::vector<flexmi::H5Dataset> ds;
};
struct fmn_loader_s {
  std::unique_ptr<flexmi::BatchRing> ring;
};

extern "C" {

const char* fmn_last_error(void) { return g_err.c_str(); }
const char* fmn_version(void) { return "flexmi-native 1"; }

// ------------------------------------------------------------------------------ strategies
fmn_strategy_t fmn_strategy_create(void) { return new fmn_strategy_s(); }

fmn_strategy_t fmn_strategy_load(const char* path) {
  auto* s = new fmn_strategy_s();
  std::string err;
  if (!flexmi::load_strategy_file(path ? path : "", s->ops, err)) {
    g_err = err;
    delete s;
    return nullptr;
  }
  return s;
}

int fmn_strategy_save(fmn_strategy_t s, const char* path) {
  if (!s || !path) return fail("null argument");
  std::string err;
  return flexmi::save_strategy_file(path, s->ops, err) ? 0 : fail(err);
}

void fmn_strategy_destroy(fmn_strategy_t s) { delete s; }

int fmn_strategy_num_ops(fmn_strategy_t s) { return s ? (int)s->ops.size() : fail("null strategy"); }

int fmn_strategy_find(fmn_strategy_t s, const char* name) {
  if (!s || !name) return fail("null argument");
  for (size_t i = 0; i < s->ops.size(); ++i)
    if (s->ops[i].name == name) return (int)i;
  return -1;
}

int fmn_strategy_get(fmn_strategy_t s, int i, char* name, size_t len, int* device_type, int* ndims, int* dims, int max_dims,
                     int* ndev, int* devs, int max_devs) {
  if (!s || i < 0 || i >= (int)s->ops.size()) return fail("op index out of range");
  const auto& o = s->ops[i];
  if (name && len) {
    std::strncpy(name, o.name.c_str(), len - 1);
    name[len - 1] = 0;
  }
  if (device_type) *device_type = o.device_type;
  if (ndims) *ndims = (int)o.dims.size();
  for (int k = 0; dims && k < (int)o.dims.size() && k < max_dims; ++k) dims[k] = o.dims[k];
  if (ndev) *ndev = (int)o.device_ids.size();
  for (int k = 0; devs && k < (int)o.device_ids.size() && k < max_devs; ++k) devs[k] = o.device_ids[k];
  return o.num_parts();
}

int fmn_strategy_set(fmn_strategy_t s, const char* name, int device_type, int ndims, const int* dims, int ndev,
                     const int* devs) {
  if (!s || !name || ndims < 0 || ndev < 0) return fail("bad argument");
  flexmi::OpStrategy o;
  o.name = name;
  o.device_type = device_type;
  o.dims.assign(dims, dims + ndims);
  o.device_ids.assign(devs, devs + ndev);
  if (o.num_parts() != ndev) return fail("device count must equal the product of dims");
  int i = fmn_strategy_find(s, name);
  if (i >= 0) s->ops[i] = o;
  else s->ops.push_back(o);
  return 0;
}

// ------------------------------------------------------------------------------ sharding
int fmn_split_extent(int64_t n, int64_t d, int64_t k, int64_t* lo, int64_t* hi) {
  if (d <= 0 || k < 0 || k >= d) return fail("bad split");
  auto r = flexmi::split_extent(n, d, k);
  *lo = r.first;
  *hi = r.second;
  return 0;
}

fmn_layout_t fmn_layout_create(int nd, const int64_t* shape, const int64_t* degrees, const int* holders, int partial) {
  return guarded(
      [&]() -> fmn_layout_t {
        auto* L = new fmn_layout_s();
        L->l.shape.assign(shape, shape + nd);
        L->l.degrees.assign(degrees, degrees + nd);
        L->l.partial = partial != 0;
        int64_t np = 1;
        for (int i = 0; i < nd; ++i) np *= degrees[i];
        L->l.holders.resize(np);
        for (int64_t p = 0; p < np; ++p) L->l.holders[p] = {holders[p]};
        L->l.validate();
        return L;
      },
      (fmn_layout_t) nullptr);
}

int fmn_layout_add_holder(fmn_layout_t l, int part, int rank) {
  if (!l || part < 0 || part >= (int)l->l.holders.size()) return fail("part out of range");
  l->l.holders[part].push_back(rank);
  return 0;
}

int64_t fmn_layout_num_parts(fmn_layout_t l) { return l ? l->l.num_parts() : fail("null layout"); }

int fmn_layout_part_box(fmn_layout_t l, int64_t part, int64_t* lo, int64_t* hi) {
  if (!l || part < 0 || part >= l->l.num_parts()) return fail("part out of range");
  auto b = l->l.part_box(part);
  for (size_t d = 0; d < b.size(); ++d) {
    lo[d] = b[d].first;
    hi[d] = b[d].second;
  }
  return 0;
}

void fmn_layout_destroy(fmn_layout_t l) { delete l; }

int fmn_reshard_transfers(fmn_layout_t src, fmn_layout_t dst, int max_n, int* src_rank, int* dst_rank, int64_t* lo,
                          int64_t* hi) {
  if (!src || !dst) return fail("null layout");
  return guarded(
      [&]() -> int {
        auto tr = flexmi::reshard_transfers(src->l, dst->l);
        const size_t nd = src->l.shape.size();
        for (int i = 0; i < (int)tr.size() && i < max_n; ++i) {
          if (src_rank) src_rank[i] = tr[i].src;
          if (dst_rank) dst_rank[i] = tr[i].dst;
          for (size_t d = 0; d < nd; ++d) {
            if (lo) lo[i * nd + d] = tr[i].box[d].first;
            if (hi) hi[i * nd + d] = tr[i].box[d].second;
          }
        }
        return (int)tr.size();
      },
      -1);
}

// ------------------------------------------------------------------------------ simulator
fmn_sim_t fmn_sim_create(int ndev, int gpus_per_node, double link_GBps, double ar_busbw_GBps) {
  if (ndev <= 0) {
    fail("ndev must be > 0");
    return nullptr;
  }
  auto* s = new fmn_sim_s();
  s->m.ndev = ndev;
  if (gpus_per_node > 0) s->m.gpus_per_node = gpus_per_node;
  if (link_GBps > 0) s->m.link_GBps = link_GBps;
  if (ar_busbw_GBps > 0) s->m.ar_busbw_GBps = ar_busbw_GBps;
  return s;
}

void fmn_sim_destroy(fmn_sim_t s) { delete s; }

int fmn_sim_add_tensor(fmn_sim_t s, int elem_bytes, int producer, int producer_out, int needs_grad) {
  if (!s || s->sim) return fail("simulator already built");
  flexmi::sim::TensorD t;
  t.elem_bytes = elem_bytes;
  t.producer = producer;
  t.producer_out = producer_out;
  t.needs_grad = needs_grad != 0;
  s->tensors.push_back(t);
  return (int)s->tensors.size() - 1;
}

int fmn_sim_add_op(fmn_sim_t s, const char* name, int n_in, const int* in_t, int n_out, const int* out_t) {
  if (!s || s->sim) return fail("simulator already built");
  flexmi::sim::OpD o;
  o.name = name ? name : "";
  o.in_t.assign(in_t, in_t + n_in);
  o.out_t.assign(out_t, out_t + n_out);
  for (int t : o.in_t)
    if (t < 0 || t >= (int)s->tensors.size()) return fail("unknown input tensor");
  s->ops.push_back(o);
  return (int)s->ops.size() - 1;
}

int fmn_sim_add_candidate(fmn_sim_t s, int nparts, const int* part_dev, const double* fwd_us, const double* bwd_us, int nd,
                          const int64_t* out_lo, const int64_t* out_hi, const int64_t* in_lo, const int64_t* in_hi,
                          double wsync_bytes, double mem_bytes, const char* label) {
  if (!s || s->sim || s->ops.empty()) return fail("no op to add a candidate to (or simulator already built)");
  if (nparts <= 0 || nd <= 0 || nd > flexmi::sim::kMaxDims) return fail("bad candidate shape");
  auto& op = s->ops.back();
  flexmi::sim::Candidate c;
  c.part_dev.assign(part_dev, part_dev + nparts);
  c.fwd_us.assign(fwd_us, fwd_us + nparts);
  c.bwd_us.assign(bwd_us, bwd_us + nparts);
  auto layouts = [&](int n, const int64_t* lo, const int64_t* hi) {
    std::vector<flexmi::sim::LayoutD> out(n);
    for (int t = 0; t < n; ++t)
      for (int p = 0; p < nparts; ++p) {
        flexmi::sim::Part part;
        part.box.nd = nd;
        for (int d = 0; d < nd; ++d) {
          part.box.lo[d] = lo[((long)t * nparts + p) * nd + d];
          part.box.hi[d] = hi[((long)t * nparts + p) * nd + d];
        }
        part.holders = {part_dev[p]};
        out[t].push_back(part);
      }
    return out;
  };
  c.out = layouts((int)op.out_t.size(), out_lo, out_hi);
  c.in = layouts((int)op.in_t.size(), in_lo, in_hi);
  if (wsync_bytes > 0) {
    flexmi::sim::WeightSync w;
    w.bytes = wsync_bytes;
    w.group = c.part_dev;
    std::sort(w.group.begin(), w.group.end());
    w.group.erase(std::unique(w.group.begin(), w.group.end()), w.group.end());
    if (w.group.size() > 1) c.wsync.push_back(w);
  }
  for (int p = 0; p < nparts; ++p) c.mem.push_back({part_dev[p], mem_bytes});
  c.label = label ? label : "";
  op.cands.push_back(c);
  return (int)op.cands.size() - 1;
}

double fmn_sim_simulate(fmn_sim_t s, const int* assign) {
  if (!s) {
    fail("null simulator");
    return -1.0;
  }
  return guarded(
      [&]() -> double {
        auto& sim = s->get();
        std::vector<int> a(assign, assign + sim.num_ops());
        return sim.simulate(a);
      },
      -1.0);
}

double fmn_sim_search(fmn_sim_t s, const int* init, long budget, double alpha, uint64_t seed, int* best) {
  if (!s) {
    fail("null simulator");
    return -1.0;
  }
  return guarded(
      [&]() -> double {
        auto& sim = s->get();
        const size_t n = sim.num_ops();
        std::vector<int> a(init, init + n);
        std::vector<char> frozen(n, 0);
        auto r = sim.search(a, budget, alpha, seed, false, frozen);
        for (size_t i = 0; i < n; ++i) best[i] = r.best[i];
        return r.best_us;
      },
      -1.0);
}

// ------------------------------------------------------------------------------ HDF5
fmn_h5_t fmn_h5_open(const char* path) {
  auto* h = new fmn_h5_s();
  h->path = path ? path : "";
  std::string err;
  if (!flexmi::h5_list_datasets(h->path, h->ds, err)) {
    g_err = err;
    delete h;
    return nullptr;
  }
  return h;
}

void fmn_h5_close(fmn_h5_t h) { delete h; }

int fmn_h5_num_datasets(fmn_h5_t h) { return h ? (int)h->ds.size() : fail("null file"); }

int fmn_h5_dataset_info(fmn_h5_t h, int i, char* name, size_t name_len, char* dtype, size_t dtype_len, int* ndims,
                        int64_t* shape, int max_dims) {
  if (!h || i < 0 || i >= (int)h->ds.size()) return fail("dataset index out of range");
  const auto& d = h->ds[i];
  if (name && name_len) {
    std::strncpy(name, d.name.c_str(), name_len - 1);
    name[name_len - 1] = 0;
  }
  if (dtype && dtype_len) {
    std::strncpy(dtype, d.dtype.c_str(), dtype_len - 1);
    dtype[dtype_len - 1] = 0;
  }
  if (ndims) *ndims = (int)d.shape.size();
  for (int k = 0; shape && k < (int)d.shape.size() && k < max_dims; ++k) shape[k] = d.shape[k];
  return 0;
}

int64_t fmn_h5_read_rows(fmn_h5_t h, const char* name, int64_t row0, int64_t nrows, void* dst, size_t dst_bytes) {
  if (!h || !name || !dst) return fail("null argument");
  const flexmi::H5Dataset* d = nullptr;
  for (const auto& x : h->ds)
    if (x.name == name) d = &x;
  if (!d) return fail(std::string("no dataset ") + name);
  if (d->offset < 0) return fail("dataset has no allocated data");
  int64_t row = itemsize(d->dtype);
  for (size_t k = 1; k < d->shape.size(); ++k) row *= d->shape[k];
  const int64_t rows = d->shape.empty() ? 1 : d->shape[0];
  if (row0 < 0 || nrows < 0 || row0 + nrows > rows) return fail("rows out of range");
  const int64_t bytes = nrows * row;
  if ((int64_t)dst_bytes < bytes) return fail("destination too small");
  FILE* f = std::fopen(h->path.c_str(), "rb");
  if (!f) return fail("cannot open " + h->path);
  int64_t got = -1;
  if (std::fseek(f, (long)(d->offset + row0 * row), SEEK_SET) == 0) got = (int64_t)std::fread(dst, 1, (size_t)bytes, f);
  std::fclose(f);
  return got == bytes ? nrows : fail("short read");
}

// ------------------------------------------------------------------------------ loader ring
fmn_loader_t fmn_loader_create(int64_t batch, int64_t num_samples, int depth, int threads, int shuffle, uint64_t seed) {
  return guarded(
      [&]() -> fmn_loader_t {
        auto* l = new fmn_loader_s();
        l->ring.reset(new flexmi::BatchRing(batch, num_samples, depth, threads, shuffle != 0, seed));
        return l;
      },
      (fmn_loader_t) nullptr);
}

int fmn_loader_add_source(fmn_loader_t l, const void* base, int64_t rows, int64_t row_bytes, int64_t col_off,
                          int64_t col_bytes, int64_t row_lo, int64_t row_hi, int64_t dst_pitch) {
  if (!l) return fail("null loader");
  return guarded([&]() -> int { return l->ring->add_source(base, rows, row_bytes, col_off, col_bytes, row_lo, row_hi, dst_pitch); },
                 -1);
}

int fmn_loader_set_slot(fmn_loader_t l, int source, int slot, void* ptr) {
  if (!l) return fail("null loader");
  return guarded([&]() -> int { l->ring->set_slot(source, slot, ptr); return 0; }, -1);
}

int fmn_loader_start(fmn_loader_t l) {
  if (!l) return fail("null loader");
  return guarded([&]() -> int { l->ring->start(); return 0; }, -1);
}

int fmn_loader_acquire(fmn_loader_t l) {
  if (!l) return fail("null loader");
  return guarded([&]() -> int { return l->ring->acquire(); }, -1);
}

int fmn_loader_release(fmn_loader_t l, int slot) {
  if (!l) return fail("null loader");
  return guarded([&]() -> int { l->ring->release(slot); return 0; }, -1);
}

int64_t fmn_loader_batches_per_epoch(fmn_loader_t l) { return l ? l->ring->batches_per_epoch() : fail("null loader"); }

int fmn_loader_batch_ids(fmn_loader_t l, int64_t n, int64_t* ids, int64_t max_ids) {
  if (!l) return fail("null loader");
  return guarded(
      [&]() -> int {
        auto v = l->ring->batch_ids(n);
        for (int64_t i = 0; i < (int64_t)v.size() && i < max_ids; ++i) ids[i] = v[i];
        return (int)v.size();
      },
      -1);
}

void fmn_loader_destroy(fmn_loader_t l) {
  if (!l) return;
  try {
    l->ring->stop();
  } catch (...) {
  }
  delete l;
}

// ------------------------------------------------------------------------------ CPU kernels
int fmn_embedding_bag_forward(const float* W, int64_t rows, int64_t D, const int64_t* idx, int64_t B, int64_t bag,
                              int64_t row_lo, float scale, float* out, int64_t ld_out) {
  if (!W || !idx || !out || D <= 0 || B < 0 || bag <= 0 || ld_out < D) return fail("bad argument");
  flexmi::cpu::embedding_bag_forward<int64_t>(W, rows, D, idx, B, bag, row_lo, scale, out, ld_out);
  return 0;
}

int fmn_embedding_bag_backward(float* target, int64_t rows, int64_t D, const int64_t* idx, int64_t B, int64_t bag,
                               int64_t row_lo, const float* dy, int64_t ld_dy, float alpha) {
  if (!target || !idx || !dy || D <= 0 || B < 0 || bag <= 0 || ld_dy < D) return fail("bad argument");
  flexmi::cpu::embedding_bag_backward<int64_t>(target, rows, D, idx, B, bag, row_lo, dy, ld_dy, alpha, 0);
  return 0;
}

}  // extern "C"

// ---- graph planner --------------------------------------------------------------------------------
struct fmn_plan_s {
  std::vector<flexmi::PlanOp> ops;
  flexmi::GraphPlan plan;
  bool planned = false;
};

extern "C" {

fmn_plan_t fmn_plan_create(void) {
  return guarded([] { return new fmn_plan_s(); }, (fmn_plan_t) nullptr);
}

int fmn_plan_add_op(fmn_plan_t p, int64_t guid, int n_out, const int64_t* outputs) {
  if (!p || n_out < 0 || (n_out > 0 && !outputs)) return fail("fmn_plan_add_op: bad arguments");
  flexmi::PlanOp op;
  op.guid = guid;
  op.outputs.assign(outputs, outputs + n_out);
  p->ops.push_back(std::move(op));
  p->planned = false;
  return (int)p->ops.size() - 1;
}

int fmn_plan_add_input(fmn_plan_t p, int64_t tensor, int64_t producer, int dtype, int64_t need, int flags) {
  if (!p || p->ops.empty()) return fail("fmn_plan_add_input: no op");
  flexmi::PlanInput in;
  in.tensor = tensor;
  in.producer = producer;
  in.dtype = dtype;
  in.need = need;
  in.is_float = flags & 1;
  in.needs_grad = (flags >> 1) & 1;
  in.reshard = (flags >> 2) & 1;
  in.remote = (flags >> 3) & 1;
  p->ops.back().inputs.push_back(in);
  return (int)p->ops.back().inputs.size() - 1;
}

int fmn_plan_run(fmn_plan_t p, int world, int input_grads) {
  if (!p) return fail("fmn_plan_run: null plan");
  return guarded(
      [&] {
        p->plan = flexmi::plan_graph(p->ops, world, input_grads != 0);
        p->planned = true;
        return 0;
      },
      -1);
}

static int64_t copy_ids(const fmn_plan_s* p, const std::vector<int64_t>& v, int64_t* out, int64_t max_n) {
  if (!p || !p->planned) return fail("plan not run");
  for (int64_t i = 0; i < (int64_t)v.size() && i < max_n; ++i) out[i] = v[i];
  return (int64_t)v.size();
}

int64_t fmn_plan_order(fmn_plan_t p, int64_t* guids, int64_t max_n) { return copy_ids(p, p ? p->plan.order : std::vector<int64_t>{}, guids, max_n); }
int64_t fmn_plan_bwd_live(fmn_plan_t p, int64_t* guids, int64_t max_n) {
  return copy_ids(p, p ? p->plan.bwd_live : std::vector<int64_t>{}, guids, max_n);
}
int64_t fmn_plan_grad_needed(fmn_plan_t p, int64_t* tensors, int64_t max_n) {
  return copy_ids(p, p ? p->plan.grad_needed : std::vector<int64_t>{}, tensors, max_n);
}

int64_t fmn_plan_steps(fmn_plan_t p, int backward, int* kind, int64_t* op, int* n_inputs, int* inputs, int64_t max_steps,
                       int64_t max_inputs) {
  if (!p || !p->planned) return fail("plan not run");
  const auto& steps = backward ? p->plan.bwd : p->plan.fwd;
  int64_t k = 0;
  for (int64_t i = 0; i < (int64_t)steps.size() && i < max_steps; ++i) {
    if (kind) kind[i] = steps[i].kind;
    if (op) op[i] = steps[i].op;
    if (n_inputs) n_inputs[i] = (int)steps[i].inputs.size();
    for (int x : steps[i].inputs) {
      if (inputs && k < max_inputs) inputs[k] = x;
      ++k;
    }
  }
  return (int64_t)steps.size();
}

void fmn_plan_destroy(fmn_plan_t p) { delete p; }

}  // extern "C"

// ---- native model -----------------------------------------------------------------------------
struct fmn_model_s {
  std::unique_ptr<flexmi::nm::Model> m;
};

extern "C" {

fmn_model_t fmn_model_create(int global_batch, int device, int rank, int world, const char* rendezvous) {
  return guarded(
      [&] {
        auto* h = new fmn_model_s();
        h->m = std::make_unique<flexmi::nm::Model>(global_batch, device, rank, world, rendezvous ? rendezvous : "");
        return h;
      },
      (fmn_model_t) nullptr);
}

void fmn_model_destroy(fmn_model_t m) { delete m; }

int fmn_model_input(fmn_model_t m, int features) {
  if (!m) return fail("fmn_model_input: null model");
  return guarded([&] { return m->m->input(features); }, -1);
}

int fmn_model_dense(fmn_model_t m, int input_tensor, int out_dim, int activation, int use_bias) {
  if (!m) return fail("fmn_model_dense: null model");
  return guarded([&] { return m->m->dense(input_tensor, out_dim, activation, use_bias != 0); }, -1);
}

int fmn_model_input_image(fmn_model_t m, int channels, int height, int width) {
  if (!m) return fail("fmn_model_input_image: null model");
  return guarded([&] { return m->m->input_image(channels, height, width); }, -1);
}

int fmn_model_conv2d(fmn_model_t m, int input_tensor, int out_channels, int kernel_h, int kernel_w, int stride_h,
                     int stride_w, int pad_h, int pad_w, int activation, int use_bias) {
  if (!m) return fail("fmn_model_conv2d: null model");
  return guarded([&] {
    return m->m->conv2d(input_tensor, out_channels, kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w, activation,
                        use_bias != 0);
  }, -1);
}

int fmn_model_pool2d(fmn_model_t m, int input_tensor, int kernel_h, int kernel_w, int stride_h, int stride_w, int pad_h,
                     int pad_w, int is_max) {
  if (!m) return fail("fmn_model_pool2d: null model");
  return guarded([&] { return m->m->pool2d(input_tensor, kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w, is_max != 0); },
                 -1);
}

int fmn_model_batch_norm(fmn_model_t m, int input_tensor, int relu) {
  if (!m) return fail("fmn_model_batch_norm: null model");
  return guarded([&] { return m->m->batch_norm(input_tensor, relu != 0); }, -1);
}

int fmn_model_sparse_input(fmn_model_t m, int bag) {
  if (!m) return fail("fmn_model_sparse_input: null model");
  return guarded([&] { return m->m->sparse_input(bag); }, -1);
}

int fmn_model_embedding(fmn_model_t m, int sparse_input, int64_t rows, int dim) {
  if (!m) return fail("fmn_model_embedding: null model");
  return guarded([&] { return m->m->embedding(sparse_input, rows, dim); }, -1);
}

int fmn_model_dot_interaction(fmn_model_t m, int bottom, int n, const int* embeddings, int pad_to) {
  if (!m || n < 1 || !embeddings) return fail("fmn_model_dot_interaction: bad arguments");
  return guarded([&] { return m->m->dot_interaction(bottom, std::vector<int>(embeddings, embeddings + n), pad_to); }, -1);
}

int fmn_model_set_table_owner(fmn_model_t m, int table, int rank) {
  if (!m) return fail("fmn_model_set_table_owner: null model");
  return guarded(
      [&] {
        m->m->set_table_owner(table, rank);
        return 0;
      },
      -1);
}

int fmn_model_set_table_columns(fmn_model_t m, int table, int n, const int* ranks) {
  if (!m || n < 1 || !ranks) return fail("fmn_model_set_table_columns: null model / empty holder list");
  return guarded(
      [&] {
        m->m->set_table_columns(table, std::vector<int>(ranks, ranks + n));
        return 0;
      },
      -1);
}

int fmn_model_set_table_rows(fmn_model_t m, int table, int n, const int* ranks) {
  if (!m || n < 1 || !ranks) return fail("fmn_model_set_table_rows: null model / empty holder list");
  return guarded(
      [&] {
        m->m->set_table_rows(table, std::vector<int>(ranks, ranks + n));
        return 0;
      },
      -1);
}

int fmn_model_set_dense_channels(fmn_model_t m, int layer, int n, const int* ranks) {
  if (!m || n < 1 || !ranks) return fail("fmn_model_set_dense_channels: null model / empty holder list");
  return guarded(
      [&] {
        m->m->set_dense_channels(layer, std::vector<int>(ranks, ranks + n));
        return 0;
      },
      -1);
}

int fmn_model_apply_strategy(fmn_model_t m, fmn_strategy_t s, int n_dense, const char* const* dense_names, int n_tables,
                             const char* const* table_names) {
  if (!m || !s) return fail("fmn_model_apply_strategy: null model / strategy");
  return guarded(
      [&] {
        auto find = [&](const char* name) -> const flexmi::OpStrategy* {
          if (!name) return nullptr;
          for (const auto& o : s->ops)
            if (o.name == name) return &o;
          return nullptr;
        };
        auto distinct = [](const std::vector<int>& v) {
          for (size_t i = 0; i < v.size(); ++i)
            for (size_t k = 0; k < i; ++k)
              if (v[k] == v[i]) return false;
          return true;
        };
        int placed = 0;
        for (int i = 0; i < n_dense && i < m->m->num_dense(); ++i) {
          const flexmi::OpStrategy* o = find(dense_names ? dense_names[i] : nullptr);
          if (!o || o->device_ids.empty()) continue;
          const int c = o->dims.empty() ? 1 : o->dims[0];
          std::vector<int> holders;
          if (c > 1) {
            for (int j = 0; j < c && j < (int)o->device_ids.size(); ++j) holders.push_back(o->device_ids[j]);
          } else if (o->num_parts() == 1) {
            holders.push_back(o->device_ids[0]);
          }
          if (holders.empty() || !distinct(holders)) continue;   // data parallel
          try {
            m->m->set_dense_channels(i, holders);
            ++placed;
          } catch (const std::invalid_argument&) {             // uneven channels: data parallel
          }
        }
        for (int t = 0; t < n_tables && t < m->m->num_tables(); ++t) {
          const flexmi::OpStrategy* o = find(table_names ? table_names[t] : nullptr);
          if (!o || o->device_ids.empty()) continue;
          std::vector<int> d = o->dims;
          d.resize(3, 1);
          const int c = d[0], n = d[1], r = d[2];
          const auto& ids = o->device_ids;
          auto dev = [&](int i, int j, int k) { return ids.at(j + c * (i + n * k)); };
          std::vector<int> holders;
          bool rows = false;
          if (c > 1) {
            for (int j = 0; j < c; ++j) holders.push_back(dev(0, j, 0));
          } else if (r > 1) {
            for (int k = 0; k < r; ++k) holders.push_back(dev(0, 0, k));
            rows = true;
          }
          try {
            if (!holders.empty() && distinct(holders)) {
              if (rows) m->m->set_table_rows(t, holders);
              else m->m->set_table_columns(t, holders);
            } else {
              m->m->set_table_owner(t, ids[0]);
            }
            ++placed;
          } catch (const std::invalid_argument&) {
            m->m->set_table_owner(t, ids[0]);
            ++placed;
          }
        }
        return placed;
      },
      -1);
}

int fmn_model_table_columns(fmn_model_t m, int table, int* ranks, int max) {
  if (!m) return fail("fmn_model_table_columns: null model");
  return guarded(
      [&] {
        const auto& h = m->m->table_holders(table);
        for (int i = 0; i < (int)h.size() && i < max; ++i) ranks[i] = h[i];
        return (int)h.size();
      },
      -1);
}

int fmn_model_table_owner(fmn_model_t m, int table) {
  if (!m) return fail("fmn_model_table_owner: null model");
  return guarded([&] { return m->m->table_owner(table); }, -1);
}

int fmn_model_param_local(fmn_model_t m, int i) {
  if (!m) return fail("fmn_model_param_local: null model");
  return guarded([&] { return m->m->param_local(i) ? 1 : 0; }, -1);
}

int fmn_model_train_step_sparse(fmn_model_t m, const float* x, const int64_t* const* sparse, const void* labels,
                                double* loss, int64_t* correct) {
  if (!m || !x || !labels) return fail("fmn_model_train_step_sparse: bad arguments");
  return guarded(
      [&] {
        const flexmi::nm::StepStat s = m->m->train_step(x, sparse, labels);
        if (loss) *loss = s.loss;
        if (correct) *correct = s.correct;
        return 0;
      },
      -1);
}

int fmn_model_set_optimizer(fmn_model_t m, int type, float momentum, int nesterov, float weight_decay, float beta1,
                            float beta2, float epsilon) {
  if (!m) return fail("fmn_model_set_optimizer: null model");
  return guarded(
      [&] {
        flexmi::nm::OptConfig o;
        o.type = type;
        o.momentum = momentum;
        o.nesterov = nesterov != 0;
        o.weight_decay = weight_decay;
        o.beta1 = beta1;
        o.beta2 = beta2;
        o.eps = epsilon;
        m->m->set_optimizer(o);
        return 0;
      },
      -1);
}

int fmn_model_set_zero(fmn_model_t m, int stage) {
  if (!m) return fail("fmn_model_set_zero: null model");
  return guarded(
      [&] {
        m->m->set_zero(stage);
        return 0;
      },
      -1);
}

int fmn_model_compile(fmn_model_t m, int loss_type, float lr, double bucket_mb) {
  if (!m) return fail("fmn_model_compile: null model");
  return guarded(
      [&] {
        m->m->compile(loss_type, lr, bucket_mb);
        return 0;
      },
      -1);
}

int fmn_model_init_weights(fmn_model_t m, uint64_t seed) {
  if (!m) return fail("fmn_model_init_weights: null model");
  return guarded(
      [&] {
        m->m->init_weights(seed);
        return 0;
      },
      -1);
}

int fmn_model_num_params(fmn_model_t m) { return m ? m->m->num_params() : fail("null model"); }

int64_t fmn_model_param_numel(fmn_model_t m, int i) {
  if (!m) return fail("null model");
  return guarded([&] { return m->m->param_numel(i); }, (int64_t)-1);
}

int fmn_model_set_param(fmn_model_t m, int i, const float* host) {
  if (!m || !host) return fail("fmn_model_set_param: bad arguments");
  return guarded(
      [&] {
        m->m->set_param(i, host);
        return 0;
      },
      -1);
}

int fmn_model_get_param(fmn_model_t m, int i, float* host) {
  if (!m || !host) return fail("fmn_model_get_param: bad arguments");
  return guarded(
      [&] {
        m->m->get_param(i, host);
        return 0;
      },
      -1);
}

int fmn_model_train_step(fmn_model_t m, const float* x, const void* labels, double* loss, int64_t* correct) {
  if (!m || !x || !labels) return fail("fmn_model_train_step: bad arguments");
  return guarded(
      [&] {
        const flexmi::nm::StepStat s = m->m->train_step(x, labels);
        if (loss) *loss = s.loss;
        if (correct) *correct = s.correct;
        return 0;
      },
      -1);
}

int64_t fmn_model_describe(fmn_model_t m, char* buf, int64_t len) {
  if (!m) return fail("null model");
  return guarded(
      [&] {
        const std::string d = m->m->describe();
        if (buf && len > 0) {
          const size_t n = std::min<size_t>(d.size(), (size_t)len - 1);
          memcpy(buf, d.data(), n);
          buf[n] = 0;
        }
        return (int64_t)d.size();
      },
      (int64_t)-1);
}

}  // extern "C"
