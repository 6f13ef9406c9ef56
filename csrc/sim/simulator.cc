// MI355X execution simulator + Metropolis SOAP search.  See simulator.h for the model.
#include "simulator.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <limits>
#include <queue>

namespace flexmi {
namespace sim {

bool intersect(const Box& a, const Box& b, Box* out) {
  if (a.nd != b.nd) return false;
  out->nd = a.nd;
  for (int i = 0; i < a.nd; ++i) {
    int64_t lo = std::max(a.lo[i], b.lo[i]);
    int64_t hi = std::min(a.hi[i], b.hi[i]);
    if (lo >= hi) return false;
    out->lo[i] = lo;
    out->hi[i] = hi;
  }
  return true;
}

int Simulator::add_op(OpD op) {
  int idx = (int)ops_.size();
  op.edge0 = (int)edges_.size();
  for (int j = 0; j < (int)op.in_t.size(); ++j) {
    int t = op.in_t[j];
    if ((int)consumers_.size() <= t) consumers_.resize(t + 1);
    consumers_[t].push_back((int)edges_.size());
    edges_.push_back({idx, j, t});
  }
  ops_.push_back(std::move(op));
  return idx;
}

static int part_on(const Candidate& c, int dev) {
  for (int p = 0; p < (int)c.part_dev.size(); ++p)
    if (c.part_dev[p] == dev) return p;
  return -1;
}

const std::vector<Simulator::Xfer>& Simulator::transfers(int edge, int pc, int cc) {
  uint64_t key = ((uint64_t)edge << 40) | ((uint64_t)pc << 20) | (uint64_t)cc;
  auto it = xcache_.find(key);
  if (it != xcache_.end()) return it->second;
  std::vector<Xfer> out;
  const Edge& e = edges_[edge];
  const TensorD& t = tensors_[e.tensor];
  if (t.producer >= 0) {
    const Candidate& cons = ops_[e.op].cands[cc];
    const Candidate& prod = ops_[t.producer].cands[pc];
    const LayoutD& need = cons.in[e.input];
    const LayoutD& home = prod.out[t.producer_out];
    std::map<std::tuple<int, int, int, int>, double> merged;
    for (int q = 0; q < (int)need.size(); ++q) {
      for (int sp = 0; sp < (int)home.size(); ++sp) {
        Box inter;
        if (!intersect(need[q].box, home[sp].box, &inter)) continue;
        const auto& sh = home[sp].holders;
        for (int d : need[q].holders) {
          int src = std::find(sh.begin(), sh.end(), d) != sh.end() ? d : sh[(q + sp) % sh.size()];
          int pp = part_on(prod, src);
          int cp = part_on(cons, d);
          if (cp < 0) continue;
          double bytes = src == d ? 0.0 : (double)inter.volume() * t.elem_bytes;
          merged[{pp, cp, src, d}] += bytes;
        }
      }
    }
    for (auto& kv : merged) {
      Xfer x;
      std::tie(x.prod_part, x.cons_part, x.src_dev, x.dst_dev) = kv.first;
      x.bytes = kv.second;
      out.push_back(x);
    }
  }
  return xcache_.emplace(key, std::move(out)).first->second;
}

double Simulator::xfer_us(int s, int d, double bytes) const {
  bool same_node = (s / m_.gpus_per_node) == (d / m_.gpus_per_node);
  if (same_node) return m_.link_lat_us + bytes / (m_.link_GBps * 1e3);
  return m_.nic_lat_us + bytes / (m_.nic_GBps * 1e3);
}

double Simulator::allreduce_us(const std::vector<int>& group, double bytes) const {
  int g = (int)group.size();
  if (g <= 1) return 0.0;
  int node0 = group[0] / m_.gpus_per_node;
  bool one_node = true;
  for (int d : group) one_node &= (d / m_.gpus_per_node) == node0;
  double busbw = one_node ? std::min(m_.ar_busbw_GBps, m_.link_GBps * (g - 1)) : m_.nic_GBps;
  double lat = one_node ? m_.ar_lat_us : m_.nic_lat_us + m_.ar_lat_us;
  return lat + 2.0 * (g - 1) / g * bytes / (busbw * 1e3);
}

std::vector<double> Simulator::memory(const std::vector<int>& assign) const {
  std::vector<double> mem(m_.ndev, 0.0);
  for (size_t i = 0; i < ops_.size(); ++i)
    for (auto& dm : ops_[i].cands[assign[i]].mem)
      if (dm.first >= 0 && dm.first < m_.ndev) mem[dm.first] += dm.second;
  return mem;
}

std::vector<int> Simulator::chunks(const std::vector<int>& assign) {
  const int nops = (int)ops_.size();
  std::vector<int> nch(nops, 1);
  const int K = m_.xchg_chunks;
  if (K <= 1 || m_.ndev <= 1) return nch;
  // the tail: the longest suffix of row-wise ops on sample-split candidates
  int s = nops;
  while (s > 0 && ops_[s - 1].rowwise && ops_[s - 1].cands[assign[s - 1]].sample_only) --s;
  // it is pipelined from the last of its ops fed across devices by an op before the tail (the
  // executor chunks the LAST cross-device exchange of the forward and everything after it)
  int r = -1;
  for (int i = s; i < nops; ++i)
    for (int j = 0; j < (int)ops_[i].in_t.size(); ++j) {
      const TensorD& t = tensors_[ops_[i].in_t[j]];
      if (t.producer < 0 || t.producer >= s) continue;
      for (const Xfer& x : transfers(ops_[i].edge0 + j, assign[t.producer], assign[i]))
        if (x.src_dev != x.dst_dev && x.bytes > 0) r = i;
    }
  if (r < 0) return nch;
  for (int i = r; i < nops; ++i) nch[i] = K;
  return nch;
}

namespace {
struct Task {
  double dur = 0, ready = 0;
  int res = -1;       // resource index, -1 none, -2 collective (uses group)
  int group = -1;
  int npred = 0;
  int kind = 0;       // 0 fwd 1 bwd 2 xfer 3 allreduce 4 update 5 barrier
  int op = -1, part = -1;
};
const char* kKind[] = {"fwd", "bwd", "xfer", "allreduce", "update", "barrier"};
}  // namespace

double Simulator::simulate(const std::vector<int>& assign, std::vector<TraceEvent>* trace) {
  const int nd = m_.ndev;
  {
    auto mem = memory(assign);
    for (double b : mem)
      if (b > m_.hbm_bytes) return std::numeric_limits<double>::infinity();
  }
  std::vector<Task> tasks;
  std::vector<std::vector<int>> succ;
  std::vector<std::vector<int>> groups;
  tasks.reserve(ops_.size() * 8);
  auto new_task = [&](int kind, double dur, int res, int op, int part) {
    Task t;
    t.kind = kind;
    t.dur = dur;
    t.res = res;
    t.op = op;
    t.part = part;
    tasks.push_back(t);
    succ.emplace_back();
    return (int)tasks.size() - 1;
  };
  auto dep = [&](int a, int b) {
    succ[a].push_back(b);
    tasks[b].npred++;
  };
  const int nops = (int)ops_.size();
  const std::vector<int> nch = chunks(assign);
  // fwd[i][p][k] / bwd[i][p][k]: task of part p, micro-batch chunk k (one chunk outside the tail)
  std::vector<std::vector<std::vector<int>>> fwd(nops), bwd(nops);
  for (int i = 0; i < nops; ++i) {
    const Candidate& c = ops_[i].cands[assign[i]];
    const int np = (int)c.part_dev.size(), K = nch[i];
    const double ov = K > 1 ? m_.chunk_us : 0.0;
    fwd[i].assign(np, std::vector<int>(K));
    bwd[i].assign(np, std::vector<int>(K));
    for (int p = 0; p < np; ++p)
      for (int k = 0; k < K; ++k) {
        fwd[i][p][k] = new_task(0, c.fwd_us[p] / K + ov, c.part_dev[p], i, p);
        bwd[i][p][k] = new_task(1, c.bwd_us[p] / K + 2.0 * ov, c.part_dev[p], i, p);
        dep(fwd[i][p][k], bwd[i][p][k]);
      }
    if (K > 1 && i == nops - 1)   // the loss runs on the whole batch: every chunk's forward first
      for (int p = 0; p < np; ++p)
        for (int k = 0; k < K; ++k)
          for (int kk = 0; kk < K; ++kk)
            if (kk != k) dep(fwd[i][p][kk], bwd[i][p][k]);
  }
  // producer -> consumer data movement (forward) and gradient return (backward).  All inputs of
  // one consumer move in ONE fused exchange (the executor's FusedExchange: one all-to-all per
  // reshard step), so the transfers of a consumer part are merged per directed link -- one
  // latency per link, after the last producer.  Inside the tail chunk k feeds chunk k; into the
  // tail the exchange is split per consumer chunk.
  struct Merged {
    double bytes = 0;
    std::vector<int> pf, pb;
  };
  for (int i = 0; i < nops; ++i) {
    const int kc = nch[i];
    std::map<std::tuple<int, int, int, int>, Merged> links;   // (cons part, chunk, src, dst)
    for (int j = 0; j < (int)ops_[i].in_t.size(); ++j) {
      const int e = ops_[i].edge0 + j;
      const TensorD& t = tensors_[edges_[e].tensor];
      if (t.producer < 0) continue;
      const int kp = nch[t.producer];
      for (const Xfer& x : transfers(e, assign[t.producer], assign[i])) {
        const bool local = x.src_dev == x.dst_dev || x.bytes <= 0;
        for (int k = 0; k < kc; ++k) {
          // producer tasks chunk k depends on: the aligned chunk, or all of them
          std::vector<int> pf, pb;
          if (x.prod_part >= 0) {
            const auto& F = fwd[t.producer][x.prod_part];
            const auto& B = bwd[t.producer][x.prod_part];
            if (kp == kc) {
              pf.push_back(F[k]);
              pb.push_back(B[k]);
            } else if (kp == 1) {
              pf.push_back(F[0]);
              pb.push_back(B[0]);
            } else {
              pf = F;
              pb = B;
            }
          }
          if (local) {
            for (int f : pf) dep(f, fwd[i][x.cons_part][k]);
            if (t.needs_grad)
              for (int q : pb) dep(bwd[i][x.cons_part][k], q);
            continue;
          }
          Merged& mg = links[{x.cons_part, k, x.src_dev, x.dst_dev}];
          mg.bytes += kp == kc || kp == 1 ? x.bytes / kc : x.bytes;
          mg.pf.insert(mg.pf.end(), pf.begin(), pf.end());
          if (t.needs_grad) mg.pb.insert(mg.pb.end(), pb.begin(), pb.end());
        }
      }
    }
    for (auto& kv : links) {
      const auto [cp, k, sd, dd] = kv.first;
      Merged& mg = kv.second;
      int cf = new_task(2, xfer_us(sd, dd, mg.bytes), link_res(sd, dd), i, cp);
      std::sort(mg.pf.begin(), mg.pf.end());
      mg.pf.erase(std::unique(mg.pf.begin(), mg.pf.end()), mg.pf.end());
      for (int f : mg.pf) dep(f, cf);
      dep(cf, fwd[i][cp][k]);
      if (!mg.pb.empty()) {
        int cb = new_task(2, xfer_us(dd, sd, mg.bytes), link_res(dd, sd), i, cp);
        dep(bwd[i][cp][k], cb);
        std::sort(mg.pb.begin(), mg.pb.end());
        mg.pb.erase(std::unique(mg.pb.begin(), mg.pb.end()), mg.pb.end());
        for (int q : mg.pb) dep(cb, q);
      }
    }
  }

  // parameter synchronisation + optimizer update
  std::vector<int> upd(nd, -1);
  std::vector<double> upd_us(nd, 0.0);
  for (int i = 0; i < nops; ++i)
    for (auto& du : ops_[i].cands[assign[i]].upd_us)
      if (du.first >= 0 && du.first < nd) upd_us[du.first] += du.second;
  for (int d = 0; d < nd; ++d) upd[d] = new_task(4, upd_us[d], d, -1, d);
  for (int i = 0; i < nops; ++i) {
    const Candidate& c = ops_[i].cands[assign[i]];
    for (int p = 0; p < (int)c.part_dev.size(); ++p)
      for (int b : bwd[i][p]) dep(b, upd[c.part_dev[p]]);
  }
  int barrier = -1;
  if (!m_.overlap) {
    barrier = new_task(5, 0.0, -1, -1, -1);
    for (int i = 0; i < nops; ++i)
      for (auto& bp : bwd[i])
        for (int b : bp) dep(b, barrier);
  }
  struct Bucket {
    double bytes = 0;
    std::vector<int> preds;
    int last_op = -1;
  };
  std::map<std::vector<int>, Bucket> open;
  auto flush = [&](const std::vector<int>& grp, Bucket& b) {
    if (b.bytes <= 0) return;
    groups.push_back(grp);
    int ct = new_task(3, allreduce_us(grp, b.bytes), -2, b.last_op, -1);
    tasks[ct].group = (int)groups.size() - 1;
    if (barrier >= 0) dep(barrier, ct);
    std::sort(b.preds.begin(), b.preds.end());
    b.preds.erase(std::unique(b.preds.begin(), b.preds.end()), b.preds.end());
    for (int p : b.preds) dep(p, ct);
    for (int d : grp) dep(ct, upd[d]);
    b = Bucket();
  };
  for (int i = nops - 1; i >= 0; --i) {   // backward order fills buckets like the executor
    const Candidate& c = ops_[i].cands[assign[i]];
    for (const WeightSync& ws : c.wsync) {
      if (ws.group.size() <= 1) continue;
      std::vector<int> grp = ws.group;
      std::sort(grp.begin(), grp.end());
      Bucket& b = open[grp];
      b.bytes += ws.bytes;
      b.last_op = i;
      for (int p = 0; p < (int)c.part_dev.size(); ++p)
        if (std::binary_search(grp.begin(), grp.end(), c.part_dev[p]))
          b.preds.insert(b.preds.end(), bwd[i][p].begin(), bwd[i][p].end());
      if (b.bytes >= m_.bucket_bytes) flush(grp, b);
    }
  }
  for (auto& kv : open) flush(kv.first, kv.second);

  // list scheduling over resources: compute d, collective channel nd+d, link 2nd + s*nd + t
  std::vector<double> free_at(2 * nd + nd * nd, 0.0);
  using QE = std::pair<double, int>;
  std::priority_queue<QE, std::vector<QE>, std::greater<QE>> q;
  for (int i = 0; i < (int)tasks.size(); ++i)
    if (tasks[i].npred == 0) q.push({0.0, i});
  double makespan = 0;
  size_t done = 0;
  while (!q.empty()) {
    auto [rdy, id] = q.top();
    q.pop();
    Task& t = tasks[id];
    double start = rdy, end;
    if (t.res >= 0) {
      start = std::max(rdy, free_at[t.res]);
      end = start + t.dur;
      free_at[t.res] = end;
    } else if (t.res == -2) {
      for (int d : groups[t.group]) start = std::max(start, free_at[nd + d]);
      end = start + t.dur;
      for (int d : groups[t.group]) free_at[nd + d] = end;
    } else {
      end = start + t.dur;
    }
    ++done;
    makespan = std::max(makespan, end);
    if (trace && t.kind != 5) {
      std::string nm = t.op >= 0 ? ops_[t.op].name : std::string("optimizer");
      int res = t.res >= 0 ? t.res : (t.res == -2 ? nd + groups[t.group][0] : -1);
      trace->push_back({nm + (t.part >= 0 ? "[" + std::to_string(t.part) + "]" : ""), kKind[t.kind], res, start, end});
    }
    for (int s : succ[id]) {
      Task& ts = tasks[s];
      ts.ready = std::max(ts.ready, end);
      if (--ts.npred == 0) q.push({ts.ready, s});
    }
  }
  if (done != tasks.size()) return std::numeric_limits<double>::infinity();  // cycle: invalid graph
  return makespan;
}

SearchResult Simulator::search(const std::vector<int>& init, long budget, double alpha, uint64_t seed,
                               bool verbose, const std::vector<char>& frozen, int greedy_passes) {
  SearchResult r;
  std::mt19937_64 rng(seed);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  std::vector<int> movable;
  for (int i = 0; i < (int)ops_.size(); ++i)
    if (ops_[i].cands.size() > 1 && !(i < (int)frozen.size() && frozen[i])) movable.push_back(i);
  std::vector<int> cur = init;
  double cur_t = simulate(cur);
  r.init_us = cur_t;
  // greedy coordinate descent (each op in turn takes its best candidate given the others):
  // lands next to hand-written strategies such as table-wise DLRM placement, so the walk
  // starts from a good basin instead of from data parallelism
  for (int pass = 0; pass < greedy_passes; ++pass) {
    bool improved = false;
    for (int op : movable) {
      int keep = cur[op];
      for (int c = 0; c < (int)ops_[op].cands.size(); ++c) {
        if (c == keep) continue;
        cur[op] = c;
        double t = simulate(cur);
        if (t < cur_t) {
          cur_t = t;
          keep = c;
          improved = true;
        }
      }
      cur[op] = keep;
    }
    if (!improved) break;
  }
  r.best = cur;
  r.best_us = cur_t;
  int last = -1;
  for (long it = 0; it < budget && !movable.empty(); ++it) {
    int op;
    do {
      op = movable[rng() % movable.size()];
    } while (movable.size() > 1 && op == last);   // reference: a different op than last time
    last = op;
    int nc = (int)ops_[op].cands.size();
    int c = (int)(rng() % (nc - 1));
    if (c >= cur[op]) ++c;
    int prev = cur[op];
    cur[op] = c;
    double t = simulate(cur);
    // Metropolis on the RELATIVE slowdown: alpha=1 accepts a 1 % slower strategy with p=1/e
    // (the reference used absolute ms, which for sub-millisecond iterations is a random walk)
    bool accept = t < cur_t || (std::isfinite(t) && U(rng) < std::exp(-alpha * 100.0 * (t - cur_t) / cur_t));
    if (accept) {
      cur_t = t;
      ++r.accepted;
      if (t < r.best_us) {
        r.best_us = t;
        r.best = cur;
      }
    } else {
      cur[op] = prev;
    }
    if (it % 100 == 0) {
      r.history.emplace_back(it, cur_t, r.best_us);
      if (verbose)
        std::fprintf(stderr, "[search] iter(%ld) cur(%.3f ms) best(%.3f ms)\n", it, cur_t * 1e-3, r.best_us * 1e-3);
    }
  }
  return r;
}

}  // namespace sim
}  // namespace flexmi
