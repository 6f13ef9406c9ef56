// MI355X execution simulator + MCMC (Metropolis) SOAP strategy search.
//
// Reference behaviour (what is modelled, not how): FlexFlow's Simulator builds a task graph
// of per-shard forward/backward tasks, producer->consumer intersection copies and parameter
// synchronisation, then list-schedules it over per-device timelines
// (src/runtime/simulator.cc:275-448, include/simulator.h:29-130); FFModel::optimize runs a
// Metropolis walk that re-draws one op's ParallelConfig per step (src/runtime/model.cc:1082-1144).
//
// flexmi design: the graph is compiled ONCE into candidate tables (per op: a list of
// candidate configs with per-part device, per-part fwd/bwd cost from the MI355X cost model,
// output/needed-input shard boxes with holders, weight-sync groups and per-device memory);
// a proposal only changes one op's candidate index.  Producer/consumer transfer lists are
// memoised per (edge, producer cand, consumer cand), so a simulation is a pure list-schedule
// over O(tasks) with no box math.  The machine model is MI355X: one compute queue + one
// collective channel per GPU, a directed xGMI link per GPU pair (full mesh inside a node),
// NIC links between nodes, RCCL ring/all-reduce cost = latency + 2(g-1)/g * bytes / busbw.
#pragma once
#include <cstdint>
#include <map>
#include <random>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

namespace flexmi {
namespace sim {

constexpr int kMaxDims = 6;

struct Box {
  int nd = 0;
  int64_t lo[kMaxDims] = {0};
  int64_t hi[kMaxDims] = {0};
  int64_t volume() const {
    int64_t v = 1;
    for (int i = 0; i < nd; ++i) v *= (hi[i] - lo[i]);
    return v;
  }
};

bool intersect(const Box& a, const Box& b, Box* out);

struct Part {
  Box box;
  std::vector<int> holders;
};
using LayoutD = std::vector<Part>;

struct WeightSync {
  double bytes = 0;          // bytes of the gradient to reduce
  std::vector<int> group;    // devices holding replicas (size > 1 => all-reduce)
};

struct Candidate {
  std::vector<int> part_dev;             // device of compute part p
  std::vector<double> fwd_us, bwd_us;    // per part
  std::vector<LayoutD> out;              // per output: home layout
  std::vector<LayoutD> in;               // per input: needed layout
  std::vector<WeightSync> wsync;         // replicated weight parts
  std::vector<std::pair<int, double>> mem;     // (device, bytes)
  std::vector<std::pair<int, double>> upd_us;  // (device, optimizer update time)
  std::string label;                     // for traces / debugging
  // one-holder sample split over every device (dim 0 only): may run as micro-batch chunks
  bool sample_only = false;
};

struct TensorD {
  int elem_bytes = 4;
  int producer = -1;      // op index, -1 = graph input (loaded in place, no transfer)
  int producer_out = 0;
  bool needs_grad = true;
};

struct OpD {
  std::string name;
  std::vector<int> in_t, out_t;
  std::vector<Candidate> cands;
  bool rowwise = false;   // every output row depends on the same input rows only (Linear, interaction, concat)
  int edge0 = 0;          // index of the edge of input 0
};

struct Machine {
  int ndev = 1;
  int gpus_per_node = 8;
  double link_GBps = 64.0;         // effective per-direction xGMI bandwidth per GPU pair
  double link_lat_us = 6.0;        // per point-to-point transfer (RCCL send/recv / a2a chunk)
  double nic_GBps = 50.0;          // inter-node per GPU pair (RCCL net)
  double nic_lat_us = 12.0;
  double ar_busbw_GBps = 300.0;    // RCCL all-reduce bus bandwidth inside one node (8 GPUs)
  double ar_lat_us = 15.0;
  double hbm_bytes = 288e9 * 0.92;
  double bucket_bytes = 32.0 * (1 << 20);
  bool overlap = true;             // gradient sync overlapped with backward (else BSP barrier)
  // micro-batch pipelining of the last exchange into a sample-split row-wise tail (executor:
  // FLEXMI_XCHG_CHUNKS): the tail's tasks and its inbound / gradient transfers split in this
  // many chunks, each chunk op paying chunk_us of extra kernel boundaries
  int xchg_chunks = 1;
  double chunk_us = 1.6;
};

struct TraceEvent {
  std::string name;
  std::string kind;   // fwd | bwd | xfer | allreduce | update
  int resource;       // compute d, channel ndev+d, link 2*ndev + s*ndev + t
  double start, end;
};

struct SearchResult {
  std::vector<int> best;
  double best_us = 0, init_us = 0;
  std::vector<std::tuple<long, double, double>> history;  // (iter, current, best)
  long accepted = 0;
};

class Simulator {
 public:
  explicit Simulator(const Machine& m) : m_(m) {}
  int add_tensor(const TensorD& t) {
    tensors_.push_back(t);
    return (int)tensors_.size() - 1;
  }
  int add_op(OpD op);
  size_t num_ops() const { return ops_.size(); }
  const OpD& op(int i) const { return ops_[i]; }

  // makespan (us) of one training iteration; +inf if a device runs out of memory
  double simulate(const std::vector<int>& assign, std::vector<TraceEvent>* trace = nullptr);
  std::vector<double> memory(const std::vector<int>& assign) const;
  SearchResult search(const std::vector<int>& init, long budget, double alpha, uint64_t seed,
                      bool verbose, const std::vector<char>& frozen, int greedy_passes = 2);

 private:
  struct Xfer {
    int src_dev, dst_dev;   // data movement src -> dst (forward direction)
    int prod_part;          // producer compute part (-1: graph input)
    int cons_part;          // consumer compute part
    double bytes;
  };
  struct Edge {             // consumer op input
    int op, input, tensor;
  };
  const std::vector<Xfer>& transfers(int edge, int pc, int cc);
  std::vector<int> chunks(const std::vector<int>& assign);   // micro-batch chunks per op
  double xfer_us(int s, int d, double bytes) const;
  double allreduce_us(const std::vector<int>& group, double bytes) const;
  int link_res(int s, int d) const { return 2 * m_.ndev + s * m_.ndev + d; }

  Machine m_;
  std::vector<TensorD> tensors_;
  std::vector<OpD> ops_;
  std::vector<Edge> edges_;
  std::vector<std::vector<int>> consumers_;   // tensor -> edges
  std::unordered_map<uint64_t, std::vector<Xfer>> xcache_;
};

}  // namespace sim
}  // namespace flexmi
