// flexmi native graph planner: the graph-level half of the per-rank plan compiler.
//
// Given the operator graph (ops in model order, each input tagged with its producer, dtype and
// whether the consumer's needed layout differs from the tensor's home layout), it derives
//   * the communication-first topological order: producers of cross-device reshards and their
//     ancestors first, so asynchronous exchanges overlap the independent ops (DLRM: embeddings
//     first, their all-to-all hides behind the bottom MLP);
//   * the forward schedule: per op, the input reshards it needs (one exchange per dtype, each
//     (tensor, needed layout) resharded once) followed by the op;
//   * backward liveness: ops whose outputs reach the loss, and the tensors that need gradients;
//   * the backward schedule: live ops in reverse order, each followed by the reduction of the
//     gradients of its resharded inputs back to their home layout.
// Every rank derives the same plan from the same graph, so collectives are issued in the same
// order everywhere.  Buffers, kernels and communicators stay with the caller (executor.py).
//
// Reference counterpart: the graph walk of FFModel::compile / the per-op task launches in
// src/runtime/model.cc:374-1180 (Legion derives the dependencies from region requirements
// at run time; here they are resolved once, ahead of time).
#pragma once

#include <cstdint>
#include <vector>

namespace flexmi {

struct PlanInput {
  int64_t tensor = -1;     // tensor guid
  int64_t producer = -1;   // producing op guid, -1 for a model input
  int dtype = 0;           // storage dtype code (reshards are grouped per dtype)
  int64_t need = -1;       // id of the needed layout (dedupes reshards of one (tensor, layout))
  bool is_float = true;
  bool needs_grad = true;  // the op produces a gradient for this input
  bool reshard = false;    // needed layout != home layout
  bool remote = false;     // ... and the reshard moves data between ranks
};

struct PlanOp {
  int64_t guid = -1;
  std::vector<PlanInput> inputs;
  std::vector<int64_t> outputs;
};

struct PlanStep {
  int kind = 0;              // 0 = op, 1 = reshard (fwd) / reduce (bwd)
  int64_t op = -1;
  std::vector<int> inputs;   // input indices of `op` handled by this step
};

struct GraphPlan {
  std::vector<int64_t> order;        // op guids, communication-first topological order
  std::vector<PlanStep> fwd;
  std::vector<int64_t> bwd_live;     // op guids (reverse order)
  std::vector<int64_t> grad_needed;  // tensor guids
  std::vector<PlanStep> bwd;
};

// ops in model order; the loss is attached to the first output of the LAST op.
// Throws std::runtime_error on a cyclic graph.
GraphPlan plan_graph(const std::vector<PlanOp>& ops, int world, bool input_grads);

}  // namespace flexmi
