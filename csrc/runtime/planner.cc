// flexmi native graph planner (see planner.h).
#include "planner.h"

#include <algorithm>
#include <map>
#include <queue>
#include <set>
#include <stdexcept>
#include <tuple>
#include <unordered_map>
#include <unordered_set>

namespace flexmi {

namespace {

// Kahn's algorithm; ready ops pop by (not hot, model position): producers of cross-device
// reshards and everything they depend on run as early as the dependencies allow.
std::vector<int64_t> comm_first_order(const std::vector<PlanOp>& ops, int world) {
  std::vector<int64_t> order;
  order.reserve(ops.size());
  if (world == 1) {
    for (auto& op : ops) order.push_back(op.guid);
    return order;
  }
  std::unordered_map<int64_t, size_t> pos;
  for (size_t k = 0; k < ops.size(); ++k) pos[ops[k].guid] = k;
  std::vector<std::vector<size_t>> deps(ops.size()), users(ops.size());
  for (size_t k = 0; k < ops.size(); ++k) {
    std::set<size_t> d;
    for (auto& in : ops[k].inputs) {
      auto it = pos.find(in.producer);
      if (in.producer >= 0 && it != pos.end()) d.insert(it->second);
    }
    deps[k].assign(d.begin(), d.end());
    for (size_t x : deps[k]) users[x].push_back(k);
  }
  std::vector<char> hot(ops.size(), 0);
  std::vector<size_t> stack;
  for (size_t k = 0; k < ops.size(); ++k)
    for (auto& in : ops[k].inputs) {
      auto it = pos.find(in.producer);
      if (in.producer >= 0 && it != pos.end() && in.reshard && in.remote && !hot[it->second]) {
        hot[it->second] = 1;
        stack.push_back(it->second);
      }
    }
  while (!stack.empty()) {
    size_t g = stack.back();
    stack.pop_back();
    for (size_t d : deps[g])
      if (!hot[d]) {
        hot[d] = 1;
        stack.push_back(d);
      }
  }
  std::vector<size_t> indeg(ops.size());
  using Key = std::tuple<int, size_t>;
  std::priority_queue<Key, std::vector<Key>, std::greater<Key>> ready;
  for (size_t k = 0; k < ops.size(); ++k) {
    indeg[k] = deps[k].size();
    if (indeg[k] == 0) ready.emplace(hot[k] ? 0 : 1, k);
  }
  while (!ready.empty()) {
    const size_t g = std::get<1>(ready.top());
    ready.pop();
    order.push_back(ops[g].guid);
    for (size_t u : users[g])
      if (--indeg[u] == 0) ready.emplace(hot[u] ? 0 : 1, u);
  }
  if (order.size() != ops.size()) throw std::runtime_error("plan_graph: graph has a cycle");
  return order;
}

}  // namespace

GraphPlan plan_graph(const std::vector<PlanOp>& ops, int world, bool input_grads) {
  GraphPlan plan;
  if (ops.empty()) return plan;
  std::unordered_map<int64_t, const PlanOp*> by_guid;
  for (auto& op : ops) by_guid[op.guid] = &op;
  plan.order = comm_first_order(ops, world);

  // forward: input reshards (grouped per dtype, in first-seen order) then the op
  std::set<std::pair<int64_t, int64_t>> made;
  for (int64_t g : plan.order) {
    const PlanOp& op = *by_guid.at(g);
    std::vector<std::pair<int, std::vector<int>>> groups;   // dtype -> input indices
    for (size_t i = 0; i < op.inputs.size(); ++i) {
      const PlanInput& in = op.inputs[i];
      if (!in.reshard || !made.insert({in.tensor, in.need}).second) continue;
      auto it = std::find_if(groups.begin(), groups.end(), [&](auto& p) { return p.first == in.dtype; });
      if (it == groups.end()) groups.push_back({in.dtype, {(int)i}});
      else it->second.push_back((int)i);
    }
    for (auto& grp : groups) plan.fwd.push_back(PlanStep{1, g, grp.second});
    plan.fwd.push_back(PlanStep{0, g, {}});
  }

  // backward liveness: the loss reads the first output of the last op in MODEL order
  std::unordered_set<int64_t> grad_needed;
  const PlanOp& final_op = ops.back();
  if (!final_op.outputs.empty()) grad_needed.insert(final_op.outputs[0]);
  std::unordered_set<int64_t> live;
  for (auto it = plan.order.rbegin(); it != plan.order.rend(); ++it) {
    const PlanOp& op = *by_guid.at(*it);
    bool reaches = false;
    for (int64_t o : op.outputs) reaches = reaches || grad_needed.count(o);
    if (!reaches) continue;
    live.insert(op.guid);
    plan.bwd_live.push_back(op.guid);
    for (auto& in : op.inputs) {
      const bool src_ok = in.producer >= 0 || input_grads;
      if (src_ok && in.needs_grad && in.is_float) grad_needed.insert(in.tensor);
    }
  }
  plan.grad_needed.assign(grad_needed.begin(), grad_needed.end());
  std::sort(plan.grad_needed.begin(), plan.grad_needed.end());

  // backward: live ops in reverse order, each followed by its resharded-input gradient reduce
  for (auto it = plan.order.rbegin(); it != plan.order.rend(); ++it) {
    if (!live.count(*it)) continue;
    const PlanOp& op = *by_guid.at(*it);
    plan.bwd.push_back(PlanStep{0, op.guid, {}});
    std::vector<int> red;
    for (size_t i = 0; i < op.inputs.size(); ++i) {
      const PlanInput& in = op.inputs[i];
      if (grad_needed.count(in.tensor) && in.needs_grad && in.reshard) red.push_back((int)i);
    }
    if (!red.empty()) plan.bwd.push_back(PlanStep{1, op.guid, red});
  }
  return plan;
}

}  // namespace flexmi
