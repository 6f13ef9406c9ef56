// flexmi native model: graph -> per-rank execution plan -> execution, entirely in C++ (no Python).
//
// Reference: FFModel::compile / init_layers / forward / backward / update
// (src/runtime/model.cc:374-1180) build the per-op regions, the replica gradient regions and
// the task launches; here the PLAN COMPILER lays out one rank's buffers for data parallelism
// over `world` ranks (sample split of every activation, replicated weights in ONE flat 256-B
// aligned parameter / gradient buffer), groups the gradients into all-reduce buckets in backward
// order (a bucket is reduced as soon as its last gradient is final), decides the fused
// epilogues (activation backward of layer i folded into layer i+1's dX GEMM, bias gradients as
// the dW GEMM's row sums, sigmoid + BCE folded into the loss), and emits the step program.  An
// Engine executes it: CPU (reference fp32 loops) or HIP (flexmi's gfx950 kernels + RCCL, in
// native_hip.cc).  plan_weights() is the same bucket planner the Python executor uses.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace flexmi {

// ---- weight / bucket plan (shared with the Python executor through flexmi._native) ----------
struct WeightPlan {
  std::vector<int64_t> offset;                 // element offset of each entry (64-float aligned)
  int64_t numel = 0;                           // flat buffer size
  std::vector<std::vector<int64_t>> buckets;   // [begin, end, entry ids...] per bucket
};
// entries in BACKWARD order (their gradients become final in this order); a bucket closes when
// adding the next entry would exceed cap_elems and the bucket is not empty
WeightPlan plan_weights(const std::vector<int64_t>& numels, int64_t cap_elems);

namespace nm {

enum Act { ACT_NONE = 10, ACT_RELU = 11, ACT_SIGMOID = 12, ACT_TANH = 13 };
enum Loss { LOSS_SCCE = 51, LOSS_MSE_AVG = 52, LOSS_BCE = 54 };

struct Dense {
  int x = -1, y = -1;          // tensor ids
  int K = 0, N = 0;            // in / out features
  int act = ACT_NONE;
  bool bias = true;
  int w = -1, b = -1;          // parameter entry ids
  // plan
  bool grad_is_dpre = false;   // the consumer's dX epilogue already applied this layer's act'
  bool fuse_below = false;     // this layer's dX epilogue applies the producer layer's act'
  bool skip_act_grad = false;  // sigmoid folded into BCE
  bool need_dx = true;
};

struct StepStat {
  double loss = 0.0;
  int64_t samples = 0;
  int64_t correct = 0;
};

class Engine;

class Model {
 public:
  Model(int global_batch, int device, int rank, int world, const std::string& rendezvous);
  ~Model();
  int input(int features);
  int dense(int x, int out_dim, int act, bool bias);
  void compile(int loss_type, float lr, double bucket_mb);
  void init_weights(uint64_t seed);            // Glorot-uniform weights, zero biases (host RNG)
  int num_params() const { return (int)pnumel_.size(); }
  int64_t param_numel(int i) const { return pnumel_.at(i); }
  void set_param(int i, const float* host);
  void get_param(int i, float* host) const;
  // x: the GLOBAL batch [B][features]; labels: [B] int32 (SCCE) or [B][out] float
  StepStat train_step(const float* x, const void* labels);
  std::string describe() const;
  const WeightPlan& weight_plan() const { return wplan_; }

 private:
  int B_, Bl_, device_, rank_, world_;
  std::string rendezvous_;
  std::vector<int> cols_;                     // tensor id -> features
  int input_ = -1;
  std::vector<Dense> ops_;
  std::vector<int64_t> pnumel_;               // parameter entries (model order: w, b per layer)
  std::vector<int> porder_;                   // backward order of entries
  WeightPlan wplan_;
  std::vector<int64_t> pofs_;                 // entry -> flat offset
  int loss_ = LOSS_MSE_AVG;
  float lr_ = 0.01f;
  bool compiled_ = false;
  std::unique_ptr<Engine> eng_;
  // device buffers
  float* params_ = nullptr;
  float* grads_ = nullptr;
  std::vector<float*> act_;                   // tensor id -> [Bl][cols]
  std::vector<float*> grad_;                  // tensor id -> [Bl][cols]
  float* probs_ = nullptr;                    // SCCE: softmax of the logits
  void* labels_ = nullptr;
  float* stats_ = nullptr;                    // [loss, correct] accumulators
};

// ---- execution engines ----------------------------------------------------------------------
class Engine {
 public:
  virtual ~Engine() = default;
  virtual void* alloc(size_t bytes) = 0;      // zero-initialised
  virtual void release(void* p) = 0;
  virtual void h2d(void* dst, const void* src, size_t bytes) = 0;
  virtual void d2h(void* dst, const void* src, size_t bytes) = 0;
  virtual void sync() = 0;
  // y[M][N] = act(x[M][K] W[N][K]^T + b)
  virtual void dense_fwd(const float* x, const float* W, const float* b, float* y, int M, int K, int N, int act) = 0;
  // one layer's backward: dpre = act'(y) dy (unless grad_is_dpre / act none); dW += dpre^T x;
  // db += colsum(dpre); dx = dpre W, then dx *= act_below'(y_below) when y_below != nullptr
  virtual void dense_bwd(const float* x, const float* W, const float* y, const float* dy, float* dx, float* dW, float* db,
                         int M, int K, int N, int act, bool grad_is_dpre, const float* y_below, int act_below) = 0;
  virtual void softmax(const float* x, float* y, int M, int C) = 0;
  // grad = (p - target) * scale; stats[0] += loss sum, stats[1] += correct predictions
  virtual void loss(int type, const float* p, const void* labels, float* grad, int M, int C, float scale,
                    float* stats) = 0;
  virtual void sgd(float* w, float* g, int64_t n, float lr) = 0;   // w -= lr g; g = 0
  // gradient bucket reduction (sum over ranks): start after the bucket's last gradient, wait
  // before the update
  virtual void allreduce_start(float* buf, int64_t n) = 0;
  virtual void allreduce_wait() = 0;
};

std::unique_ptr<Engine> make_cpu_engine();
// HIP engine (native_hip.cc): flexmi's gfx950 kernels, RCCL over the ranks of `rendezvous`
std::unique_ptr<Engine> make_hip_engine(int rank, int world, const std::string& rendezvous);

}  // namespace nm
}  // namespace flexmi
