// flexmi native model: graph -> per-rank execution plan -> execution, entirely in C++ (no Python).
// Graphs: dense (MLP) chains, embedding tables and the DLRM dot interaction (a DLRM-shaped DAG:
// bottom MLP + tables -> interaction -> top MLP), and CNN chains (image input -> convolutions /
// poolings -> dense layers on the flattened features, AlexNet-shaped); tables are placed
// table-wise, column-split or row-split over the ranks, dense layers are data parallel or
// channel-split (output features over a set of ranks), convolutions data parallel.
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

#include <array>
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
constexpr double kBnEps = 1e-5;   // batch-norm epsilon (flexmi.ops.conv.BatchNorm.eps)
enum Loss { LOSS_SCCE = 51, LOSS_MSE_AVG = 52, LOSS_BCE = 54 };

// optimizer of the dense parameters (reference: SGDOptimizer / AdamOptimizer, src/runtime/optimizer.cc
// and optimizer_kernel.cu).  SGD: gt = g + wd w; v = momentum v + gt; gt = nesterov ? gt + momentum v
// : v (momentum > 0); w -= lr gt.  Adam: gt = g + wd w; m = b1 m + (1-b1) gt; v = b2 v + (1-b2) gt^2;
// w -= alpha_t m / (sqrt(v) + eps) with alpha_t = alpha sqrt(1 - b2^t) / (1 - b1^t) (the host keeps
// b1^t, b2^t in fp32 as AdamOptimizer::next does)
enum OptType { OPT_SGD = 0, OPT_ADAM = 1 };
struct OptConfig {
  int type = OPT_SGD;
  float momentum = 0.f;
  bool nesterov = false;
  float weight_decay = 0.f;
  float beta1 = 0.9f, beta2 = 0.999f, eps = 1e-8f;
  int states() const { return type == OPT_ADAM ? 2 : momentum > 0.f ? 1 : 0; }
  bool plain() const { return type == OPT_SGD && momentum == 0.f && weight_decay == 0.f; }
};
// one update: lr = the SGD learning rate or Adam's alpha_t of this step
struct OptStep {
  OptConfig c;
  float lr = 0.f;
};

struct Dense {
  int x = -1, y = -1;          // tensor ids
  int K = 0, N = 0;            // in / out features
  int act = ACT_NONE;
  bool bias = true;
  int w = -1, b = -1;          // parameter entry ids
  // plan
  bool grad_is_dpre = false;   // the consumer's dX epilogue already applied this layer's act'
  bool fuse_below = false;     // this layer's dX epilogue applies the producer layer's act'
  int below = -1;              // dense node whose activation backward that is
  bool skip_act_grad = false;  // sigmoid folded into BCE
  bool need_dx = true;
  // channel split (the reference's Linear partitioned over its output channels, ParallelConfig
  // [1, c] on the channel dim; src/ops/linear.cu:188-293 with the input replicated): holders[j]
  // keeps output features [j*Nc, (j+1)*Nc) of W and b and computes them for the GLOBAL batch.
  // Forward: the ranks' input shards are gathered on every holder (all-to-all), each holder sends
  // every rank its sample rows of its feature slice (the columns are assembled as for a
  // column-split table).  Backward: every holder receives the output gradient of its slice for
  // the global batch, updates its slice (no all-reduce), and the partial input gradients of the
  // holders are summed on each rank's sample shard (reduce-scatter through the all-to-all).
  // Empty holders: data parallel (replicated W, bucketed gradient all-reduce).
  std::vector<int> holders;
  int Nc = 0;
  int j = -1;                  // this rank's slice (plan), -1: not a holder
};

// An embedding table (SUM bag lookups of one sparse input), placed WHOLE on one rank: table-wise
// model parallelism (the reference's DLRM strategy, src/runtime/dlrm_strategy.cc:242-296; the
// embedding op src/ops/embedding.cu:173-224).  The owner looks up the GLOBAL batch; an all-to-all
// hands every rank its sample shard; the reverse all-to-all returns the row gradients, and the
// owner applies sparse SGD to the touched rows (no dense table gradient).
struct Emb {
  int sparse = -1;             // sparse input id
  int64_t rows = 0;
  int D = 0, bag = 1;
  int y = -1;                  // tensor id of the [local batch][D] output
  int w = -1;                  // parameter entry id (the table)
  int owner = 0;               // rank holding the table (plan; the first holder of a split table)
  // column split (the reference's attribute/parameter split of the embedding weight over its
  // columns, ParallelConfig [c, 1] with c > 1; bench "table" plan for the ~40 M-row tables):
  // holders[j] keeps columns [j*Dc, (j+1)*Dc) of every row, looks them up for the global batch
  // and sends each rank its sample shard of that slice; table-wise = one holder, Dc = D
  std::vector<int> holders;
  int Dc = 0;
  // row split (the flexmi [c, n, r] extension: r row blocks): holder j keeps rows [lo_j, lo_{j+1})
  // of all D columns and looks up the global batch; lookups outside its rows add nothing, and each
  // rank SUMS the holders' partial bag sums for its sample shard (gradients go to every holder,
  // which updates the rows it keeps)
  bool rows_split = false;
  int64_t lo = 0, nrows = 0;   // this rank's row block (plan)
};

// DLRM dot interaction (src/ops/tests/test_harness.py:96-186 DotCompressor; caveat C3):
// y = [x | strictly-lower(Z Z^T) | 0 pad], Z = [x; e_1; ..; e_{F-1}] per sample
struct Dot {
  std::vector<int> in;         // tensor ids: bottom output first, then the embeddings
  int y = -1, D = 0, W = 0, npairs = 0;
  int act0 = ACT_NONE;         // the bottom layer's activation, applied by the dot backward to its gradient
};

// 2-D convolution (the reference's Conv2D, src/ops/conv_2d.cu): x [B][C][H][W] (NCHW, a sample's
// C*H*W features contiguous) -> y [B][K][P][Q], kernel [K][C][R][S], symmetric zero padding, bias +
// activation fused; data parallel (replicated kernel in the flat buffer, bucketed all-reduce).
struct Conv {
  int x = -1, y = -1;
  int C = 0, H = 0, W = 0, K = 0, R = 0, S = 0, P = 0, Q = 0;
  int sh = 1, sw = 1, ph = 0, pw = 0;
  int act = ACT_NONE;
  bool bias = true;
  int w = -1, b = -1;          // parameter entry ids
  bool need_dx = true;
};

// 2-D pooling (src/ops/pool_2d.cu): max (padding never wins) or average excluding the padding
struct Pool {
  int x = -1, y = -1;
  int C = 0, H = 0, W = 0, P = 0, Q = 0;
  int kh = 1, kw = 1, sh = 1, sw = 1, ph = 0, pw = 0;
  bool max = true;
  bool need_dx = true;
};

// spatial batch normalisation (src/ops/batch_norm.cu:348-503): training-mode statistics over the
// local shard's samples and pixels per channel, y = act(gamma * xhat + beta), optional ReLU
struct BNorm {
  int x = -1, y = -1;
  int C = 0, H = 0, W = 0;
  bool relu = true;
  int g = -1, b = -1;          // parameter entry ids (scale, bias)
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
  // image input [B][C][H][W] (its C*H*W features per sample, NCHW)
  int input_image(int channels, int height, int width);
  int dense(int x, int out_dim, int act, bool bias);
  // convolution of an image tensor; returns the [B][K][P][Q] output tensor id (dense layers take it
  // flattened)
  int conv2d(int x, int out_channels, int kh, int kw, int sh, int sw, int ph, int pw, int act, bool bias);
  int pool2d(int x, int kh, int kw, int sh, int sw, int ph, int pw, bool max);
  // batch norm of an image tensor (scale 1, bias 0 at init); returns the normalised tensor id
  int batch_norm(int x, bool relu);
  // sparse index input [B][bag] (int64, the GLOBAL batch on every rank); returns its id
  int sparse_input(int bag);
  // embedding table rows x dim looked up by sparse input `sparse` (SUM over the bag); returns the
  // [B][dim] output tensor id
  int embedding(int sparse, int64_t rows, int dim);
  // dot interaction of the bottom tensor and the embedding tensors (all [B][D]); the output width
  // D + F(F-1)/2 is padded up to a multiple of pad_to
  int dot_interaction(int bottom, const std::vector<int>& embs, int pad_to);
  // table placement before compile (default: greedy by rows over the ranks)
  void set_table_owner(int table, int rank);
  // column split of a table over `ranks` (D % ranks.size() == 0); holder j keeps columns
  // [j*D/n, (j+1)*D/n)
  void set_table_columns(int table, const std::vector<int>& ranks);
  // row split of a table over `ranks`: holder j keeps rows [j*rows/n, (j+1)*rows/n); its parameters
  // move as the FULL host array (this rank's rows read / written)
  void set_table_rows(int table, const std::vector<int>& ranks);
  // channel split of dense layer `layer` (creation order among the dense layers) over `ranks`
  // (N % ranks.size() == 0): holder j keeps output features [j*N/n, (j+1)*N/n); W [N][K] and b [N]
  // move as FULL host arrays (this rank's rows / entries read / written)
  void set_dense_channels(int layer, const std::vector<int>& ranks);
  int num_dense() const { return (int)ops_.size(); }
  // optimizer (before compile; default plain SGD at compile's lr).  Embedding tables train with the
  // sparse in-place SGD, so a model with tables needs plain SGD (no momentum / weight decay / Adam).
  void set_optimizer(const OptConfig& o);
  // ZeRO stage 1 (before compile): data-parallel dense parameters keep optimizer state for this rank's
  // 1/world slice of every gradient bucket only -- buckets are reduce-scattered instead of
  // all-reduced, each rank updates its fp32 slice, the fresh slices are all-gathered (the reference
  // has no ZeRO; SURVEY P13, flexmi.runtime.executor._zero_layout)
  void set_zero(int stage);
  void compile(int loss_type, float lr, double bucket_mb);
  void init_weights(uint64_t seed);            // Glorot-uniform weights, zero biases, U(+-sqrt(1/rows)) tables
  int num_params() const { return (int)pnumel_.size(); }
  int64_t param_numel(int i) const { return pnumel_.at(i); }
  // tables: only the owner holds the rows (param_local(i) == false elsewhere)
  bool param_local(int i) const;
  int table_owner(int table) const { return embs_.at(table).owner; }
  const std::vector<int>& table_holders(int table) const { return embs_.at(table).holders; }
  // parameters of a column-split table move as the FULL [rows][D] host array: set_param reads this
  // rank's columns from it, get_param writes them into it (the other columns untouched)
  int num_tables() const { return (int)embs_.size(); }
  void set_param(int i, const float* host);
  void get_param(int i, float* host) const;
  // x: the GLOBAL dense batch [B][features]; sparse[s]: the GLOBAL [B][bag] int64 indices of
  // sparse input s (null for a model without embeddings); labels: [B] int32 (SCCE) or [B][out]
  StepStat train_step(const float* x, const void* labels) { return train_step(x, nullptr, labels); }
  StepStat train_step(const float* x, const int64_t* const* sparse, const void* labels);
  std::string describe() const;
  const WeightPlan& weight_plan() const { return wplan_; }

 private:
  enum Kind { K_DENSE = 0, K_EMB = 1, K_DOT = 2, K_CONV = 3, K_POOL = 4, K_BN = 5 };
  struct Node {
    int kind, idx;
  };
  int dense_out_node() const;
  int slice_of(const Emb& e, int r) const;    // this rank's column slice of e, -1: none
  void check_tensor(int t, const char* what) const;

  int B_, Bl_, device_, rank_, world_;
  std::string rendezvous_;
  std::vector<int> cols_;                     // tensor id -> features
  std::vector<std::vector<int>> shape_;       // tensor id -> per-sample shape ({C, H, W} or {features})
  std::vector<Conv> convs_;
  std::vector<Pool> pools_;
  std::vector<unsigned char*> pool_code_;     // pool id -> max-pool argmax codes (engine scratch)
  std::vector<BNorm> bns_;
  std::vector<float*> bn_buf_;                // bn id -> [6C] engine scratch (statistics, mean / 1/std, sums)
  int new_tensor(const std::vector<int>& shape);
  std::vector<int> consumers_;                // tensor id -> number of consumers
  int input_ = -1;
  std::vector<Node> nodes_;                   // creation (= topological) order
  std::vector<Dense> ops_;
  std::vector<Emb> embs_;
  std::vector<Dot> dots_;
  std::vector<int> sparse_bag_;
  std::vector<int> entry_table_;              // parameter entry -> table id (-1: dense entry)
  std::vector<int> entry_dense_;              // parameter entry -> dense op id (-1: table)
  std::vector<int64_t> pnumel_;               // parameter entries (model order)
  std::vector<int> porder_;                   // backward order of the dense entries
  WeightPlan wplan_;
  std::vector<int64_t> pofs_;                 // dense entry -> flat offset
  int loss_ = LOSS_MSE_AVG;
  float lr_ = 0.01f;
  OptConfig opt_;
  float b1t_ = 1.f, b2t_ = 1.f;               // Adam: beta1^t, beta2^t
  OptStep next_step();
  int zero_ = 0;                              // ZeRO stage (1: sharded optimizer state, world > 1)
  bool zero_on() const { return zero_ >= 1 && world_ > 1; }
  std::vector<int64_t> zshard_off_;           // bucket -> offset of this rank's slice in the shard buffers
  int64_t zshard_n_ = 0;
  float* zmaster_ = nullptr;                  // [zshard_n_] fp32 master slices (ZeRO)
  float* zgrad_ = nullptr;                    // [zshard_n_] reduce-scattered gradient slices
  bool zdirty_ = true;                        // params_ changed on the host side: refresh zmaster_
  float* ostate_[2] = {nullptr, nullptr};     // optimizer state of the flat (or shard) buffer
  std::vector<std::array<float*, 4>> chan_state_;   // channel-split slices: w state x2, b state x2
  bool compiled_ = false;
  std::unique_ptr<Engine> eng_;
  // device buffers
  float* params_ = nullptr;
  float* grads_ = nullptr;
  std::vector<float*> act_;                   // tensor id -> [Bl][cols]
  std::vector<float*> grad_;                  // tensor id -> [Bl][cols]
  std::vector<float*> table_;                 // table id -> [rows][Dc] (holders only)
  std::vector<float*> emb_full_;              // table id -> [B][Dc] holder-side lookups (world > 1)
  std::vector<int64_t*> idx_;                 // table id -> [B][bag] indices (owner only)
  // channel-split dense layers (holders only; indexed by dense op id): the gathered global-batch
  // input [B][K], this slice's output / output gradient [B][Nc], the partial input gradient [B][K],
  // the slice's parameters and gradients
  struct ChanBufs {
    float *x = nullptr, *y = nullptr, *dy = nullptr, *dx = nullptr, *w = nullptr, *b = nullptr, *gw = nullptr,
          *gb = nullptr;
  };
  std::vector<ChanBufs> chan_;
  float* csend_ = nullptr;                    // channel-split exchange staging (world > 1)
  float* crecv_ = nullptr;
  void dense_split_fwd(const Dense& d, int di);
  void dense_split_bwd(const Dense& d, int di, const Dense* below, bool is_dpre);
  float* xsend_ = nullptr;                    // all-to-all staging (world > 1)
  float* xrecv_ = nullptr;
  std::vector<int64_t> xcount_send_, xcount_recv_;
  float* probs_ = nullptr;                    // SCCE: softmax of the logits
  void* labels_ = nullptr;
  float* stats_ = nullptr;                    // [loss, correct] accumulators
  // the per-step inputs (dense shard, labels, owned tables' indices) carved from ONE device arena in
  // the order of a host-side packing, so a pinned engine uploads a batch with one copy
  char* in_arena_ = nullptr;
  std::vector<std::pair<size_t, size_t>> in_parts_;   // (offset, bytes): input, labels, idx of each owned table
  size_t in_bytes_ = 0;
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
  // grad = (p - target) * scale; stats (16 floats, zeroed by the caller each step): loss sum at
  // stats[stat_slot(0)], correct predictions at stats[stat_slot(1)]
  virtual void loss(int type, const float* p, const void* labels, float* grad, int M, int C, float scale,
                    float* stats) = 0;
  virtual int stat_slot(int which) const { return which; }
  virtual void sgd(float* w, float* g, int64_t n, float lr) = 0;   // w -= lr g; g = 0
  // one optimizer update of n parameters (OptConfig); s1 / s2: its state (momentum v, or Adam m / v);
  // consumes g (left zeroed)
  virtual void opt_update(float* w, float* g, float* s1, float* s2, int64_t n, const OptStep& o) = 0;
  virtual void zero(void* p, size_t bytes) = 0;
  // ZeRO: out[n / world] = this rank's slice of sum-over-ranks(buf[n]) (asynchronous like
  // allreduce_start, completed by allreduce_wait); all_gather: buf[world * n] = every rank's in[n]
  virtual void reduce_scatter_start(const float* buf, int64_t n, float* out) = 0;
  virtual void all_gather(const float* in, int64_t n, float* buf) = 0;
  // gradient bucket reduction (sum over ranks): start after the bucket's last gradient, wait
  // before the update
  virtual void allreduce_start(float* buf, int64_t n) = 0;
  virtual void allreduce_wait() = 0;
  // ---- embeddings / interaction / exchange (DLRM plans) ----
  virtual void copy(void* dst, const void* src, size_t bytes) = 0;   // device -> device
  // rows x width_bytes from src (row pitch spitch bytes) to dst (pitch dpitch), device -> device
  virtual void copy2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width_bytes, size_t rows) = 0;
  // out[b] = sum_j W[idx[b][j] - lo]  (b < B; an index outside [lo, lo + rows) contributes nothing)
  virtual void emb_fwd(const float* W, int64_t rows, const int64_t* idx, int bag, float* out, int64_t B, int D,
                       int64_t lo) = 0;
  // W[idx[b][j] - lo] -= lr * g[b]  (duplicates accumulate; indices outside the rows skipped)
  virtual void emb_sgd(float* W, int64_t rows, const int64_t* idx, int bag, const float* g, int64_t B, int D, float lr,
                       int64_t lo) = 0;
  // every local table in one call (default: one emb_fwd / emb_sgd each; the HIP engine batches them
  // into one multi-table launch, as the executor's fused embedding groups do)
  struct EmbJob {
    float* W;
    int64_t rows;
    const int64_t* idx;
    int bag;
    float* io;       // forward: the output rows; backward: the gradient rows
    int D;
    int64_t lo;
  };
  virtual void emb_fwd_multi(const std::vector<EmbJob>& jobs, int64_t B) {
    for (const EmbJob& j : jobs) emb_fwd(j.W, j.rows, j.idx, j.bag, j.io, B, j.D, j.lo);
  }
  virtual void emb_sgd_multi(const std::vector<EmbJob>& jobs, int64_t B, float lr) {
    for (const EmbJob& j : jobs) emb_sgd(j.W, j.rows, j.idx, j.bag, j.io, B, j.D, lr, j.lo);
  }
  // a second in-order queue for independent work (the embedding lookups beside the bottom MLP, the
  // table updates beside its backward): side_begin -> later work runs after everything issued so
  // far but beside what follows side_end; side_join -> later work waits for the side work.  No-ops
  // on engines with one queue.
  virtual void side_begin() {}
  virtual void side_end() {}
  virtual void side_join() {}
  // page-locked host memory (grow-only, owned by the engine; nullptr: the engine has none) -- the batch
  // is packed there and uploaded by ONE asynchronous copy
  virtual void* pinned(size_t bytes) {
    (void)bytes;
    return nullptr;
  }
  // host -> device without the per-copy sync (the caller syncs before the host buffers change)
  virtual void h2d_nosync(void* dst, const void* src, size_t bytes) { h2d(dst, src, bytes); }
  virtual void add(float* dst, const float* src, int64_t n) = 0;   // dst += src (device)
  // y[M][W] = [z0 | lower(Z Z^T) | 0] ; dz[i] = (S Z)_i (+ dy[:, :D] for i = 0), S = dG + dG^T
  virtual void dot_fwd(const float* const* z, int F, float* y, int M, int D, int W) = 0;
  // act0 != ACT_NONE: dz[0] leaves as act0'(z[0]) * dz[0] (the bottom layer's pre-activation gradient)
  virtual void dot_bwd(const float* const* z, int F, const float* dy, float* const* dz, int M, int D, int W, int act0) = 0;
  // per-peer float counts; send / recv contiguous by peer
  virtual void all_to_all(const float* send, const int64_t* send_counts, float* recv, const int64_t* recv_counts) = 0;
  // ---- convolution / pooling (CNN plans), NCHW fp32 ----
  // y = act(conv(x, W) + b)
  virtual void conv_fwd(const float* x, const float* W, const float* b, float* y, int N, const Conv& c) = 0;
  // g = act'(y) dy; dW += g (x) x, db += sum g, dx = W^T (x) g (overwritten; skipped when null)
  virtual void conv_bwd(const float* x, const float* W, const float* y, const float* dy, float* dx, float* dW, float* db,
                        int N, const Conv& c) = 0;
  // code: one byte per output (the argmax offset inside the max window), written by the forward
  virtual void pool_fwd(const float* x, float* y, unsigned char* code, int N, const Pool& p) = 0;
  virtual void pool_bwd(const float* x, const float* y, const float* dy, float* dx, const unsigned char* code, int N,
                        const Pool& p) = 0;
  // batch norm: buf [6C] floats of engine scratch kept from the forward to the backward; the
  // backward writes dgamma / dbeta and overwrites dx (skipped when null)
  virtual void bn_fwd(const float* x, float* y, const float* gamma, const float* beta, float* buf, int N, const BNorm& b) = 0;
  virtual void bn_bwd(const float* x, const float* y, const float* dy, const float* gamma, float* buf, float* dgamma,
                      float* dbeta, float* dx, int N, const BNorm& b) = 0;
};

// CPU engine; world > 1 ranks (one process each) exchange through a HostComm in `rendezvous`
// staging up to slot_bytes per rank
std::unique_ptr<Engine> make_cpu_engine(int rank = 0, int world = 1, const std::string& rendezvous = "",
                                        size_t slot_bytes = 0);
// HIP engine (native_hip.cc): flexmi's gfx950 kernels, RCCL over the ranks of `rendezvous`
std::unique_ptr<Engine> make_hip_engine(int rank, int world, const std::string& rendezvous);

}  // namespace nm
}  // namespace flexmi
