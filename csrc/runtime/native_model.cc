// flexmi native model: plan compiler + CPU engine (see native_model.h).
#include "native_model.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <sstream>
#include <stdexcept>

namespace flexmi {

WeightPlan plan_weights(const std::vector<int64_t>& numels, int64_t cap_elems) {
  WeightPlan p;
  p.offset.resize(numels.size());
  int64_t off = 0, start = 0;
  std::vector<int64_t> ids;
  for (size_t e = 0; e < numels.size(); ++e) {
    const int64_t sz = (numels[e] + 63) / 64 * 64;   // 256-B aligned views: 16-B loads everywhere
    const int64_t end = off + sz;
    if (!ids.empty() && end - start > cap_elems) {
      std::vector<int64_t> b{start, off};
      b.insert(b.end(), ids.begin(), ids.end());
      p.buckets.push_back(std::move(b));
      start = off;
      ids.clear();
    }
    p.offset[e] = off;
    off = end;
    ids.push_back((int64_t)e);
  }
  if (!ids.empty()) {
    std::vector<int64_t> b{start, off};
    b.insert(b.end(), ids.begin(), ids.end());
    p.buckets.push_back(std::move(b));
  }
  p.numel = off;
  return p;
}

namespace nm {

namespace {

inline float act_f(int act, float v) {
  if (act == ACT_RELU) return v > 0.f ? v : 0.f;
  if (act == ACT_SIGMOID) return 1.f / (1.f + std::exp(-v));
  if (act == ACT_TANH) return std::tanh(v);
  return v;
}
inline float act_b(int act, float y, float g) {
  if (act == ACT_RELU) return y > 0.f ? g : 0.f;
  if (act == ACT_SIGMOID) return g * y * (1.f - y);
  if (act == ACT_TANH) return g * (1.f - y * y);
  return g;
}

// reference fp32 engine: plain loops in the executor's order of operations
class CpuEngine : public Engine {
 public:
  void* alloc(size_t bytes) override { return std::calloc(std::max<size_t>(bytes, 16), 1); }
  void release(void* p) override { std::free(p); }
  void h2d(void* dst, const void* src, size_t bytes) override { std::memcpy(dst, src, bytes); }
  void d2h(void* dst, const void* src, size_t bytes) override { std::memcpy(dst, src, bytes); }
  void sync() override {}
  void dense_fwd(const float* x, const float* W, const float* b, float* y, int M, int K, int N, int act) override {
    for (int m = 0; m < M; ++m)
      for (int n = 0; n < N; ++n) {
        float s = 0.f;
        const float* xr = x + (int64_t)m * K;
        const float* wr = W + (int64_t)n * K;
        for (int k = 0; k < K; ++k) s += xr[k] * wr[k];
        y[(int64_t)m * N + n] = act_f(act, s + (b ? b[n] : 0.f));
      }
  }
  void dense_bwd(const float* x, const float* W, const float* y, const float* dy, float* dx, float* dW, float* db, int M,
                 int K, int N, int act, bool grad_is_dpre, const float* y_below, int act_below) override {
    std::vector<float> dpre((size_t)M * N);
    for (int64_t i = 0; i < (int64_t)M * N; ++i) dpre[i] = grad_is_dpre ? dy[i] : act_b(act, y[i], dy[i]);
    for (int n = 0; n < N; ++n)
      for (int k = 0; k < K; ++k) {
        float s = 0.f;
        for (int m = 0; m < M; ++m) s += dpre[(int64_t)m * N + n] * x[(int64_t)m * K + k];
        dW[(int64_t)n * K + k] += s;
      }
    if (db)
      for (int n = 0; n < N; ++n) {
        float s = 0.f;
        for (int m = 0; m < M; ++m) s += dpre[(int64_t)m * N + n];
        db[n] += s;
      }
    if (!dx) return;
    for (int m = 0; m < M; ++m)
      for (int k = 0; k < K; ++k) {
        float s = 0.f;
        for (int n = 0; n < N; ++n) s += dpre[(int64_t)m * N + n] * W[(int64_t)n * K + k];
        const int64_t i = (int64_t)m * K + k;
        dx[i] = y_below ? act_b(act_below, y_below[i], s) : s;
      }
  }
  void softmax(const float* x, float* y, int M, int C) override {
    for (int m = 0; m < M; ++m) {
      const float* r = x + (int64_t)m * C;
      float mx = r[0];
      for (int c = 1; c < C; ++c) mx = std::max(mx, r[c]);
      float s = 0.f;
      for (int c = 0; c < C; ++c) s += std::exp(r[c] - mx);
      for (int c = 0; c < C; ++c) y[(int64_t)m * C + c] = std::exp(r[c] - mx) / s;
    }
  }
  void loss(int type, const float* p, const void* labels, float* grad, int M, int C, float scale, float* stats) override {
    for (int m = 0; m < M; ++m) {
      const float* pr = p + (int64_t)m * C;
      if (type == LOSS_SCCE) {
        const int lab = reinterpret_cast<const int*>(labels)[m];
        int best = 0;
        for (int c = 0; c < C; ++c) {
          grad[(int64_t)m * C + c] = (pr[c] - (c == lab ? 1.f : 0.f)) * scale;
          if (pr[c] > pr[best]) best = c;
        }
        stats[0] += -std::log(std::max(pr[lab], 1e-7f));
        stats[1] += best == lab ? 1.f : 0.f;
      } else {
        const float* t = reinterpret_cast<const float*>(labels) + (int64_t)m * C;
        for (int c = 0; c < C; ++c) {
          grad[(int64_t)m * C + c] = (pr[c] - t[c]) * scale;
          if (type == LOSS_BCE) {
            const float q = std::min(std::max(pr[c], 1e-7f), 1.f - 1e-7f);
            stats[0] += -(t[c] * std::log(q) + (1.f - t[c]) * std::log(1.f - q));
            stats[1] += ((pr[c] >= 0.5f) == (t[c] >= 0.5f)) ? 1.f : 0.f;
          } else {
            const float d = pr[c] - t[c];
            stats[0] += d * d;
          }
        }
      }
    }
  }
  void sgd(float* w, float* g, int64_t n, float lr) override {
    for (int64_t i = 0; i < n; ++i) {
      w[i] -= lr * g[i];
      g[i] = 0.f;
    }
  }
  void allreduce_start(float*, int64_t) override {}
  void allreduce_wait() override {}
};

uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

}  // namespace

std::unique_ptr<Engine> make_cpu_engine() { return std::make_unique<CpuEngine>(); }

// strong definition in native_hip.cc (libflexmi_native_c); builds without it report the engine
// as unavailable
__attribute__((weak)) std::unique_ptr<Engine> make_hip_engine(int, int, const std::string&) {
  throw std::runtime_error("flexmi native model: this build has no HIP engine");
}

Model::Model(int global_batch, int device, int rank, int world, const std::string& rendezvous)
    : B_(global_batch), device_(device), rank_(rank), world_(world), rendezvous_(rendezvous) {
  if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("native model: bad rank / world");
  if (global_batch % world) throw std::invalid_argument("native model: the global batch must divide over the ranks");
  Bl_ = global_batch / world;
  if (device == 0 && world > 1) throw std::invalid_argument("native model: the CPU engine runs one rank");
}

Model::~Model() {
  if (!eng_) return;
  eng_->sync();
  auto rel = [&](void* p) {
    if (p) eng_->release(p);
  };
  rel(params_);
  rel(grads_);
  for (auto* p : act_) rel(p);
  for (auto* p : grad_) rel(p);
  rel(probs_);
  rel(labels_);
  rel(stats_);
}

int Model::input(int features) {
  if (compiled_ || input_ >= 0) throw std::logic_error("native model: one input, before compile");
  cols_.push_back(features);
  input_ = (int)cols_.size() - 1;
  return input_;
}

int Model::dense(int x, int out_dim, int act, bool bias) {
  if (compiled_) throw std::logic_error("native model: dense after compile");
  if (x < 0 || x >= (int)cols_.size()) throw std::invalid_argument("native model: unknown input tensor");
  if (!ops_.empty() && x != ops_.back().y) throw std::invalid_argument("native model: layers form a chain");
  if (act != ACT_NONE && act != ACT_RELU && act != ACT_SIGMOID && act != ACT_TANH)
    throw std::invalid_argument("native model: activation");
  Dense d;
  d.x = x;
  d.K = cols_[x];
  d.N = out_dim;
  d.act = act;
  d.bias = bias;
  cols_.push_back(out_dim);
  d.y = (int)cols_.size() - 1;
  d.w = (int)pnumel_.size();
  pnumel_.push_back((int64_t)d.N * d.K);
  if (bias) {
    d.b = (int)pnumel_.size();
    pnumel_.push_back(d.N);
  }
  ops_.push_back(d);
  return d.y;
}

void Model::compile(int loss_type, float lr, double bucket_mb) {
  if (ops_.empty()) throw std::logic_error("native model: no layers");
  if (loss_type != LOSS_SCCE && loss_type != LOSS_MSE_AVG && loss_type != LOSS_BCE)
    throw std::invalid_argument("native model: loss type");
  loss_ = loss_type;
  lr_ = lr;
  Dense& last = ops_.back();
  if (loss_ == LOSS_BCE) {
    if (last.act != ACT_SIGMOID) throw std::invalid_argument("native model: BCE needs a sigmoid output layer");
    last.skip_act_grad = true;   // the loss emits dL/dz = p - y
  }
  if (loss_ == LOSS_SCCE && last.act != ACT_NONE) throw std::invalid_argument("native model: SCCE takes logits");
  ops_.front().need_dx = false;
  // fused epilogues: layer i+1's dX GEMM applies layer i's activation backward (and then layer
  // i's backward reads its incoming gradient as dpre); GEMM layers only (N > 1 both sides)
  for (size_t i = 0; i + 1 < ops_.size(); ++i) {
    Dense& lo = ops_[i];
    Dense& hi = ops_[i + 1];
    if (lo.act != ACT_NONE && lo.N > 1 && hi.N > 1 && !lo.skip_act_grad) {
      hi.fuse_below = true;
      lo.grad_is_dpre = true;
    }
  }
  // parameter entries in backward order -> one flat buffer, all-reduce buckets
  porder_.clear();
  for (auto it = ops_.rbegin(); it != ops_.rend(); ++it) {
    porder_.push_back(it->w);
    if (it->b >= 0) porder_.push_back(it->b);
  }
  std::vector<int64_t> nums;
  for (int e : porder_) nums.push_back(pnumel_[e]);
  const int64_t cap = std::max<int64_t>(1, (int64_t)(bucket_mb * (1 << 20) / 4));
  wplan_ = plan_weights(nums, cap);
  pofs_.assign(pnumel_.size(), 0);
  for (size_t j = 0; j < porder_.size(); ++j) pofs_[porder_[j]] = wplan_.offset[j];
  // engine + buffers
  eng_ = device_ == 1 ? make_hip_engine(rank_, world_, rendezvous_) : make_cpu_engine();
  params_ = (float*)eng_->alloc(wplan_.numel * 4);
  grads_ = (float*)eng_->alloc(wplan_.numel * 4);
  act_.assign(cols_.size(), nullptr);
  grad_.assign(cols_.size(), nullptr);
  for (size_t t = 0; t < cols_.size(); ++t) {
    act_[t] = (float*)eng_->alloc((size_t)Bl_ * cols_[t] * 4);
    if ((int)t != input_) grad_[t] = (float*)eng_->alloc((size_t)Bl_ * cols_[t] * 4);
  }
  const int C = last.N;
  if (loss_ == LOSS_SCCE) probs_ = (float*)eng_->alloc((size_t)Bl_ * C * 4);
  labels_ = eng_->alloc((size_t)Bl_ * C * 4);
  stats_ = (float*)eng_->alloc(64);
  compiled_ = true;
}

void Model::init_weights(uint64_t seed) {
  if (!compiled_) throw std::logic_error("native model: init after compile");
  for (const Dense& d : ops_) {
    std::vector<float> w((size_t)d.N * d.K);
    const float lim = std::sqrt(6.f / (float)(d.K + d.N));
    uint64_t s = seed * 1000003ULL + (uint64_t)d.w;
    for (auto& v : w) v = ((float)(splitmix(s) >> 40) / (float)(1ULL << 24) * 2.f - 1.f) * lim;
    set_param(d.w, w.data());
    if (d.b >= 0) {
      std::vector<float> z(d.N, 0.f);
      set_param(d.b, z.data());
    }
  }
}

void Model::set_param(int i, const float* host) {
  if (!compiled_) throw std::logic_error("native model: set_param after compile");
  eng_->h2d(params_ + pofs_.at(i), host, pnumel_.at(i) * 4);
  eng_->sync();
}

void Model::get_param(int i, float* host) const {
  if (!compiled_) throw std::logic_error("native model: get_param after compile");
  eng_->sync();
  eng_->d2h(host, params_ + pofs_.at(i), pnumel_.at(i) * 4);
}

StepStat Model::train_step(const float* x, const void* labels) {
  if (!compiled_) throw std::logic_error("native model: train_step before compile");
  const Dense& last = ops_.back();
  const int C = last.N;
  // this rank's sample shard of the global batch
  const int64_t r0 = (int64_t)rank_ * Bl_;
  eng_->h2d(act_[input_], x + r0 * cols_[input_], (size_t)Bl_ * cols_[input_] * 4);
  const size_t lab_row = loss_ == LOSS_SCCE ? 4 : (size_t)C * 4;
  eng_->h2d(labels_, static_cast<const char*>(labels) + r0 * lab_row, (size_t)Bl_ * lab_row);
  float zero[2] = {0.f, 0.f};
  eng_->h2d(stats_, zero, sizeof(zero));
  // forward
  for (const Dense& d : ops_)
    eng_->dense_fwd(act_[d.x], params_ + pofs_[d.w], d.b >= 0 ? params_ + pofs_[d.b] : nullptr, act_[d.y], Bl_, d.K, d.N,
                    d.act);
  // loss: gradient scaled by 1 / global batch (the reference's convention), so summing the
  // ranks' gradients gives the global mean gradient
  const float* pred = act_[last.y];
  if (loss_ == LOSS_SCCE) {
    eng_->softmax(act_[last.y], probs_, Bl_, C);
    pred = probs_;
  }
  eng_->loss(loss_, pred, labels_, grad_[last.y], Bl_, C, 1.f / (float)B_, stats_);
  // backward (reverse layer order) with bucketed gradient all-reduces
  std::vector<int> left;
  for (auto& b : wplan_.buckets) left.push_back((int)b.size() - 2);
  std::vector<int> bucket_of(pnumel_.size(), -1);
  for (size_t bi = 0; bi < wplan_.buckets.size(); ++bi)
    for (size_t k = 2; k < wplan_.buckets[bi].size(); ++k) bucket_of[porder_[wplan_.buckets[bi][k]]] = (int)bi;
  for (int i = (int)ops_.size() - 1; i >= 0; --i) {
    const Dense& d = ops_[i];
    const Dense* below = i > 0 ? &ops_[i - 1] : nullptr;
    const bool fuse = d.fuse_below && below;
    const bool is_dpre = d.grad_is_dpre || d.skip_act_grad;
    eng_->dense_bwd(act_[d.x], params_ + pofs_[d.w], act_[d.y], grad_[d.y], d.need_dx ? grad_[d.x] : nullptr,
                    grads_ + pofs_[d.w], d.b >= 0 ? grads_ + pofs_[d.b] : nullptr, Bl_, d.K, d.N, d.act, is_dpre,
                    fuse ? act_[below->y] : nullptr, fuse ? below->act : ACT_NONE);
    if (world_ > 1) {
      for (int e : {d.w, d.b}) {
        if (e < 0) continue;
        const int bi = bucket_of[e];
        if (--left[bi] == 0)
          eng_->allreduce_start(grads_ + wplan_.buckets[bi][0], wplan_.buckets[bi][1] - wplan_.buckets[bi][0]);
      }
    }
  }
  if (world_ > 1) eng_->allreduce_wait();
  eng_->sgd(params_, grads_, wplan_.numel, lr_);
  float st[2];
  eng_->sync();
  eng_->d2h(st, stats_, sizeof(st));
  StepStat s;
  s.loss = st[0] / Bl_;
  s.correct = (int64_t)st[1];
  s.samples = Bl_;
  return s;
}

std::string Model::describe() const {
  std::ostringstream o;
  o << "native model: global batch " << B_ << " over " << world_ << " rank(s) (" << Bl_ << " per rank), engine "
    << (device_ == 1 ? "hip" : "cpu") << "\n";
  for (size_t i = 0; i < ops_.size(); ++i) {
    const Dense& d = ops_[i];
    o << "  dense" << i << ": " << d.K << " -> " << d.N << " act " << d.act << (d.fuse_below ? " [dX epilogue: act' below]" : "")
      << (d.grad_is_dpre ? " [grad arrives as dpre]" : "") << (d.skip_act_grad ? " [sigmoid folded into BCE]" : "") << "\n";
  }
  o << "  flat parameters " << wplan_.numel << " floats, " << wplan_.buckets.size() << " all-reduce bucket(s)\n";
  for (auto& b : wplan_.buckets) {
    o << "    [" << b[0] << ", " << b[1] << ") entries";
    for (size_t k = 2; k < b.size(); ++k) o << " " << porder_[b[k]];
    o << "\n";
  }
  return o.str();
}

}  // namespace nm
}  // namespace flexmi
