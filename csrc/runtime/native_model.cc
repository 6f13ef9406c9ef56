// flexmi native model: plan compiler + CPU engine (see native_model.h).
#include "native_model.h"

#include "host_comm.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <sstream>
#include <stdexcept>
#include <vector>

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

// reference fp32 engine: plain loops in the executor's order of operations; a HostComm carries
// the collectives between rank processes
class CpuEngine : public Engine {
 public:
  CpuEngine(int rank, int world, const std::string& dir, size_t slot_bytes) : rank_(rank), world_(world) {
    if (world > 1) comm_ = std::make_unique<HostComm>(dir, rank, world, slot_bytes);
  }
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
  void opt_update(float* w, float* g, float* s1, float* s2, int64_t n, const OptStep& o) override {
    const OptConfig& c = o.c;
    for (int64_t i = 0; i < n; ++i) {
      float gt = g[i] + c.weight_decay * w[i];
      if (c.type == OPT_ADAM) {
        s1[i] = s1[i] * c.beta1 + (1.f - c.beta1) * gt;
        s2[i] = s2[i] * c.beta2 + (1.f - c.beta2) * gt * gt;
        w[i] -= o.lr * s1[i] / (std::sqrt(s2[i]) + c.eps);
      } else {
        if (c.momentum > 0.f) {
          s1[i] = s1[i] * c.momentum + gt;
          gt = c.nesterov ? gt + c.momentum * s1[i] : s1[i];
        }
        w[i] -= o.lr * gt;
      }
      g[i] = 0.f;
    }
  }
  void zero(void* p, size_t bytes) override { std::memset(p, 0, bytes); }
  void allreduce_start(float* buf, int64_t n) override {
    if (comm_) comm_->all_reduce_sum(buf, n);   // host collectives complete in place
  }
  // the host communicator has no reduce-scatter / all-gather: the sum-in-rank-order all-reduce, then
  // this rank's slice (the same fp32 sums); the gather as an all-reduce of a buffer that is zero
  // outside this rank's slice (x + 0 is exact)
  void reduce_scatter_start(const float* buf, int64_t n, float* out) override {
    const int64_t k = n / world_;
    if (!comm_) {
      std::memcpy(out, buf, (size_t)k * 4);
      return;
    }
    std::vector<float> t(buf, buf + n);
    comm_->all_reduce_sum(t.data(), n);
    std::memcpy(out, t.data() + (int64_t)rank_ * k, (size_t)k * 4);
  }
  void all_gather(const float* in, int64_t n, float* buf) override {
    if (!comm_) {
      std::memcpy(buf, in, (size_t)n * 4);
      return;
    }
    std::memset(buf, 0, (size_t)n * world_ * 4);
    std::memcpy(buf + (int64_t)rank_ * n, in, (size_t)n * 4);
    comm_->all_reduce_sum(buf, n * world_);
  }
  void allreduce_wait() override {}
  void copy(void* dst, const void* src, size_t bytes) override { std::memcpy(dst, src, bytes); }
  void add(float* dst, const float* src, int64_t n) override {
    for (int64_t i = 0; i < n; ++i) dst[i] += src[i];
  }
  void copy2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t rows) override {
    for (size_t r = 0; r < rows; ++r)
      std::memcpy(static_cast<char*>(dst) + r * dpitch, static_cast<const char*>(src) + r * spitch, width);
  }
  void emb_fwd(const float* W, int64_t rows, const int64_t* idx, int bag, float* out, int64_t B, int D,
               int64_t lo) override {
    for (int64_t b = 0; b < B; ++b) {
      float* o = out + b * D;
      for (int d = 0; d < D; ++d) o[d] = 0.f;
      for (int j = 0; j < bag; ++j) {
        const int64_t r = idx[b * bag + j] - lo;
        if (r < 0 || r >= rows) continue;
        const float* w = W + r * D;
        for (int d = 0; d < D; ++d) o[d] += w[d];
      }
    }
  }
  void emb_sgd(float* W, int64_t rows, const int64_t* idx, int bag, const float* g, int64_t B, int D, float lr,
               int64_t lo) override {
    for (int64_t b = 0; b < B; ++b)
      for (int j = 0; j < bag; ++j) {
        const int64_t r = idx[b * bag + j] - lo;
        if (r < 0 || r >= rows) continue;
        float* w = W + r * D;
        const float* gr = g + b * D;
        for (int d = 0; d < D; ++d) w[d] -= lr * gr[d];
      }
  }
  void dot_fwd(const float* const* z, int F, float* y, int M, int D, int W) override {
    for (int m = 0; m < M; ++m) {
      float* o = y + (int64_t)m * W;
      for (int c = 0; c < W; ++c) o[c] = 0.f;
      for (int d = 0; d < D; ++d) o[d] = z[0][(int64_t)m * D + d];
      int p = D;
      for (int i = 0; i < F; ++i)
        for (int j = 0; j < i; ++j) {
          const float* a = z[i] + (int64_t)m * D;
          const float* b = z[j] + (int64_t)m * D;
          float s = 0.f;
          for (int d = 0; d < D; ++d) s += a[d] * b[d];
          o[p++] = s;
        }
    }
  }
  void dot_bwd(const float* const* z, int F, const float* dy, float* const* dz, int M, int D, int W, int act0) override {
    std::vector<float> S((size_t)F * F);
    for (int m = 0; m < M; ++m) {
      const float* g = dy + (int64_t)m * W;
      int p = D;
      std::fill(S.begin(), S.end(), 0.f);
      for (int i = 0; i < F; ++i)
        for (int j = 0; j < i; ++j) {
          S[(size_t)i * F + j] = g[p];
          S[(size_t)j * F + i] = g[p];
          ++p;
        }
      for (int i = 0; i < F; ++i) {
        if (!dz[i]) continue;
        float* o = dz[i] + (int64_t)m * D;
        for (int d = 0; d < D; ++d) {
          float s = i == 0 ? g[d] : 0.f;
          for (int j = 0; j < F; ++j) s += S[(size_t)i * F + j] * z[j][(int64_t)m * D + d];
          o[d] = i == 0 ? act_b(act0, z[0][(int64_t)m * D + d], s) : s;
        }
      }
    }
  }
  void all_to_all(const float* send, const int64_t* send_counts, float* recv, const int64_t* recv_counts) override {
    if (comm_) {
      comm_->all_to_all(send, send_counts, recv, recv_counts);
      return;
    }
    std::memcpy(recv, send, (size_t)send_counts[0] * sizeof(float));
  }
  // direct convolution loops (double accumulation: the reference result the executor's torch
  // convolution is compared against)
  void conv_fwd(const float* x, const float* W, const float* b, float* y, int N, const Conv& c) override {
    for (int n = 0; n < N; ++n)
      for (int k = 0; k < c.K; ++k)
        for (int p = 0; p < c.P; ++p)
          for (int q = 0; q < c.Q; ++q) {
            double s = b ? b[k] : 0.0;
            for (int ch = 0; ch < c.C; ++ch)
              for (int r = 0; r < c.R; ++r) {
                const int h = p * c.sh - c.ph + r;
                if (h < 0 || h >= c.H) continue;
                for (int t = 0; t < c.S; ++t) {
                  const int w = q * c.sw - c.pw + t;
                  if (w < 0 || w >= c.W) continue;
                  s += (double)x[(((int64_t)n * c.C + ch) * c.H + h) * c.W + w] *
                       W[(((int64_t)k * c.C + ch) * c.R + r) * c.S + t];
                }
              }
            y[(((int64_t)n * c.K + k) * c.P + p) * c.Q + q] = act_f(c.act, (float)s);
          }
  }
  void conv_bwd(const float* x, const float* W, const float* y, const float* dy, float* dx, float* dW, float* db, int N,
                const Conv& c) override {
    const int64_t ny = (int64_t)N * c.K * c.P * c.Q;
    std::vector<float> g(ny);
    for (int64_t i = 0; i < ny; ++i) g[i] = act_b(c.act, y[i], dy[i]);
    auto G = [&](int n, int k, int p, int q) { return g[(((int64_t)n * c.K + k) * c.P + p) * c.Q + q]; };
    for (int k = 0; k < c.K; ++k) {
      if (db) {
        double s = 0.0;
        for (int n = 0; n < N; ++n)
          for (int p = 0; p < c.P; ++p)
            for (int q = 0; q < c.Q; ++q) s += G(n, k, p, q);
        db[k] += (float)s;
      }
      for (int ch = 0; ch < c.C; ++ch)
        for (int r = 0; r < c.R; ++r)
          for (int t = 0; t < c.S; ++t) {
            double s = 0.0;
            for (int n = 0; n < N; ++n)
              for (int p = 0; p < c.P; ++p) {
                const int h = p * c.sh - c.ph + r;
                if (h < 0 || h >= c.H) continue;
                for (int q = 0; q < c.Q; ++q) {
                  const int w = q * c.sw - c.pw + t;
                  if (w < 0 || w >= c.W) continue;
                  s += (double)G(n, k, p, q) * x[(((int64_t)n * c.C + ch) * c.H + h) * c.W + w];
                }
              }
            dW[(((int64_t)k * c.C + ch) * c.R + r) * c.S + t] += (float)s;
          }
    }
    if (!dx) return;
    std::vector<double> acc((size_t)N * c.C * c.H * c.W, 0.0);
    for (int n = 0; n < N; ++n)
      for (int k = 0; k < c.K; ++k)
        for (int p = 0; p < c.P; ++p)
          for (int q = 0; q < c.Q; ++q) {
            const double gv = G(n, k, p, q);
            if (gv == 0.0) continue;
            for (int ch = 0; ch < c.C; ++ch)
              for (int r = 0; r < c.R; ++r) {
                const int h = p * c.sh - c.ph + r;
                if (h < 0 || h >= c.H) continue;
                for (int t = 0; t < c.S; ++t) {
                  const int w = q * c.sw - c.pw + t;
                  if (w < 0 || w >= c.W) continue;
                  acc[(((size_t)n * c.C + ch) * c.H + h) * c.W + w] += gv * W[(((int64_t)k * c.C + ch) * c.R + r) * c.S + t];
                }
              }
          }
    for (size_t i = 0; i < acc.size(); ++i) dx[i] = (float)acc[i];
  }
  void pool_fwd(const float* x, float* y, unsigned char* code, int N, const Pool& pl) override {
    for (int n = 0; n < N; ++n)
      for (int ch = 0; ch < pl.C; ++ch) {
        const float* xc = x + ((int64_t)n * pl.C + ch) * pl.H * pl.W;
        for (int p = 0; p < pl.P; ++p)
          for (int q = 0; q < pl.Q; ++q) {
            float best = -INFINITY;
            int arg = 0, cnt = 0;
            double sum = 0.0;
            for (int r = 0; r < pl.kh; ++r) {
              const int h = p * pl.sh - pl.ph + r;
              if (h < 0 || h >= pl.H) continue;
              for (int t = 0; t < pl.kw; ++t) {
                const int w = q * pl.sw - pl.pw + t;
                if (w < 0 || w >= pl.W) continue;
                const float v = xc[(int64_t)h * pl.W + w];
                if (v > best) {
                  best = v;
                  arg = r * pl.kw + t;
                }
                sum += v;
                ++cnt;
              }
            }
            const int64_t o = (((int64_t)n * pl.C + ch) * pl.P + p) * pl.Q + q;
            y[o] = pl.max ? best : (float)(sum / std::max(cnt, 1));
            if (code) code[o] = (unsigned char)arg;
          }
      }
  }
  void pool_bwd(const float* x, const float* y, const float* dy, float* dx, const unsigned char* code, int N,
                const Pool& pl) override {
    (void)x;
    (void)y;
    std::fill(dx, dx + (int64_t)N * pl.C * pl.H * pl.W, 0.f);
    for (int n = 0; n < N; ++n)
      for (int ch = 0; ch < pl.C; ++ch) {
        float* dc = dx + ((int64_t)n * pl.C + ch) * pl.H * pl.W;
        for (int p = 0; p < pl.P; ++p)
          for (int q = 0; q < pl.Q; ++q) {
            const int64_t o = (((int64_t)n * pl.C + ch) * pl.P + p) * pl.Q + q;
            if (pl.max) {
              const int r = code[o] / pl.kw, t = code[o] % pl.kw;
              dc[(int64_t)(p * pl.sh - pl.ph + r) * pl.W + (q * pl.sw - pl.pw + t)] += dy[o];
              continue;
            }
            int cnt = 0;
            for (int r = 0; r < pl.kh; ++r)
              for (int t = 0; t < pl.kw; ++t) {
                const int h = p * pl.sh - pl.ph + r, w = q * pl.sw - pl.pw + t;
                cnt += h >= 0 && h < pl.H && w >= 0 && w < pl.W;
              }
            for (int r = 0; r < pl.kh; ++r)
              for (int t = 0; t < pl.kw; ++t) {
                const int h = p * pl.sh - pl.ph + r, w = q * pl.sw - pl.pw + t;
                if (h >= 0 && h < pl.H && w >= 0 && w < pl.W) dc[(int64_t)h * pl.W + w] += dy[o] / (float)std::max(cnt, 1);
              }
          }
      }
  }
  // batch norm in double: buf[0..C) mean, buf[C..2C) 1/sqrt(var + eps)
  void bn_fwd(const float* x, float* y, const float* gamma, const float* beta, float* buf, int N, const BNorm& b) override {
    const int64_t HW = (int64_t)b.H * b.W, m = (int64_t)N * HW;
    for (int c = 0; c < b.C; ++c) {
      double s = 0.0, s2 = 0.0;
      for (int n = 0; n < N; ++n) {
        const float* xc = x + ((int64_t)n * b.C + c) * HW;
        for (int64_t i = 0; i < HW; ++i) s += xc[i];
      }
      const double mean = s / (double)m;
      for (int n = 0; n < N; ++n) {
        const float* xc = x + ((int64_t)n * b.C + c) * HW;
        for (int64_t i = 0; i < HW; ++i) s2 += ((double)xc[i] - mean) * ((double)xc[i] - mean);
      }
      const double inv = 1.0 / std::sqrt(s2 / (double)m + kBnEps);
      buf[c] = (float)mean;
      buf[b.C + c] = (float)inv;
      for (int n = 0; n < N; ++n) {
        const float* xc = x + ((int64_t)n * b.C + c) * HW;
        float* yc = y + ((int64_t)n * b.C + c) * HW;
        for (int64_t i = 0; i < HW; ++i) {
          const float v = (float)(((double)xc[i] - mean) * inv) * gamma[c] + beta[c];
          yc[i] = b.relu ? std::max(v, 0.f) : v;
        }
      }
    }
  }
  void bn_bwd(const float* x, const float* y, const float* dy, const float* gamma, float* buf, float* dgamma, float* dbeta,
              float* dx, int N, const BNorm& b) override {
    const int64_t HW = (int64_t)b.H * b.W, m = (int64_t)N * HW;
    for (int c = 0; c < b.C; ++c) {
      const double mean = buf[c], inv = buf[b.C + c];
      double sg = 0.0, sgx = 0.0;
      auto G = [&](int n, int64_t i) {
        const int64_t o = ((int64_t)n * b.C + c) * HW + i;
        return (double)(b.relu && !(y[o] > 0.f) ? 0.f : dy[o]);
      };
      for (int n = 0; n < N; ++n)
        for (int64_t i = 0; i < HW; ++i) {
          const double g = G(n, i);
          sg += g;
          sgx += g * ((double)x[((int64_t)n * b.C + c) * HW + i] - mean) * inv;
        }
      dbeta[c] = (float)sg;
      dgamma[c] = (float)sgx;
      if (!dx) continue;
      for (int n = 0; n < N; ++n)
        for (int64_t i = 0; i < HW; ++i) {
          const int64_t o = ((int64_t)n * b.C + c) * HW + i;
          const double xh = ((double)x[o] - mean) * inv;
          dx[o] = (float)(gamma[c] * inv / (double)m * ((double)m * G(n, i) - sg - xh * sgx));
        }
    }
  }

 private:
  int rank_, world_;
  std::unique_ptr<HostComm> comm_;
};

uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

}  // namespace

std::unique_ptr<Engine> make_cpu_engine(int rank, int world, const std::string& rendezvous, size_t slot_bytes) {
  return std::make_unique<CpuEngine>(rank, world, rendezvous, slot_bytes);
}

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
}

Model::~Model() {
  if (!eng_) return;
  eng_->sync();
  auto rel = [&](void* p) {
    if (p) eng_->release(p);
  };
  rel(params_);
  rel(grads_);
  if (input_ >= 0 && input_ < (int)act_.size()) act_[input_] = nullptr;   // carved from in_arena_
  for (auto* p : act_) rel(p);
  for (auto* p : grad_) rel(p);
  for (auto* p : table_) rel(p);
  for (auto* p : emb_full_) rel(p);
  rel(in_arena_);   // idx_ and labels_ are views into it
  for (auto& c : chan_)
    for (float* q : {c.x, c.y, c.dy, c.dx, c.w, c.b, c.gw, c.gb}) rel(q);
  rel(csend_);
  rel(crecv_);
  rel(xsend_);
  rel(xrecv_);
  rel(probs_);
  rel(stats_);
  for (auto* p : pool_code_) rel(p);
  for (auto* p : bn_buf_) rel(p);
  rel(zmaster_);
  rel(zgrad_);
  for (auto* p : ostate_) rel(p);
  for (auto& a : chan_state_)
    for (float* q : a) rel(q);
}

void Model::check_tensor(int t, const char* what) const {
  if (t < 0 || t >= (int)cols_.size()) throw std::invalid_argument(std::string("native model: unknown tensor for ") + what);
  if (consumers_[t] > 0) throw std::invalid_argument(std::string("native model: tensor consumed twice (") + what + ")");
}

int Model::new_tensor(const std::vector<int>& shape) {
  int64_t n = 1;
  for (int v : shape) n *= v;
  if (n <= 0 || n > (1LL << 30)) throw std::invalid_argument("native model: tensor shape");
  cols_.push_back((int)n);
  shape_.push_back(shape);
  consumers_.push_back(0);
  return (int)cols_.size() - 1;
}

int Model::input(int features) {
  if (compiled_ || input_ >= 0) throw std::logic_error("native model: one input, before compile");
  input_ = new_tensor({features});
  return input_;
}

int Model::input_image(int channels, int height, int width) {
  if (compiled_ || input_ >= 0) throw std::logic_error("native model: one input, before compile");
  if (channels <= 0 || height <= 0 || width <= 0) throw std::invalid_argument("native model: image shape");
  input_ = new_tensor({channels, height, width});
  return input_;
}

int Model::conv2d(int x, int out_channels, int kh, int kw, int sh, int sw, int ph, int pw, int act, bool bias) {
  if (compiled_) throw std::logic_error("native model: conv2d after compile");
  check_tensor(x, "conv2d");
  if (shape_[x].size() != 3) throw std::invalid_argument("native model: conv2d needs an image tensor [C][H][W]");
  if (act != ACT_NONE && act != ACT_RELU && act != ACT_SIGMOID && act != ACT_TANH)
    throw std::invalid_argument("native model: activation");
  Conv c;
  c.x = x;
  c.C = shape_[x][0];
  c.H = shape_[x][1];
  c.W = shape_[x][2];
  c.K = out_channels;
  c.R = kh;
  c.S = kw;
  c.sh = sh;
  c.sw = sw;
  c.ph = ph;
  c.pw = pw;
  c.act = act;
  c.bias = bias;
  if (out_channels <= 0 || kh <= 0 || kw <= 0 || sh <= 0 || sw <= 0 || ph < 0 || pw < 0)
    throw std::invalid_argument("native model: conv2d geometry");
  c.P = (c.H + 2 * ph - kh) / sh + 1;
  c.Q = (c.W + 2 * pw - kw) / sw + 1;
  if (c.P <= 0 || c.Q <= 0) throw std::invalid_argument("native model: conv2d output is empty");
  consumers_[x]++;
  c.y = new_tensor({c.K, c.P, c.Q});
  c.w = (int)pnumel_.size();
  pnumel_.push_back((int64_t)c.K * c.C * c.R * c.S);
  entry_table_.push_back(-1);
  entry_dense_.push_back(-1);
  if (bias) {
    c.b = (int)pnumel_.size();
    pnumel_.push_back(c.K);
    entry_table_.push_back(-1);
    entry_dense_.push_back(-1);
  }
  convs_.push_back(c);
  nodes_.push_back({K_CONV, (int)convs_.size() - 1});
  return c.y;
}

int Model::pool2d(int x, int kh, int kw, int sh, int sw, int ph, int pw, bool max) {
  if (compiled_) throw std::logic_error("native model: pool2d after compile");
  check_tensor(x, "pool2d");
  if (shape_[x].size() != 3) throw std::invalid_argument("native model: pool2d needs an image tensor [C][H][W]");
  if (kh <= 0 || kw <= 0 || sh <= 0 || sw <= 0 || ph < 0 || pw < 0 || ph >= kh || pw >= kw || kh * kw > 255)
    throw std::invalid_argument("native model: pool2d geometry");
  Pool pl;
  pl.x = x;
  pl.C = shape_[x][0];
  pl.H = shape_[x][1];
  pl.W = shape_[x][2];
  pl.kh = kh;
  pl.kw = kw;
  pl.sh = sh;
  pl.sw = sw;
  pl.ph = ph;
  pl.pw = pw;
  pl.max = max;
  pl.P = (pl.H + 2 * ph - kh) / sh + 1;
  pl.Q = (pl.W + 2 * pw - kw) / sw + 1;
  if (pl.P <= 0 || pl.Q <= 0) throw std::invalid_argument("native model: pool2d output is empty");
  consumers_[x]++;
  pl.y = new_tensor({pl.C, pl.P, pl.Q});
  pools_.push_back(pl);
  nodes_.push_back({K_POOL, (int)pools_.size() - 1});
  return pl.y;
}

int Model::batch_norm(int x, bool relu) {
  if (compiled_) throw std::logic_error("native model: batch_norm after compile");
  check_tensor(x, "batch_norm");
  if (shape_[x].size() != 3) throw std::invalid_argument("native model: batch_norm needs an image tensor [C][H][W]");
  BNorm b;
  b.x = x;
  b.C = shape_[x][0];
  b.H = shape_[x][1];
  b.W = shape_[x][2];
  b.relu = relu;
  consumers_[x]++;
  b.y = new_tensor({b.C, b.H, b.W});
  for (int* e : {&b.g, &b.b}) {
    *e = (int)pnumel_.size();
    pnumel_.push_back(b.C);
    entry_table_.push_back(-1);
    entry_dense_.push_back(-1);
  }
  bns_.push_back(b);
  nodes_.push_back({K_BN, (int)bns_.size() - 1});
  return b.y;
}

int Model::dense(int x, int out_dim, int act, bool bias) {
  if (compiled_) throw std::logic_error("native model: dense after compile");
  check_tensor(x, "dense");
  if (act != ACT_NONE && act != ACT_RELU && act != ACT_SIGMOID && act != ACT_TANH)
    throw std::invalid_argument("native model: activation");
  Dense d;
  d.x = x;
  d.K = cols_[x];
  d.N = out_dim;
  d.act = act;
  d.bias = bias;
  consumers_[x]++;
  d.y = new_tensor({out_dim});
  d.w = (int)pnumel_.size();
  pnumel_.push_back((int64_t)d.N * d.K);
  entry_table_.push_back(-1);
  entry_dense_.push_back((int)ops_.size());
  if (bias) {
    d.b = (int)pnumel_.size();
    pnumel_.push_back(d.N);
    entry_table_.push_back(-1);
    entry_dense_.push_back((int)ops_.size());
  }
  ops_.push_back(d);
  nodes_.push_back({K_DENSE, (int)ops_.size() - 1});
  return d.y;
}

int Model::sparse_input(int bag) {
  if (compiled_) throw std::logic_error("native model: sparse input after compile");
  if (bag < 1) throw std::invalid_argument("native model: bag >= 1");
  sparse_bag_.push_back(bag);
  return (int)sparse_bag_.size() - 1;
}

int Model::embedding(int sparse, int64_t rows, int dim) {
  if (compiled_) throw std::logic_error("native model: embedding after compile");
  if (sparse < 0 || sparse >= (int)sparse_bag_.size()) throw std::invalid_argument("native model: unknown sparse input");
  for (const Emb& e : embs_)
    if (e.sparse == sparse) throw std::invalid_argument("native model: sparse input used twice");
  if (rows < 1 || dim < 1) throw std::invalid_argument("native model: embedding shape");
  Emb e;
  e.sparse = sparse;
  e.rows = rows;
  e.D = dim;
  e.bag = sparse_bag_[sparse];
  e.y = new_tensor({dim});
  e.w = (int)pnumel_.size();
  pnumel_.push_back(rows * dim);
  entry_table_.push_back((int)embs_.size());
  entry_dense_.push_back(-1);
  e.owner = -1;
  embs_.push_back(e);
  nodes_.push_back({K_EMB, (int)embs_.size() - 1});
  return e.y;
}

int Model::dot_interaction(int bottom, const std::vector<int>& embs, int pad_to) {
  if (compiled_) throw std::logic_error("native model: interaction after compile");
  if (embs.empty() || embs.size() > 31) throw std::invalid_argument("native model: 1..31 embeddings per interaction");
  Dot d;
  d.in.push_back(bottom);
  for (int t : embs) d.in.push_back(t);
  check_tensor(bottom, "interaction");
  d.D = cols_[bottom];
  for (int t : d.in) {
    check_tensor(t, "interaction");
    if (cols_[t] != d.D) throw std::invalid_argument("native model: interaction inputs of different widths");
  }
  for (int t : d.in) consumers_[t]++;
  const int F = (int)d.in.size();
  d.npairs = F * (F - 1) / 2;
  const int p = std::max(1, pad_to);
  d.W = (d.D + d.npairs + p - 1) / p * p;
  d.y = new_tensor({d.W});
  dots_.push_back(d);
  nodes_.push_back({K_DOT, (int)dots_.size() - 1});
  return d.y;
}

void Model::set_table_owner(int table, int rank) {
  if (compiled_) throw std::logic_error("native model: placement after compile");
  if (table < 0 || table >= (int)embs_.size() || rank < 0 || rank >= world_)
    throw std::invalid_argument("native model: table / rank");
  embs_[table].owner = rank;
  embs_[table].holders.clear();
  embs_[table].rows_split = false;
}

void Model::set_table_columns(int table, const std::vector<int>& ranks) {
  if (compiled_) throw std::logic_error("native model: placement after compile");
  if (table < 0 || table >= (int)embs_.size() || ranks.empty()) throw std::invalid_argument("native model: table / ranks");
  Emb& e = embs_[table];
  if (e.D % (int)ranks.size() != 0) throw std::invalid_argument("native model: columns not divisible by the holders");
  for (size_t i = 0; i < ranks.size(); ++i) {
    if (ranks[i] < 0 || ranks[i] >= world_) throw std::invalid_argument("native model: holder rank");
    for (size_t j = 0; j < i; ++j)
      if (ranks[j] == ranks[i]) throw std::invalid_argument("native model: holder listed twice");
  }
  e.holders = ranks;
  e.owner = ranks[0];
  e.rows_split = false;
}

void Model::set_table_rows(int table, const std::vector<int>& ranks) {
  // every check before any field changes: a rejected call leaves the table's placement as it was
  if (compiled_) throw std::logic_error("native model: placement after compile");
  if (table < 0 || table >= (int)embs_.size() || ranks.empty()) throw std::invalid_argument("native model: table / ranks");
  Emb& e = embs_[table];
  for (size_t i = 0; i < ranks.size(); ++i) {
    if (ranks[i] < 0 || ranks[i] >= world_) throw std::invalid_argument("native model: holder rank");
    for (size_t j = 0; j < i; ++j)
      if (ranks[j] == ranks[i]) throw std::invalid_argument("native model: holder listed twice");
  }
  if ((int64_t)ranks.size() > e.rows) throw std::invalid_argument("native model: more row blocks than rows");
  e.holders = ranks;
  e.owner = ranks[0];
  e.rows_split = ranks.size() > 1;
}

void Model::set_dense_channels(int layer, const std::vector<int>& ranks) {
  if (compiled_) throw std::logic_error("native model: placement after compile");
  if (layer < 0 || layer >= (int)ops_.size() || ranks.empty()) throw std::invalid_argument("native model: dense layer / ranks");
  Dense& d = ops_[layer];
  if (d.N % (int)ranks.size() != 0) throw std::invalid_argument("native model: output features not divisible by the holders");
  for (size_t i = 0; i < ranks.size(); ++i) {
    if (ranks[i] < 0 || ranks[i] >= world_) throw std::invalid_argument("native model: holder rank");
    for (size_t k = 0; k < i; ++k)
      if (ranks[k] == ranks[i]) throw std::invalid_argument("native model: holder listed twice");
  }
  d.holders = ranks;
}

int Model::slice_of(const Emb& e, int r) const {
  for (size_t j = 0; j < e.holders.size(); ++j)
    if (e.holders[j] == r) return (int)j;
  return -1;
}

int Model::dense_out_node() const {
  if (nodes_.empty() || nodes_.back().kind != K_DENSE) throw std::logic_error("native model: the last op must be dense");
  return nodes_.back().idx;
}

bool Model::param_local(int i) const {
  const int t = entry_table_.at(i);
  if (t >= 0) return slice_of(embs_[t], rank_) >= 0;
  const Dense& d = ops_[entry_dense_.at(i)];
  return d.holders.empty() || std::find(d.holders.begin(), d.holders.end(), rank_) != d.holders.end();
}

void Model::set_optimizer(const OptConfig& o) {
  if (compiled_) throw std::logic_error("native model: set_optimizer after compile");
  if (o.type != OPT_SGD && o.type != OPT_ADAM) throw std::invalid_argument("native model: optimizer type");
  if (o.momentum < 0.f || o.weight_decay < 0.f || o.beta1 < 0.f || o.beta1 >= 1.f || o.beta2 < 0.f || o.beta2 >= 1.f ||
      o.eps <= 0.f)
    throw std::invalid_argument("native model: optimizer hyper-parameters");
  opt_ = o;
}

void Model::set_zero(int stage) {
  if (compiled_) throw std::logic_error("native model: set_zero after compile");
  if (stage < 0 || stage > 1) throw std::invalid_argument("native model: ZeRO stage (0 or 1)");
  zero_ = stage;
}

OptStep Model::next_step() {
  OptStep s;
  s.c = opt_;
  s.lr = lr_;
  if (opt_.type == OPT_ADAM) {   // AdamOptimizer::next (src/runtime/optimizer.cc:167-173), fp32 counters
    b1t_ *= opt_.beta1;
    b2t_ *= opt_.beta2;
    s.lr = lr_ * std::sqrt(1.f - b2t_) / (1.f - b1t_);
  }
  return s;
}

void Model::compile(int loss_type, float lr, double bucket_mb) {
  if (ops_.empty()) throw std::logic_error("native model: no layers");
  if (!embs_.empty() && !opt_.plain())
    throw std::invalid_argument(
        "native model: embedding tables train with the sparse in-place SGD; momentum / weight decay / Adam "
        "need dense table gradients (not planned natively)");
  if (loss_type != LOSS_SCCE && loss_type != LOSS_MSE_AVG && loss_type != LOSS_BCE)
    throw std::invalid_argument("native model: loss type");
  loss_ = loss_type;
  lr_ = lr;
  Dense& last = ops_[dense_out_node()];
  if (loss_ == LOSS_BCE) {
    if (last.act != ACT_SIGMOID) throw std::invalid_argument("native model: BCE needs a sigmoid output layer");
    last.skip_act_grad = true;   // the loss emits dL/dz = p - y
  }
  if (loss_ == LOSS_SCCE && last.act != ACT_NONE) throw std::invalid_argument("native model: SCCE takes logits");
  // producers of the dense tensors
  std::vector<int> dense_of(cols_.size(), -1);
  for (size_t i = 0; i < ops_.size(); ++i) dense_of[ops_[i].y] = (int)i;
  for (Dense& d : ops_) d.need_dx = d.x != input_;
  for (Conv& c : convs_) c.need_dx = c.x != input_;
  for (Pool& pl : pools_) pl.need_dx = pl.x != input_;
  for (BNorm& b : bns_) b.need_dx = b.x != input_;
  // fused epilogues: a dense layer whose input is another dense layer's output applies that
  // layer's activation backward in its dX GEMM (the producer then reads its gradient as dpre)
  for (Dense& hi : ops_) {
    const int lo_i = dense_of[hi.x];
    if (lo_i < 0) continue;
    Dense& lo = ops_[lo_i];
    if (lo.act != ACT_NONE && lo.N > 1 && hi.N > 1 && !lo.skip_act_grad) {
      hi.fuse_below = true;
      hi.below = lo_i;
      lo.grad_is_dpre = true;
    }
  }
  // the dot interaction's backward applies the bottom layer's activation derivative to the gradient it
  // writes (flexmi/runtime/executor.py _build_interaction_act_fusion): that layer reads it as dpre
  for (Dot& d : dots_) {
    const int li = dense_of[d.in[0]];
    if (li < 0) continue;
    Dense& L = ops_[li];
    if (L.holders.empty() && L.act != ACT_NONE && L.N > 1 && !L.grad_is_dpre && !L.skip_act_grad) {
      d.act0 = L.act;
      L.grad_is_dpre = true;
    }
  }
  // table-wise placement: unplaced tables go to the rank with the fewest rows (largest first)
  {
    std::vector<int64_t> load(world_, 0);
    for (const Emb& e : embs_)
      if (e.owner >= 0) load[e.owner] += e.rows;
    std::vector<int> order;
    for (int t = 0; t < (int)embs_.size(); ++t)
      if (embs_[t].owner < 0) order.push_back(t);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return embs_[a].rows > embs_[b].rows; });
    for (int t : order) {
      const int r = (int)(std::min_element(load.begin(), load.end()) - load.begin());
      embs_[t].owner = r;
      load[r] += embs_[t].rows;
    }
    for (Emb& e : embs_) {
      if (e.holders.empty()) e.holders = {e.owner};
      const int n = (int)e.holders.size();
      e.Dc = e.rows_split ? e.D : e.D / n;
      const int j = slice_of(e, rank_);
      e.lo = e.rows_split && j >= 0 ? e.rows * j / n : 0;
      e.nrows = e.rows_split ? (j >= 0 ? e.rows * (j + 1) / n - e.lo : 0) : e.rows;
    }
  }
  // channel-split dense layers: this rank's slice
  for (Dense& d : ops_) {
    d.j = -1;
    d.Nc = d.N;
    if (d.holders.empty()) continue;
    d.Nc = d.N / (int)d.holders.size();
    for (size_t k = 0; k < d.holders.size(); ++k)
      if (d.holders[k] == rank_) d.j = (int)k;
  }
  // data-parallel dense parameter entries in backward order -> one flat buffer, all-reduce buckets
  // (channel-split slices are updated by their holders, never reduced)
  porder_.clear();
  for (auto it = nodes_.rbegin(); it != nodes_.rend(); ++it) {   // backward (reverse creation) order
    int w = -1, b = -1;
    if (it->kind == K_DENSE) {
      const Dense& d = ops_[it->idx];
      if (!d.holders.empty()) continue;
      w = d.w;
      b = d.b;
    } else if (it->kind == K_CONV) {
      w = convs_[it->idx].w;
      b = convs_[it->idx].b;
    } else if (it->kind == K_BN) {
      w = bns_[it->idx].g;
      b = bns_[it->idx].b;
    } else {
      continue;
    }
    porder_.push_back(w);
    if (b >= 0) porder_.push_back(b);
  }
  std::vector<int64_t> nums;
  for (int e : porder_) nums.push_back(pnumel_[e]);
  const int64_t cap = std::max<int64_t>(1, (int64_t)(bucket_mb * (1 << 20) / 4));
  if (zero_on()) {
    // ZeRO-1 layout (flexmi.runtime.executor._zero_layout): 64-float aligned entries, every bucket
    // padded to a multiple of world x 64 floats so each rank owns an equal 256-B aligned slice
    const int64_t quant = (int64_t)world_ * 64;
    WeightPlan p;
    p.offset.resize(nums.size());
    int64_t off = 0, start = 0;
    std::vector<int64_t> ids;
    auto close = [&] {
      const int64_t end = start + (off - start + quant - 1) / quant * quant;
      std::vector<int64_t> b{start, end};
      b.insert(b.end(), ids.begin(), ids.end());
      p.buckets.push_back(std::move(b));
      start = off = end;
      ids.clear();
    };
    for (size_t e = 0; e < nums.size(); ++e) {
      const int64_t sz = (nums[e] + 63) / 64 * 64;
      if (!ids.empty() && off + sz - start > cap) close();
      p.offset[e] = off;
      off += sz;
      ids.push_back((int64_t)e);
    }
    if (!ids.empty()) close();
    p.numel = off;
    wplan_ = std::move(p);
    zshard_off_.clear();
    zshard_n_ = 0;
    for (auto& b : wplan_.buckets) {
      zshard_off_.push_back(zshard_n_);
      zshard_n_ += (b[1] - b[0]) / world_;
    }
  } else {
    wplan_ = plan_weights(nums, cap);
  }
  pofs_.assign(pnumel_.size(), 0);
  for (size_t j = 0; j < porder_.size(); ++j) pofs_[porder_[j]] = wplan_.offset[j];
  // embedding exchange: every holder sends each peer that peer's sample rows of its column slice
  // of every held table (table order); each rank receives, per peer, the slices that peer holds
  // (table order) and assembles the columns
  xcount_send_.assign(world_, 0);
  xcount_recv_.assign(world_, 0);
  for (const Emb& e : embs_)
    for (int p = 0; p < world_; ++p) {
      if (slice_of(e, rank_) >= 0) xcount_send_[p] += (int64_t)Bl_ * e.Dc;
      if (slice_of(e, p) >= 0) xcount_recv_[p] += (int64_t)Bl_ * e.Dc;
    }
  int64_t xs = 0, xr = 0;
  for (int p = 0; p < world_; ++p) {
    xs += xcount_send_[p];
    xr += xcount_recv_[p];
  }
  // engine + buffers.  The host communicator's slot size must be the SAME on every rank (rank 0
  // publishes it, peers require an exact match, and the chunk strides of all_reduce_sum /
  // all_to_all depend on it), so it is sized from global quantities every rank derives from the
  // deterministic placement: the largest send total of any rank (world * Bl * the D of the tables
  // it owns) and the receive total (Bl * the D of every table, the same for all ranks).
  int64_t xmax = xr;
  {
    std::vector<int64_t> own(world_, 0);
    for (const Emb& e : embs_)
      for (int h : e.holders) own[h] += (int64_t)world_ * Bl_ * e.Dc;
    for (int64_t v : own) xmax = std::max(xmax, v);
  }
  // channel-split exchanges (every quantity global): input gather (each rank sends n * Bl * K, a
  // holder receives B * K), output slices (a holder sends B * Nc, each rank receives Bl * N), their
  // gradients back, the partial input gradients (a holder sends B * K, each rank receives
  // n * Bl * K)
  int64_t cmax = 0;
  for (const Dense& d : ops_) {
    if (d.holders.empty()) continue;
    const int64_t n = (int64_t)d.holders.size();
    cmax = std::max({cmax, (int64_t)B_ * d.K, (int64_t)B_ * d.Nc, n * Bl_ * d.K, (int64_t)Bl_ * d.N});
  }
  xmax = std::max(xmax, cmax);
  const size_t slot = std::max<size_t>((size_t)std::max<int64_t>(xmax, std::max(xs, xr)) * 4 + 4096, 4u << 20);
  eng_ = device_ == 1 ? make_hip_engine(rank_, world_, rendezvous_) : make_cpu_engine(rank_, world_, rendezvous_, slot);
  params_ = (float*)eng_->alloc(wplan_.numel * 4);
  grads_ = (float*)eng_->alloc(wplan_.numel * 4);
  act_.assign(cols_.size(), nullptr);
  grad_.assign(cols_.size(), nullptr);
  // input arena: [dense input shard | labels | indices of every owned table], 256-B aligned parts
  {
    const Dense& lastd = ops_[dense_out_node()];
    auto part = [&](size_t bytes) {
      in_parts_.push_back({in_bytes_, bytes});
      in_bytes_ += (bytes + 255) / 256 * 256;
    };
    in_parts_.clear();
    in_bytes_ = 0;
    part((size_t)Bl_ * cols_[input_] * 4);
    part((size_t)Bl_ * (loss_ == LOSS_SCCE ? 4 : (size_t)lastd.N * 4));   // int32 class ids / float targets
    for (const Emb& e : embs_)
      if (slice_of(e, rank_) >= 0) part((size_t)B_ * e.bag * 8);
    in_arena_ = (char*)eng_->alloc(in_bytes_);
  }
  for (size_t t = 0; t < cols_.size(); ++t) {
    if ((int)t == input_) {
      act_[t] = reinterpret_cast<float*>(in_arena_ + in_parts_[0].first);
      continue;
    }
    act_[t] = (float*)eng_->alloc((size_t)Bl_ * cols_[t] * 4);
    if ((int)t != input_) grad_[t] = (float*)eng_->alloc((size_t)Bl_ * cols_[t] * 4);
  }
  table_.assign(embs_.size(), nullptr);
  emb_full_.assign(embs_.size(), nullptr);
  idx_.assign(embs_.size(), nullptr);
  int next_in_part = 0;
  for (size_t t = 0; t < embs_.size(); ++t) {
    const Emb& e = embs_[t];
    if (slice_of(e, rank_) < 0) continue;
    table_[t] = (float*)eng_->alloc((size_t)e.nrows * e.Dc * 4);
    idx_[t] = reinterpret_cast<int64_t*>(in_arena_ + in_parts_[2 + (next_in_part++)].first);
    if (world_ > 1) emb_full_[t] = (float*)eng_->alloc((size_t)B_ * e.Dc * 4);
  }
  if (world_ > 1 && !embs_.empty()) {
    xsend_ = (float*)eng_->alloc((size_t)std::max<int64_t>(xs, 1) * 4);
    xrecv_ = (float*)eng_->alloc((size_t)std::max<int64_t>(xr, 1) * 4);
  }
  chan_.assign(ops_.size(), ChanBufs{});
  for (size_t i = 0; i < ops_.size(); ++i) {
    const Dense& d = ops_[i];
    if (d.j < 0) continue;
    ChanBufs& c = chan_[i];
    c.x = (float*)eng_->alloc((size_t)B_ * d.K * 4);
    c.y = (float*)eng_->alloc((size_t)B_ * d.Nc * 4);
    c.dy = (float*)eng_->alloc((size_t)B_ * d.Nc * 4);
    if (d.need_dx) c.dx = (float*)eng_->alloc((size_t)B_ * d.K * 4);
    c.w = (float*)eng_->alloc((size_t)d.Nc * d.K * 4);
    c.gw = (float*)eng_->alloc((size_t)d.Nc * d.K * 4);
    if (d.b >= 0) {
      c.b = (float*)eng_->alloc((size_t)d.Nc * 4);
      c.gb = (float*)eng_->alloc((size_t)d.Nc * 4);
    }
  }
  if (cmax > 0) {
    csend_ = (float*)eng_->alloc((size_t)cmax * 4);
    crecv_ = (float*)eng_->alloc((size_t)cmax * 4);
  }
  pool_code_.assign(pools_.size(), nullptr);
  for (size_t i = 0; i < pools_.size(); ++i)
    pool_code_[i] = (unsigned char*)eng_->alloc((size_t)Bl_ * pools_[i].C * pools_[i].P * pools_[i].Q);
  bn_buf_.assign(bns_.size(), nullptr);
  for (size_t i = 0; i < bns_.size(); ++i) bn_buf_[i] = (float*)eng_->alloc((size_t)6 * bns_[i].C * 4);
  const int C = last.N;
  if (loss_ == LOSS_SCCE) probs_ = (float*)eng_->alloc((size_t)Bl_ * C * 4);
  labels_ = in_arena_ + in_parts_[1].first;
  stats_ = (float*)eng_->alloc(64);
  // optimizer state (momentum v / Adam m, v) for the flat buffer -- or, under ZeRO-1, for this
  // rank's slices only -- and for the channel-split slices this rank holds
  const int64_t on = zero_on() ? zshard_n_ : wplan_.numel;
  for (int k = 0; k < opt_.states(); ++k) ostate_[k] = (float*)eng_->alloc((size_t)std::max<int64_t>(on, 1) * 4);
  if (zero_on()) {
    zmaster_ = (float*)eng_->alloc((size_t)std::max<int64_t>(zshard_n_, 1) * 4);
    zgrad_ = (float*)eng_->alloc((size_t)std::max<int64_t>(zshard_n_, 1) * 4);
  }
  chan_state_.assign(ops_.size(), {nullptr, nullptr, nullptr, nullptr});
  for (size_t i = 0; i < ops_.size(); ++i) {
    const Dense& d = ops_[i];
    if (d.j < 0) continue;
    for (int k = 0; k < opt_.states(); ++k) {
      chan_state_[i][k] = (float*)eng_->alloc((size_t)d.Nc * d.K * 4);
      if (d.b >= 0) chan_state_[i][2 + k] = (float*)eng_->alloc((size_t)d.Nc * 4);
    }
  }
  b1t_ = b2t_ = 1.f;
  zdirty_ = true;
  compiled_ = true;
}

void Model::init_weights(uint64_t seed) {
  if (!compiled_) throw std::logic_error("native model: init after compile");
  for (const Dense& d : ops_) {
    std::vector<float> w((size_t)d.N * d.K);
    const float lim = std::sqrt(6.f / (float)(d.K + d.N));
    uint64_t s = seed * 1000003ULL + (uint64_t)d.w;
    for (auto& v : w) v = ((float)(splitmix(s) >> 40) / (float)(1ULL << 24) * 2.f - 1.f) * lim;
    if (!param_local(d.w)) continue;
    set_param(d.w, w.data());
    if (d.b >= 0) {
      std::vector<float> z(d.N, 0.f);
      set_param(d.b, z.data());
    }
  }
  for (const Conv& c : convs_) {   // Glorot-uniform over fan-in C*R*S and fan-out K*R*S, zero bias
    std::vector<float> w((size_t)c.K * c.C * c.R * c.S);
    const float lim = std::sqrt(6.f / (float)((c.C + c.K) * c.R * c.S));
    uint64_t s = seed * 1000003ULL + (uint64_t)c.w;
    for (auto& v : w) v = ((float)(splitmix(s) >> 40) / (float)(1ULL << 24) * 2.f - 1.f) * lim;
    set_param(c.w, w.data());
    if (c.b >= 0) {
      std::vector<float> z(c.K, 0.f);
      set_param(c.b, z.data());
    }
  }
  for (const BNorm& b : bns_) {    // scale 1, bias 0
    std::vector<float> one(b.C, 1.f), zero(b.C, 0.f);
    set_param(b.g, one.data());
    set_param(b.b, zero.data());
  }
  for (const Emb& e : embs_) {
    if (slice_of(e, rank_) < 0) continue;
    std::vector<float> w((size_t)e.rows * e.D);   // the whole table; this rank keeps its columns
    const float lim = std::sqrt(1.f / (float)e.rows);
    uint64_t s = seed * 1000003ULL + (uint64_t)e.w;
    for (auto& v : w) v = ((float)(splitmix(s) >> 40) / (float)(1ULL << 24) * 2.f - 1.f) * lim;
    set_param(e.w, w.data());
  }
}

void Model::set_param(int i, const float* host) {
  if (!compiled_) throw std::logic_error("native model: set_param after compile");
  const int t = entry_table_.at(i);
  if (t >= 0) {
    const Emb& e = embs_[t];
    const int j = slice_of(e, rank_);
    if (j < 0) throw std::invalid_argument("native model: table not on this rank");
    if (e.rows_split) {
      eng_->h2d(table_[t], host + e.lo * e.D, (size_t)e.nrows * e.D * 4);
    } else if (e.Dc == e.D) {
      eng_->h2d(table_[t], host, pnumel_[i] * 4);
    } else {
      std::vector<float> sl((size_t)e.rows * e.Dc);
      for (int64_t r = 0; r < e.rows; ++r)
        std::memcpy(&sl[(size_t)r * e.Dc], host + r * e.D + (int64_t)j * e.Dc, (size_t)e.Dc * 4);
      eng_->h2d(table_[t], sl.data(), sl.size() * 4);
    }
  } else if (entry_dense_.at(i) >= 0 && !ops_[entry_dense_[i]].holders.empty()) {
    const int di = entry_dense_[i];
    const Dense& d = ops_[di];
    if (d.j < 0) throw std::invalid_argument("native model: dense slice not on this rank");
    if (i == d.w) eng_->h2d(chan_[di].w, host + (int64_t)d.j * d.Nc * d.K, (size_t)d.Nc * d.K * 4);
    else eng_->h2d(chan_[di].b, host + (int64_t)d.j * d.Nc, (size_t)d.Nc * 4);
  } else {
    eng_->h2d(params_ + pofs_.at(i), host, pnumel_.at(i) * 4);
    zdirty_ = true;   // the ZeRO master slices are refreshed from params_ before the next update
  }
  eng_->sync();
}

void Model::get_param(int i, float* host) const {
  if (!compiled_) throw std::logic_error("native model: get_param after compile");
  eng_->sync();
  const int t = entry_table_.at(i);
  if (t >= 0) {
    const Emb& e = embs_[t];
    const int j = slice_of(e, rank_);
    if (j < 0) throw std::invalid_argument("native model: table not on this rank");
    if (e.rows_split) {
      eng_->d2h(host + e.lo * e.D, table_[t], (size_t)e.nrows * e.D * 4);
    } else if (e.Dc == e.D) {
      eng_->d2h(host, table_[t], pnumel_[i] * 4);
    } else {
      std::vector<float> sl((size_t)e.rows * e.Dc);
      eng_->d2h(sl.data(), table_[t], sl.size() * 4);
      for (int64_t r = 0; r < e.rows; ++r)
        std::memcpy(host + r * e.D + (int64_t)j * e.Dc, &sl[(size_t)r * e.Dc], (size_t)e.Dc * 4);
    }
  } else if (entry_dense_.at(i) >= 0 && !ops_[entry_dense_[i]].holders.empty()) {
    const int di = entry_dense_[i];
    const Dense& d = ops_[di];
    if (d.j < 0) throw std::invalid_argument("native model: dense slice not on this rank");
    if (i == d.w) eng_->d2h(host + (int64_t)d.j * d.Nc * d.K, chan_[di].w, (size_t)d.Nc * d.K * 4);
    else eng_->d2h(host + (int64_t)d.j * d.Nc, chan_[di].b, (size_t)d.Nc * 4);
  } else {
    eng_->d2h(host, params_ + pofs_.at(i), pnumel_.at(i) * 4);
  }
}

// forward of a channel-split dense layer (every rank takes part in the exchanges)
void Model::dense_split_fwd(const Dense& d, int di) {
  const ChanBufs& c = chan_[di];
  const int n = (int)d.holders.size();
  if (world_ == 1) {   // one rank holds every slice
    eng_->dense_fwd(act_[d.x], c.w, c.b, act_[d.y], Bl_, d.K, d.N, d.act);
    return;
  }
  std::vector<int64_t> sc(world_, 0), rc(world_, 0);
  // 1. gather the input shards on the holders (peer order = sample order)
  int64_t o = 0;
  for (int p = 0; p < world_; ++p)
    if (std::find(d.holders.begin(), d.holders.end(), p) != d.holders.end()) {
      eng_->copy(csend_ + o, act_[d.x], (size_t)Bl_ * d.K * 4);
      sc[p] = (int64_t)Bl_ * d.K;
      o += sc[p];
    }
  if (d.j >= 0) std::fill(rc.begin(), rc.end(), (int64_t)Bl_ * d.K);
  eng_->all_to_all(csend_, sc.data(), d.j >= 0 ? c.x : crecv_, rc.data());
  // 2. the slice for the global batch
  if (d.j >= 0) eng_->dense_fwd(c.x, c.w, c.b, c.y, B_, d.K, d.Nc, d.act);
  // 3. every rank gets its sample rows of every slice (the slice's rows are contiguous by peer)
  std::fill(sc.begin(), sc.end(), d.j >= 0 ? (int64_t)Bl_ * d.Nc : 0);
  std::fill(rc.begin(), rc.end(), 0);
  for (int h : d.holders) rc[h] = (int64_t)Bl_ * d.Nc;
  eng_->all_to_all(d.j >= 0 ? c.y : csend_, sc.data(), crecv_, rc.data());
  o = 0;
  for (int p = 0; p < world_; ++p) {
    if (rc[p] == 0) continue;
    const int jj = (int)(std::find(d.holders.begin(), d.holders.end(), p) - d.holders.begin());
    eng_->copy2d(act_[d.y] + (int64_t)jj * d.Nc, (size_t)d.N * 4, crecv_ + o, (size_t)d.Nc * 4, (size_t)d.Nc * 4, Bl_);
    o += rc[p];
  }
  (void)n;
}

// backward of a channel-split dense layer: output-gradient slices to the holders, the slice's
// weight gradients for the global batch, the holders' partial input gradients summed per shard
void Model::dense_split_bwd(const Dense& d, int di, const Dense* below, bool is_dpre) {
  const ChanBufs& c = chan_[di];
  if (world_ == 1) {
    eng_->dense_bwd(act_[d.x], c.w, act_[d.y], grad_[d.y], d.need_dx ? grad_[d.x] : nullptr, c.gw, c.gb, Bl_, d.K, d.N,
                    d.act, is_dpre, below ? act_[below->y] : nullptr, below ? below->act : ACT_NONE);
    return;
  }
  std::vector<int64_t> sc(world_, 0), rc(world_, 0);
  int64_t o = 0;
  for (int p = 0; p < world_; ++p) {
    const auto it = std::find(d.holders.begin(), d.holders.end(), p);
    if (it == d.holders.end()) continue;
    const int jj = (int)(it - d.holders.begin());
    eng_->copy2d(csend_ + o, (size_t)d.Nc * 4, grad_[d.y] + (int64_t)jj * d.Nc, (size_t)d.N * 4, (size_t)d.Nc * 4, Bl_);
    sc[p] = (int64_t)Bl_ * d.Nc;
    o += sc[p];
  }
  if (d.j >= 0) std::fill(rc.begin(), rc.end(), (int64_t)Bl_ * d.Nc);
  eng_->all_to_all(csend_, sc.data(), d.j >= 0 ? c.dy : crecv_, rc.data());
  // the layer below's activation output for the global batch is this layer's gathered input
  if (d.j >= 0)
    eng_->dense_bwd(c.x, c.w, c.y, c.dy, d.need_dx ? c.dx : nullptr, c.gw, c.gb, B_, d.K, d.Nc, d.act, is_dpre,
                    below ? c.x : nullptr, below ? below->act : ACT_NONE);
  if (!d.need_dx) return;
  std::fill(sc.begin(), sc.end(), d.j >= 0 ? (int64_t)Bl_ * d.K : 0);
  std::fill(rc.begin(), rc.end(), 0);
  for (int h : d.holders) rc[h] = (int64_t)Bl_ * d.K;
  eng_->all_to_all(d.j >= 0 ? c.dx : csend_, sc.data(), crecv_, rc.data());
  o = 0;
  bool first = true;
  for (int p = 0; p < world_; ++p) {
    if (rc[p] == 0) continue;
    if (first) eng_->copy(grad_[d.x], crecv_ + o, (size_t)Bl_ * d.K * 4);
    else eng_->add(grad_[d.x], crecv_ + o, (int64_t)Bl_ * d.K);
    first = false;
    o += rc[p];
  }
}

StepStat Model::train_step(const float* x, const int64_t* const* sparse, const void* labels) {
  if (!compiled_) throw std::logic_error("native model: train_step before compile");
  if (!embs_.empty() && !sparse) throw std::invalid_argument("native model: this model needs sparse inputs");
  const Dense& last = ops_[dense_out_node()];
  const int C = last.N;
  // this rank's sample shard of the global batch; the owned tables' GLOBAL indices
  const int64_t r0 = (int64_t)rank_ * Bl_;
  // the batch uploads are issued back to back with ONE sync (the caller's host arrays may change after
  // train_step returns)
  const size_t lab_row = loss_ == LOSS_SCCE ? 4 : (size_t)C * 4;
  std::vector<const void*> srcs{x + r0 * cols_[input_], static_cast<const char*>(labels) + r0 * lab_row};
  for (size_t t = 0; t < embs_.size(); ++t)
    if (slice_of(embs_[t], rank_) >= 0) srcs.push_back(sparse[embs_[t].sparse]);
  std::function<void()> idx_upload;
  if (char* pin = static_cast<char*>(eng_->pinned(in_bytes_))) {
    // packed into page-locked memory, one asynchronous upload (the previous step's final sync has
    // released the staging buffer)
    for (size_t k = 0; k < srcs.size(); ++k) std::memcpy(pin + in_parts_[k].first, srcs[k], in_parts_[k].second);
    // the dense input and labels on the compute stream; the table indices (most of the bytes) go up
    // with the lookups (on the side queue at one rank), so the bottom MLP starts after the small copy
    const size_t head = srcs.size() > 2 ? in_parts_[2].first : in_bytes_;
    eng_->h2d_nosync(in_arena_, pin, head);
    if (head < in_bytes_) idx_upload = [this, pin, head]() { eng_->h2d_nosync(in_arena_ + head, pin + head, in_bytes_ - head); };
  } else {
    for (size_t k = 0; k < srcs.size(); ++k) eng_->h2d_nosync(in_arena_ + in_parts_[k].first, srcs[k], in_parts_[k].second);
    eng_->sync();
  }
  eng_->zero(stats_, 16 * sizeof(float));

  // embedding lookups (owners, global batch) and the exchange to the sample shards, issued ahead
  // of the first consumer
  auto emb_forward = [&]() {
    std::vector<Engine::EmbJob> jobs;
    for (size_t t = 0; t < embs_.size(); ++t) {
      const Emb& e = embs_[t];
      if (slice_of(e, rank_) < 0) continue;
      jobs.push_back({table_[t], e.nrows, idx_[t], e.bag, world_ > 1 ? emb_full_[t] : act_[e.y], e.Dc, e.lo});
    }
    if (!jobs.empty()) eng_->emb_fwd_multi(jobs, B_);
    if (world_ == 1 || embs_.empty()) return;
    // pack: per peer p, every held slice's rows [p*Bl, (p+1)*Bl)
    int64_t o = 0;
    for (int p = 0; p < world_; ++p)
      for (size_t t = 0; t < embs_.size(); ++t) {
        const Emb& e = embs_[t];
        if (slice_of(e, rank_) < 0) continue;
        eng_->copy(xsend_ + o, emb_full_[t] + (int64_t)p * Bl_ * e.Dc, (size_t)Bl_ * e.Dc * 4);
        o += (int64_t)Bl_ * e.Dc;
      }
    eng_->all_to_all(xsend_, xcount_send_.data(), xrecv_, xcount_recv_.data());
    o = 0;
    // row blocks: the holders' partial bag sums add up -- the FIRST block received (peer order, which
    // need not be slice order: holders {3, 1}) initialises the output, later ones add to it
    std::vector<char> first(embs_.size(), 1);
    for (int p = 0; p < world_; ++p)
      for (size_t t = 0; t < embs_.size(); ++t) {
        const Emb& e = embs_[t];
        const int j = slice_of(e, p);
        if (j < 0) continue;
        if (e.rows_split && !first[t])
          eng_->add(act_[e.y], xrecv_ + o, (int64_t)Bl_ * e.D);
        else
          eng_->copy2d(act_[e.y] + (e.rows_split ? 0 : (int64_t)j * e.Dc), (size_t)e.D * 4, xrecv_ + o, (size_t)e.Dc * 4,
                       (size_t)e.Dc * 4, Bl_);
        first[t] = 0;
        o += (int64_t)Bl_ * e.Dc;
      }
  };
  // one rank: the lookups run on the engine's side queue beside the bottom MLP, joined before the
  // interaction (with ranks, the exchange's RCCL calls stay in program order on one stream)
  const bool side = world_ == 1 && !embs_.empty();
  if (side) eng_->side_begin();
  if (idx_upload) idx_upload();
  emb_forward();
  if (side) eng_->side_end();
  // forward in creation order
  for (const Node& n : nodes_) {
    if (n.kind == K_DENSE) {
      const Dense& d = ops_[n.idx];
      if (!d.holders.empty()) {
        dense_split_fwd(d, n.idx);
        continue;
      }
      eng_->dense_fwd(act_[d.x], params_ + pofs_[d.w], d.b >= 0 ? params_ + pofs_[d.b] : nullptr, act_[d.y], Bl_, d.K,
                      d.N, d.act);
    } else if (n.kind == K_DOT) {
      const Dot& d = dots_[n.idx];
      std::vector<const float*> z;
      for (int t : d.in) z.push_back(act_[t]);
      eng_->side_join();
      eng_->dot_fwd(z.data(), (int)z.size(), act_[d.y], Bl_, d.D, d.W);
    } else if (n.kind == K_CONV) {
      const Conv& c = convs_[n.idx];
      eng_->conv_fwd(act_[c.x], params_ + pofs_[c.w], c.b >= 0 ? params_ + pofs_[c.b] : nullptr, act_[c.y], Bl_, c);
    } else if (n.kind == K_POOL) {
      const Pool& pl = pools_[n.idx];
      eng_->pool_fwd(act_[pl.x], act_[pl.y], pool_code_[n.idx], Bl_, pl);
    } else if (n.kind == K_BN) {
      const BNorm& b = bns_[n.idx];
      eng_->bn_fwd(act_[b.x], act_[b.y], params_ + pofs_[b.g], params_ + pofs_[b.b], bn_buf_[n.idx], Bl_, b);
    }
  }
  // loss: gradient scaled by 1 / global batch (the reference's convention), so summing the
  // ranks' gradients gives the global mean gradient
  const float* pred = act_[last.y];
  if (loss_ == LOSS_SCCE) {
    eng_->softmax(act_[last.y], probs_, Bl_, C);
    pred = probs_;
  }
  eng_->loss(loss_, pred, labels_, grad_[last.y], Bl_, C, 1.f / (float)B_, stats_);
  // backward (reverse creation order) with bucketed gradient all-reduces of the dense entries
  std::vector<int> left;
  for (auto& b : wplan_.buckets) left.push_back((int)b.size() - 2);
  std::vector<int> bucket_of(pnumel_.size(), -1);
  for (size_t bi = 0; bi < wplan_.buckets.size(); ++bi)
    for (size_t k = 2; k < wplan_.buckets[bi].size(); ++k) bucket_of[porder_[wplan_.buckets[bi][k]]] = (int)bi;
  // a final bucket: all-reduced, or under ZeRO-1 reduce-scattered into this rank's gradient slice
  auto bucket_done = [&](int bi) {
    const int64_t b0 = wplan_.buckets[bi][0], n = wplan_.buckets[bi][1] - b0;
    if (zero_on()) eng_->reduce_scatter_start(grads_ + b0, n, zgrad_ + zshard_off_[bi]);
    else eng_->allreduce_start(grads_ + b0, n);
  };
  // embedding gradients back to the owners (reverse exchange), then sparse SGD of the touched rows;
  // with one rank issued on the side queue right after the interaction backward (beside the bottom
  // MLP's backward), else after the dense backward
  bool emb_bwd_done = embs_.empty();
  auto emb_backward = [&]() {
    if (world_ > 1) {
      int64_t o = 0;
      for (int p = 0; p < world_; ++p)
        for (size_t t = 0; t < embs_.size(); ++t) {
          const Emb& e = embs_[t];
          const int j = slice_of(e, p);
          if (j < 0) continue;
          // (row blocks: every holder gets the whole gradient, j * Dc = 0 columns offset)
          eng_->copy2d(xrecv_ + o, (size_t)e.Dc * 4, grad_[e.y] + (e.rows_split ? 0 : (int64_t)j * e.Dc), (size_t)e.D * 4,
                       (size_t)e.Dc * 4, Bl_);
          o += (int64_t)Bl_ * e.Dc;
        }
      eng_->all_to_all(xrecv_, xcount_recv_.data(), xsend_, xcount_send_.data());
      o = 0;
      for (int p = 0; p < world_; ++p)
        for (size_t t = 0; t < embs_.size(); ++t) {
          const Emb& e = embs_[t];
          if (slice_of(e, rank_) < 0) continue;
          eng_->copy(emb_full_[t] + (int64_t)p * Bl_ * e.Dc, xsend_ + o, (size_t)Bl_ * e.Dc * 4);
          o += (int64_t)Bl_ * e.Dc;
        }
    }
    std::vector<Engine::EmbJob> jobs;
    for (size_t t = 0; t < embs_.size(); ++t) {
      const Emb& e = embs_[t];
      if (slice_of(e, rank_) < 0) continue;
      jobs.push_back({table_[t], e.nrows, idx_[t], e.bag, world_ > 1 ? emb_full_[t] : grad_[e.y], e.Dc, e.lo});
    }
    if (!jobs.empty()) eng_->emb_sgd_multi(jobs, B_, lr_);
    emb_bwd_done = true;
  };
  for (int ni = (int)nodes_.size() - 1; ni >= 0; --ni) {
    const Node& n = nodes_[ni];
    if (n.kind == K_DENSE) {
      const Dense& d = ops_[n.idx];
      const Dense* below = d.fuse_below ? &ops_[d.below] : nullptr;
      const bool is_dpre = d.grad_is_dpre || d.skip_act_grad;
      if (!d.holders.empty()) {
        dense_split_bwd(d, n.idx, below, is_dpre);
        continue;
      }
      eng_->dense_bwd(act_[d.x], params_ + pofs_[d.w], act_[d.y], grad_[d.y], d.need_dx ? grad_[d.x] : nullptr,
                      grads_ + pofs_[d.w], d.b >= 0 ? grads_ + pofs_[d.b] : nullptr, Bl_, d.K, d.N, d.act, is_dpre,
                      below ? act_[below->y] : nullptr, below ? below->act : ACT_NONE);
      if (world_ > 1) {
        for (int e : {d.w, d.b}) {
          if (e < 0) continue;
          const int bi = bucket_of[e];
          if (--left[bi] == 0)
            bucket_done(bi);
        }
      }
    } else if (n.kind == K_CONV) {
      const Conv& c = convs_[n.idx];
      eng_->conv_bwd(act_[c.x], params_ + pofs_[c.w], act_[c.y], grad_[c.y], c.need_dx ? grad_[c.x] : nullptr,
                     grads_ + pofs_[c.w], c.b >= 0 ? grads_ + pofs_[c.b] : nullptr, Bl_, c);
      if (world_ > 1) {
        for (int e : {c.w, c.b}) {
          if (e < 0) continue;
          const int bi = bucket_of[e];
          if (--left[bi] == 0)
            bucket_done(bi);
        }
      }
    } else if (n.kind == K_POOL) {
      const Pool& pl = pools_[n.idx];
      if (pl.need_dx) eng_->pool_bwd(act_[pl.x], act_[pl.y], grad_[pl.y], grad_[pl.x], pool_code_[n.idx], Bl_, pl);
    } else if (n.kind == K_BN) {
      const BNorm& b = bns_[n.idx];
      eng_->bn_bwd(act_[b.x], act_[b.y], grad_[b.y], params_ + pofs_[b.g], bn_buf_[n.idx], grads_ + pofs_[b.g],
                   grads_ + pofs_[b.b], b.need_dx ? grad_[b.x] : nullptr, Bl_, b);
      if (world_ > 1) {
        for (int e : {b.g, b.b}) {
          const int bi = bucket_of[e];
          if (--left[bi] == 0)
            bucket_done(bi);
        }
      }
    } else if (n.kind == K_DOT) {
      const Dot& d = dots_[n.idx];
      std::vector<const float*> z;
      std::vector<float*> dz;
      for (int t : d.in) {
        z.push_back(act_[t]);
        dz.push_back(grad_[t]);
      }
      eng_->dot_bwd(z.data(), (int)z.size(), grad_[d.y], dz.data(), Bl_, d.D, d.W, d.act0);
      if (side && !emb_bwd_done) {
        eng_->side_begin();
        emb_backward();
        eng_->side_end();
      }
    }
  }
  if (!emb_bwd_done) emb_backward();
  eng_->side_join();
  if (world_ > 1) eng_->allreduce_wait();
  const OptStep os = next_step();
  if (zero_on()) {
    // ZeRO-1: update this rank's fp32 slices with their state, then all-gather the fresh slices
    if (zdirty_) {
      for (size_t bi = 0; bi < wplan_.buckets.size(); ++bi) {
        const int64_t b0 = wplan_.buckets[bi][0], k = (wplan_.buckets[bi][1] - b0) / world_;
        eng_->copy(zmaster_ + zshard_off_[bi], params_ + b0 + (int64_t)rank_ * k, (size_t)k * 4);
      }
      zdirty_ = false;
    }
    eng_->zero(grads_, (size_t)wplan_.numel * 4);   // the reduce-scatter consumed the gradients
    eng_->opt_update(zmaster_, zgrad_, ostate_[0], ostate_[1], zshard_n_, os);
    for (size_t bi = 0; bi < wplan_.buckets.size(); ++bi) {
      const int64_t b0 = wplan_.buckets[bi][0], k = (wplan_.buckets[bi][1] - b0) / world_;
      eng_->all_gather(zmaster_ + zshard_off_[bi], k, params_ + b0);
    }
  } else if (opt_.plain()) {
    eng_->sgd(params_, grads_, wplan_.numel, lr_);
  } else {
    eng_->opt_update(params_, grads_, ostate_[0], ostate_[1], wplan_.numel, os);
  }
  for (size_t i = 0; i < ops_.size(); ++i) {
    const Dense& d = ops_[i];
    if (d.j < 0) continue;
    const auto& cs = chan_state_[i];
    if (opt_.plain()) {
      eng_->sgd(chan_[i].w, chan_[i].gw, (int64_t)d.Nc * d.K, lr_);
      if (chan_[i].b) eng_->sgd(chan_[i].b, chan_[i].gb, d.Nc, lr_);
    } else {
      eng_->opt_update(chan_[i].w, chan_[i].gw, cs[0], cs[1], (int64_t)d.Nc * d.K, os);
      if (chan_[i].b) eng_->opt_update(chan_[i].b, chan_[i].gb, cs[2], cs[3], d.Nc, os);
    }
  }
  float st[16];
  eng_->sync();
  eng_->d2h(st, stats_, sizeof(st));
  StepStat s;
  s.loss = st[eng_->stat_slot(0)] / Bl_;
  s.correct = (int64_t)st[eng_->stat_slot(1)];
  s.samples = Bl_;
  return s;
}

std::string Model::describe() const {
  std::ostringstream o;
  o << "native model: global batch " << B_ << " over " << world_ << " rank(s) (" << Bl_ << " per rank), engine "
    << (device_ == 1 ? "hip" : "cpu") << "\n";
  for (const Node& n : nodes_) {
    if (n.kind == K_DENSE) {
      const Dense& d = ops_[n.idx];
      o << "  dense" << n.idx << ": " << d.K << " -> " << d.N << " act " << d.act
        << (d.fuse_below ? " [dX epilogue: act' below]" : "") << (d.grad_is_dpre ? " [grad arrives as dpre]" : "")
        << (d.skip_act_grad ? " [sigmoid folded into BCE]" : "");
      if (!d.holders.empty()) {
        o << " channel-split over ranks";
        for (int h : d.holders) o << " " << h;
        o << " (" << d.Nc << " features each" << (d.j >= 0 ? "; local slice" : "") << ")";
      }
      o << "\n";
    } else if (n.kind == K_EMB) {
      const Emb& e = embs_[n.idx];
      if (e.rows_split) {
        o << "  embedding" << n.idx << ": " << e.rows << " x " << e.D << " bag " << e.bag << " row-split over ranks";
        for (int h : e.holders) o << " " << h;
        o << " (partial bag sums added" << (slice_of(e, rank_) >= 0 ? "; local rows " : "");
        if (slice_of(e, rank_) >= 0) o << e.lo << ".." << e.lo + e.nrows;
        o << ")\n";
      } else if (e.holders.size() > 1) {
        o << "  embedding" << n.idx << ": " << e.rows << " x " << e.D << " bag " << e.bag << " column-split over ranks";
        for (int h : e.holders) o << " " << h;
        o << " (" << e.Dc << " columns each" << (slice_of(e, rank_) >= 0 ? "; local slice" : "") << ")\n";
      } else {
        o << "  embedding" << n.idx << ": " << e.rows << " x " << e.D << " bag " << e.bag << " on rank " << e.owner
          << (e.owner == rank_ ? " (local: global-batch lookups, sparse SGD)" : "") << "\n";
      }
    } else if (n.kind == K_CONV) {
      const Conv& c = convs_[n.idx];
      o << "  conv" << n.idx << ": " << c.C << "x" << c.H << "x" << c.W << " -> " << c.K << "x" << c.P << "x" << c.Q << " kernel "
        << c.R << "x" << c.S << " stride " << c.sh << "x" << c.sw << " pad " << c.ph << "x" << c.pw << " act " << c.act
        << " (data parallel)\n";
    } else if (n.kind == K_BN) {
      const BNorm& b = bns_[n.idx];
      o << "  batchnorm" << n.idx << ": " << b.C << "x" << b.H << "x" << b.W << (b.relu ? " relu" : "")
        << " (local-shard statistics, data parallel)\n";
    } else if (n.kind == K_POOL) {
      const Pool& pl = pools_[n.idx];
      o << "  pool" << n.idx << " " << (pl.max ? "max" : "avg") << ": " << pl.C << "x" << pl.H << "x" << pl.W << " -> " << pl.C
        << "x" << pl.P << "x" << pl.Q << " window " << pl.kh << "x" << pl.kw << " stride " << pl.sh << "x" << pl.sw << "\n";
    } else {
      const Dot& d = dots_[n.idx];
      o << "  dot interaction: " << d.in.size() << " features x " << d.D << " -> " << d.W
        << (d.act0 != ACT_NONE ? " [backward applies the bottom layer's act']" : "") << "\n";
    }
  }
  if (!embs_.empty() && world_ > 1) {
    o << "  embedding exchange (all-to-all) floats per peer: send";
    for (auto c : xcount_send_) o << " " << c;
    o << " / recv";
    for (auto c : xcount_recv_) o << " " << c;
    o << "\n";
  }
  if (opt_.type == OPT_ADAM)
    o << "  optimizer: adam alpha " << lr_ << " beta1 " << opt_.beta1 << " beta2 " << opt_.beta2 << " eps " << opt_.eps
      << " weight decay " << opt_.weight_decay << "\n";
  else
    o << "  optimizer: sgd lr " << lr_ << " momentum " << opt_.momentum << (opt_.nesterov ? " nesterov" : "")
      << " weight decay " << opt_.weight_decay << "\n";
  if (zero_on())
    o << "  ZeRO-1: buckets reduce-scattered, optimizer state for this rank's " << zshard_n_ << " of " << wplan_.numel
      << " floats, slices all-gathered after the update\n";
  o << "  flat parameters " << wplan_.numel << " floats, " << wplan_.buckets.size()
    << (zero_on() ? " reduce-scatter bucket(s)\n" : " all-reduce bucket(s)\n");
  for (auto& b : wplan_.buckets) {
    o << "    [" << b[0] << ", " << b[1] << ") entries";
    for (size_t k = 2; k < b.size(); ++k) o << " " << porder_[b[k]];
    o << "\n";
  }
  return o.str();
}

}  // namespace nm
}  // namespace flexmi
