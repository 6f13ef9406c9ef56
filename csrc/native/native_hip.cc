// HIP engine of the native model (native_model.h): flexmi's gfx950 kernels (linked from
// libflexmi_kernels.so, no PyTorch) and flexmi's own RCCL communicator.
//
//   dense forward  fm_gemm_f32 (the exact three-way bf16 split or v_mfma_f32_16x16x4_f32, bias +
//                  activation in the epilogue; the executor's measured GEMM table picks the form) or
//                  the skinny N = 1 kernel
//   dense backward fm_act_bwd_bias (act'), fm_gemm_f32 dW (+= , bias gradient as the staged A
//                  tiles' row sums) and dX (activation backward of the layer below fused into
//                  the epilogue) -- the same kernel sequence as flexmi/ops/_kernels.py linear_backward
//   loss / SGD     fm_loss_fwd_bwd, fm_sgd_update (zeroes the consumed gradients)
//   embeddings     fm_embedding_fwd (global-batch lookups on the owner), fm_embedding_bwd with a
//                  device lr (fused sparse SGD of the touched rows); fm_dot_interaction_{fwd,bwd}_f32
//                  (v_mfma_f32_32x32x2_f32); the exchange = RCCL grouped send / recv per peer
//   convolutions   fm_conv_fwd / fm_conv_act_bwd / fm_conv_wgrad / fm_conv_dgrad (fp32 implicit GEMM
//                  on MFMA), fm_pool_fwd / fm_pool_bwd, fm_bn_fwd / fm_bn_bwd -- the Python executor's Conv2D /
//                  Pool2D / BatchNorm kernels
//   communication  one RCCL communicator per model (unique id handed over through a file in the
//                  rendezvous directory); bucket all-reduces on a second HIP stream, started as
//                  soon as the bucket's last gradient kernel is enqueued (event dependency) and
//                  joined before the update -- overlapped with the rest of the backward.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <unistd.h>
#include <unordered_map>
#include <vector>

#include "native_model.h"

extern "C" {
int fm_gemm_f32(const float* A, long lda, long sA, int a_kcontig, const float* B, long ldb, long sB, int b_kcontig, float* C,
                long ldc, long sC, const float* bias, int M, int N, int K, int batch, float alpha, int beta, int act, float* ws,
                long ws_bytes, int ksplit_req, const float* act_y, long lday, int bwd_act, float* colsum, float* rowsum_a,
                hipStream_t stream);
void fm_skinny_fwd_f32_launch(const float* x, long ldx, const float* w, const float* bias, float* y, long ldy, long B, int K,
                              int act, hipStream_t s);
void fm_skinny_bwd_f32_launch(const float* x, long ldx, const float* w, const float* y, long ldy, const float* dy, long lddy,
                              float* dx, long lddx, int dx_acc, float* dw, float* db, long B, int K, int act, int bact,
                              hipStream_t s);
void fm_act_bwd_bias(const void* y, const void* dy, void* dpre, float* db, long B, int N, int act, int bf16, hipStream_t s);
void fm_softmax_fwd(const void* x, void* y, long rows, int C, int bf16, hipStream_t s);
void fm_loss_fwd_bwd(const void* logits, int logits_bf16, const void* labels, void* grad, int grad_bf16, long B, int C,
                     int loss_type, float scale, float* acc, int mask, float clamp_t, hipStream_t s);
void fm_sgd_update(float* W, float* G, float* V, unsigned short* Wc, const float* lr, long n, float wd, float mom, int nesterov,
                   int zero_g, hipStream_t s);
int fm_smallk_fwd_launch(const void* x, long ldx, const void* w, const float* bias, void* y, long ldy, long M, int K, int N,
                         int act, int bf16, hipStream_t s);
int fm_smallk_dw_launch(const void* dpre, long ldd, const void* x, long ldx, float* dw, float* db, long M, int K, int N,
                        float* ws, long ws_bytes, float* V, unsigned short* Wc, const float* lr, float wd, float mom,
                        int nesterov, int bf16, hipStream_t s);
void fm_adam_update(float* W, float* G, float* M, float* V, unsigned short* Wc, long n, const float* alpha_t, float b1, float b2,
                    float wd, float eps, int zero_g, hipStream_t s);
void fm_embedding_fwd_multi(int n, const float* const* W, const void* const* idx, const int* idx64, void* const* out,
                            const long* ldo, const long* lo, const int* rows, const int* D, const int* bag,
                            const float* scale, int out_bf16, long B, hipStream_t st);
void fm_embedding_bwd_multi(int n, float* const* W, const void* const* idx, const int* idx64, const void* const* dy,
                            const long* ldg, const long* lo, const int* rows, const int* D, const int* bag,
                            const float* scale, int dy_bf16, const float* lr, long B, int* const* owner,
                            int* const* dups, int* const* ndup, hipStream_t st);
void fm_binary_forward(int code, const void* a, const void* b, void* y, long n, int relu, int bf16, hipStream_t s);
void fm_embedding_fwd(const void* idx, int idx64, const float* W, void* out, int out_bf16, long B, int bag, int rows, int D,
                      long ldo, float scale, hipStream_t s);
void fm_embedding_bwd(const void* idx, int idx64, const void* dy, int dy_bf16, float* W, const float* lr, long B, int bag,
                      int rows, int D, long ldg, float scale, hipStream_t s);
void fm_dot_interaction_fwd_f32(const float* const* z, int F, long ldz, float* out, long ldo, long B, int D, int W, int self,
                                hipStream_t s);
void fm_dot_interaction_bwd_f32(const float* const* z, int F, long ldz, const float* dout, long ldo, float* const* dz,
                                long lddz, unsigned acc_mask, long B, int D, int self, int act0, hipStream_t s);
int fm_conv_lda(int cols);
int fm_conv_fwd(const void* x, const void* w, void* wpad, const float* bias, void* y, int bf16, int N, int C, int H, int W,
                int K, int R, int S, int P, int Q, int sh, int sw, int pt, int pl, int act, hipStream_t s);
int fm_conv_dgrad(const void* g, const void* w, void* wt, void* dx, int accum, int bf16, int N, int C, int H, int W, int K,
                  int R, int S, int P, int Q, int sh, int sw, int pt, int pl, hipStream_t s);
int fm_conv_wgrad(const void* g, const void* x, float* dw, int bf16, int N, int C, int H, int W, int K, int R, int S, int P,
                  int Q, int sh, int sw, int pt, int pl, hipStream_t s);
void fm_conv_act_bwd(const void* dy, const void* y, void* g, float* db, int bf16, int N, int K, int PQ, int act,
                     hipStream_t s);
void fm_pool_fwd(const void* x, void* y, unsigned char* code, int N, int C, int H, int W, int P, int Q, int kh, int kw,
                 int sh, int sw, int pt, int pl, int is_max, int act, int bf16, hipStream_t st);
void fm_pool_bwd(const void* x, const void* y, const void* dy, void* dx, unsigned char* code, int code_ready, int N, int C,
                 int H, int W, int P, int Q, int kh, int kw, int sh, int sw, int pt, int pl, int is_max, int act, int acc,
                 int bf16, hipStream_t st);
void fm_bn_fwd(const void* x, void* y, const float* gamma, const float* beta, float* stats, float* meaninv, int N, int C,
               int HW, float eps, int relu, int bf16, hipStream_t st);
void fm_bn_bwd(const void* x, const void* y, const void* dy, const float* meaninv, const float* gamma, float* gsum,
               float* dgamma, float* dbeta, void* dx, int N, int C, int HW, int relu, int acc, int bf16, hipStream_t st);
}

namespace flexmi {
namespace nm {

namespace {

#define HIPX(x)                                                                                            \
  do {                                                                                                     \
    hipError_t e_ = (x);                                                                                   \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("native hip engine: ") + #x + ": " + hipGetErrorString(e_)); \
  } while (0)
#define NCCLX(x)                                                                                           \
  do {                                                                                                     \
    ncclResult_t r_ = (x);                                                                                 \
    if (r_ != ncclSuccess) throw std::runtime_error(std::string("native hip engine: ") + #x + ": " + ncclGetErrorString(r_)); \
  } while (0)

constexpr long WS_BYTES = 64L << 20;   // split-K slabs of the dW GEMMs

// The measured GEMM configuration table the Python executor uses (flexmi/ops/gemm_tune.py: key ->
// cfg = split depth | form << 8), read from flexmi/ops/tuned/gemm_mi355x.json next to this library
// (FM_GEMM_TUNE: 0 = off, or another table's path).  Keys as gemm_tune.key: dtype|MxNxK|orientations
// |batch|fused epilogues|C dtype.  A missing table or key means the kernels' own heuristic.
class TuneTable {
 public:
  static const TuneTable& get() {
    static const TuneTable t;
    return t;
  }
  int cfg(int M, int N, int K, bool a_k, bool b_k, bool act_y, bool rowsum) const {
    if (m_.empty()) return 0;
    char k[160];
    std::snprintf(k, sizeof(k), "fp32|%dx%dx%d|%c%c|b1|%s|c32", M, N, K, a_k ? 'k' : 'm', b_k ? 'k' : 'm',
                  act_y ? "y" : rowsum ? "r" : "-");
    auto it = m_.find(k);
    return it == m_.end() ? 0 : it->second;
  }

 private:
  TuneTable() {
    const char* env = std::getenv("FM_GEMM_TUNE");
    std::string path;
    if (env && std::string(env) == "0") return;
    if (env && *env && std::string(env) != "1") {
      path = env;
    } else {
      Dl_info info;
      if (!dladdr(reinterpret_cast<void*>(&TuneTable::get), &info) || !info.dli_fname) return;
      const std::string lib = info.dli_fname;
      const size_t slash = lib.rfind('/');
      path = (slash == std::string::npos ? std::string(".") : lib.substr(0, slash)) + "/ops/tuned/gemm_mi355x.json";
    }
    std::ifstream f(path);
    if (!f) return;
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string j = ss.str();
    // entries: "<key with '|'>": { ... "cfg": <int>, ... }
    size_t pos = 0;
    while ((pos = j.find('"', pos)) != std::string::npos) {
      const size_t end = j.find('"', pos + 1);
      if (end == std::string::npos) break;
      const std::string key = j.substr(pos + 1, end - pos - 1);
      pos = end + 1;
      if (key.find('|') == std::string::npos) continue;
      const size_t open = j.find('{', pos), close = j.find('}', pos);
      if (open == std::string::npos || close == std::string::npos || open > close) continue;
      const size_t c = j.find("\"cfg\"", open);
      if (c == std::string::npos || c > close) continue;
      const size_t colon = j.find(':', c);
      const int v = std::atoi(j.c_str() + colon + 1);
      if (v > 0) m_[key] = v;
      pos = close + 1;
    }
  }
  std::unordered_map<std::string, int> m_;
};

// the multi-table embedding launchers' parallel arrays
struct EmbArrays {
  explicit EmbArrays(const std::vector<Engine::EmbJob>& jobs) : n((int)jobs.size()) {
    for (const Engine::EmbJob& j : jobs) {
      W.push_back(j.W);
      Wc.push_back(j.W);
      ix.push_back(j.idx);
      i64.push_back(1);
      o.push_back(j.io);
      ld.push_back(j.D);
      l0.push_back((long)j.lo);
      r.push_back((int)j.rows);
      D.push_back(j.D);
      bag.push_back(j.bag);
      sc.push_back(1.f);
    }
  }
  int n;
  std::vector<float*> W;
  std::vector<const float*> Wc;
  std::vector<const void*> ix;
  std::vector<int> i64;
  std::vector<void*> o;
  std::vector<long> ld, l0;
  std::vector<int> r, D, bag;
  std::vector<float> sc;
};

class HipEngine : public Engine {
 public:
  HipEngine(int rank, int world, const std::string& rendezvous) : rank_(rank), world_(world) {
    int ndev = 0;
    HIPX(hipGetDeviceCount(&ndev));
    if (ndev <= 0) throw std::runtime_error("native hip engine: no GPU");
    HIPX(hipSetDevice(rank % ndev));
    HIPX(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
    HIPX(hipStreamCreateWithFlags(&comm_st_, hipStreamNonBlocking));
    HIPX(hipStreamCreateWithFlags(&side_st_, hipStreamNonBlocking));
    main_st_ = st_;
    HIPX(hipMalloc(&ws_, WS_BYTES));
    HIPX(hipMalloc(&slots_, 16 * sizeof(float)));
    HIPX(hipMalloc(&lr_, sizeof(float)));
    if (world > 1) init_comm(rendezvous);
  }
  ~HipEngine() override {
    hipStreamSynchronize(st_);
    hipStreamSynchronize(comm_st_);
    hipStreamSynchronize(side_st_);
    for (auto e : events_) hipEventDestroy(e);
    if (comm_) ncclCommDestroy(comm_);
    hipFree(ws_);
    for (float* b : bufs_)
      if (b) hipFree(b);
    hipFree(slots_);
    hipFree(lr_);
    hipStreamDestroy(comm_st_);
    hipStreamDestroy(side_st_);
    if (pinned_) hipHostFree(pinned_);
    for (auto& kv : claim_) {
      hipFree(kv.second.owner);
      hipFree(kv.second.dups);
      hipFree(kv.second.ndup);
    }
    hipStreamDestroy(st_);
  }

  void* alloc(size_t bytes) override {
    void* p = nullptr;
    HIPX(hipMalloc(&p, std::max<size_t>(bytes, 256)));
    HIPX(hipMemsetAsync(p, 0, std::max<size_t>(bytes, 256), st_));
    return p;
  }
  void release(void* p) override { hipFree(p); }
  void h2d(void* dst, const void* src, size_t bytes) override {
    HIPX(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st_));
    HIPX(hipStreamSynchronize(st_));   // the host buffer may be reused right after
  }
  void d2h(void* dst, const void* src, size_t bytes) override {
    HIPX(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st_));
    HIPX(hipStreamSynchronize(st_));
  }
  void sync() override {
    HIPX(hipStreamSynchronize(main_st_));
    HIPX(hipStreamSynchronize(side_st_));
    if (!pending_) ev_next_ = 0;   // every recorded event has completed: the pool is reusable
  }
  // the side queue: every kernel launch goes to st_, which points at the main or the side stream
  void side_begin() override {
    if (st_ == side_st_) return;
    hipEvent_t e = event();
    HIPX(hipEventRecord(e, main_st_));
    HIPX(hipStreamWaitEvent(side_st_, e, 0));
    st_ = side_st_;
  }
  void side_end() override {
    if (st_ != side_st_) return;
    st_ = main_st_;
    side_pending_ = true;
  }
  void side_join() override {
    if (!side_pending_) return;
    hipEvent_t e = event();
    HIPX(hipEventRecord(e, side_st_));
    HIPX(hipStreamWaitEvent(main_st_, e, 0));
    side_pending_ = false;
  }

  void dense_fwd(const float* x, const float* W, const float* b, float* y, int M, int K, int N, int act) override {
    // thin inputs (K <= 32, K % 4 == 0: the DLRM bottom layer on its padded 16 features) on the
    // executor's gemm_small kernel
    if (K <= 32 && fm_smallk_fwd_launch(x, K, W, b, y, N, M, K, N, act, 0, st_) == 0) return;
    if (N == 1) {
      fm_skinny_fwd_f32_launch(x, K, W, b, y, 1, M, K, act, st_);
      return;
    }
    const int cfg = TuneTable::get().cfg(M, N, K, true, true, false, false);
    fm_gemm_f32(x, K, 0, 1, W, K, 0, 1, y, N, 0, b, M, N, K, 1, 1.f, 0, act, ws_, WS_BYTES, cfg, nullptr, 0, ACT_NONE, nullptr,
                nullptr, st_);
  }

  void dense_bwd(const float* x, const float* W, const float* y, const float* dy, float* dx, float* dW, float* db, int M,
                 int K, int N, int act, bool grad_is_dpre, const float* y_below, int act_below) override {
    if (N == 1 && K % 4 == 0 && y_below == nullptr) {
      fm_skinny_bwd_f32_launch(x, K, W, y, 1, dy, 1, dx, K, 0, dW, db, M, K, grad_is_dpre ? ACT_NONE : act, ACT_NONE, st_);
      return;
    }
    const float* dpre = dy;
    if (!grad_is_dpre && act != ACT_NONE) {
      float* t = scratch((size_t)M * N);
      fm_act_bwd_bias(y, dy, t, nullptr, M, N, act, 0, st_);
      dpre = t;
    }
    // dW[N][K] += dpre^T x (both operands MN-contiguous), db += column sums of dpre (thin inputs:
    // gemm_small's partial / reduce pair)
    const bool thin = K <= 32 && fm_smallk_dw_launch(dpre, N, x, K, dW, db, M, K, N, ws_, WS_BYTES, nullptr, nullptr, nullptr,
                                                     0.f, 0.f, 0, 0, st_) == 0;
    if (!thin)
      fm_gemm_f32(dpre, N, 0, 0, x, K, 0, 0, dW, K, 0, nullptr, N, K, M, 1, 1.f, 1, ACT_NONE, ws_, WS_BYTES,
                  TuneTable::get().cfg(N, K, M, false, false, false, db != nullptr), nullptr, 0, ACT_NONE, nullptr, db, st_);
    if (!dx) return;
    // dX[M][K] = dpre W (+ act' of the layer below)
    fm_gemm_f32(dpre, N, 0, 1, W, K, 0, 0, dx, K, 0, nullptr, M, K, N, 1, 1.f, 0, ACT_NONE, ws_, WS_BYTES,
                TuneTable::get().cfg(M, K, N, true, false, y_below != nullptr, false), y_below, y_below ? K : 0,
                y_below ? act_below : ACT_NONE, nullptr, nullptr, st_);
  }

  void softmax(const float* x, float* y, int M, int C) override { fm_softmax_fwd(x, y, M, C, 0, st_); }

  void loss(int type, const float* p, const void* labels, float* grad, int M, int C, float scale, float* stats) override {
    // the kernel's metric slots ARE the model's stats buffer ([1] correct, [7] loss sum): no copies
    fm_loss_fwd_bwd(p, 0, labels, grad, 0, M, C, type, scale, stats, 1, 0.f, st_);
  }
  int stat_slot(int which) const override { return which == 0 ? 7 : 1; }

  void sgd(float* w, float* g, int64_t n, float lr) override {
    set_lr(lr);
    fm_sgd_update(w, g, nullptr, nullptr, lr_, n, 0.f, 0.f, 0, 1, st_);
  }

  // the executor's optimizer kernels (optim.hip): SGD with momentum / Nesterov / weight decay, Adam
  // with the device-side alpha_t; both consume the gradient
  void opt_update(float* w, float* g, float* s1, float* s2, int64_t n, const OptStep& o) override {
    set_lr(o.lr);
    const OptConfig& c = o.c;
    if (c.type == OPT_ADAM)
      fm_adam_update(w, g, s1, s2, nullptr, n, lr_, c.beta1, c.beta2, c.weight_decay, c.eps, 1, st_);
    else
      fm_sgd_update(w, g, c.momentum > 0.f ? s1 : nullptr, nullptr, lr_, n, c.weight_decay, c.momentum, c.nesterov ? 1 : 0,
                    1, st_);
  }
  void zero(void* p, size_t bytes) override { HIPX(hipMemsetAsync(p, 0, bytes, st_)); }
  // ZeRO-1 collectives on RCCL: the reduce-scatter runs on the communication stream like the bucket
  // all-reduces (overlapping the rest of the backward), the all-gather in order on the compute stream
  void reduce_scatter_start(const float* buf, int64_t n, float* out) override {
    if (!comm_) {
      HIPX(hipMemcpyAsync(out, buf, (size_t)n * sizeof(float), hipMemcpyDeviceToDevice, st_));
      return;
    }
    hipEvent_t ready = event();
    HIPX(hipEventRecord(ready, st_));
    HIPX(hipStreamWaitEvent(comm_st_, ready, 0));
    NCCLX(ncclReduceScatter(buf, out, (size_t)(n / world_), ncclFloat32, ncclSum, comm_, comm_st_));
    pending_ = true;
  }
  void all_gather(const float* in, int64_t n, float* buf) override {
    if (!comm_) {
      HIPX(hipMemcpyAsync(buf, in, (size_t)n * sizeof(float), hipMemcpyDeviceToDevice, st_));
      return;
    }
    NCCLX(ncclAllGather(in, buf, (size_t)n, ncclFloat32, comm_, st_));
  }

  void copy(void* dst, const void* src, size_t bytes) override {
    HIPX(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st_));
  }
  void copy2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t rows) override {
    HIPX(hipMemcpy2DAsync(dst, dpitch, src, spitch, width, rows, hipMemcpyDeviceToDevice, st_));
  }

  void emb_fwd(const float* W, int64_t rows, const int64_t* idx, int bag, float* out, int64_t B, int D,
               int64_t lo) override {
    const void* ix = idx;
    const int i64 = 1, r = (int)rows;
    void* o = out;
    const long ld = D, l0 = (long)lo;
    const float sc = 1.f;
    fm_embedding_fwd_multi(1, &W, &ix, &i64, &o, &ld, &l0, &r, &D, &bag, &sc, 0, B, st_);
  }
  void emb_sgd(float* W, int64_t rows, const int64_t* idx, int bag, const float* g, int64_t B, int D, float lr,
               int64_t lo) override {
    set_lr(lr);
    const void* ix = idx;
    const void* dy = g;
    const int i64 = 1, r = (int)rows;
    const long ld = D, l0 = (long)lo;
    const float sc = 1.f;
    fm_embedding_bwd_multi(1, &W, &ix, &i64, &dy, &ld, &l0, &r, &D, &bag, &sc, 0, lr_, B, nullptr, nullptr, nullptr, st_);
  }
  void emb_fwd_multi(const std::vector<EmbJob>& jobs, int64_t B) override {
    EmbArrays a(jobs);
    fm_embedding_fwd_multi(a.n, a.Wc.data(), a.ix.data(), a.i64.data(), a.o.data(), a.ld.data(), a.l0.data(), a.r.data(),
                           a.D.data(), a.bag.data(), a.sc.data(), 0, B, st_);
  }
  // the executor's owner-computes sparse SGD for mostly-unique tables (rows > 0.2 x lookups per step,
  // flexmi.ops.embedding CLAIM_RATIO): a per-row claim slot (-1 = free, restored by the owner kernel),
  // the duplicate list and its counter per table, allocated on the table's first update; the other
  // tables keep the atomic / LDS kernels
  void emb_sgd_multi(const std::vector<EmbJob>& jobs, int64_t B, float lr) override {
    set_lr(lr);
    EmbArrays a(jobs);
    std::vector<const void*> dy(a.o.begin(), a.o.end());
    std::vector<int*> owner(a.n, nullptr), dups(a.n, nullptr), ndup(a.n, nullptr);
    for (int i = 0; i < a.n; ++i) {
      const EmbJob& j = jobs[i];
      const int64_t lookups = B * j.bag;
      if ((double)j.rows <= 0.2 * (double)lookups || j.D % 4 != 0) continue;
      ClaimBufs& c = claim_[j.W];
      if (!c.owner) {
        HIPX(hipMalloc(&c.owner, (size_t)j.rows * sizeof(int)));
        HIPX(hipMemsetAsync(c.owner, 0xff, (size_t)j.rows * sizeof(int), st_));   // -1: free
        HIPX(hipMalloc(&c.dups, (size_t)std::max<int64_t>(lookups, 1) * sizeof(int)));
        HIPX(hipMalloc(&c.ndup, sizeof(int)));
        HIPX(hipMemsetAsync(c.ndup, 0, sizeof(int), st_));
        HIPX(hipStreamSynchronize(st_));
      }
      owner[i] = c.owner;
      dups[i] = c.dups;
      ndup[i] = c.ndup;
    }
    fm_embedding_bwd_multi(a.n, a.W.data(), a.ix.data(), a.i64.data(), dy.data(), a.ld.data(), a.l0.data(), a.r.data(),
                           a.D.data(), a.bag.data(), a.sc.data(), 0, lr_, B, owner.data(), dups.data(), ndup.data(), st_);
  }
  void* pinned(size_t bytes) override {
    if (bytes > pinned_n_) {
      if (pinned_) {
        HIPX(hipStreamSynchronize(main_st_));
        HIPX(hipHostFree(pinned_));
      }
      HIPX(hipHostMalloc(&pinned_, bytes, hipHostMallocDefault));
      pinned_n_ = bytes;
    }
    return pinned_;
  }
  void h2d_nosync(void* dst, const void* src, size_t bytes) override {
    HIPX(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st_));
  }
  void add(float* dst, const float* src, int64_t n) override { fm_binary_forward(0, dst, src, dst, n, 0, 0, st_); }
  void dot_fwd(const float* const* z, int F, float* y, int M, int D, int W) override {
    fm_dot_interaction_fwd_f32(z, F, D, y, W, M, D, W, 0, st_);
  }
  void dot_bwd(const float* const* z, int F, const float* dy, float* const* dz, int M, int D, int W, int act0) override {
    fm_dot_interaction_bwd_f32(z, F, D, dy, W, dz, D, 0u, M, D, 0, act0, st_);
  }
  void all_to_all(const float* send, const int64_t* send_counts, float* recv, const int64_t* recv_counts) override {
    if (!comm_) {
      HIPX(hipMemcpyAsync(recv, send, (size_t)send_counts[0] * sizeof(float), hipMemcpyDeviceToDevice, st_));
      return;
    }
    int64_t so = 0, ro = 0;
    NCCLX(ncclGroupStart());
    for (int p = 0; p < world_; ++p) {
      if (send_counts[p]) NCCLX(ncclSend(send + so, (size_t)send_counts[p], ncclFloat32, p, comm_, st_));
      if (recv_counts[p]) NCCLX(ncclRecv(recv + ro, (size_t)recv_counts[p], ncclFloat32, p, comm_, st_));
      so += send_counts[p];
      ro += recv_counts[p];
    }
    NCCLX(ncclGroupEnd());
  }

  // convolutions on flexmi's implicit-GEMM MFMA kernels (conv_igemm.hip, fp32 operands), pooling on
  // cnn.hip -- the kernels the Python executor's Conv2D / Pool2D ops run
  void conv_fwd(const float* x, const float* W, const float* b, float* y, int N, const Conv& c) override {
    float* wpad = buf(1, (size_t)c.K * fm_conv_lda(c.C * c.R * c.S));
    if (fm_conv_fwd(x, W, wpad, b, y, 0, N, c.C, c.H, c.W, c.K, c.R, c.S, c.P, c.Q, c.sh, c.sw, c.ph, c.pw, c.act, st_) != 0)
      throw std::runtime_error("native hip engine: conv forward");
  }
  void conv_bwd(const float* x, const float* W, const float* y, const float* dy, float* dx, float* dW, float* db, int N,
                const Conv& c) override {
    const float* g = dy;
    if (c.act != ACT_NONE || db) {
      float* t = c.act != ACT_NONE ? buf(0, (size_t)N * c.K * c.P * c.Q) : nullptr;
      fm_conv_act_bwd(dy, y, t ? t : const_cast<float*>(dy), db, 0, N, c.K, c.P * c.Q, c.act, st_);
      if (t) g = t;
    }
    if (fm_conv_wgrad(g, x, dW, 0, N, c.C, c.H, c.W, c.K, c.R, c.S, c.P, c.Q, c.sh, c.sw, c.ph, c.pw, st_) != 0)
      throw std::runtime_error("native hip engine: conv weight gradient");
    if (!dx) return;
    float* wt = buf(2, (size_t)c.C * fm_conv_lda(c.K * c.R * c.S));
    if (fm_conv_dgrad(g, W, wt, dx, 0, 0, N, c.C, c.H, c.W, c.K, c.R, c.S, c.P, c.Q, c.sh, c.sw, c.ph, c.pw, st_) != 0)
      throw std::runtime_error("native hip engine: conv data gradient");
  }
  void pool_fwd(const float* x, float* y, unsigned char* code, int N, const Pool& p) override {
    fm_pool_fwd(x, y, code, N, p.C, p.H, p.W, p.P, p.Q, p.kh, p.kw, p.sh, p.sw, p.ph, p.pw, p.max ? 1 : 0, ACT_NONE, 0, st_);
  }
  void pool_bwd(const float* x, const float* y, const float* dy, float* dx, const unsigned char* code, int N,
                const Pool& p) override {
    fm_pool_bwd(x, y, dy, dx, const_cast<unsigned char*>(code), 1, N, p.C, p.H, p.W, p.P, p.Q, p.kh, p.kw, p.sh, p.sw, p.ph,
                p.pw, p.max ? 1 : 0, ACT_NONE, 0, 0, st_);
  }
  // batch norm on the executor's kernels (cnn.hip): buf = stats [2C] | mean, 1/std [2C] | sums [2C]
  void bn_fwd(const float* x, float* y, const float* gamma, const float* beta, float* buf, int N, const BNorm& b) override {
    fm_bn_fwd(x, y, gamma, beta, buf, buf + 2 * b.C, N, b.C, b.H * b.W, (float)kBnEps, b.relu ? 1 : 0, 0, st_);
  }
  void bn_bwd(const float* x, const float* y, const float* dy, const float* gamma, float* buf, float* dgamma, float* dbeta,
              float* dx, int N, const BNorm& b) override {
    fm_bn_bwd(x, y, dy, buf + 2 * b.C, gamma, buf + 4 * b.C, dgamma, dbeta, dx, N, b.C, b.H * b.W, b.relu ? 1 : 0, 0, 0, st_);
  }

  void allreduce_start(float* buf, int64_t n) override {
    if (!comm_) return;
    hipEvent_t ready = event();
    HIPX(hipEventRecord(ready, st_));
    HIPX(hipStreamWaitEvent(comm_st_, ready, 0));
    NCCLX(ncclAllReduce(buf, buf, (size_t)n, ncclFloat32, ncclSum, comm_, comm_st_));
    pending_ = true;
  }
  void allreduce_wait() override {
    if (!pending_) return;
    hipEvent_t done = event();
    HIPX(hipEventRecord(done, comm_st_));
    HIPX(hipStreamWaitEvent(st_, done, 0));
    pending_ = false;
    ev_next_ = 0;
  }

 private:
  void set_lr(float lr) {
    if (lr != lr_host_) {
      HIPX(hipMemcpyAsync(lr_, &lr, sizeof(float), hipMemcpyHostToDevice, st_));
      HIPX(hipStreamSynchronize(st_));
      lr_host_ = lr;
    }
  }
  hipEvent_t event() {
    if (ev_next_ == events_.size()) {
      hipEvent_t e;
      HIPX(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      events_.push_back(e);
    }
    return events_[ev_next_++];
  }
  // grow-only scratch slots (0: conv act' gradient, 1 / 2: repacked conv kernels)
  float* buf(int k, size_t n) {
    if (n > bufn_[k]) {
      if (bufs_[k]) {
        HIPX(hipStreamSynchronize(st_));
        hipFree(bufs_[k]);
      }
      HIPX(hipMalloc(&bufs_[k], n * sizeof(float)));
      bufn_[k] = n;
    }
    return bufs_[k];
  }
  float* scratch(size_t n) {
    if (n > scratch_n_) {
      if (scratch_) {
        HIPX(hipStreamSynchronize(st_));
        hipFree(scratch_);
      }
      HIPX(hipMalloc(&scratch_, n * sizeof(float)));
      scratch_n_ = n;
    }
    return scratch_;
  }
  // rank 0 creates the RCCL unique id and publishes it as <rendezvous>/rccl_id (written to a
  // temporary name, then renamed: readers never see a partial file); the others poll for it
  void init_comm(const std::string& dir) {
    if (dir.empty()) throw std::runtime_error("native hip engine: world > 1 needs a rendezvous directory");
    ncclUniqueId id;
    const std::string path = dir + "/rccl_id";
    if (rank_ == 0) {
      NCCLX(ncclGetUniqueId(&id));
      const std::string tmp = path + ".tmp";
      {
        std::ofstream f(tmp, std::ios::binary);
        f.write(reinterpret_cast<const char*>(&id), sizeof(id));
      }
      if (std::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("native hip engine: publish rccl id");
    } else {
      const auto t0 = std::chrono::steady_clock::now();
      while (true) {
        std::ifstream f(path, std::ios::binary);
        if (f && f.read(reinterpret_cast<char*>(&id), sizeof(id)) && f.gcount() == sizeof(id)) break;
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120))
          throw std::runtime_error("native hip engine: no rccl id from rank 0 in " + dir);
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
      }
    }
    NCCLX(ncclCommInitRank(&comm_, world_, id, rank_));
  }

  int rank_, world_;
  hipStream_t st_ = nullptr, comm_st_ = nullptr, main_st_ = nullptr, side_st_ = nullptr;
  bool side_pending_ = false;
  void* pinned_ = nullptr;
  size_t pinned_n_ = 0;
  struct ClaimBufs {
    int *owner = nullptr, *dups = nullptr, *ndup = nullptr;
  };
  std::unordered_map<const float*, ClaimBufs> claim_;   // table -> owner-computes buffers
  ncclComm_t comm_ = nullptr;
  float* ws_ = nullptr;
  float* slots_ = nullptr;
  float* lr_ = nullptr;
  float lr_host_ = -1.f;
  float* scratch_ = nullptr;
  size_t scratch_n_ = 0;
  float* bufs_[3] = {nullptr, nullptr, nullptr};
  size_t bufn_[3] = {0, 0, 0};
  std::vector<hipEvent_t> events_;
  size_t ev_next_ = 0;
  bool pending_ = false;
};

}  // namespace

std::unique_ptr<Engine> make_hip_engine(int rank, int world, const std::string& rendezvous) {
  return std::make_unique<HipEngine>(rank, world, rendezvous);
}

}  // namespace nm
}  // namespace flexmi
