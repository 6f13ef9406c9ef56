// Native CPU initialisers and loss / metrics (flexmi/_cpu): the CPU-backend counterparts of
// csrc/kernels/init.hip and csrc/kernels/loss.hip.
//
// Reference behaviour: the CPU init tasks of src/runtime/initializer.cc (Glorot / uniform /
// normal / constant / zero, initializer_kernel.cu:24-295 for the GPU side) and the CPU metrics
// task of src/metrics_functions/metrics_functions.cc (accuracy, categorical / sparse categorical
// cross-entropy, MSE / RMSE / MAE accumulated into a PerfMetrics record).
//
// Initialisation is counter-based -- element i of the LOGICAL tensor gets f(seed, i) with the same
// lowbias32 hash as the HIP kernel -- so a CPU-initialised shard equals the GPU-initialised one and
// any sharding reproduces the unsharded values.  Uniform draws are bit-identical to the GPU; normal
// draws go through the host libm log/cos (within 1 ulp of the device ones).
#include <torch/extension.h>
#include <ATen/Parallel.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <mutex>
#include <vector>

namespace {

inline uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

inline double u01(uint32_t seed, uint64_t idx) {
  const uint32_t lo = (uint32_t)(idx & 0xFFFFFFFFull), hi = (uint32_t)(idx >> 32);
  const uint32_t h = lowbias32(hi ^ lowbias32(seed ^ 0x9E3779B9u));
  return (double)(lowbias32(lo ^ h) >> 8) * (1.0 / 16777216.0);
}

// Fill `out` (dense fp32, the sub-box `box` = [(lo, hi)...] of a logical tensor of `shape`).
// kind: 0 zero, 1 constant a, 2 uniform[a, b), 3 normal(mean a, stddev b)
void counter_fill(torch::Tensor out, std::vector<int64_t> shape, std::vector<std::pair<int64_t, int64_t>> box, int64_t kind,
                  int64_t seed, double a, double b) {
  TORCH_CHECK(out.device().is_cpu() && out.scalar_type() == torch::kFloat32 && out.is_contiguous(),
              "counter_fill: contiguous fp32 CPU tensor");
  TORCH_CHECK(box.size() == shape.size(), "counter_fill: box rank != shape rank");
  const int nd = (int)shape.size();
  std::vector<int64_t> ext(nd), gstride(nd);
  int64_t total = 1, gs = 1;
  for (int d = nd - 1; d >= 0; --d) {
    TORCH_CHECK(box[d].first >= 0 && box[d].second <= shape[d] && box[d].first <= box[d].second, "counter_fill: box outside shape");
    ext[d] = box[d].second - box[d].first;
    gstride[d] = gs;
    gs *= shape[d];
    total *= ext[d];
  }
  TORCH_CHECK(out.numel() == total, "counter_fill: out has ", out.numel(), " elements, box ", total);
  float* o = out.data_ptr<float>();
  if (total == 0) return;
  if (kind == 0 || kind == 1) {
    std::fill(o, o + total, kind == 0 ? 0.f : (float)a);
    return;
  }
  TORCH_CHECK(kind == 2 || kind == 3, "counter_fill: unknown kind ", kind);
  const uint32_t sd = (uint32_t)(seed & 0xFFFFFFFF);
  // rows = all but the innermost box dimension; each row is a contiguous run of logical indices
  const int64_t inner = nd ? ext[nd - 1] : 1, rows = total / std::max<int64_t>(inner, 1);
  at::parallel_for(0, rows, std::max<int64_t>(1, 16384 / std::max<int64_t>(inner, 1)), [&](int64_t r0, int64_t r1) {
    for (int64_t r = r0; r < r1; ++r) {
      int64_t rem = r, base = 0;
      for (int d = nd - 2; d >= 0; --d) {
        base += (box[d].first + rem % ext[d]) * gstride[d];
        rem /= ext[d];
      }
      if (nd) base += box[nd - 1].first;
      float* dst = o + r * inner;
      if (kind == 2) {
        for (int64_t c = 0; c < inner; ++c) dst[c] = (float)(a + (b - a) * u01(sd, (uint64_t)(base + c)));
      } else {
        for (int64_t c = 0; c < inner; ++c) {
          const uint64_t gi = (uint64_t)(base + c);
          const double x1 = u01(sd, 2 * gi), x2 = u01(sd, 2 * gi + 1);
          dst[c] = (float)(a + b * (std::sqrt(-2.0 * std::log(1.0 - x1)) * std::cos(6.283185307179586 * x2)));
        }
      }
    }
  });
}

// metric slots (flexmi/core/loss_metrics.py M_*) and loss codes (flexmi/core/types.py LossType)
enum { M_ALL, M_CORRECT, M_CCE, M_SCCE, M_MSE, M_RMSE, M_MAE, M_LOSS, NUM_SLOTS };
enum { L_CCE = 50, L_SCCE = 51, L_MSE_AVG = 52, L_MSE_SUM = 53, L_BCE = 54 };
constexpr double LOG_MIN = 1e-7;

// One pass over the batch: gradient (p - y) * scale (zero where the DLRM loss threshold clamped the
// prediction), and the metrics selected by `mask` (bit i = metric i of metrics_mask()) summed into
// acc[NUM_SLOTS] in double per worker.
void loss_metrics(int64_t loss_type, torch::Tensor logits, torch::Tensor labels, c10::optional<torch::Tensor> grad,
                  double scale, torch::Tensor acc, int64_t mask, double clamp) {
  TORCH_CHECK(logits.device().is_cpu() && logits.scalar_type() == torch::kFloat32 && logits.is_contiguous(),
              "loss_metrics: contiguous fp32 CPU logits");
  TORCH_CHECK(acc.scalar_type() == torch::kFloat32 && acc.numel() >= NUM_SLOTS && acc.is_contiguous(), "loss_metrics: acc");
  TORCH_CHECK(loss_type >= L_CCE && loss_type <= L_BCE, "loss_metrics: unknown loss ", loss_type);
  const int64_t B = logits.size(0), C = B ? logits.numel() / B : 1;
  const bool sparse = loss_type == L_SCCE;
  torch::Tensor lab = labels.contiguous();
  if (sparse) {
    lab = lab.to(torch::kInt64).reshape({B});
  } else {
    lab = lab.to(torch::kFloat32).reshape({B, C});
  }
  float* g = nullptr;
  if (grad) {
    TORCH_CHECK(grad->scalar_type() == torch::kFloat32 && grad->is_contiguous() && grad->numel() == B * C, "loss_metrics: grad");
    g = grad->data_ptr<float>();
  }
  const float* p = logits.data_ptr<float>();
  const int64_t* li = sparse ? lab.data_ptr<int64_t>() : nullptr;
  const float* lf = sparse ? nullptr : lab.data_ptr<float>();
  const float lo = (float)clamp, hi = (float)(1.0 - clamp);
  const bool clamped = clamp > 0.0;

  std::array<double, NUM_SLOTS> tot{};
  std::mutex mu;
  at::parallel_for(0, B, 256, [&](int64_t b0, int64_t b1) {
    std::array<double, NUM_SLOTS> s{};
    for (int64_t b = b0; b < b1; ++b) {
      const float* pr = p + b * C;
      auto pv = [&](int64_t c) { float v = pr[c]; return clamped ? std::min(std::max(v, lo), hi) : v; };
      auto yv = [&](int64_t c) -> float { return sparse ? (c == li[b] ? 1.f : 0.f) : lf[b * C + c]; };
      int64_t ap = 0, ay = 0;
      float bp = -INFINITY, by = -INFINITY;
      double se = 0.0, ae = 0.0, cce = 0.0, bce = 0.0;
      for (int64_t c = 0; c < C; ++c) {
        const float x = pv(c), y = yv(c), d = x - y;
        if (g) g[b * C + c] = (clamped && x != pr[c]) ? 0.f : (float)(d * scale);
        if (x > bp) { bp = x; ap = c; }
        if (y > by) { by = y; ay = c; }
        se += (double)d * d;
        ae += std::fabs((double)d);
        cce -= (double)y * std::log(std::max((double)x, LOG_MIN));
        if (loss_type == L_BCE) {
          const double pc = std::min(std::max((double)x, LOG_MIN), 1.0 - LOG_MIN);
          bce -= y * std::log(pc) + (1.0 - y) * std::log(1.0 - pc);
        }
      }
      if (mask & 1) s[M_CORRECT] += C == 1 ? ((pv(0) >= 0.5f) == (yv(0) >= 0.5f)) : (ap == ay);
      if (mask & 2) s[M_CCE] += cce;
      if (mask & 4) s[M_SCCE] -= std::log(std::max((double)pv(ay), LOG_MIN));
      if (mask & 8) s[M_MSE] += se;
      if (mask & 16) s[M_RMSE] += std::sqrt(se);
      if (mask & 32) s[M_MAE] += ae;
      s[M_LOSS] += loss_type == L_BCE ? bce : (loss_type == L_CCE || loss_type == L_SCCE) ? cce : se;
    }
    std::lock_guard<std::mutex> lk(mu);
    for (int k = 0; k < NUM_SLOTS; ++k) tot[k] += s[k];
  });
  tot[M_ALL] = (double)B;
  float* ac = acc.data_ptr<float>();
  for (int k = 0; k < NUM_SLOTS; ++k) ac[k] += (float)tot[k];
}

}  // namespace

void register_init_metrics(pybind11::module& m) {
  m.def("counter_fill", &counter_fill, "counter-based init of a sub-box of a logical tensor (same values as init.hip)");
  m.def("loss_metrics", &loss_metrics, "loss gradient + metrics accumulation (same semantics as loss.hip)",
        pybind11::arg("loss_type"), pybind11::arg("logits"), pybind11::arg("labels"), pybind11::arg("grad"),
        pybind11::arg("scale"), pybind11::arg("acc"), pybind11::arg("mask"), pybind11::arg("clamp") = 0.0);
}
