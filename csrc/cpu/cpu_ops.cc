// flexmi native CPU kernels (flexmi/_cpu): the embedding-bag lookup / gradient / fused sparse SGD
// of the CPU backend and of host-placed tables.  The kernels themselves are
// torch-free (emb_kernels.cc, also behind the native C API); this file binds them to torch
// tensors and runs them on ATen's intra-op thread pool.
//
// Reference behaviour: src/ops/embedding.cc:87-163 (CPU forward / backward tasks, sum and avg
// aggregation) and the AVX2 lookup of src/ops/embedding_avx2.cc:5-296.
#include <torch/extension.h>
#include <ATen/Parallel.h>

#include <algorithm>
#include <cstdint>

#include "emb_kernels.h"

namespace {

void use_aten_pool() {
  static const bool done = [] {
    flexmi::cpu::set_parallel_for([](int64_t n, int64_t grain, int64_t max_threads,
                                     const std::function<void(int64_t, int64_t)>& fn) {
      if (max_threads > 0 && max_threads <= n) grain = std::max<int64_t>(grain, (n + max_threads - 1) / max_threads);
      at::parallel_for(0, n, grain, [&](int64_t b, int64_t e) { fn(b, e); });
    });
    return true;
  }();
  (void)done;
}

void check(const torch::Tensor& W, const torch::Tensor& idx, const torch::Tensor& rowt, const char* what) {
  TORCH_CHECK(W.device().is_cpu() && idx.device().is_cpu() && rowt.device().is_cpu(), what, ": CPU tensors");
  TORCH_CHECK(W.scalar_type() == torch::kFloat32 && W.dim() == 2 && W.is_contiguous(), what, ": contiguous fp32 table [R,D]");
  TORCH_CHECK(idx.dim() == 2 && idx.is_contiguous() &&
                  (idx.scalar_type() == torch::kInt32 || idx.scalar_type() == torch::kInt64), what,
              ": contiguous int32/int64 indices [B,bag]");
  TORCH_CHECK(rowt.scalar_type() == torch::kFloat32 && rowt.dim() == 2 && rowt.size(0) == idx.size(0) &&
                  rowt.size(1) == W.size(1) && rowt.stride(1) == 1, what, ": fp32 rows [B,D] with unit column stride");
}

// out[b] = scale * sum_j W[idx[b, j] - row_lo]
void embedding_fwd(torch::Tensor W, torch::Tensor idx, torch::Tensor out, int64_t row_lo, double scale) {
  check(W, idx, out, "embedding_fwd");
  use_aten_pool();
  if (idx.scalar_type() == torch::kInt32)
    flexmi::cpu::embedding_bag_forward<int32_t>(W.data_ptr<float>(), W.size(0), W.size(1), idx.data_ptr<int32_t>(),
                                                idx.size(0), idx.size(1), row_lo, (float)scale, out.data_ptr<float>(),
                                                out.stride(0));
  else
    flexmi::cpu::embedding_bag_forward<int64_t>(W.data_ptr<float>(), W.size(0), W.size(1), idx.data_ptr<int64_t>(),
                                                idx.size(0), idx.size(1), row_lo, (float)scale, out.data_ptr<float>(),
                                                out.stride(0));
}

// target[idx[b, j] - row_lo] += alpha * dy[b]  (dense gradient: alpha = scale; fused SGD:
// alpha = -lr * scale, target = the table itself)
void embedding_bwd(torch::Tensor target, torch::Tensor idx, torch::Tensor dy, int64_t row_lo, double alpha) {
  check(target, idx, dy, "embedding_bwd");
  use_aten_pool();
  const int64_t B = idx.size(0), bag = idx.size(1), D = target.size(1);
  const int workers = (int)std::max<int64_t>(1, std::min<int64_t>(at::get_num_threads(), (B * bag * D) / 16384 + 1));
  if (idx.scalar_type() == torch::kInt32)
    flexmi::cpu::embedding_bag_backward<int32_t>(target.data_ptr<float>(), target.size(0), D, idx.data_ptr<int32_t>(), B,
                                                 bag, row_lo, dy.data_ptr<float>(), dy.stride(0), (float)alpha, workers);
  else
    flexmi::cpu::embedding_bag_backward<int64_t>(target.data_ptr<float>(), target.size(0), D, idx.data_ptr<int64_t>(), B,
                                                 bag, row_lo, dy.data_ptr<float>(), dy.stride(0), (float)alpha, workers);
}

bool avx2() { return flexmi::cpu::has_avx2(); }

}  // namespace

void register_init_metrics(pybind11::module& m);  // init_metrics.cc

PYBIND11_MODULE(_cpu, m) {
  m.doc() = "flexmi native CPU kernels (embedding bag forward / backward / fused sparse SGD, counter-based init, loss + metrics)";
  m.def("embedding_fwd", &embedding_fwd, "out = scale * bag-sum of table rows");
  m.def("embedding_bwd", &embedding_bwd, "table rows += alpha * dy (dense grad or fused SGD)");
  m.def("avx2", &avx2);
  register_init_metrics(m);
}
