// flexmi native CPU kernels (flexmi/_cpu): the embedding-bag lookup / gradient / fused sparse SGD
// of the CPU backend and of host-placed tables.
//
// Reference behaviour: src/ops/embedding.cc:87-163 (CPU forward / backward tasks, sum and avg
// aggregation) and the AVX2 lookup of src/ops/embedding_avx2.cc:5-296.  flexmi's version is one
// kernel per direction over any bag size and any row shard (row_lo: the first table row this
// shard holds; lookups outside [row_lo, row_lo + rows) contribute nothing), parallel on ATen's
// intra-op pool:
//   * forward: samples split over threads, each bag accumulated in registers with 8-wide AVX2
//     FMAs (scalar tail / non-AVX2 fallback), written once into a possibly strided output row;
//   * backward / sparse SGD: target[row] += alpha * dy[sample] for every lookup.  Threads own
//     disjoint ROW sets (row % threads) -- no atomics, no locks, deterministic order within a
//     row; alpha = scale for the dense gradient, -lr * scale for the fused SGD update (SGD is
//     linear, so applying duplicates one by one equals summing them first).
#include <torch/extension.h>
#include <ATen/Parallel.h>
#include <immintrin.h>

#include <algorithm>
#include <cstdint>

namespace {

bool has_avx2() {
  static const bool ok = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
  return ok;
}

__attribute__((target("avx2,fma"))) void axpy_avx2(float* __restrict__ y, const float* __restrict__ x, float a, int64_t n) {
  const __m256 va = _mm256_set1_ps(a);
  int64_t i = 0;
  for (; i + 8 <= n; i += 8) _mm256_storeu_ps(y + i, _mm256_fmadd_ps(va, _mm256_loadu_ps(x + i), _mm256_loadu_ps(y + i)));
  for (; i < n; ++i) y[i] += a * x[i];
}

void axpy_scalar(float* __restrict__ y, const float* __restrict__ x, float a, int64_t n) {
  for (int64_t i = 0; i < n; ++i) y[i] += a * x[i];
}

inline void axpy(float* y, const float* x, float a, int64_t n) {
  if (has_avx2()) axpy_avx2(y, x, a, n);
  else axpy_scalar(y, x, a, n);
}

// one bag: out = scale * sum_j W[idx_j - row_lo] (rows outside the shard skipped)
template <typename I>
__attribute__((target("avx2,fma"))) void bag_avx2(const float* W, int64_t rows, int64_t D, const I* idx, int64_t bag,
                                                 int64_t row_lo, float scale, float* out) {
  int64_t d = 0;
  for (; d + 32 <= D; d += 32) {   // 4 independent accumulators per 32 columns
    __m256 a0 = _mm256_setzero_ps(), a1 = a0, a2 = a0, a3 = a0;
    for (int64_t j = 0; j < bag; ++j) {
      const int64_t r = (int64_t)idx[j] - row_lo;
      if (r < 0 || r >= rows) continue;
      const float* w = W + r * D + d;
      a0 = _mm256_add_ps(a0, _mm256_loadu_ps(w));
      a1 = _mm256_add_ps(a1, _mm256_loadu_ps(w + 8));
      a2 = _mm256_add_ps(a2, _mm256_loadu_ps(w + 16));
      a3 = _mm256_add_ps(a3, _mm256_loadu_ps(w + 24));
    }
    const __m256 s = _mm256_set1_ps(scale);
    _mm256_storeu_ps(out + d, _mm256_mul_ps(a0, s));
    _mm256_storeu_ps(out + d + 8, _mm256_mul_ps(a1, s));
    _mm256_storeu_ps(out + d + 16, _mm256_mul_ps(a2, s));
    _mm256_storeu_ps(out + d + 24, _mm256_mul_ps(a3, s));
  }
  for (; d + 8 <= D; d += 8) {
    __m256 a = _mm256_setzero_ps();
    for (int64_t j = 0; j < bag; ++j) {
      const int64_t r = (int64_t)idx[j] - row_lo;
      if (r < 0 || r >= rows) continue;
      a = _mm256_add_ps(a, _mm256_loadu_ps(W + r * D + d));
    }
    _mm256_storeu_ps(out + d, _mm256_mul_ps(a, _mm256_set1_ps(scale)));
  }
  for (; d < D; ++d) {
    float a = 0.f;
    for (int64_t j = 0; j < bag; ++j) {
      const int64_t r = (int64_t)idx[j] - row_lo;
      if (r >= 0 && r < rows) a += W[r * D + d];
    }
    out[d] = a * scale;
  }
}

template <typename I>
void bag_scalar(const float* W, int64_t rows, int64_t D, const I* idx, int64_t bag, int64_t row_lo, float scale,
                float* out) {
  for (int64_t d = 0; d < D; ++d) out[d] = 0.f;
  for (int64_t j = 0; j < bag; ++j) {
    const int64_t r = (int64_t)idx[j] - row_lo;
    if (r < 0 || r >= rows) continue;
    for (int64_t d = 0; d < D; ++d) out[d] += W[r * D + d];
  }
  for (int64_t d = 0; d < D; ++d) out[d] *= scale;
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
  const int64_t B = idx.size(0), bag = idx.size(1), D = W.size(1), rows = W.size(0), ld = out.stride(0);
  const float* w = W.data_ptr<float>();
  float* o = out.data_ptr<float>();
  const float sc = (float)scale;
  const bool avx = has_avx2();
  AT_DISPATCH_INDEX_TYPES(idx.scalar_type(), "embedding_fwd", [&] {
    const index_t* ix = idx.data_ptr<index_t>();
    at::parallel_for(0, B, std::max<int64_t>(1, 2048 / std::max<int64_t>(1, D * bag / 64)), [&](int64_t b0, int64_t b1) {
      for (int64_t b = b0; b < b1; ++b) {
        if (avx) bag_avx2<index_t>(w, rows, D, ix + b * bag, bag, row_lo, sc, o + b * ld);
        else bag_scalar<index_t>(w, rows, D, ix + b * bag, bag, row_lo, sc, o + b * ld);
      }
    });
  });
}

// target[idx[b, j] - row_lo] += alpha * dy[b]  (dense gradient: alpha = scale; fused SGD:
// alpha = -lr * scale, target = the table itself)
void embedding_bwd(torch::Tensor target, torch::Tensor idx, torch::Tensor dy, int64_t row_lo, double alpha) {
  check(target, idx, dy, "embedding_bwd");
  const int64_t B = idx.size(0), bag = idx.size(1), D = target.size(1), rows = target.size(0), ld = dy.stride(0);
  float* t = target.data_ptr<float>();
  const float* g = dy.data_ptr<float>();
  const float a = (float)alpha;
  const int64_t nthr = std::max<int64_t>(1, std::min<int64_t>(at::get_num_threads(), (B * bag * D) / 16384 + 1));
  AT_DISPATCH_INDEX_TYPES(idx.scalar_type(), "embedding_bwd", [&] {
    const index_t* ix = idx.data_ptr<index_t>();
    // thread p owns the rows r with r % nthr == p: every row is updated by exactly one thread
    at::parallel_for(0, nthr, 1, [&](int64_t p0, int64_t p1) {
      for (int64_t p = p0; p < p1; ++p)
        for (int64_t b = 0; b < B; ++b)
          for (int64_t j = 0; j < bag; ++j) {
            const int64_t r = (int64_t)ix[b * bag + j] - row_lo;
            if (r < 0 || r >= rows || r % nthr != p) continue;
            axpy(t + r * D, g + b * ld, a, D);
          }
    });
  });
}

bool avx2() { return has_avx2(); }

}  // namespace

PYBIND11_MODULE(_cpu, m) {
  m.doc() = "flexmi native CPU kernels (embedding bag forward / backward / fused sparse SGD)";
  m.def("embedding_fwd", &embedding_fwd, "out = scale * bag-sum of table rows");
  m.def("embedding_bwd", &embedding_bwd, "table rows += alpha * dy (dense grad or fused SGD)");
  m.def("avx2", &avx2);
}
