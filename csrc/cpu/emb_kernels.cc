// Native CPU embedding-bag kernels: AVX2 (8-wide FMA, 4 accumulators per 32 columns) with a
// scalar fallback, samples split over workers in the forward, rows owned per worker in the
// backward.  See emb_kernels.h.
#include "emb_kernels.h"

#include <immintrin.h>

#include <algorithm>
#include <thread>
#include <vector>

namespace flexmi {
namespace cpu {

namespace {

ParallelFor g_pf;

void default_parallel_for(int64_t n, int64_t grain, int64_t max_threads, const std::function<void(int64_t, int64_t)>& fn) {
  const int64_t hw = std::max<int64_t>(1, (int64_t)std::thread::hardware_concurrency());
  const int64_t nt = std::max<int64_t>(1, std::min<int64_t>({hw, max_threads > 0 ? max_threads : hw, (n + grain - 1) / grain}));
  if (nt <= 1) {
    fn(0, n);
    return;
  }
  std::vector<std::thread> th;
  const int64_t per = (n + nt - 1) / nt;
  for (int64_t t = 0; t < nt; ++t) {
    const int64_t b = t * per, e = std::min(n, b + per);
    if (b < e) th.emplace_back([&fn, b, e] { fn(b, e); });
  }
  for (auto& t : th) t.join();
}

void pfor(int64_t n, int64_t grain, int64_t max_threads, const std::function<void(int64_t, int64_t)>& fn) {
  if (g_pf) g_pf(n, grain, max_threads, fn);
  else default_parallel_for(n, grain, max_threads, fn);
}

__attribute__((target("avx2,fma"))) void axpy_avx2(float* __restrict__ y, const float* __restrict__ x, float a, int64_t n) {
  const __m256 va = _mm256_set1_ps(a);
  int64_t i = 0;
  for (; i + 8 <= n; i += 8) _mm256_storeu_ps(y + i, _mm256_fmadd_ps(va, _mm256_loadu_ps(x + i), _mm256_loadu_ps(y + i)));
  for (; i < n; ++i) y[i] += a * x[i];
}

void axpy(float* y, const float* x, float a, int64_t n) {
  if (has_avx2()) {
    axpy_avx2(y, x, a, n);
  } else {
    for (int64_t i = 0; i < n; ++i) y[i] += a * x[i];
  }
}

template <typename I>
__attribute__((target("avx2,fma"))) void bag_avx2(const float* W, int64_t rows, int64_t D, const I* idx, int64_t bag,
                                                 int64_t row_lo, float scale, float* out) {
  int64_t d = 0;
  for (; d + 32 <= D; d += 32) {
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

}  // namespace

void set_parallel_for(ParallelFor pf) { g_pf = std::move(pf); }

bool has_avx2() {
  static const bool ok = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
  return ok;
}

template <typename I>
void embedding_bag_forward(const float* W, int64_t rows, int64_t D, const I* idx, int64_t B, int64_t bag, int64_t row_lo,
                           float scale, float* out, int64_t ld_out) {
  const bool avx = has_avx2();
  pfor(B, std::max<int64_t>(1, 2048 / std::max<int64_t>(1, D * bag / 64)), 0, [&](int64_t b0, int64_t b1) {
    for (int64_t b = b0; b < b1; ++b) {
      if (avx) bag_avx2<I>(W, rows, D, idx + b * bag, bag, row_lo, scale, out + b * ld_out);
      else bag_scalar<I>(W, rows, D, idx + b * bag, bag, row_lo, scale, out + b * ld_out);
    }
  });
}

template <typename I>
void embedding_bag_backward(float* target, int64_t rows, int64_t D, const I* idx, int64_t B, int64_t bag, int64_t row_lo,
                            const float* dy, int64_t ld_dy, float alpha, int workers) {
  const int64_t nw = std::max<int64_t>(1, workers > 0 ? workers : (B * bag * D) / 16384 + 1);
  pfor(nw, 1, nw, [&](int64_t p0, int64_t p1) {
    for (int64_t p = p0; p < p1; ++p)
      for (int64_t b = 0; b < B; ++b)
        for (int64_t j = 0; j < bag; ++j) {
          const int64_t r = (int64_t)idx[b * bag + j] - row_lo;
          if (r < 0 || r >= rows || r % nw != p) continue;
          axpy(target + r * D, dy + b * ld_dy, alpha, D);
        }
  });
}

template void embedding_bag_forward<int32_t>(const float*, int64_t, int64_t, const int32_t*, int64_t, int64_t, int64_t, float,
                                             float*, int64_t);
template void embedding_bag_forward<int64_t>(const float*, int64_t, int64_t, const int64_t*, int64_t, int64_t, int64_t, float,
                                             float*, int64_t);
template void embedding_bag_backward<int32_t>(float*, int64_t, int64_t, const int32_t*, int64_t, int64_t, int64_t,
                                              const float*, int64_t, float, int);
template void embedding_bag_backward<int64_t>(float*, int64_t, int64_t, const int64_t*, int64_t, int64_t, int64_t,
                                              const float*, int64_t, float, int);

}  // namespace cpu
}  // namespace flexmi
