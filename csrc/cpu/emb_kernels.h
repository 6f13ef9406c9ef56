// Torch-free native CPU embedding-bag kernels (shared by flexmi/_cpu and the native C API).
//
// Reference behaviour: src/ops/embedding.cc:87-163 (CPU forward / backward, sum and avg
// aggregation) and the AVX2 lookup of src/ops/embedding_avx2.cc:5-296.  Row shard semantics:
// the table holds rows [row_lo, row_lo + rows); lookups outside contribute nothing.
#pragma once
#include <cstdint>
#include <functional>

namespace flexmi {
namespace cpu {

// run fn(begin, end) over [0, n) on `threads` workers (<= 1: inline); the torch binding passes
// ATen's pool instead through emb_parallel_hook
using ParallelFor = std::function<void(int64_t, int64_t, int64_t, const std::function<void(int64_t, int64_t)>&)>;
void set_parallel_for(ParallelFor pf);   // default: std::thread workers

bool has_avx2();

// out[b * ld_out + d] = scale * sum_j W[(idx[b * bag + j] - row_lo) * D + d]
template <typename I>
void embedding_bag_forward(const float* W, int64_t rows, int64_t D, const I* idx, int64_t B, int64_t bag, int64_t row_lo,
                           float scale, float* out, int64_t ld_out);

// target[(idx[b * bag + j] - row_lo) * D + d] += alpha * dy[b * ld_dy + d]  (dense gradient:
// alpha = scale; fused sparse SGD: target = the table, alpha = -lr * scale).  Rows are owned by
// one worker each (row % workers): no atomics, deterministic per-row order.
template <typename I>
void embedding_bag_backward(float* target, int64_t rows, int64_t D, const I* idx, int64_t B, int64_t bag, int64_t row_lo,
                            const float* dy, int64_t ld_dy, float alpha, int workers);

}  // namespace cpu
}  // namespace flexmi
