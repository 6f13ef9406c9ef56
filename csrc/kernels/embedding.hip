// Embedding-bag kernels (replace src/ops/embedding.cu:173-224 embed_forward / embed_backward).
//
// Forward: thread = (sample, 4 consecutive columns); a table row of D fp32 is read by D/4
// consecutive lanes with 16-B loads (one 512-B row = 32 lanes for D=128), summed over the bag,
// written as bf16 (or fp32) activations with 8-B / 16-B stores.  Multi-table variant ("TBE")
// processes every table of an embedding collection in ONE launch from a descriptor array and
// writes straight into the interaction input buffer [B, F, D] (concat fused away).
//
// Backward (fused sparse SGD, no dense gradient): W[idx] -= lr * dy.  Large tables: one
// wave-instruction = 64 consecutive fp32 atomic adds (256 contiguous bytes: full atomic rate on
// gfx950).  Tiny tables (rows*D fits LDS): block-private LDS accumulation first, then one
// global atomic per (touched row, column) per block -- avoids the 14x slowdown of many adders on
// one row.  Dense-gradient variant for replicated (data-parallel) tables.
#include "common.h"

namespace {

template <typename OutT, typename IdxT>
__global__ void fm_emb_fwd_kernel(const IdxT* __restrict__ idx, const float* __restrict__ W, OutT* __restrict__ out,
                                  long B, int bag, int D, long ldo, float scale) {
  const int D4 = D >> 2;
  const long total = B * D4;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    long b = e / D4;
    int c = (int)(e % D4) * 4;
    f32x4_t s = {0.f, 0.f, 0.f, 0.f};
    const IdxT* ib = idx + b * bag;
    for (int j = 0; j < bag; ++j) {
      long r = (long)ib[j];
      s += *reinterpret_cast<const f32x4_t*>(W + r * D + c);
    }
    s *= scale;
    OutT* o = out + b * ldo + c;
    if constexpr (sizeof(OutT) == 4) {
      *reinterpret_cast<f32x4_t*>(o) = s;
    } else {
      bf16x4_t v;
      v[0] = (short)f2bf(s[0]); v[1] = (short)f2bf(s[1]); v[2] = (short)f2bf(s[2]); v[3] = (short)f2bf(s[3]);
      *reinterpret_cast<bf16x4_t*>(o) = v;
    }
  }
}

// scalar fallback for D % 4 != 0
template <typename OutT, typename IdxT>
__global__ void fm_emb_fwd_scalar(const IdxT* __restrict__ idx, const float* __restrict__ W, OutT* __restrict__ out,
                                  long B, int bag, int D, long ldo, float scale) {
  const long total = B * D;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    long b = e / D;
    int c = (int)(e % D);
    float s = 0.f;
    for (int j = 0; j < bag; ++j) s += W[(long)idx[b * bag + j] * D + c];
    st<OutT>(out + b * ldo + c, s * scale);
  }
}

// ---- backward: atomics (large tables) --------------------------------------------------
template <typename GT, typename IdxT>
__global__ void fm_emb_bwd_atomic(const IdxT* __restrict__ idx, const GT* __restrict__ dy, float* __restrict__ W,
                                  const float* __restrict__ lr, long B, int bag, int D, long ldg, float scale) {
  const float neg = lr ? -lr[0] * scale : scale;
  const long total = B * (long)bag * D;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    long bj = e / D;
    int c = (int)(e % D);
    long b = bj / bag;
    float g = ld<GT>(dy + b * ldg + c) * neg;
    atomicAdd(W + (long)idx[bj] * D + c, g);
  }
}

// ---- backward: LDS-privatised (tiny tables) --------------------------------------------
template <typename GT, typename IdxT>
__global__ void fm_emb_bwd_lds(const IdxT* __restrict__ idx, const GT* __restrict__ dy, float* __restrict__ W,
                               const float* __restrict__ lr, long B, int bag, int rows, int D, long ldg, float scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* acc = reinterpret_cast<float*>(smem);
  const int n = rows * D;
  for (int i = threadIdx.x; i < n; i += blockDim.x) acc[i] = 0.f;
  __syncthreads();
  const long total = B * (long)bag * D;
  const long per_block = (total + gridDim.x - 1) / gridDim.x;
  const long e0 = blockIdx.x * per_block;
  const long e1 = min(total, e0 + per_block);
  for (long e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
    long bj = e / D;
    int c = (int)(e % D);
    long b = bj / bag;
    atomicAdd(acc + (int)idx[bj] * D + c, ld<GT>(dy + b * ldg + c));
  }
  __syncthreads();
  const float neg = lr ? -lr[0] * scale : scale;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    float v = acc[i];
    if (v != 0.f) atomicAdd(W + i, v * neg);
  }
}

}  // namespace

// idx64: 1 => int64 indices else int32; out_bf16: output storage
extern "C" void fm_embedding_fwd(const void* idx, int idx64, const float* W, void* out, int out_bf16, long B, int bag,
                                 int D, long ldo, float scale, hipStream_t s) {
  if (B <= 0) return;
  bool vec = (D % 4 == 0) && (ldo % 4 == 0);
  long work = vec ? B * (D / 4) : B * D;
  dim3 g(fm_grid(work, 256, 16384)), blk(256);
#define FM_EMB_FWD(OT, IT)                                                                                      \
  if (vec) hipLaunchKernelGGL((fm_emb_fwd_kernel<OT, IT>), g, blk, 0, s, (const IT*)idx, W, (OT*)out, B, bag, D, ldo, scale); \
  else hipLaunchKernelGGL((fm_emb_fwd_scalar<OT, IT>), g, blk, 0, s, (const IT*)idx, W, (OT*)out, B, bag, D, ldo, scale);
  if (out_bf16) {
    if (idx64) { FM_EMB_FWD(unsigned short, long long) } else { FM_EMB_FWD(unsigned short, int) }
  } else {
    if (idx64) { FM_EMB_FWD(float, long long) } else { FM_EMB_FWD(float, int) }
  }
#undef FM_EMB_FWD
}

// lr != nullptr: fused SGD update of W (W -= lr*scale*grad); lr == nullptr: dense grad accumulate
// into W (W := dW buffer, +scale*grad).
extern "C" void fm_embedding_bwd(const void* idx, int idx64, const void* dy, int dy_bf16, float* W, const float* lr,
                                 long B, int bag, int rows, int D, long ldg, float scale, hipStream_t s) {
  if (B <= 0) return;
  long total = B * (long)bag * D;
  const long lds_bytes = (long)rows * D * 4;
  if (lds_bytes <= 64 * 1024 && total >= 4L * rows * D) {
    int blocks = (int)std::min<long>(512, std::max<long>(1, total / (64L * 256)));
#define FM_EMB_LDS(GT, IT) \
  hipLaunchKernelGGL((fm_emb_bwd_lds<GT, IT>), dim3(blocks), dim3(256), lds_bytes, s, (const IT*)idx, (const GT*)dy, W, lr, B, bag, rows, D, ldg, scale);
    if (dy_bf16) { if (idx64) { FM_EMB_LDS(unsigned short, long long) } else { FM_EMB_LDS(unsigned short, int) } }
    else { if (idx64) { FM_EMB_LDS(float, long long) } else { FM_EMB_LDS(float, int) } }
#undef FM_EMB_LDS
    return;
  }
  dim3 g(fm_grid(total, 256, 16384)), blk(256);
#define FM_EMB_AT(GT, IT) \
  hipLaunchKernelGGL((fm_emb_bwd_atomic<GT, IT>), g, blk, 0, s, (const IT*)idx, (const GT*)dy, W, lr, B, bag, D, ldg, scale);
  if (dy_bf16) { if (idx64) { FM_EMB_AT(unsigned short, long long) } else { FM_EMB_AT(unsigned short, int) } }
  else { if (idx64) { FM_EMB_AT(float, long long) } else { FM_EMB_AT(float, int) } }
#undef FM_EMB_AT
}
