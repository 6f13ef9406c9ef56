// Embedding-bag kernels (replace src/ops/embedding.cu:173-224 embed_forward / embed_backward, which
// ran one thread per (sample, column) with the bag loop inside and one launch per table).
//
// All kernels take a TABLE DESCRIPTOR ARRAY and process every table of an embedding group in ONE
// launch (blockIdx.y = table) -- the executor fuses the independent per-table Embedding ops of a
// DLRM graph (26 ops in the MLPerf config) into one forward and two backward launches.
//
// Forward: lane = 4 consecutive columns of one sample (D/4 lanes per row: a 512-B fp32 row of a
// D=128 table is read by 32 lanes with 16-B loads), sum over the bag, bf16/fp32 output written
// with 8/16-B stores straight into the consumer's buffer (row stride ldo).  No 64-bit div/mod in
// the loop (lane->column mapping fixed per block).
// Backward (fused sparse SGD: W[idx] -= lr*scale*dy; or dense-grad accumulate when lr == null):
//   * large tables: one wave-instruction = 64 consecutive fp32 atomic adds (256 contiguous bytes:
//     the full gfx950 atomic rate, MI355X_MICROARCH "Global float atomics");
//   * tiny tables (rows*D*4 <= 64 KiB): block-private LDS accumulation over a chunk of samples, then
//     one global atomic per (row, column) per block -- avoids the ~14x slowdown of many adders on
//     one row (table with 3 rows in the MLPerf set).
#include "common.h"

#include <algorithm>
#include <vector>

namespace {

constexpr int MAXT = 32;

struct TabDesc {
  const float* W;     // fwd: table (read); bwd: table or dense grad (written)
  const void* idx;    // [B, bag] int32/int64
  void* act;          // fwd: out [B, *] (row stride ld); bwd: dy
  long ld;
  int rows, D, bag, idx64;
  float scale;
};
struct TabSet {
  TabDesc t[MAXT];
  int n;
};

FM_DEVICE long load_idx(const void* p, long i, int idx64) {
  return idx64 ? (long)reinterpret_cast<const long long*>(p)[i] : (long)reinterpret_cast<const int*>(p)[i];
}

template <typename OutT>
__global__ void __launch_bounds__(256) fm_emb_fwd_multi(TabSet s, long B) {
  const TabDesc& d = s.t[blockIdx.y];
  const int D4 = d.D >> 2;
  const int lpr = D4 < 64 ? D4 : 64;              // lanes per row (D <= 256)
  const int rpi = 256 / lpr;                       // rows per block-iteration
  const int sub = threadIdx.x / lpr, lc = threadIdx.x - sub * lpr;
  if (sub >= rpi) return;
  for (long b = (long)blockIdx.x * rpi + sub; b < B; b += (long)gridDim.x * rpi) {
    for (int c4 = lc; c4 < D4; c4 += lpr) {
      const int c = c4 * 4;
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
      for (int j = 0; j < d.bag; ++j) {
        long r = load_idx(d.idx, b * d.bag + j, d.idx64);
        acc += *reinterpret_cast<const f32x4_t*>(d.W + r * d.D + c);
      }
      acc *= d.scale;
      OutT* o = reinterpret_cast<OutT*>(d.act) + b * d.ld + c;
      if constexpr (sizeof(OutT) == 4) {
        *reinterpret_cast<f32x4_t*>(o) = acc;
      } else {
        bf16x4_t v;
        v[0] = (short)f2bf(acc[0]); v[1] = (short)f2bf(acc[1]); v[2] = (short)f2bf(acc[2]); v[3] = (short)f2bf(acc[3]);
        *reinterpret_cast<bf16x4_t*>(o) = v;
      }
    }
  }
}

// scalar fallback for D % 4 != 0 (any D)
template <typename OutT>
__global__ void __launch_bounds__(256) fm_emb_fwd_multi_scalar(TabSet s, long B) {
  const TabDesc& d = s.t[blockIdx.y];
  const int lpr = d.D < 256 ? d.D : 256;
  const int rpi = 256 / lpr;
  const int sub = threadIdx.x / lpr, lc = threadIdx.x - sub * lpr;
  if (sub >= rpi) return;
  for (long b = (long)blockIdx.x * rpi + sub; b < B; b += (long)gridDim.x * rpi)
    for (int c = lc; c < d.D; c += lpr) {
      float acc = 0.f;
      for (int j = 0; j < d.bag; ++j) acc += d.W[load_idx(d.idx, b * d.bag + j, d.idx64) * d.D + c];
      st<OutT>(reinterpret_cast<OutT*>(d.act) + b * d.ld + c, acc * d.scale);
    }
}

template <typename GT>
__global__ void __launch_bounds__(256) fm_emb_bwd_atomic_multi(TabSet s, const float* __restrict__ lr, long B) {
  const TabDesc& d = s.t[blockIdx.y];
  const float mul = (lr ? -lr[0] : 1.f) * d.scale;
  const int lpr = d.D < 256 ? d.D : 256;
  const int rpi = 256 / lpr;
  const int sub = threadIdx.x / lpr, lc = threadIdx.x - sub * lpr;
  if (sub >= rpi) return;
  float* W = const_cast<float*>(d.W);
  const GT* dy = reinterpret_cast<const GT*>(d.act);
  for (long b = (long)blockIdx.x * rpi + sub; b < B; b += (long)gridDim.x * rpi)
    for (int c = lc; c < d.D; c += lpr) {
      const float g = ld<GT>(dy + b * d.ld + c) * mul;
      for (int j = 0; j < d.bag; ++j) atomicAdd(W + load_idx(d.idx, b * d.bag + j, d.idx64) * d.D + c, g);
    }
}

// Tiny tables: block-private LDS copy of the table's gradient.  One WAVE per sample row
// (lane = column, columns l, l+64, ... so every LDS add of a wave hits 64 distinct banks and
// no two lanes of a wave ever add to the same address), U samples in flight per wave, a short
// chunk of samples per block so that the grid has >= 1024 blocks (latency-bound otherwise:
// the previous 32-block grid ran 128 dependent samples per wave).  The flush adds only touched
// rows (nonzero) into the table: <= chunk rows per block.
template <typename GT>
__global__ void __launch_bounds__(256) fm_emb_bwd_lds_multi(TabSet s, const float* __restrict__ lr, long B,
                                                             int chunk) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* acc = reinterpret_cast<float*>(smem);
  const TabDesc& d = s.t[blockIdx.y];
  const long b0 = (long)blockIdx.x * chunk;
  if (b0 >= B) return;
  const long b1 = min(B, b0 + chunk);
  const int n = d.rows * d.D;
  for (int i = threadIdx.x; i < n; i += 256) acc[i] = 0.f;
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const GT* dy = reinterpret_cast<const GT*>(d.act);
  constexpr int U = 4;
  for (long b = b0 + wave; b < b1; b += 4 * U) {
    long r[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long bb = b + 4L * u;
      ok[u] = bb < b1;
      r[u] = ok[u] ? load_idx(d.idx, bb * d.bag, d.idx64) : 0;
    }
    for (int c = lane; c < d.D; c += 64) {
      float g[U];
#pragma unroll
      for (int u = 0; u < U; ++u) g[u] = ok[u] ? ld<GT>(dy + (b + 4L * u) * d.ld + c) : 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (ok[u]) atomicAdd(acc + r[u] * d.D + c, g[u]);
    }
    if (d.bag > 1) {   // remaining bag entries (same gradient row)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (!ok[u]) continue;
        const long bb = b + 4L * u;
        for (int j = 1; j < d.bag; ++j) {
          const long rj = load_idx(d.idx, bb * d.bag + j, d.idx64);
          for (int c = lane; c < d.D; c += 64) atomicAdd(acc + rj * d.D + c, ld<GT>(dy + bb * d.ld + c));
        }
      }
    }
  }
  __syncthreads();
  const float mul = (lr ? -lr[0] : 1.f) * d.scale;
  float* W = const_cast<float*>(d.W);
  for (int i = threadIdx.x; i < n; i += 256) {
    float v = acc[i];
    if (v != 0.f) atomicAdd(W + i, v * mul);
  }
}

constexpr long TINY_BYTES = 64 * 1024;

}  // namespace

// ------------------------------------------------------------------------------------------
// Launchers.  Arrays describe n tables; act/ld = outputs (fwd) or output grads (bwd).
extern "C" void fm_embedding_fwd_multi(int n, const float* const* W, const void* const* idx, const int* idx64,
                                       void* const* out, const long* ldo, const int* rows, const int* D, const int* bag,
                                       const float* scale, int out_bf16, long B, hipStream_t st) {
  if (B <= 0) return;
  for (int base = 0; base < n; base += MAXT) {
    TabSet s;
    int m = std::min(MAXT, n - base);
    bool vec = true;
    for (int i = 0; i < m; ++i) {
      int k = base + i;
      s.t[i] = TabDesc{W[k], idx[k], out[k], ldo[k], rows[k], D[k], bag[k], idx64[k], scale[k]};
      vec = vec && (D[k] % 4 == 0) && (ldo[k] % 4 == 0) && D[k] <= 256;
    }
    s.n = m;
    const int rpi = std::max(1, 256 / std::min(64, std::max(1, D[base] / 4)));
    dim3 grid((unsigned)std::max<long>(1, std::min<long>((B + rpi - 1) / rpi, 2048)), m);
    if (vec) {
      if (out_bf16) hipLaunchKernelGGL(fm_emb_fwd_multi<unsigned short>, grid, dim3(256), 0, st, s, B);
      else hipLaunchKernelGGL(fm_emb_fwd_multi<float>, grid, dim3(256), 0, st, s, B);
    } else {
      if (out_bf16) hipLaunchKernelGGL(fm_emb_fwd_multi_scalar<unsigned short>, grid, dim3(256), 0, st, s, B);
      else hipLaunchKernelGGL(fm_emb_fwd_multi_scalar<float>, grid, dim3(256), 0, st, s, B);
    }
  }
}

// lr != nullptr: fused sparse SGD into W; lr == nullptr: W is a dense grad buffer (accumulate).
extern "C" void fm_embedding_bwd_multi(int n, float* const* W, const void* const* idx, const int* idx64,
                                       const void* const* dy, const long* ldg, const int* rows, const int* D,
                                       const int* bag, const float* scale, int dy_bf16, const float* lr, long B,
                                       hipStream_t st) {
  if (B <= 0) return;
  // partition: tiny tables -> LDS kernel, others -> atomic kernel
  for (int pass = 0; pass < 2; ++pass) {
    std::vector<int> sel;
    for (int k = 0; k < n; ++k) {
      bool tiny = (long)rows[k] * D[k] * 4 <= TINY_BYTES && B * (long)bag[k] >= 4L * rows[k];
      if ((pass == 0) == tiny) sel.push_back(k);
    }
    for (size_t base = 0; base < sel.size(); base += MAXT) {
      TabSet s;
      int m = (int)std::min<size_t>(MAXT, sel.size() - base);
      int maxD = 1, maxrows = 1;
      for (int i = 0; i < m; ++i) {
        int k = sel[base + i];
        s.t[i] = TabDesc{W[k], idx[k], const_cast<void*>(dy[k]), ldg[k], rows[k], D[k], bag[k], idx64[k], scale[k]};
        maxD = std::max(maxD, D[k]);
        maxrows = std::max(maxrows, rows[k]);
      }
      s.n = m;
      if (pass == 0) {
        size_t lds = (size_t)0;
        for (int i = 0; i < m; ++i) lds = std::max(lds, (size_t)s.t[i].rows * s.t[i].D * 4);
        // chunk: >= 64 samples (16 per wave), more for larger tables (flush <= rows*D adds per block)
        int chunk = std::max(64, std::min(512, ((2 * maxrows + 31) / 32) * 32));
        dim3 grid((unsigned)((B + chunk - 1) / chunk), m);
        if (dy_bf16) hipLaunchKernelGGL(fm_emb_bwd_lds_multi<unsigned short>, grid, dim3(256), lds, st, s, lr, B, chunk);
        else hipLaunchKernelGGL(fm_emb_bwd_lds_multi<float>, grid, dim3(256), lds, st, s, lr, B, chunk);
      } else {
        const int rpi = std::max(1, 256 / std::min(256, maxD));
        dim3 grid((unsigned)std::max<long>(1, std::min<long>((B + rpi - 1) / rpi, 2048)), m);
        if (dy_bf16) hipLaunchKernelGGL(fm_emb_bwd_atomic_multi<unsigned short>, grid, dim3(256), 0, st, s, lr, B);
        else hipLaunchKernelGGL(fm_emb_bwd_atomic_multi<float>, grid, dim3(256), 0, st, s, lr, B);
      }
    }
  }
}

// single-table conveniences
extern "C" void fm_embedding_fwd(const void* idx, int idx64, const float* W, void* out, int out_bf16, long B, int bag,
                                 int D, long ldo, float scale, hipStream_t s) {
  int rows = 0;
  fm_embedding_fwd_multi(1, &W, &idx, &idx64, &out, &ldo, &rows, &D, &bag, &scale, out_bf16, B, s);
}

extern "C" void fm_embedding_bwd(const void* idx, int idx64, const void* dy, int dy_bf16, float* W, const float* lr,
                                 long B, int bag, int rows, int D, long ldg, float scale, hipStream_t s) {
  fm_embedding_bwd_multi(1, &W, &idx, &idx64, &dy, &ldg, &rows, &D, &bag, &scale, dy_bf16, lr, B, s);
}
