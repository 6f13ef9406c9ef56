// Embedding-bag kernels (replace src/ops/embedding.cu:173-224 embed_forward / embed_backward, which
// ran one thread per (sample, column) with the bag loop inside and one launch per table).
//
// All kernels take a TABLE DESCRIPTOR ARRAY and process every table of an embedding group in ONE
// launch (blockIdx.y = table) -- the executor fuses the independent per-table Embedding ops of a
// DLRM graph (26 ops in the MLPerf config) into one forward and two backward launches.
// The index width (int32/int64) is a template parameter and every load in the hot loops is
// unconditional (clamped address, predicated use): a runtime width test or a guarded load makes
// the compiler emit a branch + s_waitcnt vmcnt(0) per load, i.e. one HBM round trip per sample
// (measured 3-8x slowdowns before this rule was applied).
//
// Forward: lane = 4 consecutive columns of one sample (D/4 lanes per row: a 512-B fp32 row of a
// D=128 table is read by 32 lanes with 16-B loads), sum over the bag, bf16/fp32 output written
// with 8/16-B stores straight into the consumer's buffer (row stride ldo).
// Backward (fused sparse SGD: W[idx] -= lr*scale*dy; or dense-grad accumulate when lr == null):
//   * regular tables: one wave-instruction = 64 consecutive fp32 atomic adds (256 contiguous bytes:
//     the full gfx950 atomic rate, MI355X_MICROARCH "Global float atomics");
//   * tiny tables (<= 64 rows: 3, 4, 10, 14, 36, 63 rows in the MLPerf set): thousands of samples hit the
//     same few addresses, which L2 serialises; each wave accumulates into a PRIVATE LDS copy of the
//     table gradient with plain read-add-write (row index wave-uniform, lane = column: 64 distinct
//     banks, no atomics), the block sums its waves' copies and flushes one atomic per (row, col).
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {

constexpr int MAXT = 32;
constexpr int TINY_ROWS = 16;

// Row-sharded tables (SOAP row split of the embedding weight): a shard holds the global rows
// [lo, lo + rows); lookups outside it contribute nothing here (their partial sums come from the
// shards that hold them).  Whole tables have lo = 0, and out-of-range indices are dropped, never
// read or written out of bounds.  The range test is a select AFTER an unconditional (clamped)
// load, so the hot loops keep their branch-free loads.
struct TabDesc {
  const float* W;     // fwd: table (read); bwd: table or dense grad (written)
  const void* idx;    // [B, bag] int32/int64
  void* act;          // fwd: out [B, *] (row stride ld); bwd: dy
  long ld;
  long lo;            // first global row held by this shard
  int rows, D, bag;   // rows: rows held by this shard
  float scale;
};

// local row of a lookup, clamped into the shard (ok = the shard holds it)
FM_DEVICE long local_row(long r, long lo, int rows, bool& ok) {
  const long l = r - lo;
  ok = (unsigned long)l < (unsigned long)rows;
  return ok ? l : 0;
}
struct TabSet {
  TabDesc t[MAXT];
  int n;
};

template <bool I64>
FM_DEVICE long ldi(const void* p, long i) {
  if constexpr (I64) return (long)reinterpret_cast<const long long*>(p)[i];
  else return (long)reinterpret_cast<const int*>(p)[i];
}

template <typename OutT, bool I64>
__global__ void __launch_bounds__(256) fm_emb_fwd_multi(TabSet s, long B, int su) {
  const TabDesc& d = s.t[blockIdx.y];
  const int D4 = d.D >> 2;
  const int lpr = D4 < 64 ? D4 : 64;              // lanes per row (D <= 256)
  const int rpi = 256 / lpr;                       // rows per block-iteration
  const int sub = threadIdx.x / lpr, lc = threadIdx.x - sub * lpr;
  if (sub >= rpi) return;
  const long bstride = (long)gridDim.x * rpi;
  if (su && d.bag == 1 && D4 <= 64) {
    // one lookup per sample (the MLPerf tables): SU samples' index loads, then their row loads in
    // flight per lane, so a small grid still streams at the HBM rate and leaves CU slots to the
    // bottom-MLP GEMMs running beside it on the other stream
    constexpr int SU = 4;
    const int c = lc * 4;
    for (long b0 = (long)blockIdx.x * rpi + sub; b0 < B; b0 += SU * bstride) {
      long r[SU];
      bool ok[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) r[u] = local_row(ldi<I64>(d.idx, min(b0 + u * bstride, B - 1)), d.lo, d.rows, ok[u]);
      f32x4_t v[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) v[u] = *reinterpret_cast<const f32x4_t*>(d.W + r[u] * d.D + c);
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const long b = b0 + u * bstride;
        if (b >= B) break;
        f32x4_t acc = ok[u] ? v[u] * d.scale : f32x4_t{0.f, 0.f, 0.f, 0.f};
        OutT* o = reinterpret_cast<OutT*>(d.act) + b * d.ld + c;
        if constexpr (sizeof(OutT) == 4) {
          *reinterpret_cast<f32x4_t*>(o) = acc;
        } else {
          bf16x4_t w;
          w[0] = (short)f2bf(acc[0]); w[1] = (short)f2bf(acc[1]); w[2] = (short)f2bf(acc[2]); w[3] = (short)f2bf(acc[3]);
          *reinterpret_cast<bf16x4_t*>(o) = w;
        }
      }
    }
    return;
  }
  for (long b = (long)blockIdx.x * rpi + sub; b < B; b += bstride) {
    for (int c4 = lc; c4 < D4; c4 += lpr) {
      const int c = c4 * 4;
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
      int j = 0;
      // long bags (summit_large: 100 lookups per sample, 256 samples): 8 index loads, then 8 row
      // loads in flight per lane instead of one dependent index -> row round trip per lookup
      for (; j + 8 <= d.bag; j += 8) {
        long r[8];
        bool ok[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) r[u] = local_row(ldi<I64>(d.idx, b * d.bag + j + u), d.lo, d.rows, ok[u]);
        f32x4_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const f32x4_t*>(d.W + r[u] * d.D + c);
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (ok[u]) acc += v[u];
      }
      for (; j < d.bag; ++j) {
        bool ok;
        const long r = local_row(ldi<I64>(d.idx, b * d.bag + j), d.lo, d.rows, ok);
        const f32x4_t v = *reinterpret_cast<const f32x4_t*>(d.W + r * d.D + c);
        if (ok) acc += v;
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

// Long bags on small batches (summit_large: 256 samples x 100 lookups per table): one lane group
// per sample leaves ~100 blocks for 256 CUs, each lane walking the whole bag.  Here SP lane groups
// share a sample -- group k sums lookups k, k+SP, ... -- and the block folds the SP partial rows
// through LDS.  D <= 256 (one 16-B column chunk per lane, lpr = D/4 lanes per row).
template <typename OutT, bool I64>
__global__ void __launch_bounds__(256) fm_emb_fwd_split(TabSet s, long B, int sp) {
  __shared__ f32x4_t part[256];
  const TabDesc& d = s.t[blockIdx.y];
  const int lpr = d.D >> 2;                        // <= 64
  const int rpi = 256 / lpr;                       // lane groups per block
  const int spb = rpi / sp;                        // samples per block
  const int sub = threadIdx.x / lpr, lc = threadIdx.x - sub * lpr;
  const bool live = sub < spb * sp;                // whole sample groups only
  const int si = sub / sp, k = sub - si * sp;
  const long b = (long)blockIdx.x * spb + si;
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  if (live && b < B) {
    const int c = lc * 4;
    int j = k;
    for (; j + 3 * sp < d.bag; j += 4 * sp) {
      long r[4];
      bool ok[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) r[u] = local_row(ldi<I64>(d.idx, b * d.bag + j + u * sp), d.lo, d.rows, ok[u]);
      f32x4_t v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const f32x4_t*>(d.W + r[u] * d.D + c);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (ok[u]) acc += v[u];
    }
    for (; j < d.bag; j += sp) {
      bool ok;
      const long r = local_row(ldi<I64>(d.idx, b * d.bag + j), d.lo, d.rows, ok);
      const f32x4_t v = *reinterpret_cast<const f32x4_t*>(d.W + r * d.D + c);
      if (ok) acc += v;
    }
  }
  part[threadIdx.x] = acc;
  __syncthreads();
  if (!live || k != 0 || b >= B) return;
  for (int q = 1; q < sp; ++q) acc += part[threadIdx.x + q * lpr];
  acc *= d.scale;
  OutT* o = reinterpret_cast<OutT*>(d.act) + b * d.ld + lc * 4;
  if constexpr (sizeof(OutT) == 4) {
    *reinterpret_cast<f32x4_t*>(o) = acc;
  } else {
    bf16x4_t v;
    v[0] = (short)f2bf(acc[0]); v[1] = (short)f2bf(acc[1]); v[2] = (short)f2bf(acc[2]); v[3] = (short)f2bf(acc[3]);
    *reinterpret_cast<bf16x4_t*>(o) = v;
  }
}

// scalar fallback for D % 4 != 0 (any D)
template <typename OutT, bool I64>
__global__ void __launch_bounds__(256) fm_emb_fwd_multi_scalar(TabSet s, long B) {
  const TabDesc& d = s.t[blockIdx.y];
  const int lpr = d.D < 256 ? d.D : 256;
  const int rpi = 256 / lpr;
  const int sub = threadIdx.x / lpr, lc = threadIdx.x - sub * lpr;
  if (sub >= rpi) return;
  for (long b = (long)blockIdx.x * rpi + sub; b < B; b += (long)gridDim.x * rpi)
    for (int c = lc; c < d.D; c += lpr) {
      float acc = 0.f;
      for (int j = 0; j < d.bag; ++j) {
        bool ok;
        const long r = local_row(ldi<I64>(d.idx, b * d.bag + j), d.lo, d.rows, ok);
        const float v = d.W[r * d.D + c];
        if (ok) acc += v;
      }
      st<OutT>(reinterpret_cast<OutT*>(d.act) + b * d.ld + c, acc * d.scale);
    }
}

template <typename GT, bool I64>
__global__ void __launch_bounds__(256) fm_emb_bwd_atomic_multi(TabSet s, const float* __restrict__ lr, long B) {
  const TabDesc& d = s.t[blockIdx.y];
  const float mul = (lr ? -lr[0] : 1.f) * d.scale;
  const int lpr = d.D < 256 ? d.D : 256;
  const int rpi = 256 / lpr;
  const int sub = threadIdx.x / lpr, lc = threadIdx.x - sub * lpr;
  if (sub >= rpi) return;
  float* W = const_cast<float*>(d.W);
  const GT* dy = reinterpret_cast<const GT*>(d.act);
  for (long b = (long)blockIdx.x * rpi + sub; b < B; b += (long)gridDim.x * rpi) {
    bool ok0;
    const long r0 = local_row(ldi<I64>(d.idx, b * d.bag), d.lo, d.rows, ok0);
    for (int c = lc; c < d.D; c += lpr) {
      const float g = ld<GT>(dy + b * d.ld + c) * mul;
      if (ok0) atomicAdd(W + r0 * d.D + c, g);
      for (int j = 1; j < d.bag; ++j) {
        bool ok;
        const long r = local_row(ldi<I64>(d.idx, b * d.bag + j), d.lo, d.rows, ok);
        if (ok) atomicAdd(W + r * d.D + c, g);
      }
    }
  }
}

template <typename GT, bool I64>
__global__ void __launch_bounds__(256) fm_emb_bwd_tiny_multi(TabSet s, const float* __restrict__ lr, long B, int chunk) {
  constexpr int S = 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red = reinterpret_cast<float*>(smem);     // [4][rows*D]
  const TabDesc& d = s.t[blockIdx.y];
  const long b0 = (long)blockIdx.x * chunk;
  if (b0 >= B) return;
  const long b1 = min(B, b0 + chunk);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n = d.rows * d.D;
  float* mine = red + wave * n;
  for (int i = lane; i < n; i += 64) mine[i] = 0.f;
  const GT* dy = reinterpret_cast<const GT*>(d.act);
  for (long bw = b0 + (long)wave * S; bw < b1; bw += 4L * S) {
    for (int c0 = 0; c0 < d.D; c0 += 128) {
      const int ca = c0 + lane, cb = c0 + 64 + lane;
      const int sa = min(ca, d.D - 1), sb = min(cb, d.D - 1);   // clamped: loads stay unconditional
      long r[S];
      bool rok[S];
      float ga[S], gb[S];
#pragma unroll
      for (int u = 0; u < S; ++u) {
        const long bu = min(bw + u, b1 - 1);
        r[u] = local_row(ldi<I64>(d.idx, bu * d.bag), d.lo, d.rows, rok[u]);
        ga[u] = ld<GT>(dy + bu * d.ld + sa);
        gb[u] = ld<GT>(dy + bu * d.ld + sb);
      }
#pragma unroll
      for (int u = 0; u < S; ++u) {
        if (bw + u >= b1) break;                       // wave-uniform
        float* p = mine + r[u] * d.D;
        if (rok[u] && ca < d.D) p[ca] += ga[u];
        if (rok[u] && cb < d.D) p[cb] += gb[u];
        for (int j = 1; j < d.bag; ++j) {              // further bag entries share the gradient row
          bool ok;
          float* q = mine + local_row(ldi<I64>(d.idx, (bw + u) * d.bag + j), d.lo, d.rows, ok) * d.D;
          if (ok && ca < d.D) q[ca] += ga[u];
          if (ok && cb < d.D) q[cb] += gb[u];
        }
      }
    }
  }
  __syncthreads();
  const float mul = (lr ? -lr[0] : 1.f) * d.scale;
  float* W = const_cast<float*>(d.W);
  for (int i = threadIdx.x; i < n; i += 256) {
    const float v = red[i] + red[n + i] + red[2 * n + i] + red[3 * n + i];
    if (v != 0.f) atomicAdd(W + i, v * mul);
  }
}

template <bool I64>
void launch_fwd(const TabSet& s, int m, bool vec, bool out_bf16, long B, int D0, hipStream_t st) {
  const int rpi = std::max(1, 256 / std::min(64, std::max(1, D0 / 4)));
  // long bags with too few samples to fill the chip: split every bag over SP lane groups
  // (measured on summit_large, profiles/README.md)
  int minbag = 1 << 30, maxD = 0, minD = 1 << 30;
  for (int i = 0; i < m; ++i) {
    minbag = std::min(minbag, s.t[i].bag);
    maxD = std::max(maxD, s.t[i].D);
    minD = std::min(minD, s.t[i].D);
  }
  if (vec && maxD == minD && maxD <= 256 && minbag >= 16 && (B + rpi - 1) / rpi * m < 1024) {
    int sp = 1;
    while (sp * 2 <= rpi && sp * 2 <= minbag / 4 && (B * sp * 2 + rpi - 1) / rpi * m <= 2048) sp *= 2;
    if (sp > 1) {
      const int spb = rpi / sp;
      dim3 grid((unsigned)((B + spb - 1) / spb), m);
      if (out_bf16) hipLaunchKernelGGL((fm_emb_fwd_split<unsigned short, I64>), grid, dim3(256), 0, st, s, B, sp);
      else hipLaunchKernelGGL((fm_emb_fwd_split<float, I64>), grid, dim3(256), 0, st, s, B, sp);
      return;
    }
  }
  // 256 blocks per table: the forward runs beside the bottom MLP on a second stream; fewer,
  // longer-running blocks leave CUs to its GEMMs: MLPerf fp32 step 1.181 ms at 2048 blocks per
  // table, 1.164 at 256, 1.172 at 64 (profiles/bench_ab_x3_sched_embgrid_r5n.txt).  Single-lookup
  // bags take two samples per lane-group iteration (su; profiles/bench_ab_emb_fwd_su_r5zc.txt)
  dim3 grid((unsigned)std::max<long>(1, std::min<long>((B + rpi - 1) / rpi, 256L)), m);
  const int su = 1;
  if (vec) {
    if (out_bf16) hipLaunchKernelGGL((fm_emb_fwd_multi<unsigned short, I64>), grid, dim3(256), 0, st, s, B, su);
    else hipLaunchKernelGGL((fm_emb_fwd_multi<float, I64>), grid, dim3(256), 0, st, s, B, su);
  } else {
    if (out_bf16) hipLaunchKernelGGL((fm_emb_fwd_multi_scalar<unsigned short, I64>), grid, dim3(256), 0, st, s, B);
    else hipLaunchKernelGGL((fm_emb_fwd_multi_scalar<float, I64>), grid, dim3(256), 0, st, s, B);
  }
}

// ---- mostly-unique tables (rows > B*bag): owner-computes sparse SGD without row atomics -------
// claim: every lookup entry e CASes its row's owner slot (-1 -> e); the winner owns the row, the
// others are appended to a per-table duplicate list.  dup: one wave per duplicate adds its row
// update with float atomics (few for large tables).  owner (after dup, kernel boundary): each
// owner does a plain 16-B read-modify-write of its row and releases the claim (-1), so the table
// is touched with full-line stores at the HBM rate instead of the ~1.3 TB/s atomic rate.
struct ClaimDesc {
  float* W;
  const void* idx;
  const void* dy;
  long ld;
  long lo;
  int rows, D, bag;
  float scale;
  int* owner;   // [rows] int32, -1 = free (restored by the owner kernel)
  int* dups;    // [B*bag]
  int* ndup;    // [1]
};
struct ClaimSet {
  ClaimDesc t[MAXT];
  int n;
};

template <bool I64>
__global__ void __launch_bounds__(256) fm_emb_claim_multi(ClaimSet s, long B) {
  const ClaimDesc& d = s.t[blockIdx.y];
  const long n = B * d.bag;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    bool ok;
    const long r = local_row(ldi<I64>(d.idx, e), d.lo, d.rows, ok);
    if (!ok) continue;                               // row held by another shard
    const int prev = atomicCAS(d.owner + r, -1, (int)e);
    if (prev != -1) d.dups[atomicAdd(d.ndup, 1)] = (int)e;
  }
}

template <typename GT, bool I64>
__global__ void __launch_bounds__(256) fm_emb_dup_multi(ClaimSet s, const float* __restrict__ lr) {
  const ClaimDesc& d = s.t[blockIdx.y];
  const int nd = *d.ndup;
  const float mul = -lr[0] * d.scale;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const GT* dy = reinterpret_cast<const GT*>(d.dy);
  for (long k = blockIdx.x * 4L + wave; k < nd; k += (long)gridDim.x * 4) {
    const long e = d.dups[k];
    const long b = e / d.bag, r = ldi<I64>(d.idx, e) - d.lo;   // dups hold in-shard entries only
    for (int c = lane; c < d.D; c += 64) atomicAdd(d.W + r * d.D + c, ld<GT>(dy + b * d.ld + c) * mul);
  }
}

template <typename GT, bool I64>
__global__ void __launch_bounds__(256) fm_emb_owner_multi(ClaimSet s, const float* __restrict__ lr, long B) {
  const ClaimDesc& d = s.t[blockIdx.y];
  const float mul = -lr[0] * d.scale;
  const int D4 = d.D >> 2;
  const int lpr = D4 < 64 ? D4 : 64;
  const int rpi = 256 / lpr;
  const int sub = threadIdx.x / lpr, lc = threadIdx.x - sub * lpr;
  const long n = B * d.bag;
  const GT* dy = reinterpret_cast<const GT*>(d.dy);
  if (sub < rpi) {
    for (long e = (long)blockIdx.x * rpi + sub; e < n; e += (long)gridDim.x * rpi) {
      bool ok;
      const long r = local_row(ldi<I64>(d.idx, e), d.lo, d.rows, ok);
      if (!ok || d.owner[r] != (int)e) continue;   // uniform across the row's lanes
      const long b = e / d.bag;
      for (int c4 = lc; c4 < D4; c4 += lpr) {
        const int c = c4 * 4;
        f32x4_t* wp = reinterpret_cast<f32x4_t*>(d.W + r * d.D + c);
        f32x4_t w = *wp;
        if constexpr (sizeof(GT) == 2) {
          const bf16x4_t g = *reinterpret_cast<const bf16x4_t*>(dy + b * d.ld + c);
#pragma unroll
          for (int j = 0; j < 4; ++j) w[j] += mul * bf2f((unsigned short)g[j]);
        } else {
          const f32x4_t g = *reinterpret_cast<const f32x4_t*>(dy + b * d.ld + c);
          w += mul * g;
        }
        *wp = w;
      }
      if (lc == 0) d.owner[r] = -1;                // release the claim for the next step
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *d.ndup = 0;   // the dup kernel has finished reading it
}

// ---- count-based sparse SGD (fm_embedding_set_bwd_mode(1)): two launches for every non-tiny table ---
// count: every in-shard lookup e adds one to its row's slot (slot = lookups - 1; -1 = untouched)
// and records in own[e] (the dups array) whether it arrived first.  update: a lookup whose row was
// hit exactly once (slot == 0) applies a plain 16-B read-modify-write and frees the slot; rows hit
// more often take float atomics (lane = column: 256 contiguous bytes per wave-instruction) and
// their first arrival frees the slot.  A freed slot reads -1, never 0, so the plain path stays
// exclusive to single-lookup rows whatever the order of the lookups -- the claim / dup / owner
// kernels' work in one pass, and the mid-size tables (where most rows repeat) no longer need a
// kernel of their own.
template <bool I64>
__global__ void __launch_bounds__(256) fm_emb_count_multi(ClaimSet s, long B) {
  const ClaimDesc& d = s.t[blockIdx.y];
  const long n = B * d.bag;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    bool ok;
    const long r = local_row(ldi<I64>(d.idx, e), d.lo, d.rows, ok);
    int own = 0;
    if (ok) own = atomicAdd(d.owner + r, 1) == -1;
    d.dups[e] = own;
  }
}

template <typename GT, bool I64>
__global__ void __launch_bounds__(256) fm_emb_update_multi(ClaimSet s, const float* __restrict__ lr, long B) {
  const ClaimDesc& d = s.t[blockIdx.y];
  const float mul = -lr[0] * d.scale;
  const int D4 = d.D >> 2;
  const int lpr = D4 < 64 ? D4 : 64;
  const int rpi = 256 / lpr;
  const int sub = threadIdx.x / lpr, lc = threadIdx.x - sub * lpr;
  const long n = B * d.bag;
  const GT* dy = reinterpret_cast<const GT*>(d.dy);
  if (sub >= rpi) return;
  for (long e = (long)blockIdx.x * rpi + sub; e < n; e += (long)gridDim.x * rpi) {
    bool ok;
    const long r = local_row(ldi<I64>(d.idx, e), d.lo, d.rows, ok);
    if (!ok) continue;                                // uniform across the row's lanes
    const int c = __hip_atomic_load(d.owner + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int own = d.dups[e];
    const long b = e / d.bag;
    const GT* g = dy + b * d.ld;
    float* wr = d.W + r * d.D;
    if (c == 0) {                                     // the row's only lookup: plain 16-B RMW
      for (int c4 = lc; c4 < D4; c4 += lpr) {
        const int col = c4 * 4;
        f32x4_t* wp = reinterpret_cast<f32x4_t*>(wr + col);
        f32x4_t w = *wp;
        if constexpr (sizeof(GT) == 2) {
          const bf16x4_t gv = *reinterpret_cast<const bf16x4_t*>(g + col);
#pragma unroll
          for (int j = 0; j < 4; ++j) w[j] += mul * bf2f((unsigned short)gv[j]);
        } else {
          w += mul * *reinterpret_cast<const f32x4_t*>(g + col);
        }
        *wp = w;
      }
    } else {                                          // repeated row: lane = column atomics
      for (int col = lc; col < d.D; col += lpr) atomicAdd(wr + col, mul * ld<GT>(g + col));
    }
    if (lc == 0 && (c == 0 || own)) __hip_atomic_store(d.owner + r, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <bool I64>
void launch_count(const ClaimSet& s, int m, bool dy_bf16, const float* lr, long B, int maxbag, int minD4,
                  hipStream_t st) {
  const long n = B * maxbag;
  dim3 gc((unsigned)std::max<long>(1, std::min<long>((n + 255) / 256, 1024)), m);
  hipLaunchKernelGGL((fm_emb_count_multi<I64>), gc, dim3(256), 0, st, s, B);
  const int rpi = 256 / std::min(64, std::max(1, minD4));
  dim3 gu((unsigned)std::max<long>(1, std::min<long>((n + rpi - 1) / rpi, 2048)), m);
  if (dy_bf16) hipLaunchKernelGGL((fm_emb_update_multi<unsigned short, I64>), gu, dim3(256), 0, st, s, lr, B);
  else hipLaunchKernelGGL((fm_emb_update_multi<float, I64>), gu, dim3(256), 0, st, s, lr, B);
}

// blocks per table of the grid-stride backward kernels (claim / dup / owner / atomic): uncapped
long emb_bwd_cap(long want) { return want; }

template <bool I64>
void launch_claim(const ClaimSet& s, int m, bool dy_bf16, const float* lr, long B, int maxbag, int minD4,
                  hipStream_t st) {
  const long n = B * maxbag;
  dim3 gc((unsigned)std::max<long>(1, emb_bwd_cap(std::min<long>((n + 255) / 256, 1024))), m);
  hipLaunchKernelGGL((fm_emb_claim_multi<I64>), gc, dim3(256), 0, st, s, B);
  // (a 64-block grid measured 18.4 vs 9.5 us/step: 12k..40k-row tables still see thousands of dups)
  dim3 gd((unsigned)std::max<long>(1, emb_bwd_cap(std::min<long>((n + 3) / 4, 1024))), m);
  if (dy_bf16) hipLaunchKernelGGL((fm_emb_dup_multi<unsigned short, I64>), gd, dim3(256), 0, st, s, lr);
  else hipLaunchKernelGGL((fm_emb_dup_multi<float, I64>), gd, dim3(256), 0, st, s, lr);
  const int rpi = 256 / std::min(64, std::max(1, minD4));
  dim3 go((unsigned)std::max<long>(1, emb_bwd_cap(std::min<long>((n + rpi - 1) / rpi, 2048))), m);
  if (dy_bf16) hipLaunchKernelGGL((fm_emb_owner_multi<unsigned short, I64>), go, dim3(256), 0, st, s, lr, B);
  else hipLaunchKernelGGL((fm_emb_owner_multi<float, I64>), go, dim3(256), 0, st, s, lr, B);
}

template <bool I64>
void launch_bwd(const TabSet& s, int m, bool tiny, bool dy_bf16, const float* lr, long B, int maxD, hipStream_t st) {
  if (tiny) {
    size_t lds = 0;
    for (int i = 0; i < m; ++i) lds = std::max(lds, (size_t)s.t[i].rows * s.t[i].D * 4 * 4);  // one copy per wave
    static bool attr = false;
    if (!attr) {   // > 64 KiB of dynamic LDS (above 32 rows at D = 128) needs the opt-in
      (void)hipFuncSetAttribute((const void*)fm_emb_bwd_tiny_multi<unsigned short, I64>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 << 10);
      (void)hipFuncSetAttribute((const void*)fm_emb_bwd_tiny_multi<float, I64>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 << 10);
      attr = true;
    }
    // 64-sample chunks keep the per-wave chain to one round trip; at large B more blocks would
    // pile onto the same few addresses in the flush (tools/bench_embedding.py: B=8192 -> 64,
    // B=65536 -> 128..256)
    const int chunk = B <= 16384 ? 64 : B <= 32768 ? 128 : 256;
    dim3 grid((unsigned)((B + chunk - 1) / chunk), m);
    if (dy_bf16) hipLaunchKernelGGL((fm_emb_bwd_tiny_multi<unsigned short, I64>), grid, dim3(256), lds, st, s, lr, B, chunk);
    else hipLaunchKernelGGL((fm_emb_bwd_tiny_multi<float, I64>), grid, dim3(256), lds, st, s, lr, B, chunk);
  } else {
    const int rpi = std::max(1, 256 / std::min(256, maxD));
    dim3 grid((unsigned)std::max<long>(1, emb_bwd_cap(std::min<long>((B + rpi - 1) / rpi, 2048))), m);
    if (dy_bf16) hipLaunchKernelGGL((fm_emb_bwd_atomic_multi<unsigned short, I64>), grid, dim3(256), 0, st, s, lr, B);
    else hipLaunchKernelGGL((fm_emb_bwd_atomic_multi<float, I64>), grid, dim3(256), 0, st, s, lr, B);
  }
}

// ---- sparse data parallelism for replicated tables ---------------------------------------------
// A table replicated over R ranks (DP on its sample dim) is trained WITHOUT a dense gradient: each
// replica coalesces its own lookups into (unique local row, summed gradient) pairs, the replica set
// all-gathers those payloads, and every replica applies the R segments in rank order -- the same
// fp32 operations in the same order everywhere, so the replicas stay bit-identical.  Within one
// segment the rows are unique: the apply is a plain read-modify-write, no atomics.
//   claim  : every in-shard lookup e CASes its row's slot (-1 -> e)
//   assign : the winner takes a compact id u (one atomic per unique row), writes cid[e] = u,
//            ids[u] = row and g[u] = scale * dy[b] with plain stores
//   dups   : every other lookup of the row atomically adds its gradient into g[cid[slot[row]]]
//   apply  : per segment r: W[ids[u]] -= lr * g[u] for u < count; the own segment also frees the
//            slots (slot = -1) and zeroes its count for the next step
struct SdpDesc {
  const void* idx;    // [B, bag] int32/int64 (global rows)
  const void* dy;     // [B, *] bf16/fp32, row stride ld
  long ld;
  long lo;            // first global row of this shard
  int rows, D, bag;
  float scale;
  int* slot;          // [rows] int32, -1 = free
  int* cid;           // [B*bag] compact id of an owner entry (scratch)
  int* ids;           // [nmax] unique local rows      (payload)
  float* g;           // [nmax][D] summed gradients   (payload)
  int* count;         // [1] unique rows              (payload)
};
struct SdpSet {
  SdpDesc t[MAXT];
  int n;
};

template <bool I64>
__global__ void __launch_bounds__(256) fm_sdp_claim(SdpSet s, long B) {
  const SdpDesc& d = s.t[blockIdx.y];
  const long n = B * d.bag;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    bool ok;
    const long r = local_row(ldi<I64>(d.idx, e), d.lo, d.rows, ok);
    if (ok) atomicCAS(d.slot + r, -1, (int)e);
  }
}

// one wave per lookup entry (lane = column): the row's owner entry takes the compact id
template <typename GT, bool I64>
__global__ void __launch_bounds__(256) fm_sdp_assign(SdpSet s, long B) {
  const SdpDesc& d = s.t[blockIdx.y];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long n = B * d.bag;
  const GT* dy = reinterpret_cast<const GT*>(d.dy);
  for (long e = blockIdx.x * 4L + wave; e < n; e += (long)gridDim.x * 4) {
    bool ok;
    const long r = local_row(ldi<I64>(d.idx, e), d.lo, d.rows, ok);
    if (!ok || d.slot[r] != (int)e) continue;       // wave-uniform
    int u = 0;
    if (lane == 0) u = atomicAdd(d.count, 1);
    u = __shfl(u, 0, 64);
    const long b = e / d.bag;
    float* gu = d.g + (long)u * d.D;
    for (int c = lane; c < d.D; c += 64) gu[c] = ld<GT>(dy + b * d.ld + c) * d.scale;
    if (lane == 0) {
      d.ids[u] = (int)r;
      d.cid[e] = u;
    }
  }
}

template <typename GT, bool I64>
__global__ void __launch_bounds__(256) fm_sdp_dups(SdpSet s, long B) {
  const SdpDesc& d = s.t[blockIdx.y];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long n = B * d.bag;
  const GT* dy = reinterpret_cast<const GT*>(d.dy);
  for (long e = blockIdx.x * 4L + wave; e < n; e += (long)gridDim.x * 4) {
    bool ok;
    const long r = local_row(ldi<I64>(d.idx, e), d.lo, d.rows, ok);
    if (!ok) continue;
    const int own = d.slot[r];
    if (own == (int)e) continue;                     // the owner entry wrote g[u] itself
    const long b = e / d.bag;
    float* gu = d.g + (long)d.cid[own] * d.D;
    for (int c = lane; c < d.D; c += 64) atomicAdd(gu + c, ld<GT>(dy + b * d.ld + c) * d.scale);
  }
}

// one segment of the gathered payloads: W[ids[u]] -= lr * g[u] (rows unique within a segment)
struct SdpApply {
  float* W;
  const int* ids;
  const float* g;
  const int* count;
  int D;
  int* slot;          // own segment: free the claimed slots; else nullptr
  int* own_count;     // own segment: this rank's count, zeroed after use; else nullptr
};
struct SdpApplySet {
  SdpApply t[MAXT];
  int n;
};

__global__ void __launch_bounds__(256) fm_sdp_apply(SdpApplySet s, const float* __restrict__ lr, int nmax) {
  const SdpApply& d = s.t[blockIdx.y];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int cnt = min(*d.count, nmax);
  const float mlr = -lr[0];
  for (long u = blockIdx.x * 4L + wave; u < cnt; u += (long)gridDim.x * 4) {
    const long r = d.ids[u];
    float* w = d.W + r * d.D;
    const float* gu = d.g + u * d.D;
    for (int c = lane; c < d.D; c += 64) w[c] += mlr * gu[c];
    if (d.slot && lane == 0) d.slot[r] = -1;
  }
}

// zero the own counts once every segment has been applied (a separate tiny launch: the own
// segment's count may be read by later segments' launches only through the gathered copy)
__global__ void fm_sdp_reset_counts(SdpApplySet s) {
  if (threadIdx.x < s.n && s.t[threadIdx.x].own_count) *s.t[threadIdx.x].own_count = 0;
}

}  // namespace

// ------------------------------------------------------------------------------------------
// Launchers.  Arrays describe n tables; act/ld = outputs (fwd) or output grads (bwd).  Tables
// are batched by index width (and, in backward, by kernel kind) into launches of <= 32 tables.
// lo: first global row of each table shard (nullptr = whole tables); rows: rows held
extern "C" void fm_embedding_fwd_multi(int n, const float* const* W, const void* const* idx, const int* idx64,
                                       void* const* out, const long* ldo, const long* lo, const int* rows, const int* D,
                                       const int* bag, const float* scale, int out_bf16, long B, hipStream_t st) {
  if (B <= 0) return;
  for (int wide = 0; wide < 2; ++wide) {
    std::vector<int> sel;
    for (int k = 0; k < n; ++k)
      if ((idx64[k] != 0) == (wide != 0)) sel.push_back(k);
    for (size_t base = 0; base < sel.size(); base += MAXT) {
      TabSet s;
      int m = (int)std::min<size_t>(MAXT, sel.size() - base);
      bool vec = true;
      for (int i = 0; i < m; ++i) {
        int k = sel[base + i];
        s.t[i] = TabDesc{W[k], idx[k], out[k], ldo[k], lo ? lo[k] : 0, rows[k], D[k], bag[k], scale[k]};
        vec = vec && (D[k] % 4 == 0) && (ldo[k] % 4 == 0) && D[k] <= 256;
      }
      s.n = m;
      if (wide) launch_fwd<true>(s, m, vec, out_bf16, B, D[sel[base]], st);
      else launch_fwd<false>(s, m, vec, out_bf16, B, D[sel[base]], st);
    }
  }
}

static int g_emb_count = 0;    // fm_embedding_set_bwd_mode: 1 = the count / update pair
extern "C" void fm_embedding_set_bwd_mode(int count) { g_emb_count = count ? 1 : 0; }

// lr != nullptr: fused sparse SGD into W; lr == nullptr: W is a dense grad buffer (accumulate).
extern "C" void fm_embedding_bwd_multi(int n, float* const* W, const void* const* idx, const int* idx64,
                                       const void* const* dy, const long* ldg, const long* lo, const int* rows, const int* D,
                                       const int* bag, const float* scale, int dy_bf16, const float* lr, long B,
                                       int* const* owner, int* const* dups, int* const* ndup, hipStream_t st) {
  if (B <= 0) return;
  // owner-computes path: fused SGD, claim buffers given, 16-B rows; count mode: the count / update
  // pair instead of claim / dup / owner (the buffers are the same)
  const bool count_mode = g_emb_count == 1;
  auto claimable = [&](int k) {
    return lr != nullptr && owner != nullptr && owner[k] != nullptr && D[k] % 4 == 0 && ldg[k] % 4 == 0 &&
           D[k] <= 256;
  };
  for (int wide = 0; wide < 2; ++wide) {
    std::vector<int> sel;
    for (int k = 0; k < n; ++k)
      if (claimable(k) && (idx64[k] != 0) == (wide != 0)) sel.push_back(k);
    for (size_t base = 0; base < sel.size(); base += MAXT) {
      ClaimSet s;
      int m = (int)std::min<size_t>(MAXT, sel.size() - base);
      int maxbag = 1, minD4 = 64;
      for (int i = 0; i < m; ++i) {
        int k = sel[base + i];
        s.t[i] = ClaimDesc{W[k], idx[k], dy[k], ldg[k], lo ? lo[k] : 0, rows[k], D[k], bag[k], scale[k], owner[k], dups[k],
                           ndup[k]};
        maxbag = std::max(maxbag, bag[k]);
        minD4 = std::min(minD4, D[k] / 4);
      }
      s.n = m;
      if (count_mode) {
        if (wide) launch_count<true>(s, m, dy_bf16, lr, B, maxbag, minD4, st);
        else launch_count<false>(s, m, dy_bf16, lr, B, maxbag, minD4, st);
      } else if (wide) {
        launch_claim<true>(s, m, dy_bf16, lr, B, maxbag, minD4, st);
      } else {
        launch_claim<false>(s, m, dy_bf16, lr, B, maxbag, minD4, st);
      }
    }
  }
  // kind: 0 tiny (wave-private LDS copies), 2 regular (atomics).  Measured and deleted in r6: a
  // block-shared LDS copy for 36..155-row tables (113 vs 16.6 us of regular atomics) and row-block
  // ownership for <= 8192-row tables (76 vs 48 us; profiles/emb_bwd_rowblock_r5u.jsonl)
  auto kind_of = [&](int k) {
    // the wave-private LDS kernel up to TINY_ROWS rows while its four copies fit the LDS (rows * D *
    // 16 B).  64 takes the 36- and 63-row MLPerf tables off the same-address atomics: slower alone
    // (35.5 vs 32.3 us for the eight <= 155-row tables) but less contention beside the bottom-MLP
    // backward, step 1.145-1.164 vs 1.170-1.173 ms at 16 (profiles/emb_tiny_rows_ab_r5tr.txt).  A
    // block-shared copy with LDS float atomics for <= 160 rows measured 93.5 vs 30.5 us (r7, removed).
    constexpr int tiny_rows = 64;
    if (rows[k] <= tiny_rows && (long)rows[k] * D[k] * 16 <= (160L << 10) && D[k] <= 256 &&
        B * (long)bag[k] >= 16L * rows[k])
      return 0;
    return 2;
  };
  for (int pass = 0; pass < 4; ++pass) {
    const int kind = (pass >> 1) * 2;
    const bool tiny = kind == 0, wide = pass & 1;
    std::vector<int> sel;
    for (int k = 0; k < n; ++k) {
      if (claimable(k)) continue;
      if (kind_of(k) == kind && (idx64[k] != 0) == wide) sel.push_back(k);
    }
    for (size_t base = 0; base < sel.size(); base += MAXT) {
      TabSet s;
      int m = (int)std::min<size_t>(MAXT, sel.size() - base);
      int maxD = 1;
      for (int i = 0; i < m; ++i) {
        int k = sel[base + i];
        s.t[i] = TabDesc{W[k], idx[k], const_cast<void*>(dy[k]), ldg[k], lo ? lo[k] : 0, rows[k], D[k], bag[k], scale[k]};
        maxD = std::max(maxD, D[k]);
      }
      s.n = m;
      if (wide) {
        launch_bwd<true>(s, m, tiny, dy_bf16, lr, B, maxD, st);
      } else {
        launch_bwd<false>(s, m, tiny, dy_bf16, lr, B, maxD, st);
      }
    }
  }
}

// single-table conveniences
extern "C" void fm_embedding_fwd(const void* idx, int idx64, const float* W, void* out, int out_bf16, long B, int bag,
                                 int rows, int D, long ldo, float scale, hipStream_t s) {
  fm_embedding_fwd_multi(1, &W, &idx, &idx64, &out, &ldo, nullptr, &rows, &D, &bag, &scale, out_bf16, B, s);
}

extern "C" void fm_embedding_bwd(const void* idx, int idx64, const void* dy, int dy_bf16, float* W, const float* lr,
                                 long B, int bag, int rows, int D, long ldg, float scale, hipStream_t s) {
  fm_embedding_bwd_multi(1, &W, &idx, &idx64, &dy, &ldg, nullptr, &rows, &D, &bag, &scale, dy_bf16, lr, B, nullptr,
                         nullptr, nullptr, s);
}

// ---- sparse DP launchers -------------------------------------------------------------------
// coalesce: this rank's lookups of n replicated tables -> (count, ids, g) payloads
extern "C" void fm_sdp_coalesce(int n, const void* const* idx, const int* idx64, const void* const* dy, const long* ldg,
                                const long* lo, const int* rows, const int* D, const int* bag, const float* scale,
                                int dy_bf16, long B, int* const* slot, int* const* cid, int* const* ids, float* const* g,
                                int* const* count, hipStream_t st) {
  if (B <= 0 || n <= 0) return;
  for (int wide = 0; wide < 2; ++wide) {
    std::vector<int> sel;
    for (int k = 0; k < n; ++k)
      if ((idx64[k] != 0) == (wide != 0)) sel.push_back(k);
    for (size_t base = 0; base < sel.size(); base += MAXT) {
      SdpSet s;
      const int m = (int)std::min<size_t>(MAXT, sel.size() - base);
      int maxbag = 1;
      for (int i = 0; i < m; ++i) {
        const int k = sel[base + i];
        s.t[i] = SdpDesc{idx[k], dy[k], ldg[k], lo ? lo[k] : 0, rows[k], D[k], bag[k], scale[k], slot[k], cid[k], ids[k],
                         g[k], count[k]};
        maxbag = std::max(maxbag, bag[k]);
      }
      s.n = m;
      const long ne = B * maxbag;
      dim3 gc((unsigned)std::max<long>(1, std::min<long>((ne + 255) / 256, 1024)), m);
      dim3 gw((unsigned)std::max<long>(1, std::min<long>((ne + 3) / 4, 2048)), m);
      if (wide) {
        hipLaunchKernelGGL((fm_sdp_claim<true>), gc, dim3(256), 0, st, s, B);
        if (dy_bf16) {
          hipLaunchKernelGGL((fm_sdp_assign<unsigned short, true>), gw, dim3(256), 0, st, s, B);
          hipLaunchKernelGGL((fm_sdp_dups<unsigned short, true>), gw, dim3(256), 0, st, s, B);
        } else {
          hipLaunchKernelGGL((fm_sdp_assign<float, true>), gw, dim3(256), 0, st, s, B);
          hipLaunchKernelGGL((fm_sdp_dups<float, true>), gw, dim3(256), 0, st, s, B);
        }
      } else {
        hipLaunchKernelGGL((fm_sdp_claim<false>), gc, dim3(256), 0, st, s, B);
        if (dy_bf16) {
          hipLaunchKernelGGL((fm_sdp_assign<unsigned short, false>), gw, dim3(256), 0, st, s, B);
          hipLaunchKernelGGL((fm_sdp_dups<unsigned short, false>), gw, dim3(256), 0, st, s, B);
        } else {
          hipLaunchKernelGGL((fm_sdp_assign<float, false>), gw, dim3(256), 0, st, s, B);
          hipLaunchKernelGGL((fm_sdp_dups<float, false>), gw, dim3(256), 0, st, s, B);
        }
      }
    }
  }
}

// apply the gathered segments in order: segs x n tables; seg_ids/seg_g/seg_count[s*n + k]; the
// own segment (own_seg) frees slot[k] and zeroes own_count[k] afterwards
extern "C" void fm_sdp_apply_segments(int n, int segs, int own_seg, float* const* W, const int* D, const int* const* seg_ids,
                                      const float* const* seg_g, const int* const* seg_count, int* const* slot,
                                      int* const* own_count, const int* nmax, const float* lr, hipStream_t st) {
  if (n <= 0) return;
  for (size_t base = 0; base < (size_t)n; base += MAXT) {
    const int m = (int)std::min<size_t>(MAXT, n - base);
    int nm = 1;
    for (int i = 0; i < m; ++i) nm = std::max(nm, nmax[base + i]);
    dim3 grid((unsigned)std::max(1, std::min((nm + 3) / 4, 2048)), m);
    SdpApplySet last;
    for (int sg = 0; sg < segs; ++sg) {
      SdpApplySet s;
      for (int i = 0; i < m; ++i) {
        const int k = (int)base + i;
        const bool own = sg == own_seg;
        s.t[i] = SdpApply{W[k], seg_ids[sg * n + k], seg_g[sg * n + k], seg_count[sg * n + k], D[k], own ? slot[k] : nullptr,
                          own ? own_count[k] : nullptr};
      }
      s.n = m;
      hipLaunchKernelGGL(fm_sdp_apply, grid, dim3(256), 0, st, s, lr, nm);
      if (sg == own_seg) last = s;
    }
    if (own_seg >= 0 && own_seg < segs) hipLaunchKernelGGL(fm_sdp_reset_counts, dim3(1), dim3(64), 0, st, last);
  }
}
