// Shared pieces of flexmi's MFMA GEMM kernels (gemm.hip register-staged bf16,
// gemm_f32.hip / gemm_x3.hip fp32): LDS operand images + swizzles, MFMA fragment reads, the parameter block and the
// fused epilogue (alpha, bias, activation, fused activation-backward of the layer below, beta
// accumulate, bf16/fp32 output, split-K slabs).
#pragma once
#include "common.h"

namespace {

constexpr int BK = 64;

typedef __attribute__((address_space(3))) bf16x4_t lds_v4_t;

// MN-contiguous operand image [k][R rows]: XOR swizzle of 16-B chunks per k-row so the
// transposing ds_read_b64_tr_b16 fragment reads of a 32-lane half hit every bank once.
template <int R>
struct MNSwz;
template <>
struct MNSwz<256> {  // 512-B rows, 32 chunks (same pattern as 128: stays inside 16-chunk halves)
  static FM_DEVICE int f(int k) { return 2 * ((k & 3) | (((k >> 3) & 1) << 2)); }
};
template <>
struct MNSwz<128> {  // 256-B rows, 16 chunks
  static FM_DEVICE int f(int k) { return 2 * ((k & 3) | (((k >> 3) & 1) << 2)); }
};
template <>
struct MNSwz<64> {  // 128-B rows, 8 chunks
  static FM_DEVICE int f(int k) { return 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1)); }
};

// byte offset inside an operand LDS image.  K-contiguous image [row][64 k] (128-B rows, 16-B
// chunks XOR-swizzled by (row>>1)&7): conflict-free ds_read_b128 fragment reads.
template <bool KC, int R>
FM_DEVICE int lds_off(int row_or_k, int chunk) {
  if constexpr (KC) {
    return row_or_k * (BK * 2) + 16 * (chunk ^ ((row_or_k >> 1) & 7));
  } else {
    return row_or_k * (R * 2) + 16 * (chunk ^ MNSwz<R>::f(row_or_k));
  }
}

// ---- LDS -> MFMA fragment (8 bf16: k = 8*(lane>>4)+j for row/col lane&15) -------------
template <bool KC, int R>
FM_DEVICE bf16x8_t frag(const char* lds, int base, int kk, int lane) {
  if constexpr (KC) {
    int row = base + (lane & 15);
    int chunk = 4 * kk + (lane >> 4);
    return *reinterpret_cast<const bf16x8_t*>(lds + lds_off<true, R>(row, chunk));
  } else {
    int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    int chunk = (base >> 3) + (p >> 1);
    int k0 = 32 * kk + 8 * g + q;
    int o0 = lds_off<false, R>(k0, chunk) + 8 * (p & 1);
    int o1 = lds_off<false, R>(k0 + 4, chunk) + 8 * (p & 1);
    bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4_t*)(lds + o0));
    bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4_t*)(lds + o1));
    bf16x8_t r;
    r.lo = lo;
    r.hi = hi;
    return r;
  }
}

struct GemmP {
  const unsigned short* A; long lda; long sA;
  const unsigned short* B; long ldb; long sB;
  void* C; long ldc; long sC;
  const float* bias;
  float* ws;          // split-K slabs [batch][split][M][N]
  // fused backward epilogue of the producing layer below: v = act'(ay) * v ; colsum[n] += sum_m v
  const unsigned short* ay;
  long lday;
  float* colsum;
  float* rowsum_a;   // += sum_k A(m,k)  (MN-contiguous A only; used for bias grads in dW GEMMs)
  int bact;
  int M, N, K, act, beta, c_fp32, ksplit, batch;
  float alpha;
  int tiles_m, tiles_n;
  int n_fast;   // tile order: column tiles fastest (A row-block reused by consecutive tiles on one XCD)
  // fused SGD (dW GEMMs whose gradient has no other consumer): instead of storing the gradient,
  // the epilogue updates the fp32 master W (same [M][ldc] layout as C), its momentum and bf16 mirror
  // exactly as fm_sgd_kernel would (optim.hip) -- the gradient never round-trips through HBM
  float* uw;             // nullptr = plain GEMM
  unsigned short* uwc;   // bf16 compute mirror (nullptr: none)
  float* uv;             // momentum buffer (used when umom > 0)
  const float* ulr;      // device-side learning rate
  float uwd, umom;
  int unest;
  int ulds;              // unsplit tiles stage the update through LDS (gemm.hip sgd_epilogue_lds)
  int dma;   // operands staged by LDS-DMA (gemm.hip: full tiles, no row sums)
};

// W -= lr * (g + wd W) (momentum / Nesterov as fm_sgd_kernel), one element at offset o of W
// (P = GemmP or gemm_f32.hip's GemmF: the same uw / uwc / uv / ulr / uwd / umom / unest fields)
template <class P>
FM_DEVICE void sgd_apply1(const P& p, long o, float g) {
  const float lr = p.ulr[0];
  float w = p.uw[o];
  g += p.uwd * w;
  if (p.umom > 0.f) {
    const float v = p.uv[o] * p.umom + g;
    p.uv[o] = v;
    g = p.unest ? g + p.umom * v : v;
  }
  w -= lr * g;
  p.uw[o] = w;
  if (p.uwc) p.uwc[o] = f2bf(w);
}

// four consecutive elements at a 16-B aligned offset o
template <class P>
FM_DEVICE void sgd_apply4(const P& p, long o, f32x4_t g) {
  const float lr = p.ulr[0];
  f32x4_t w = *reinterpret_cast<const f32x4_t*>(p.uw + o);
  g += p.uwd * w;
  if (p.umom > 0.f) {
    const f32x4_t v = *reinterpret_cast<const f32x4_t*>(p.uv + o) * p.umom + g;
    *reinterpret_cast<f32x4_t*>(p.uv + o) = v;
    g = p.unest ? g + p.umom * v : v;
  }
  w -= lr * g;
  *reinterpret_cast<f32x4_t*>(p.uw + o) = w;
  if (p.uwc) {
    bf16x4_t c;
#pragma unroll
    for (int r = 0; r < 4; ++r) c[r] = (short)f2bf(w[r]);
    *reinterpret_cast<bf16x4_t*>(p.uwc + o) = c;
  }
}

// tile coordinates of remapped block id: consecutive ids share an XCD (xcd_remap), so the
// operand traversed slowest stays resident in that XCD's 4 MB L2 while the other streams
FM_DEVICE void tile_coords(const GemmP& p, int bid, int& tm, int& tn) {
  if (p.n_fast) {
    tn = bid % p.tiles_n;
    tm = bid / p.tiles_n;
  } else {
    tm = bid % p.tiles_m;
    tn = bid / p.tiles_m;
  }
}

// Sum of ks split-K slabs (MN floats apart) in slab order, with up to eight loads in flight: a
// plain `for k: s += slab[k]` waits for each load before issuing the next (one HBM round trip per
// slab -- 16 us for a 16-way reduce).  Same additions in the same order as that loop.
FM_DEVICE f32x4_t slab_sum4(const float* __restrict__ src, long MN, int ks) {
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  int k = 0;
  for (; k + 8 <= ks; k += 8) {
    f32x4_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const f32x4_t*>(src + (long)(k + u) * MN);
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  if (k + 4 <= ks) {
    f32x4_t v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const f32x4_t*>(src + (long)(k + u) * MN);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += v[u];
    k += 4;
  }
  for (; k < ks; ++k) acc += *reinterpret_cast<const f32x4_t*>(src + (long)k * MN);
  return acc;
}
FM_DEVICE float slab_sum1(const float* __restrict__ src, long MN, int ks) {
  float acc = 0.f;
  int k = 0;
  for (; k + 8 <= ks; k += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = src[(long)(k + u) * MN];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; k < ks; ++k) acc += src[(long)k * MN];
  return acc;
}

// XCD-aware bijective remap of the tile id (blocks b and b+8 share an XCD)
FM_DEVICE int xcd_remap(int bid, int ntiles) {
  int q = ntiles / 8, r = ntiles % 8, x = bid % 8;
  if (ntiles >= 8) bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  return bid;
}

// ---- epilogue: lane owns C[m][n..n+3], m = lane&15, n = 4*(lane>>4) of each 16x16 tile;
// tile (i, j) of the wave covers rows mbase+16i.., cols nbase+16j..
// SGD: the fused-SGD instantiation (dW GEMMs of fm_gemm_dw_sgd); plain GEMMs compile without it
template <int MR, int NR, bool SGD = false>
FM_DEVICE void gemm_epilogue_store(const GemmP& p, const f32x4_t (&acc)[MR][NR], int zb, int mbase, int nbase, int lane);

template <int MR, int NR, bool SGD = false>
FM_DEVICE void gemm_epilogue(const GemmP& p, const f32x4_t (&acc)[MR][NR], int zb, int split, int mbase, int nbase,
                             int lane) {
  const int mrow = lane & 15;
  const int ncol = 4 * (lane >> 4);
  if (p.ksplit > 1) {   // split-K partial tile -> fp32 slab [batch][split][M][N] (reduce launch)
    float* ws = p.ws + ((long)zb * p.ksplit + split) * (long)p.M * p.N;
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        int m = mbase + 16 * i + mrow;
        int n = nbase + 16 * j + ncol;
        if (m >= p.M) continue;
        float* dst = ws + (long)m * p.N + n;
        if (n + 3 < p.N && (p.N & 3) == 0) {
          *reinterpret_cast<f32x4_t*>(dst) = acc[i][j];
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n + r < p.N) dst[r] = acc[i][j][r];
        }
      }
    return;
  }
  gemm_epilogue_store<MR, NR, SGD>(p, acc, zb, mbase, nbase, lane);
}

template <int MR, int NR, bool SGD>
FM_DEVICE void gemm_epilogue_store(const GemmP& p, const f32x4_t (&acc)[MR][NR], int zb, int mbase, int nbase, int lane) {
  const int mrow = lane & 15;
  const int ncol = 4 * (lane >> 4);
  float csum[NR][4];
#pragma unroll
  for (int j = 0; j < NR; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) csum[j][r] = 0.f;
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int m = mbase + 16 * i + mrow;
      const int n = nbase + 16 * j + ncol;
      const bool mok = m < p.M;
      const bool full = (n + 3 < p.N);
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] * p.alpha;
      if (p.bias) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += (n + r < p.N) ? p.bias[n + r] : 0.f;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = act_fwd(p.act, v[r]);
      if (p.ay) {  // fused activation backward of the layer below (dX -> dpre)
        float yv[4] = {0.f, 0.f, 0.f, 0.f};
        if (mok) {
          const unsigned short* yp = p.ay + (long)m * p.lday + n;
          if (full && ((p.lday & 3) == 0)) {
            bf16x4_t t = *reinterpret_cast<const bf16x4_t*>(yp);
#pragma unroll
            for (int r = 0; r < 4; ++r) yv[r] = bf2f((unsigned short)t[r]);
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) yv[r] = (n + r < p.N) ? bf2f(yp[r]) : 0.f;
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = act_bwd(p.bact, yv[r], v[r]);
      }
      if (p.colsum && mok) {
#pragma unroll
        for (int r = 0; r < 4; ++r) csum[j][r] += (n + r < p.N) ? v[r] : 0.f;
      }
      if (!mok) continue;
      if constexpr (SGD) {   // fused SGD: the host guarantees ldc % 4 == 0 and 16-B aligned W / V / C
        const long o = (long)m * p.ldc + n;
        if (full) {
          sgd_apply4(p, o, f32x4_t{v[0], v[1], v[2], v[3]});
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n + r < p.N) sgd_apply1(p, o + r, v[r]);
        }
        continue;
      }
      if (p.c_fp32) {
        float* dst = reinterpret_cast<float*>(p.C) + (long)zb * p.sC + (long)m * p.ldc + n;
        if (full && ((p.ldc & 3) == 0) && ((((uintptr_t)dst) & 15) == 0)) {
          f32x4_t o = {v[0], v[1], v[2], v[3]};
          if (p.beta) o += *reinterpret_cast<f32x4_t*>(dst);
          *reinterpret_cast<f32x4_t*>(dst) = o;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n + r < p.N) dst[r] = v[r] + (p.beta ? dst[r] : 0.f);
        }
      } else {
        unsigned short* dst = reinterpret_cast<unsigned short*>(p.C) + (long)zb * p.sC + (long)m * p.ldc + n;
        if (full && ((p.ldc & 3) == 0) && ((((uintptr_t)dst) & 7) == 0)) {
          if (p.beta) {
            bf16x4_t old = *reinterpret_cast<bf16x4_t*>(dst);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += bf2f((unsigned short)old[r]);
          }
          bf16x4_t o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(v[r]);
          *reinterpret_cast<bf16x4_t*>(dst) = o;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n + r < p.N) dst[r] = f2bf(v[r] + (p.beta ? bf2f(dst[r]) : 0.f));
        }
      }
    }
  if (p.colsum) {  // bias gradient of the layer below: reduce the 16 rows of each lane group, 1 atomic/col
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float x = csum[j][r];
        x += __shfl_xor(x, 1, 64);
        x += __shfl_xor(x, 2, 64);
        x += __shfl_xor(x, 4, 64);
        x += __shfl_xor(x, 8, 64);
        const int n = nbase + 16 * j + ncol + r;
        if (mrow == 0 && n < p.N) atomicAdd(p.colsum + n, x);
      }
  }
}

}  // namespace
