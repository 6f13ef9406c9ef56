// Shared pieces of flexmi's fp32 MFMA GEMMs (gemm_f32.hip, gemm_x3.hip): the parameter block,
// LDS image helpers, fragment loads and the fused epilogues (bias / activation / activation-backward /
// bias-gradient column sums / beta accumulate / split-K slabs / fused SGD).  Internal linkage: every
// translation unit gets its own copy.
#pragma once
#include "gemm_common.h"

namespace {

constexpr int NTF = 256;   // threads per block
constexpr int BKF = 32;    // k per LDS tile (fp32)

struct GemmF {
  const float* A; long lda; long sA;
  const float* B; long ldb; long sB;
  float* C; long ldc; long sC;
  const float* bias;
  float* ws;            // split-K slabs [batch][split][M][N]
  const float* ay;      // fused act-bwd of the layer below: v = act'(ay) * v
  long lday;
  float* colsum;        // += column sums of the (post act-bwd) output
  float* rowsum_a;      // += sum_k A(m,k)  (MN-contiguous A only)
  int bact;
  int M, N, K, act, beta, ksplit, batch;
  float alpha;
  int tiles_m, tiles_n, n_fast;
  // fused SGD (fm_gemm_f32_dw_sgd; default register-staged kernel and its reduce only): the
  // epilogue updates W (same [M][ldc] layout as C) instead of storing the gradient
  float* uw;
  unsigned short* uwc;
  float* uv;
  const float* ulr;
  float uwd, umom;
  int unest;
  int ulds;             // unsplit tiles stage the update through LDS (sgd_epilogue_lds_f32)
  int dma;              // operands staged by LDS-DMA (gemm_f32.hip: full tiles, no row sums)
  // fp16 two-plane split (gemm_x3.hip F16 form): max |x| bit patterns of every A row (M index) and
  // every B column (N index) over K, from fm_f32_amax (the per-row / per-column power-of-two scales)
  const unsigned* amax_a;
  const unsigned* amax_b;
  int amax_na, amax_nb;   // partials per index (strides M / N): the scale takes their max
};

// the max over the np partials of index i (stride n)
FM_DEVICE unsigned amax_of(const unsigned* a, int np, int n, int i) {
  unsigned v = a[i];
  for (int k = 1; k < np; ++k) v = max(v, a[(long)k * n + i]);
  return v;
}

// power-of-two scale of a row / column whose max |x| has bit pattern mb: 2^sig with
// max * 2^sig in [2^14, 2^15) (an fp16 holds it with 11 significant bits and no overflow; a subnormal
// max counts by its leading bit); an all-zero row takes sig 0.  sig is clamped to the normal fp32
// exponent range, so rows below 2^-112 keep fp16 subnormal precision only (as fp32 itself does there).
FM_DEVICE int f16_sig(unsigned mb) {
  if (mb == 0) return 0;
  const int e = (int)(mb >> 23);
  const int eu = e ? e - 127 : (31 - __clz(mb)) - 149;
  const int sg = 14 - eu;
  return sg > 126 ? 126 : (sg < -126 ? -126 : sg);
}
FM_DEVICE float pow2f(int e) { return __uint_as_float((unsigned)(e + 127) << 23); }   // e in [-126, 127]

template <int N>
using fvec = float __attribute__((ext_vector_type(N)));

FM_DEVICE int xcd_remap_f(int bid, int ntiles) {
  int q = ntiles / 8, r = ntiles % 8, x = bid % 8;
  if (ntiles >= 8) bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  return bid;
}

// byte offset of 16-B chunk c (4 floats) of row r in a K-contiguous image (128-B rows)
FM_DEVICE int kc_off(int r, int c) { return r * (BKF * 4) + 16 * (c ^ ((r >> 1) & 7)); }

// ---- global -> registers -> LDS (one operand tile) ----------------------------------------
template <bool KC, int R, bool VEC, int NT = NTF>
struct StageF {
  static constexpr int CHUNKS = R * BKF / 4;
  static constexpr int PER_T = CHUNKS / NT;
  static_assert(PER_T >= 1 && CHUNKS % NT == 0, "tile too small for the block");
  f32x4_t v[PER_T];

  FM_DEVICE void load(const float* __restrict__ p, long ld, int row0, int rows, int k0, int K, int tid) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int ci = tid + NT * i;
      int gr, gk;
      if constexpr (KC) {
        gr = row0 + (ci >> 3);
        gk = k0 + 4 * (ci & 7);
      } else {
        gk = k0 + ci / (R / 4);
        gr = row0 + 4 * (ci % (R / 4));
      }
      if constexpr (VEC) {
        if (gr < rows && gk < K) {
          const float* src = KC ? (p + (long)gr * ld + gk) : (p + (long)gk * ld + gr);
          v[i] = *reinterpret_cast<const f32x4_t*>(src);
        } else {
          v[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int rr = KC ? gr : gr + j;
          const int kk = KC ? gk + j : gk;
          v[i][j] = (rr < rows && kk < K) ? (KC ? p[(long)rr * ld + kk] : p[(long)kk * ld + rr]) : 0.f;
        }
      }
    }
  }

  FM_DEVICE void store(char* lds, int tid) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int ci = tid + NT * i;
      int off;
      if constexpr (KC) off = kc_off(ci >> 3, ci & 7);
      else off = (ci / (R / 4)) * (R * 4) + 16 * (ci % (R / 4));
      *reinterpret_cast<f32x4_t*>(lds + off) = v[i];
    }
  }

  // MN-contiguous operand: every chunk of this thread covers the same 4 rows (tid % (R/4)),
  // so per-thread sums over the staged k are row partial sums (bias grad inside the dW GEMM)
  FM_DEVICE void accumulate_rows(float (&s)[4]) const {
#pragma unroll
    for (int i = 0; i < PER_T; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) s[j] += v[i][j];
  }
};

typedef __attribute__((address_space(1))) const void* gptr_s;
typedef __attribute__((address_space(3))) void* lptr_s;

// global -> LDS by LDS-DMA (global_load_lds_dwordx4: 1 KiB per wave-instruction, lane L's 16 B at
// base + 16 L): each lane loads the chunk the image layout (kc_off swizzle / linear MN rows) puts at
// its slot.  Full tiles only (the caller guarantees M, N multiples of the tile and K of BKF).
template <bool KC, int R, int NT>
struct DmaStageF {
  static constexpr int BYTES = R * BKF * 4;
  static constexpr int PER_W = BYTES / 1024 / (NT / 64);
  static_assert(PER_W >= 1 && BYTES % (1024 * (NT / 64)) == 0, "whole 1-KiB pieces per wave");
  FM_DEVICE static void issue(const float* __restrict__ p, long ld, int row0, int k0, char* lds, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < PER_W; ++i) {
      const int piece = wave * PER_W + i;
      const int o = piece * 1024 + 16 * lane;
      const float* src;
      if constexpr (KC) {
        const int row = o / (BKF * 4), slot = (o % (BKF * 4)) / 16;
        src = p + (long)(row0 + row) * ld + k0 + 4 * (slot ^ ((row >> 1) & 7));
      } else {
        const int kr = o / (R * 4), ch = (o % (R * 4)) / 16;
        src = p + (long)(k0 + kr) * ld + row0 + 4 * ch;
      }
      __builtin_amdgcn_global_load_lds((gptr_s)(const void*)src, (lptr_s)(void*)(lds + piece * 1024), 16, 0, 0);
    }
  }
};

// fragments of one operand for one 16-wide k-chunk: f[t][s] = element (tile t, k-step s)
template <bool KC, int R, int T>
FM_DEVICE void load_frags(const char* lds, int base, int kk, int lane, float (&f)[T][4]) {
  const int q = lane & 15, g = lane >> 4;
  if constexpr (KC) {
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const f32x4_t x = *reinterpret_cast<const f32x4_t*>(lds + kc_off(base + 16 * t + q, 4 * kk + g));
#pragma unroll
      for (int s = 0; s < 4; ++s) f[t][s] = x[s];
    }
  } else {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int k = 16 * kk + 4 * g + s;
      const fvec<T> x = *reinterpret_cast<const fvec<T>*>(lds + k * (R * 4) + 4 * (base + T * q));
#pragma unroll
      for (int t = 0; t < T; ++t) f[t][s] = x[t];
    }
  }
}

// ---- epilogue ---------------------------------------------------------------------------------
// lane (q = lane&15, g = lane>>4) holds acc[i][j][r] = C[m(i, q)][n(j, 4g + r)] with
//   m = IL_A ? mbase + MR*q + i : mbase + 16i + q          (IL = MN-contiguous operand)
//   n = IL_B ? nbase + NR*qn + j : nbase + 16j + qn        (qn = 4g + r)
// processed as NR quads of 4 consecutive columns per row.
template <int MR, int NR, bool IL_A, bool IL_B>
FM_DEVICE void quad_of(const f32x4_t (&acc)[MR][NR], int i, int u, int nbase, int g, int& n0, float (&v)[4]) {
  if constexpr (IL_B) {
    n0 = nbase + 4 * NR * g + 4 * u;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = acc[i][(4 * u + e) % NR][(4 * u + e) / NR];
  } else {
    n0 = nbase + 16 * u + 4 * g;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = acc[i][u][e];
  }
}

template <int MR, int NR, bool IL_A, bool IL_B, bool SGD = false>
FM_DEVICE void epilogue_f32(const GemmF& p, const f32x4_t (&acc)[MR][NR], int zb, int split, int mbase, int nbase,
                            int lane) {
  const int q = lane & 15, g = lane >> 4;
  if (p.ksplit > 1) {
    float* ws = p.ws + ((long)zb * p.ksplit + split) * (long)p.M * p.N;
    const bool v4 = (p.N & 3) == 0;
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      const int m = IL_A ? mbase + MR * q + i : mbase + 16 * i + q;
      if (m >= p.M) continue;
#pragma unroll
      for (int u = 0; u < NR; ++u) {
        int n0;
        float v[4];
        quad_of<MR, NR, IL_A, IL_B>(acc, i, u, nbase, g, n0, v);
        float* dst = ws + (long)m * p.N + n0;
        if (v4 && n0 + 3 < p.N) {
          *reinterpret_cast<f32x4_t*>(dst) = f32x4_t{v[0], v[1], v[2], v[3]};
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (n0 + e < p.N) dst[e] = v[e];
        }
      }
    }
    return;
  }
  float csum[NR][4];
#pragma unroll
  for (int u = 0; u < NR; ++u)
#pragma unroll
    for (int e = 0; e < 4; ++e) csum[u][e] = 0.f;
  float* Cz = p.C + (long)zb * p.sC;
#pragma unroll
  for (int i = 0; i < MR; ++i) {
    const int m = IL_A ? mbase + MR * q + i : mbase + 16 * i + q;
    const bool mok = m < p.M;
#pragma unroll
    for (int u = 0; u < NR; ++u) {
      int n0;
      float v[4];
      quad_of<MR, NR, IL_A, IL_B>(acc, i, u, nbase, g, n0, v);
      const bool full = n0 + 3 < p.N;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] *= p.alpha;
        if (p.bias) v[e] += (n0 + e < p.N) ? p.bias[n0 + e] : 0.f;
        v[e] = act_fwd(p.act, v[e]);
      }
      if (p.ay) {
        float yv[4] = {0.f, 0.f, 0.f, 0.f};
        if (mok) {
          const float* yp = p.ay + (long)m * p.lday + n0;
          if (full && ((p.lday & 3) == 0)) {
            const f32x4_t t = *reinterpret_cast<const f32x4_t*>(yp);
#pragma unroll
            for (int e = 0; e < 4; ++e) yv[e] = t[e];
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) yv[e] = (n0 + e < p.N) ? yp[e] : 0.f;
          }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = act_bwd(p.bact, yv[e], v[e]);
      }
      if (p.colsum && mok) {
#pragma unroll
        for (int e = 0; e < 4; ++e) csum[u][e] += (n0 + e < p.N) ? v[e] : 0.f;
      }
      if (!mok) continue;
      if constexpr (SGD) {
        const long o = (long)m * p.ldc + n0;
        if (full) {
          sgd_apply4(p, o, f32x4_t{v[0], v[1], v[2], v[3]});
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (n0 + e < p.N) sgd_apply1(p, o + e, v[e]);
        }
        continue;
      }
      float* dst = Cz + (long)m * p.ldc + n0;
      if (full && ((p.ldc & 3) == 0) && ((((uintptr_t)dst) & 15) == 0)) {
        f32x4_t o = {v[0], v[1], v[2], v[3]};
        if (p.beta) o += *reinterpret_cast<const f32x4_t*>(dst);
        *reinterpret_cast<f32x4_t*>(dst) = o;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (n0 + e < p.N) dst[e] = v[e] + (p.beta ? dst[e] : 0.f);
      }
    }
  }
  if (p.colsum) {   // the 16 lanes of a group share every column: reduce over q, one atomic per column
#pragma unroll
    for (int u = 0; u < NR; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x = csum[u][e];
        x += __shfl_xor(x, 1, 64);
        x += __shfl_xor(x, 2, 64);
        x += __shfl_xor(x, 4, 64);
        x += __shfl_xor(x, 8, 64);
        const int n = (IL_B ? nbase + 4 * NR * g + 4 * u : nbase + 16 * u + 4 * g) + e;
        if (q == 0 && n < p.N) atomicAdd(p.colsum + n, x);
      }
  }
}

// Fused-SGD epilogue of an unsplit fp32 dW tile through LDS (same scheme as gemm.hip
// sgd_epilogue_lds): the accumulator quads (quad_of, incl. the interleaved layouts) are parked in
// the free operand LDS with row-XOR-swizzled 16-B chunks, then whole rows of W are updated with
// contiguous BN*4-byte accesses.  BM*BN*4 <= 2*(BM+BN)*BKF*4: the tile fits the K-loop LDS.
template <int BM, int BN, int NT, int MR, int NR, bool IL_A, bool IL_B, int LDSB>
FM_DEVICE void sgd_epilogue_lds_f32(const GemmF& p, const f32x4_t (&acc)[MR][NR], char* smem, int m0, int n0,
                                    int mbase, int nbase, int lane, int tid) {
  constexpr int CPR = BN / 4;
  static_assert(BM * BN * 4 <= LDSB, "fp32 tile must fit the kernel's LDS");
  static_assert(CPR >= 8, "row XOR swizzle (r & 7) needs >= 8 chunks per row");
  f32x4_t* t = reinterpret_cast<f32x4_t*>(smem);
  const int q = lane & 15, g = lane >> 4;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < MR; ++i) {
    const int r = (IL_A ? mbase + MR * q + i : mbase + 16 * i + q) - m0;
#pragma unroll
    for (int u = 0; u < NR; ++u) {
      int nn;
      float v[4];
      quad_of<MR, NR, IL_A, IL_B>(acc, i, u, nbase, g, nn, v);
      const int c = (nn - n0) >> 2;
      t[r * CPR + (c ^ (r & 7))] = f32x4_t{v[0], v[1], v[2], v[3]} * p.alpha;
    }
  }
  __syncthreads();
  const bool n4 = (p.N & 3) == 0;
#pragma unroll 4
  for (int e = tid; e < BM * CPR; e += NT) {
    const int r = e / CPR, c = e % CPR;
    const int m = m0 + r, n = n0 + 4 * c;
    if (m >= p.M || n >= p.N) continue;
    const f32x4_t gv = t[r * CPR + (c ^ (r & 7))];
    const long o = (long)m * p.ldc + n;
    if (n4 && n + 3 < p.N) {
      sgd_apply4(p, o, gv);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (n + k < p.N) sgd_apply1(p, o + k, gv[k]);
    }
  }
}


typedef __attribute__((address_space(1))) const void* gptr_f;
typedef __attribute__((address_space(3))) void* lptr_f;

template <int N>
FM_DEVICE void wait_vmcnt_f() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

}  // namespace
