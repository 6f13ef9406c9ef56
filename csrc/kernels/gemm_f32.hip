// flexmi fp32 MFMA GEMM for gfx950 (MI355X / CDNA4) -- the reference-precision path.
//
//   C[M,N] (+)= epilogue( alpha * sum_k A(m,k) * B(k,n) )      fp32 in, fp32 accumulate, fp32 out
//
// The reference is fp32 end to end (cublasSgemm, src/ops/linear.cu:432-441 fwd, :616-634 dW/dX,
// src/ops/batch_matmul.cu:199-201).  CDNA4 has an exact f32-input MFMA
// (v_mfma_f32_16x16x4_f32: one k-ordered fmaf chain per output, 64 FLOP/clk/SIMD = 157 TF/s chip
// peak) and no xf32, so this kernel runs the fp32 products on the matrix cores and leaves the
// VALU for the fused epilogue.
//
// Tile BM x BN x 32 (fp32), 256 threads = 4 waves (2x2); a wave owns (BM/2) x (BN/2) as MR x NR
// 16x16 MFMA tiles.  The K index inside a 16-wide k-chunk is permuted per lane group
// (g = lane>>4 takes k = 4g + s at MFMA step s) so that ONE 16-B LDS read feeds several MFMAs:
//   * K-contiguous operand (A [M][K] / B [N][K]): LDS image [row][32 floats] (128-B rows, 16-B
//     chunks XOR-swizzled by (row>>1)&7 -> conflict-free ds_read_b128); one b128 read = the 4
//     k-steps of one 16x16 tile.
//   * MN-contiguous operand (A [K][M] / B [K][N]): LDS image [k][R floats]; the wave's rows are
//     INTERLEAVED over its tiles (tile t, lane row q -> row base + T*q + t) so one b128 read at a
//     fixed k gives the fragments of all T tiles.  No transposed copies, no scalar LDS reads.
// The epilogue undoes the interleave: each lane owns groups of 4 consecutive output columns
// (16-B stores).  Fused epilogue like the bf16 kernel (gemm_common.h): alpha, bias[n],
// activation, activation-backward of the layer below (y fp32) + its bias-gradient column sums,
// beta accumulate; dW GEMMs fold the bias gradient in as row sums of the staged A tiles.
// Split-K writes fp32 slabs reduced by one vectorised reduce launch.  XCD-aware tile order.
#include "gemm_f32_common.h"

#include <algorithm>
#include <cstdlib>

namespace {

// OPT: 1 = s_setprio(1) around each MFMA cluster (A/B only); 2 = fragment double buffer (default):
// the second k-chunk's LDS fragments are read before the first chunk's MFMAs and interleaved with
// them (sched_group_barrier).  Measured A/B, incl. removed experiments (de-phased blocks, diagnostic
// kernels without the K-loop loads / stores): profiles/gemm_f32_variants_ab.jsonl, gemm_f32_diag.jsonl.
// NT = 256 (4 waves, 2x2, wave tile BM/2 x BN/2) or 512 (8 waves, 2x4 for BN >= 128, else 4x2:
// twice the waves per SIMD to cover the LDS-read and barrier latency of each K tile).
template <int BM, int BN, bool AK, bool BKC, bool VEC, int OPT = 0, int NT = NTF, int MINB = 2, bool SGD = false>
__global__ void __launch_bounds__(NT, MINB) fm_gemm_f32_kernel(GemmF p) {
  constexpr int A_BYTES = BM * BKF * 4;
  constexpr int B_BYTES = BN * BKF * 4;
  constexpr int WN = (NT == 512 && BN >= 128) ? 4 : 2;
  constexpr int WM = NT / 64 / WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MR = TM / 16;
  constexpr int NR = TN / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  const int bid = xcd_remap_f(blockIdx.x, p.tiles_m * p.tiles_n);
  int tm, tn;
  if (p.n_fast) { tn = bid % p.tiles_n; tm = bid / p.tiles_n; }
  else { tm = bid % p.tiles_m; tn = bid / p.tiles_m; }
  const int zb = blockIdx.y;
  const int split = blockIdx.z;
  const int m0 = tm * BM, n0 = tn * BN;
  const float* A = p.A + (long)zb * p.sA;
  const float* B = p.B + (long)zb * p.sB;

  const int ktiles_total = (p.K + BKF - 1) / BKF;
  const int kt_per = (ktiles_total + p.ksplit - 1) / p.ksplit;
  const int kt0 = split * kt_per;
  const int kt1 = min(ktiles_total, kt0 + kt_per);

  f32x4_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  StageF<AK, BM, VEC, NT> sa;
  StageF<BKC, BN, VEC, NT> sb;
  const bool rowsum = (!AK) && (p.rowsum_a != nullptr) && (tn == 0);
  float rs[4] = {0.f, 0.f, 0.f, 0.f};
#define LDSF_A(b) (smem + (b) * (A_BYTES + B_BYTES))
#define LDSF_B(b) (smem + (b) * (A_BYTES + B_BYTES) + A_BYTES)
  if (kt0 < kt1) {
    sa.load(A, p.lda, m0, p.M, kt0 * BKF, p.K, tid);
    sb.load(B, p.ldb, n0, p.N, kt0 * BKF, p.K, tid);
    sa.store(LDSF_A(0), tid);
    sb.store(LDSF_B(0), tid);
    if (rowsum) sa.accumulate_rows(rs);
  }
  __syncthreads();
  for (int kt = kt0; kt < kt1; ++kt) {
    const int cur = (kt - kt0) & 1;
    const bool more = kt + 1 < kt1;
    if (more) {
      sa.load(A, p.lda, m0, p.M, (kt + 1) * BKF, p.K, tid);
      sb.load(B, p.ldb, n0, p.N, (kt + 1) * BKF, p.K, tid);
    }
    if constexpr ((OPT & 2) != 0) {
      float af0[MR][4], bf0[NR][4], af1[MR][4], bf1[NR][4];
      load_frags<AK, BM, MR>(LDSF_A(cur), wm * TM, 0, lane, af0);
      load_frags<BKC, BN, NR>(LDSF_B(cur), wn * TN, 0, lane, bf0);
      load_frags<AK, BM, MR>(LDSF_A(cur), wm * TM, 1, lane, af1);
      load_frags<BKC, BN, NR>(LDSF_B(cur), wn * TN, 1, lane, bf1);
      if constexpr ((OPT & 1) != 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < MR; ++i)
#pragma unroll
          for (int j = 0; j < NR; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(bf0[j][s], af0[i][s], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < MR; ++i)
#pragma unroll
          for (int j = 0; j < NR; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(bf1[j][s], af1[i][s], acc[i][j], 0, 0, 0);
      if constexpr ((OPT & 1) != 0) __builtin_amdgcn_s_setprio(0);
      // first chunk's reads, then one ds_read per MFMA for the second chunk's fragments
      __builtin_amdgcn_sched_group_barrier(0x100, MR + NR, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
#pragma unroll
      for (int x = 0; x < MR + NR; ++x) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      }
    } else {
#pragma unroll
    for (int kk = 0; kk < BKF / 16; ++kk) {
      float af[MR][4], bfr[NR][4];
      load_frags<AK, BM, MR>(LDSF_A(cur), wm * TM, kk, lane, af);
      load_frags<BKC, BN, NR>(LDSF_B(cur), wn * TN, kk, lane, bfr);
      if constexpr ((OPT & 1) != 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < MR; ++i)
#pragma unroll
          for (int j = 0; j < NR; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(bfr[j][s], af[i][s], acc[i][j], 0, 0, 0);
      if constexpr ((OPT & 1) != 0) __builtin_amdgcn_s_setprio(0);
    }
    }
    if (more) {
      sa.store(LDSF_A(cur ^ 1), tid);
      sb.store(LDSF_B(cur ^ 1), tid);
      if (rowsum) sa.accumulate_rows(rs);
    }
    __syncthreads();
  }
#undef LDSF_A
#undef LDSF_B
  if constexpr (!AK) {
    if (rowsum) {   // threads with equal tid % (BM/4) share 4 rows: reduce in LDS, one atomic per row
      float* red = reinterpret_cast<float*>(smem);
      constexpr int G = BM / 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) red[(tid / G) * BM + (tid % G) * 4 + j] = rs[j];
      __syncthreads();
      if (tid < BM) {
        float x = 0.f;
        for (int t = 0; t < NT / G; ++t) x += red[t * BM + tid];
        if (m0 + tid < p.M) atomicAdd(p.rowsum_a + m0 + tid, x);
      }
      __syncthreads();
    }
  }
  if constexpr (SGD) {
    if (p.ksplit == 1 && p.ulds) {
      sgd_epilogue_lds_f32<BM, BN, NT, MR, NR, !AK, !BKC, 2 * (BM + BN) * BKF * 4>(p, acc, smem, m0, n0, m0 + wm * TM,
                                                                                   n0 + wn * TN, lane, tid);
      return;
    }
  }
  epilogue_f32<MR, NR, !AK, !BKC, SGD>(p, acc, zb, split, m0 + wm * TM, n0 + wn * TN, lane);
}

// split-K reduce: 4 consecutive outputs per thread when N % 4 == 0 (16-B slab loads)
template <bool SGD>
__global__ void fm_gemm_f32_reduce(GemmF p, int v4) {
  const long MN = (long)p.M * p.N;
  const int E = v4 ? 4 : 1;
  const long total = MN * p.batch / E;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long e0 = i * E;
    const long zb = e0 / MN, e = e0 % MN;
    const int m = (int)(e / p.N), n = (int)(e % p.N);
    const float* src = p.ws + zb * p.ksplit * MN + e;
    float* d = p.C + zb * p.sC + (long)m * p.ldc + n;
    if (v4) {
      f32x4_t s = slab_sum4(src, MN, p.ksplit);
      if constexpr (SGD) {
        sgd_apply4(p, (long)m * p.ldc + n, s * p.alpha);
        continue;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) s[r] = act_fwd(p.act, s[r] * p.alpha + (p.bias ? p.bias[n + r] : 0.f));
      if (p.beta) s += *reinterpret_cast<const f32x4_t*>(d);
      *reinterpret_cast<f32x4_t*>(d) = s;
      if (p.Cp) {
        const float fo[4] = {s[0], s[1], s[2], s[3]};
        store_planes4(p.Cp, p.psc, zb * p.sC + (long)m * p.ldc + n, fo);
      }
    } else {
      float s = slab_sum1(src, MN, p.ksplit);
      if constexpr (SGD) {
        sgd_apply1(p, (long)m * p.ldc + n, s * p.alpha);
        continue;
      }
      s = act_fwd(p.act, s * p.alpha + (p.bias ? p.bias[n] : 0.f));
      *d = s + (p.beta ? *d : 0.f);
      if (p.Cp) store_planes1(p.Cp, p.psc, zb * p.sC + (long)m * p.ldc + n, *d);
    }
  }
}

// ---- fp32 GEMM on the bf16 matrix cores by exact three-way splitting --------------------------
// CDNA4's fp32 MFMA (v_mfma_f32_16x16x4_f32, 157 TF/s) is 16x slower than its bf16 MFMA.  Every fp32
// operand x is split EXACTLY into three bf16 terms at LDS-store time: h = bf16(x), m = bf16(x - h),
// l = bf16(x - h - m) (x - h and x - h - m are exact fp32 differences; h + m + l carries 24
// significant bits, the fp32 mantissa, with a final rounding error <= 2^-25 |x|).  The products
// x*y are then sum over the six terms with i + j <= 2 (hh, hm, mh, hl, mm, lh) on
// v_mfma_f32_16x16x32_bf16 with fp32 accumulation: every bf16 x bf16 product is exact in fp32, and
// the dropped terms (ml, lm, ll) are <= 2^-24 |x y| -- the same order as the fp32 product rounding
// itself, so the result has native-fp32 accuracy (tests/test_gpu_fp32.py checks it against float64
// at the native kernel's tolerance).  Cost per k: 6 bf16 MFMA (16 cycles) vs 8 fp32 MFMA (32
// cycles) for a 16x16x32 block: 2.7x the fp32 MFMA rate.
// MEASURED (profiles/gemm_f32_split_vs_native_r4c.jsonl): accuracy at the native kernel's level
// (tests/test_gpu_fp32_split.py), speed only at parity -- 1362 vs 1391 us over the DLRM shapes,
// hipBLASLt fp32 1287 us, and the DLRM step 1.53 vs 1.45 ms (profiles/bench_ab_f32_split_r4c.txt).
// Three planes per operand triple the LDS fragment reads per k (18 b128 reads per 48 MFMAs per
// wave: ~96 B/clk/CU of the 128 B/clk LDS rate) and the 96 KB of planes leave one block per CU, so
// the kernel is LDS- and latency-bound well before the 2.7x MFMA headroom.  OPT-IN.
// Tile 128x128x64, 512 threads (8 waves, 64x32 per wave), six bf16 LDS planes (3 per operand,
// gemm_common.h images: K-contiguous 128-B rows / MN-contiguous transposed reads) = 96 KB, one
// block per CU; the next k-tile's fp32 operands are loaded into registers during this tile's MFMAs.
constexpr int X3_BK = 64;

FM_DEVICE void split3(const float (&x)[8], u32x4_t& h, u32x4_t& m, u32x4_t& l) {
  unsigned short hs[8], ms[8], ls[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    hs[t] = f2bf(x[t]);
    const float r1 = x[t] - bf2f(hs[t]);
    ms[t] = f2bf(r1);
    ls[t] = f2bf(r1 - bf2f(ms[t]));
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    h[u] = (unsigned)hs[2 * u] | ((unsigned)hs[2 * u + 1] << 16);
    m[u] = (unsigned)ms[2 * u] | ((unsigned)ms[2 * u + 1] << 16);
    l[u] = (unsigned)ls[2 * u] | ((unsigned)ls[2 * u + 1] << 16);
  }
}

template <bool KC, int R>
struct StageX3 {
  static constexpr int NTH = 512;
  static constexpr int PER_T = R * X3_BK / 8 / NTH;
  float v[PER_T][8];

  FM_DEVICE void load(const float* __restrict__ p, long ld, int row0, int rows, int k0, int K, int tid, int vec) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int ci = tid + NTH * i;
      int gr, gk;
      if constexpr (KC) {
        gr = row0 + (ci >> 3);
        gk = k0 + 8 * (ci & 7);
      } else {
        gk = k0 + ci / (R / 8);
        gr = row0 + 8 * (ci % (R / 8));
      }
      const bool full = KC ? (gr < rows && gk + 8 <= K) : (gk < K && gr + 8 <= rows);
      if (vec && full) {
        const float* src = KC ? p + (long)gr * ld + gk : p + (long)gk * ld + gr;
        const f32x4_t a = *reinterpret_cast<const f32x4_t*>(src);
        const f32x4_t b = *reinterpret_cast<const f32x4_t*>(src + 4);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          v[i][t] = a[t];
          v[i][4 + t] = b[t];
        }
      } else {
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const int r = KC ? gr : gr + t, k = KC ? gk + t : gk;
          v[i][t] = (r < rows && k < K) ? (KC ? p[(long)r * ld + k] : p[(long)k * ld + r]) : 0.f;
        }
      }
    }
  }

  FM_DEVICE void store(char* l0, char* l1, char* l2, int tid) const {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int ci = tid + NTH * i;
      int a, c;
      if constexpr (KC) {
        a = ci >> 3;
        c = ci & 7;
      } else {
        a = ci / (R / 8);
        c = ci % (R / 8);
      }
      u32x4_t h, m, l;
      split3(v[i], h, m, l);
      const int off = lds_off<KC, R>(a, c);
      *reinterpret_cast<u32x4_t*>(l0 + off) = h;
      *reinterpret_cast<u32x4_t*>(l1 + off) = m;
      *reinterpret_cast<u32x4_t*>(l2 + off) = l;
    }
  }

  // MN-contiguous operand: a thread's chunks cover the same 8 rows (bias-gradient row sums)
  FM_DEVICE void rowsum(float (&s)[8]) const {
#pragma unroll
    for (int i = 0; i < PER_T; ++i)
#pragma unroll
      for (int t = 0; t < 8; ++t) s[t] += v[i][t];
  }
};

template <bool AK, bool BKC>
__global__ void __launch_bounds__(512, 1) fm_gemm_x3_kernel(GemmF p, int vec) {
  constexpr int BM = 128, BN = 128, NTH = 512, WN = 4, TM = 64, TN = 32, MR = TM / 16, NR = TN / 16;
  constexpr int PL = 128 * X3_BK * 2;   // one bf16 plane of one operand
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const la0 = smem;
  char* const lb0 = smem + 3 * PL;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int bid = xcd_remap_f(blockIdx.x, p.tiles_m * p.tiles_n);
  int tm, tn;
  if (p.n_fast) {
    tn = bid % p.tiles_n;
    tm = bid / p.tiles_n;
  } else {
    tm = bid % p.tiles_m;
    tn = bid / p.tiles_m;
  }
  const int zb = blockIdx.y, split = blockIdx.z;
  const int m0 = tm * BM, n0 = tn * BN;
  const float* A = p.A + (long)zb * p.sA;
  const float* B = p.B + (long)zb * p.sB;
  const int ktiles = (p.K + X3_BK - 1) / X3_BK;
  const int kt_per = (ktiles + p.ksplit - 1) / p.ksplit;
  const int kt0 = split * kt_per, kt1 = min(ktiles, kt0 + kt_per);

  f32x4_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  StageX3<AK, BM> sa;
  StageX3<BKC, BN> sb;
  const bool dorow = (!AK) && p.rowsum_a != nullptr && tn == 0;
  float rs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int va = vec & 1, vb = (vec >> 1) & 1;
  if (kt0 < kt1) {
    sa.load(A, p.lda, m0, p.M, kt0 * X3_BK, p.K, tid, va);
    sb.load(B, p.ldb, n0, p.N, kt0 * X3_BK, p.K, tid, vb);
  }
  for (int kt = kt0; kt < kt1; ++kt) {
    __syncthreads();                              // every wave is done reading the previous tile
    sa.store(la0, la0 + PL, la0 + 2 * PL, tid);
    sb.store(lb0, lb0 + PL, lb0 + 2 * PL, tid);
    if constexpr (!AK) {
      if (dorow) sa.rowsum(rs);
    }
    __syncthreads();
    if (kt + 1 < kt1) {                           // next tile's operands land during the MFMAs
      sa.load(A, p.lda, m0, p.M, (kt + 1) * X3_BK, p.K, tid, va);
      sb.load(B, p.ldb, n0, p.N, (kt + 1) * X3_BK, p.K, tid, vb);
    }
#pragma unroll
    for (int kk = 0; kk < X3_BK / 32; ++kk) {
      bf16x8_t af[3][MR], bfr[3][NR];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
        for (int i = 0; i < MR; ++i) af[pl][i] = frag<AK, BM>(la0 + pl * PL, wm * TM + 16 * i, kk, lane);
#pragma unroll
        for (int j = 0; j < NR; ++j) bfr[pl][j] = frag<BKC, BN>(lb0 + pl * PL, wn * TN + 16 * j, kk, lane);
      }
      // small terms first, the dominant h*h product last
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j) {
          constexpr int PA[6] = {2, 1, 0, 1, 0, 0};
          constexpr int PB[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
          for (int t = 0; t < 6; ++t)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<bf16x8v_t*>(&bfr[PB[t]][j]),
                                                                *reinterpret_cast<bf16x8v_t*>(&af[PA[t]][i]), acc[i][j],
                                                                0, 0, 0);
        }
    }
  }
  if constexpr (!AK) {
    if (dorow) {   // reduce the threads sharing each 8-row group, one atomic per row
      __syncthreads();
      float* red = reinterpret_cast<float*>(smem);
      constexpr int G = BM / 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) red[(tid / G) * BM + (tid % G) * 8 + j] = rs[j];
      __syncthreads();
      if (tid < BM) {
        float x = 0.f;
        for (int t = 0; t < NTH / G; ++t) x += red[t * BM + tid];
        if (m0 + tid < p.M) atomicAdd(p.rowsum_a + m0 + tid, x);
      }
    }
  }

  // epilogue: lane owns C[m][n .. n+3], m = mbase + 16 i + (lane & 15), n = nbase + 16 j + 4 (lane >> 4)
  const int mbase = m0 + wm * TM, nbase = n0 + wn * TN;
  const int mrow = lane & 15, ncol = 4 * (lane >> 4);
  float csum[NR][4];
#pragma unroll
  for (int j = 0; j < NR; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) csum[j][r] = 0.f;
#pragma unroll
  for (int i = 0; i < MR; ++i) {
    const int m = mbase + 16 * i + mrow;
    const bool mok = m < p.M;
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int n = nbase + 16 * j + ncol;
      if (!mok || n >= p.N) continue;
      const bool full = n + 3 < p.N;
      if (p.ksplit > 1) {   // fp32 slab of this split: the reduce launch applies the epilogue
        float* dst = p.ws + (((long)zb * p.ksplit + split) * p.M + m) * (long)p.N + n;
        if (full && (p.N & 3) == 0) {
          *reinterpret_cast<f32x4_t*>(dst) = acc[i][j];
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n + r < p.N) dst[r] = acc[i][j][r];
        }
        continue;
      }
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool ok = n + r < p.N;
        v[r] = acc[i][j][r] * p.alpha + ((p.bias && ok) ? p.bias[n + r] : 0.f);
        v[r] = act_fwd(p.act, v[r]);
        if (p.ay) v[r] = act_bwd(p.bact, ok ? p.ay[(long)m * p.lday + n + r] : 0.f, v[r]);
        if (p.colsum && ok) csum[j][r] += v[r];
      }
      float* dst = p.C + (long)zb * p.sC + (long)m * p.ldc + n;
      if (full && (p.ldc & 3) == 0 && ((((uintptr_t)dst) & 15) == 0)) {
        f32x4_t o = {v[0], v[1], v[2], v[3]};
        if (p.beta) o += *reinterpret_cast<f32x4_t*>(dst);
        *reinterpret_cast<f32x4_t*>(dst) = o;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (n + r < p.N) dst[r] = v[r] + (p.beta ? dst[r] : 0.f);
      }
    }
  }
  if (p.colsum && p.ksplit == 1) {   // bias gradient of the layer below: 16 rows per lane group, 1 atomic/col
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

// split-K reduce of a GEMM with the FUSED BACKWARD epilogue (dX of a layer whose input has an
// activation): v = act_bwd(bact, ay, act(alpha * sum + bias)), colsum[n] += sum over rows of v.
// Thread = 4 columns x RB rows: the column sums stay in registers, one atomic per (column, block),
// so small-batch dX GEMMs (summit_large: 256 x 4096 x 4096) can split K instead of running 64
// blocks of 128x128 tiles or 64x64 tiles at ~60 % of the big-tile rate.
__global__ void __launch_bounds__(256) fm_gemm_f32_reduce_bwd(GemmF p, int RB) {
  const int n = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (n >= p.N) return;
  const int m0 = blockIdx.y * RB, m1 = min(p.M, m0 + RB);
  const long MN = (long)p.M * p.N;
  const bool v4 = n + 3 < p.N && (p.N & 3) == 0;
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  for (int m = m0; m < m1; ++m) {
    const float* src = p.ws + (long)m * p.N + n;
    float sv[4] = {0.f, 0.f, 0.f, 0.f};
    if (v4) {
      f32x4_t a = slab_sum4(src, MN, p.ksplit);
#pragma unroll
      for (int r = 0; r < 4; ++r) sv[r] = a[r];
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (n + r < p.N)
          sv[r] = slab_sum1(src + r, MN, p.ksplit);
    }
    float* d = p.C + (long)m * p.ldc + n;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (n + r >= p.N) break;
      float v = act_fwd(p.act, sv[r] * p.alpha + (p.bias ? p.bias[n + r] : 0.f));
      if (p.ay) v = act_bwd(p.bact, p.ay[(long)m * p.lday + n + r], v);
      cs[r] += v;
      d[r] = v + (p.beta ? d[r] : 0.f);
      if (p.Cp) store_planes1(p.Cp, p.psc, (long)m * p.ldc + n + r, d[r]);
    }
  }
  if (p.colsum) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (n + r < p.N) atomicAdd(p.colsum + n + r, cs[r]);
  }
}

}  // namespace

// the split-bf16 kernel, second form (gemm_x3.hip)
extern "C" int fm_gemm_x3v2_launch(const void* params, int bm, int a_kcontig, int b_kcontig, int sgd, hipStream_t s);
// the pre-split plane kernel (gemm_pl.hip)
extern "C" int fm_gemm_pl3_launch(const void* params, int bm, int a_kcontig, int b_kcontig, int sgd, hipStream_t s);
// the ring-form kernel (gemm_f32_ring.hip)
extern "C" int fm_gemm_f32_ring_cfg(int c, int* geo);
extern "C" void fm_gemm_f32_ring_launch(const void* params, int c, int a_kcontig, int b_kcontig, int sgd,
                                        hipStream_t stream);

// split-K reduce off the critical path (gemm_async.hip)
extern "C" void fm_gemm_join(hipStream_t s);
extern "C" hipStream_t fm_gemm_async_fork(hipStream_t s);
extern "C" void fm_gemm_async_forked(hipStream_t side);

namespace {

void launch_reduce_f32(const GemmF& p, int v4, long total, hipStream_t stream) {
  hipStream_t rs = fm_gemm_async_fork(stream);
  if (p.uw) hipLaunchKernelGGL(fm_gemm_f32_reduce<true>, dim3(fm_grid(total)), dim3(256), 0, rs, p, v4);
  else hipLaunchKernelGGL(fm_gemm_f32_reduce<false>, dim3(fm_grid(total)), dim3(256), 0, rs, p, v4);
  if (rs != stream) fm_gemm_async_forked(rs);
}

template <int BM, int BN, bool AK, bool BKC, bool VEC>
void launch_f(const GemmF& p, hipStream_t s, int opt) {
  constexpr int LDS = 2 * (BM + BN) * BKF * 4;
  dim3 grid(p.tiles_m * p.tiles_n, p.batch, p.ksplit);
  if constexpr (!AK && !BKC && BM <= 128) {   // fused-SGD dW GEMMs: own instantiation of the default forms
    if (p.uw) {
      if constexpr (VEC && BM == 128) {
        hipLaunchKernelGGL((fm_gemm_f32_kernel<BM, BN, AK, BKC, VEC, 2, 512, 2, true>), grid, dim3(512), LDS, s, p);
      } else {
        hipLaunchKernelGGL((fm_gemm_f32_kernel<BM, BN, AK, BKC, VEC, 0, NTF, 2, true>), grid, dim3(NTF), LDS, s, p);
      }
      return;
    }
  }
  if constexpr (VEC && BM == 256 && BN == 128) {
    // one 4-wave block per CU, one wave per SIMD with a 128x64 wave tile (the shape hipBLASLt's
    // fp32 kernel uses on these GEMMs: 8x4 16x16 accumulators, 512-VGPR budget)
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)fm_gemm_f32_kernel<BM, BN, AK, BKC, VEC, 0, 256, 1>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
      (void)hipFuncSetAttribute((const void*)fm_gemm_f32_kernel<BM, BN, AK, BKC, VEC, 2, 256, 1>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
      attr = true;
    }
    if (opt == 2) hipLaunchKernelGGL((fm_gemm_f32_kernel<BM, BN, AK, BKC, VEC, 2, 256, 1>), grid, dim3(256), LDS, s, p);
    else hipLaunchKernelGGL((fm_gemm_f32_kernel<BM, BN, AK, BKC, VEC, 0, 256, 1>), grid, dim3(256), LDS, s, p);
    return;
  } else {
  if constexpr (VEC && BM == 128 && BN == 128) {   // tuning variants only on the main tile
    // default: 8 waves (2x4, 64x32 per wave) with the fragment double buffer -- 4 waves per SIMD
    // hide the per-K-tile barrier and first-fragment latency (DLRM fp32 GEMMs -3.7 %, the
    // 1024-wide layers -5..8 %: profiles/gemm_f32_variants_ab.jsonl); opt 5 = the 4-wave kernel
    switch (opt) {
      case 0: hipLaunchKernelGGL((fm_gemm_f32_kernel<BM, BN, AK, BKC, VEC, 2, 512>), grid, dim3(512), LDS, s, p); return;
      case 5: hipLaunchKernelGGL((fm_gemm_f32_kernel<BM, BN, AK, BKC, VEC, 0, 256>), grid, dim3(NTF), LDS, s, p); return;
      case 1: hipLaunchKernelGGL((fm_gemm_f32_kernel<BM, BN, AK, BKC, VEC, 1>), grid, dim3(NTF), LDS, s, p); return;
      case 2: hipLaunchKernelGGL((fm_gemm_f32_kernel<BM, BN, AK, BKC, VEC, 2>), grid, dim3(NTF), LDS, s, p); return;
      default: break;
    }
  }
  if constexpr (VEC && BM == 128 && BN == 64) {
    // default: the 8-wave (4x2 waves of 32x32) form; opt 10 = the 4-wave kernel (A/B:
    // profiles/gemm_f32_8wave_ab.jsonl, the 512/256-wide layers' dX/dW -5..14 %)
    if (opt != 10) {
      hipLaunchKernelGGL((fm_gemm_f32_kernel<BM, BN, AK, BKC, VEC, 2, 512>), grid, dim3(512), LDS, s, p);
      return;
    }
  }
  hipLaunchKernelGGL((fm_gemm_f32_kernel<BM, BN, AK, BKC, VEC>), grid, dim3(NTF), LDS, s, p);
  }
}

template <int BM, int BN>
void launch_fbm(const GemmF& p, bool ak, bool bk, bool vec, hipStream_t s, int opt) {
  if (vec) {
    if (ak && bk) launch_f<BM, BN, true, true, true>(p, s, opt);
    else if (ak) launch_f<BM, BN, true, false, true>(p, s, opt);
    else if (bk) launch_f<BM, BN, false, true, true>(p, s, opt);
    else launch_f<BM, BN, false, false, true>(p, s, opt);
  } else {
    if (ak && bk) launch_f<BM, BN, true, true, false>(p, s, 0);
    else if (ak) launch_f<BM, BN, true, false, false>(p, s, 0);
    else if (bk) launch_f<BM, BN, false, true, false>(p, s, 0);
    else launch_f<BM, BN, false, false, false>(p, s, 0);
  }
}


// ---- LDS-DMA pipelined variant ------------------------------------------------------------
// Operands go global -> LDS with global_load_lds_dwordx4 (no staging VGPRs, no ds_write pass)
// into a 3-stage ring, two K-tiles in flight behind the one being multiplied (the same schedule
// as the bf16 gemm_glds.hip):
//   iteration t: s_waitcnt vmcnt(L) (own loads of tile t landed); lgkmcnt(0); s_barrier
//                issue tile t+2 -> stage (t+2)%3; MFMAs on stage t%3
// The DMA destination is lane-linear (wave base + 16*lane), so the K-contiguous image's chunk
// swizzle is applied to the per-lane SOURCE address; MN-contiguous images are unswizzled rows.
// Used when K-tiles are whole (K % 32 == 0) and operands allow 16-B access.

template <bool KC, int R, int NTH>
struct GldsF {
  static constexpr int INSTR = R * BKF * 4 / 1024;
  static constexpr int NWAVES = NTH / 64;
  static constexpr int PER_W = INSTR / NWAVES;
  static_assert(INSTR % NWAVES == 0, "tile bytes must split evenly over waves");

  FM_DEVICE static void issue(const float* __restrict__ p, long ld, int row0, int rows, int k0, char* lds, int wave,
                              int lane) {
#pragma unroll
    for (int i = 0; i < PER_W; ++i) {
      const int j = wave + NWAVES * i;
      const float* src;
      if constexpr (KC) {           // image [row][32 k]: 8 rows of 128 B per instruction
        const int row = 8 * j + (lane >> 3);
        const int chunk = (lane & 7) ^ ((row >> 1) & 7);
        const int gr = min(row0 + row, rows - 1);          // rows past the edge: never stored
        src = p + (long)gr * ld + k0 + 4 * chunk;
      } else {                      // image [k][R rows]: 1024/(4R) k-rows per instruction
        constexpr int CPR = R / 4;                      // 16-B chunks per k-row
        constexpr int KPI = 1024 / (4 * R);
        const int krow = KPI * j + lane / CPR;
        const int gr = min(row0 + 4 * (lane % CPR), rows - 4);
        src = p + (long)(k0 + krow) * ld + gr;
      }
      __builtin_amdgcn_global_load_lds((gptr_f)src, (lptr_f)(lds + j * 1024), 16, 0, 0);
    }
  }
};


template <int BM, int BN, int WM, int WN, bool AK, bool BKC>
__global__ void __launch_bounds__(WM * WN * 64, 1) fm_gemm_f32_glds_kernel(GemmF p) {
  constexpr int NW = WM * WN;
  constexpr int NTH = NW * 64;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MR = TM / 16, NR = TN / 16;
  constexpr int A_BYTES = BM * BKF * 4;
  constexpr int B_BYTES = BN * BKF * 4;
  constexpr int STG = A_BYTES + B_BYTES;
  constexpr int NS = 3;
  constexpr int LPT = GldsF<AK, BM, NTH>::PER_W + GldsF<BKC, BN, NTH>::PER_W;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int bid = xcd_remap_f(blockIdx.x, p.tiles_m * p.tiles_n);
  int tm, tn;
  if (p.n_fast) { tn = bid % p.tiles_n; tm = bid / p.tiles_n; }
  else { tm = bid % p.tiles_m; tn = bid / p.tiles_m; }
  const int zb = blockIdx.y;
  const int split = blockIdx.z;
  const int m0 = tm * BM, n0 = tn * BN;
  const float* A = p.A + (long)zb * p.sA;
  const float* B = p.B + (long)zb * p.sB;

  const int ktiles_total = p.K / BKF;
  const int kt_per = (ktiles_total + p.ksplit - 1) / p.ksplit;
  const int kt0 = split * kt_per;
  const int kt1 = min(ktiles_total, kt0 + kt_per);
  const int nkt = max(kt1 - kt0, 0);
  const int klast = max(min(kt1, ktiles_total) - 1, 0);

  auto issue = [&](int t, int stage) {
    const int kt = min(kt0 + t, klast);     // prefetches past the end re-read the last tile
    char* base = smem + stage * STG;
    GldsF<AK, BM, NTH>::issue(A, p.lda, m0, p.M, kt * BKF, base, wave, lane);
    GldsF<BKC, BN, NTH>::issue(B, p.ldb, n0, p.N, kt * BKF, base + A_BYTES, wave, lane);
  };

  f32x4_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const bool rowsum = (!AK) && (p.rowsum_a != nullptr) && (tn == 0);
  constexpr int CPR = BM / 4;
  float rs[4] = {0.f, 0.f, 0.f, 0.f};

  issue(0, 0);
  issue(1, 1);
  for (int t = 0; t < nkt; ++t) {
    const int stage = t % NS;
    wait_vmcnt_f<LPT>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    issue(t + 2, (t + 2) % NS);
    const char* la = smem + stage * STG;
    const char* lb = la + A_BYTES;
    if constexpr (!AK) {
      if (rowsum) {
        for (int kr = tid / CPR; kr < BKF; kr += NTH / CPR) {
          const f32x4_t v = *reinterpret_cast<const f32x4_t*>(la + kr * (BM * 4) + 16 * (tid % CPR));
#pragma unroll
          for (int e = 0; e < 4; ++e) rs[e] += v[e];
        }
      }
    }
#pragma unroll
    for (int kk = 0; kk < BKF / 16; ++kk) {
      float af[MR][4], bfr[NR][4];
      load_frags<AK, BM, MR>(la, wm * TM, kk, lane, af);
      load_frags<BKC, BN, NR>(lb, wn * TN, kk, lane, bfr);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < MR; ++i)
#pragma unroll
          for (int j = 0; j < NR; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(bfr[j][s], af[i][s], acc[i][j], 0, 0, 0);
    }
  }
  wait_vmcnt_f<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if constexpr (!AK) {
    if (rowsum) {
      float* red = reinterpret_cast<float*>(smem);
      constexpr int G = NTH / CPR;
#pragma unroll
      for (int e = 0; e < 4; ++e) red[(tid / CPR) * BM + (tid % CPR) * 4 + e] = rs[e];
      __syncthreads();
      for (int r = tid; r < BM; r += NTH) {
        float x = 0.f;
        for (int g = 0; g < G; ++g) x += red[g * BM + r];
        if (m0 + r < p.M) atomicAdd(p.rowsum_a + m0 + r, x);
      }
    }
  }
  epilogue_f32<MR, NR, !AK, !BKC>(p, acc, zb, split, m0 + wm * TM, n0 + wn * TN, lane);
}

template <int BM, int BN, int WM, int WN>
void launch_f_glds(const GemmF& p, bool ak, bool bk, hipStream_t s) {
  constexpr int NTH = WM * WN * 64;
  constexpr int LDS = 3 * (BM + BN) * BKF * 4;
  static bool attr_set = false;
  if (!attr_set) {   // > 64 KiB dynamic LDS needs the opt-in attribute
    auto set = [](const void* f) { (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS); };
    set((const void*)fm_gemm_f32_glds_kernel<BM, BN, WM, WN, true, true>);
    set((const void*)fm_gemm_f32_glds_kernel<BM, BN, WM, WN, true, false>);
    set((const void*)fm_gemm_f32_glds_kernel<BM, BN, WM, WN, false, true>);
    set((const void*)fm_gemm_f32_glds_kernel<BM, BN, WM, WN, false, false>);
    attr_set = true;
  }
  dim3 grid(p.tiles_m * p.tiles_n, p.batch, p.ksplit);
  if (ak && bk) hipLaunchKernelGGL((fm_gemm_f32_glds_kernel<BM, BN, WM, WN, true, true>), grid, dim3(NTH), LDS, s, p);
  else if (ak) hipLaunchKernelGGL((fm_gemm_f32_glds_kernel<BM, BN, WM, WN, true, false>), grid, dim3(NTH), LDS, s, p);
  else if (bk) hipLaunchKernelGGL((fm_gemm_f32_glds_kernel<BM, BN, WM, WN, false, true>), grid, dim3(NTH), LDS, s, p);
  else hipLaunchKernelGGL((fm_gemm_f32_glds_kernel<BM, BN, WM, WN, false, false>), grid, dim3(NTH), LDS, s, p);
}

// ---- 32x32x2 kernel ---------------------------------------------------------------------------
// v_mfma_f32_32x32x2_f32: half the MFMA instructions of the 16x16x4 form for the same tile (64
// cycles each, latency = issue, so two accumulators in rotation keep the pipe full), and its
// accumulator puts 32 consecutive OUTPUT COLUMNS on the 32 lanes of each half-wave: every
// accumulator register is two 128-B row segments of C -- the full-rate shape for stores and for
// no-return float atomics, so split-K partials are added straight into C (beta = 1 outputs, i.e.
// the dW GEMMs whose gradients the optimizer zeroes) instead of slabs + a reduce launch.
//   operand fragments for one 16-wide k-chunk: lane (q = lane & 31, h = lane >> 5) takes
//   k = 8h + s at MFMA step s (s = 0..7), so two 16-B LDS reads per row feed 8 MFMAs;
//   K-contiguous images [row][BK] with XOR-swizzled 16-B chunks (conflict-free ds_read_b128);
//   MN-contiguous A [k][BM] with the wave's rows interleaved over its MR tiles (one b64/b128 read
//   at a fixed k gives all MR fragments); MN-contiguous B [k][BN] read per lane (b32).
template <int BK>
FM_DEVICE int kcx_off(int r, int c) {
  constexpr int CPR = BK / 4;                                 // 16-B chunks per row
  constexpr int RPL = (256 / (BK * 4)) > 0 ? 256 / (BK * 4) : 1;   // rows per 256-B bank line
  return r * (BK * 4) + 16 * (c ^ ((r / RPL) & (CPR - 1)));
}

template <bool KC, int R, int BK, int NT>
struct StageX {
  static constexpr int CHUNKS = R * BK / 4;
  static constexpr int PER_T = CHUNKS / NT;
  static_assert(PER_T >= 1 && CHUNKS % NT == 0, "tile too small for the block");
  f32x4_t v[PER_T];

  FM_DEVICE void load(const float* __restrict__ p, long ld, int row0, int rows, int k0, int K, int tid) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int ci = tid + NT * i;
      int gr, gk;
      if constexpr (KC) {
        gr = row0 + ci / (BK / 4);
        gk = k0 + 4 * (ci % (BK / 4));
      } else {
        gk = k0 + ci / (R / 4);
        gr = row0 + 4 * (ci % (R / 4));
      }
      if (gr < rows && gk < K) {
        const float* src = KC ? (p + (long)gr * ld + gk) : (p + (long)gk * ld + gr);
        v[i] = *reinterpret_cast<const f32x4_t*>(src);
      } else {
        v[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  FM_DEVICE void store(char* lds, int tid) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int ci = tid + NT * i;
      int off;
      if constexpr (KC) off = kcx_off<BK>(ci / (BK / 4), ci % (BK / 4));
      else off = (ci / (R / 4)) * (R * 4) + 16 * (ci % (R / 4));
      *reinterpret_cast<f32x4_t*>(lds + off) = v[i];
    }
  }
  FM_DEVICE void accumulate_rows(float (&s)[4]) const {
#pragma unroll
    for (int i = 0; i < PER_T; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) s[j] += v[i][j];
  }
};

// A fragments (M side, T = MR tiles) for k-chunk kk: f[t][s], s = 0..7
template <bool KC, int R, int BK, int T>
FM_DEVICE void frags_a32(const char* lds, int base, int kk, int lane, float (&f)[T][8]) {
  const int q = lane & 31, h = lane >> 5;
  if constexpr (KC) {
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int row = base + 32 * t + q;
      const f32x4_t x0 = *reinterpret_cast<const f32x4_t*>(lds + kcx_off<BK>(row, 4 * kk + 2 * h));
      const f32x4_t x1 = *reinterpret_cast<const f32x4_t*>(lds + kcx_off<BK>(row, 4 * kk + 2 * h + 1));
#pragma unroll
      for (int s = 0; s < 4; ++s) { f[t][s] = x0[s]; f[t][4 + s] = x1[s]; }
    }
  } else {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int k = 16 * kk + 8 * h + s;
      const fvec<T> x = *reinterpret_cast<const fvec<T>*>(lds + k * (R * 4) + 4 * (base + T * q));
#pragma unroll
      for (int t = 0; t < T; ++t) f[t][s] = x[t];
    }
  }
}

// B fragments (N side, T = NR tiles, never interleaved: lane q <-> column base + 32t + q)
template <bool KC, int R, int BK, int T>
FM_DEVICE void frags_b32(const char* lds, int base, int kk, int lane, float (&f)[T][8]) {
  const int q = lane & 31, h = lane >> 5;
  if constexpr (KC) {
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int row = base + 32 * t + q;
      const f32x4_t x0 = *reinterpret_cast<const f32x4_t*>(lds + kcx_off<BK>(row, 4 * kk + 2 * h));
      const f32x4_t x1 = *reinterpret_cast<const f32x4_t*>(lds + kcx_off<BK>(row, 4 * kk + 2 * h + 1));
#pragma unroll
      for (int s = 0; s < 4; ++s) { f[t][s] = x0[s]; f[t][4 + s] = x1[s]; }
    }
  } else {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int k = 16 * kk + 8 * h + s;
#pragma unroll
      for (int t = 0; t < T; ++t) f[t][s] = *reinterpret_cast<const float*>(lds + k * (R * 4) + 4 * (base + 32 * t + q));
    }
  }
}

// lane (q, h) holds acc[i][j][r] = C[m][n]:  n = nbase + 32 j + q,
//   im = 8 (r >> 2) + 4 h + (r & 3),  m = IL_A ? mbase + MR im + i : mbase + 32 i + im
template <int MR, int NR, bool IL_A>
FM_DEVICE void epilogue_x32(const GemmF& p, const f32x16_t (&acc)[MR][NR], int zb, int split, int mbase, int nbase,
                            int lane) {
  const int q = lane & 31, h = lane >> 5;
  if (p.ksplit > 1 && !p.atomic) {
    float* ws = p.ws + ((long)zb * p.ksplit + split) * (long)p.M * p.N;
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int im = 8 * (r >> 2) + 4 * h + (r & 3);
        const int m = IL_A ? mbase + MR * im + i : mbase + 32 * i + im;
        if (m >= p.M) continue;
#pragma unroll
        for (int j = 0; j < NR; ++j) {
          const int n = nbase + 32 * j + q;
          if (n < p.N) ws[(long)m * p.N + n] = acc[i][j][r];
        }
      }
    return;
  }
  float* Cz = p.C + (long)zb * p.sC;
  if (p.atomic) {   // split-K partials (and any beta = 1 output): no-return float atomics, 128-B rows
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int im = 8 * (r >> 2) + 4 * h + (r & 3);
        const int m = IL_A ? mbase + MR * im + i : mbase + 32 * i + im;
        if (m >= p.M) continue;
#pragma unroll
        for (int j = 0; j < NR; ++j) {
          const int n = nbase + 32 * j + q;
          if (n < p.N) atomicAdd(Cz + (long)m * p.ldc + n, p.alpha * acc[i][j][r]);
        }
      }
    return;
  }
  float bias[NR], csum[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const int n = nbase + 32 * j + q;
    bias[j] = (p.bias && n < p.N) ? p.bias[n] : 0.f;
    csum[j] = 0.f;
  }
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int im = 8 * (r >> 2) + 4 * h + (r & 3);
      const int m = IL_A ? mbase + MR * im + i : mbase + 32 * i + im;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        const int n = nbase + 32 * j + q;
        if (n >= p.N) continue;
        float v = act_fwd(p.act, acc[i][j][r] * p.alpha + bias[j]);
        if (p.ay) v = act_bwd(p.bact, p.ay[(long)m * p.lday + n], v);
        csum[j] += v;
        float* dst = Cz + (long)m * p.ldc + n;
        *dst = p.beta ? *dst + v : v;
      }
    }
  if (p.colsum) {
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const float x = csum[j] + __shfl_xor(csum[j], 32, 64);
      const int n = nbase + 32 * j + q;
      if (h == 0 && n < p.N) atomicAdd(p.colsum + n, x);
    }
  }
}

// WM x WN waves, wave tile (BM/WM) x (BN/WN) = MR x NR 32x32 tiles; BK-deep LDS tiles, two stages,
// register-staged global loads of the next tile issued before the current tile's MFMAs.
template <int BM, int BN, int BK, int WM, int WN, bool AK, bool BKC, int MINB>
__global__ void __launch_bounds__(WM * WN * 64, MINB) fm_gemm_f32x_kernel(GemmF p) {
  constexpr int NT = WM * WN * 64;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MR = TM / 32, NR = TN / 32;
  static_assert(MR >= 1 && NR >= 1 && MR * NR >= 2, "need >= 2 accumulators (MFMA latency = issue)");
  static_assert(AK || MR == 1 || MR == 2 || MR == 4, "interleaved A reads b32/b64/b128");
  constexpr int A_BYTES = BM * BK * 4;
  constexpr int B_BYTES = BN * BK * 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  const int bid = xcd_remap_f(blockIdx.x, p.tiles_m * p.tiles_n);
  int tm, tn;
  if (p.n_fast) { tn = bid % p.tiles_n; tm = bid / p.tiles_n; }
  else { tm = bid % p.tiles_m; tn = bid / p.tiles_m; }
  const int zb = blockIdx.y;
  const int split = blockIdx.z;
  const int m0 = tm * BM, n0 = tn * BN;
  const float* A = p.A + (long)zb * p.sA;
  const float* B = p.B + (long)zb * p.sB;

  const int ktiles_total = (p.K + BK - 1) / BK;
  const int kt_per = (ktiles_total + p.ksplit - 1) / p.ksplit;
  const int kt0 = split * kt_per;
  const int kt1 = min(ktiles_total, kt0 + kt_per);

  f32x16_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  StageX<AK, BM, BK, NT> sa;
  StageX<BKC, BN, BK, NT> sb;
  const bool rowsum = (!AK) && (p.rowsum_a != nullptr) && (tn == 0);
  float rs[4] = {0.f, 0.f, 0.f, 0.f};
#define LDSX(b) (smem + (b) * (A_BYTES + B_BYTES))
  if (kt0 < kt1) {
    sa.load(A, p.lda, m0, p.M, kt0 * BK, p.K, tid);
    sb.load(B, p.ldb, n0, p.N, kt0 * BK, p.K, tid);
    sa.store(LDSX(0), tid);
    sb.store(LDSX(0) + A_BYTES, tid);
    if (rowsum) sa.accumulate_rows(rs);
  }
  __syncthreads();
  for (int kt = kt0; kt < kt1; ++kt) {
    const int cur = (kt - kt0) & 1;
    const bool more = kt + 1 < kt1;
    if (more) {
      sa.load(A, p.lda, m0, p.M, (kt + 1) * BK, p.K, tid);
      sb.load(B, p.ldb, n0, p.N, (kt + 1) * BK, p.K, tid);
    }
    const char* la = LDSX(cur);
    const char* lb = la + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      float af[MR][8], bfr[NR][8];
      frags_a32<AK, BM, BK, MR>(la, wm * TM, kk, lane, af);
      frags_b32<BKC, BN, BK, NR>(lb, wn * TN, kk, lane, bfr);
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int i = 0; i < MR; ++i)
#pragma unroll
          for (int j = 0; j < NR; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bfr[j][s], acc[i][j], 0, 0, 0);
    }
    if (more) {
      sa.store(LDSX(cur ^ 1), tid);
      sb.store(LDSX(cur ^ 1) + A_BYTES, tid);
      if (rowsum) sa.accumulate_rows(rs);
    }
    __syncthreads();
  }
#undef LDSX
  if constexpr (!AK) {
    if (rowsum) {
      float* red = reinterpret_cast<float*>(smem);
      constexpr int G = BM / 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) red[(tid / G) * BM + (tid % G) * 4 + j] = rs[j];
      __syncthreads();
      for (int r = tid; r < BM; r += NT) {
        float x = 0.f;
        for (int t = 0; t < NT / G; ++t) x += red[t * BM + r];
        if (m0 + r < p.M) atomicAdd(p.rowsum_a + m0 + r, x);
      }
      __syncthreads();
    }
  }
  epilogue_x32<MR, NR, !AK>(p, acc, zb, split, m0 + wm * TM, n0 + wn * TN, lane);
}

template <int BM, int BN, int BK, int WM, int WN, int MINB>
void launch_x(const GemmF& p, bool ak, bool bk, hipStream_t s) {
  constexpr int NT = WM * WN * 64;
  constexpr int LDS = 2 * (BM + BN) * BK * 4;
  static bool attr_set = false;
  if (!attr_set) {
    auto set = [](const void* f) { (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS); };
    set((const void*)fm_gemm_f32x_kernel<BM, BN, BK, WM, WN, true, true, MINB>);
    set((const void*)fm_gemm_f32x_kernel<BM, BN, BK, WM, WN, true, false, MINB>);
    set((const void*)fm_gemm_f32x_kernel<BM, BN, BK, WM, WN, false, true, MINB>);
    set((const void*)fm_gemm_f32x_kernel<BM, BN, BK, WM, WN, false, false, MINB>);
    attr_set = true;
  }
  dim3 grid(p.tiles_m * p.tiles_n, p.batch, p.ksplit);
  if (ak && bk) hipLaunchKernelGGL((fm_gemm_f32x_kernel<BM, BN, BK, WM, WN, true, true, MINB>), grid, dim3(NT), LDS, s, p);
  else if (ak) hipLaunchKernelGGL((fm_gemm_f32x_kernel<BM, BN, BK, WM, WN, true, false, MINB>), grid, dim3(NT), LDS, s, p);
  else if (bk) hipLaunchKernelGGL((fm_gemm_f32x_kernel<BM, BN, BK, WM, WN, false, true, MINB>), grid, dim3(NT), LDS, s, p);
  else hipLaunchKernelGGL((fm_gemm_f32x_kernel<BM, BN, BK, WM, WN, false, false, MINB>), grid, dim3(NT), LDS, s, p);
}

// tile configurations of the 32x32 kernel (index = FM_GEMM_F32_VARIANT - 1000 for A/B runs)
struct XCfg { int bm, bn, bk, wm, wn; };
constexpr XCfg kXCfgs[] = {
    {128, 128, 32, 2, 2},   // 0: 4 waves of 64x64, 64 KB LDS -> 2 blocks / CU
    {128, 128, 32, 4, 2},   // 1: 8 waves of 32x64
    {256, 128, 32, 4, 2},   // 2: 8 waves of 64x64, 96 KB LDS -> 1 block / CU
    {256, 128, 16, 4, 2},   // 3: 8 waves of 64x64, 48 KB LDS -> 2 blocks / CU (VGPR permitting)
    {128, 256, 32, 2, 4},   // 4: 8 waves of 64x64
    {128, 128, 16, 2, 2},   // 5: 4 waves, 32 KB LDS
    {128, 64, 32, 2, 2},    // 6: 4 waves of 64x32
    {64, 64, 32, 2, 1},     // 7: 2 waves of 32x64
};
constexpr int kNumXCfgs = sizeof(kXCfgs) / sizeof(kXCfgs[0]);

void launch_x_cfg(int c, const GemmF& p, bool ak, bool bk, hipStream_t s) {
  switch (c) {
    case 0: launch_x<128, 128, 32, 2, 2, 2>(p, ak, bk, s); break;
    case 1: launch_x<128, 128, 32, 4, 2, 2>(p, ak, bk, s); break;
    case 2: launch_x<256, 128, 32, 4, 2, 1>(p, ak, bk, s); break;
    case 3: launch_x<256, 128, 16, 4, 2, 2>(p, ak, bk, s); break;
    case 4: launch_x<128, 256, 32, 2, 4, 1>(p, ak, bk, s); break;
    case 5: launch_x<128, 128, 16, 2, 2, 2>(p, ak, bk, s); break;
    case 6: launch_x<128, 64, 32, 2, 2, 2>(p, ak, bk, s); break;
    default: launch_x<64, 64, 32, 2, 1, 4>(p, ak, bk, s); break;
  }
}

}  // namespace

// Tile and split-K depth of the plane kernel: 256x128 (8 waves) when those tiles cover >= 3/4 of the
// 256 CUs, else 128x128 (4 waves, 3-stage ring); K split until the grid reaches one block per CU
// (a fused backward epilogue needs the whole sum).  FM_PL_BM / FM_PL_KS force them (lab A/B).
static void pl3_choose(int M, int N, int K, bool fused, int ksplit_req, const float* ws, long ws_bytes, int& bm, int& ks) {
  static const int bm_env = getenv("FM_PL_BM") ? atoi(getenv("FM_PL_BM")) : 0;
  static const int ks_env = getenv("FM_PL_KS") ? atoi(getenv("FM_PL_KS")) : 0;
  const long t256 = (long)((M + 255) / 256) * ((N + 127) / 128);
  bm = (bm_env == 128 || bm_env == 256) ? bm_env : (t256 >= 192 ? 256 : 128);
  const long tiles = (long)((M + bm - 1) / bm) * ((N + 127) / 128);
  const int ktiles = K / 32;
  ks = 1;
  if (ksplit_req > 0) ks = ksplit_req;
  else if (ks_env > 0) ks = ks_env;
  else if (ws != nullptr)
    while (tiles * ks < 256 && ks * 2 <= ktiles / 4 && ks < 16) ks *= 2;
  if (fused) ks = 1;
  while (ks > 1 && (ws == nullptr || (long)ks * M * (long)N * 4 > ws_bytes)) ks /= 2;
  if (ks > ktiles) ks = ktiles > 0 ? ktiles : 1;
}

static int g_f32_variant = getenv("FM_GEMM_F32_VARIANT") ? atoi(getenv("FM_GEMM_F32_VARIANT")) : 0;
extern "C" void fm_gemm_f32_set_variant(int v) { g_f32_variant = v; }

// Same contract as fm_gemm (gemm.hip) with fp32 operands and output:
//   A_kcontig: A stored [M][K] (lda >= K) else [K][M] (lda >= M)
//   B_kcontig: B stored [N][K] (ldb >= K) else [K][N] (ldb >= N)
static int g_f32_split = -1;   // -1: from FM_F32_SPLIT at the first call
extern "C" void fm_gemm_f32_set_split(int on) { g_f32_split = on < 0 ? 0 : on; }
// default 3: the split kernel (gemm_x3.hip) for the big GEMMs, where it beat both the native
// fp32 MFMA kernel and hipBLASLt on every DLRM shape and orientation (profiles/gemm_f32_lab_r5i_*)
static int f32_split_mode() {
  if (g_f32_split < 0) g_f32_split = getenv("FM_F32_SPLIT") != nullptr ? std::max(0, atoi(getenv("FM_F32_SPLIT"))) : 3;
  return g_f32_split;
}
extern "C" int fm_gemm_f32_get_split() { return f32_split_mode(); }

struct SgdUpdF {
  float* w; unsigned short* wc; float* v; const float* lr; float wd, mom; int nest;
};

struct PlanesF {
  const unsigned short* a; long psa;
  const unsigned short* b; long psb;
  unsigned short* c; long psc;
};

static int gemm_f32_run(const float* A, long lda, long sA, int a_kcontig, const float* B, long ldb, long sB,
                        int b_kcontig, float* C, long ldc, long sC, const float* bias, int M, int N, int K, int batch,
                        float alpha, int beta, int act, float* ws, long ws_bytes, int ksplit_req, const float* act_y,
                        long lday, int bwd_act, float* colsum, float* rowsum_a, const SgdUpdF* upd, const PlanesF* pl,
                        hipStream_t stream);

extern "C" int fm_gemm_f32(const float* A, long lda, long sA, int a_kcontig, const float* B, long ldb, long sB,
                           int b_kcontig, float* C, long ldc, long sC, const float* bias, int M, int N, int K, int batch,
                           float alpha, int beta, int act, float* ws, long ws_bytes, int ksplit_req, const float* act_y,
                           long lday, int bwd_act, float* colsum, float* rowsum_a, hipStream_t stream) {
  return gemm_f32_run(A, lda, sA, a_kcontig, B, ldb, sB, b_kcontig, C, ldc, sC, bias, M, N, K, batch, alpha, beta, act, ws,
                      ws_bytes, ksplit_req, act_y, lday, bwd_act, colsum, rowsum_a, nullptr, nullptr, stream);
}

// fm_gemm_f32 with exact bf16 operand planes (gemm_pl.hip): Ap / Bp (or nullptr) are the planes of
// A / B with A's / B's leading dims, plane p at base + p * ps; Cp (or nullptr) receives the planes
// of the stored C (C's leading dim, plane stride psc).  With both operand planes the plane kernel
// runs wherever its shape constraints hold (else the fp32 kernels, which still emit Cp).
extern "C" int fm_gemm_f32_pl(const float* A, long lda, long sA, int a_kcontig, const float* B, long ldb, long sB,
                              int b_kcontig, float* C, long ldc, long sC, const float* bias, int M, int N, int K, int batch,
                              float alpha, int beta, int act, float* ws, long ws_bytes, int ksplit_req, const float* act_y,
                              long lday, int bwd_act, float* colsum, float* rowsum_a, const unsigned short* Ap, long psa,
                              const unsigned short* Bp, long psb, unsigned short* Cp, long psc, hipStream_t stream) {
  PlanesF pl{Ap, psa, Bp, psb, Cp, psc};
  return gemm_f32_run(A, lda, sA, a_kcontig, B, ldb, sB, b_kcontig, C, ldc, sC, bias, M, N, K, batch, alpha, beta, act, ws,
                      ws_bytes, ksplit_req, act_y, lday, bwd_act, colsum, rowsum_a, nullptr, &pl, stream);
}

// fp32 weight-gradient GEMM with the SGD update fused in (same contract as gemm.hip fm_gemm_dw_sgd):
// A = dpre [K][M], B = x [K][N], W [M][ldw] updated in place, the gradient never stored; -1 when
// the fused form does not apply (the caller falls back to GEMM + optimizer kernel).  Always the
// default register-staged kernel (the split-bf16 and A/B variants carry no update epilogue).
extern "C" int fm_gemm_f32_dw_sgd(const float* A, long lda, const float* B, long ldb, float* W, long ldw,
                                  unsigned short* Wc, float* V, const float* lr, float wd, float mom, int nesterov,
                                  int M, int N, int K, float* ws, long ws_bytes, float* rowsum_a, hipStream_t stream) {
  SgdUpdF u{W, Wc, V, lr, wd, mom, nesterov};
  return gemm_f32_run(A, lda, 0, 0, B, ldb, 0, 0, W, ldw, 0, nullptr, M, N, K, 1, 1.f, 0, 10, ws, ws_bytes, 0, nullptr, 0,
                      10, nullptr, rowsum_a, &u, nullptr, stream);
}

// fm_gemm_f32_dw_sgd with the operand planes of dpre (Ap) and x (Bp), see fm_gemm_f32_pl
extern "C" int fm_gemm_f32_dw_sgd_pl(const float* A, long lda, const float* B, long ldb, float* W, long ldw,
                                     unsigned short* Wc, float* V, const float* lr, float wd, float mom, int nesterov,
                                     int M, int N, int K, float* ws, long ws_bytes, float* rowsum_a,
                                     const unsigned short* Ap, long psa, const unsigned short* Bp, long psb,
                                     hipStream_t stream) {
  SgdUpdF u{W, Wc, V, lr, wd, mom, nesterov};
  PlanesF pl{Ap, psa, Bp, psb, nullptr, 0};
  return gemm_f32_run(A, lda, 0, 0, B, ldb, 0, 0, W, ldw, 0, nullptr, M, N, K, 1, 1.f, 0, 10, ws, ws_bytes, 0, nullptr, 0,
                      10, nullptr, rowsum_a, &u, &pl, stream);
}

static int gemm_f32_run(const float* A, long lda, long sA, int a_kcontig, const float* B, long ldb, long sB,
                        int b_kcontig, float* C, long ldc, long sC, const float* bias, int M, int N, int K, int batch,
                        float alpha, int beta, int act, float* ws, long ws_bytes, int ksplit_req, const float* act_y,
                        long lday, int bwd_act, float* colsum, float* rowsum_a, const SgdUpdF* upd, const PlanesF* pl,
                        hipStream_t stream) {
  if (M <= 0 || N <= 0 || batch <= 0) return 0;
  if (upd && (K <= 0 || ldc % 4 != 0 || (((uintptr_t)upd->w | (uintptr_t)(upd->v ? upd->v : upd->w)) & 15) ||
              (((uintptr_t)(upd->wc ? (void*)upd->wc : (void*)upd->w)) & 7)))
    return -1;
  if (beta) fm_gemm_join(stream);      // C may be a gradient an async reduce is still writing
  GemmF p;
  p.A = A; p.lda = lda; p.sA = sA;
  p.B = B; p.ldb = ldb; p.sB = sB;
  p.C = C; p.ldc = ldc; p.sC = sC;
  p.bias = bias; p.ws = ws; p.ay = act_y; p.lday = lday; p.colsum = colsum; p.rowsum_a = rowsum_a;
  p.bact = bwd_act; p.M = M; p.N = N; p.K = K; p.act = act; p.beta = beta; p.batch = batch; p.alpha = alpha;
  p.n_fast = M >= N;
  p.uw = upd ? upd->w : nullptr;
  p.uwc = upd ? upd->wc : nullptr;
  p.uv = upd ? upd->v : nullptr;
  p.ulr = upd ? upd->lr : nullptr;
  p.uwd = upd ? upd->wd : 0.f;
  p.umom = upd ? upd->mom : 0.f;
  p.unest = upd ? upd->nest : 0;
  static const bool sgd_direct = getenv("FM_SGD_EPI_DIRECT") != nullptr && atoi(getenv("FM_SGD_EPI_DIRECT")) == 1;
  p.ulds = upd && !sgd_direct;
  p.Ap = pl ? pl->a : nullptr;
  p.psa = pl ? pl->psa : 0;
  p.Bp = pl ? pl->b : nullptr;
  p.psb = pl ? pl->psb : 0;
  p.Cp = (pl && !upd) ? pl->c : nullptr;
  p.psc = pl ? pl->psc : 0;
  static const int pvar_env = getenv("FM_PL_VAR") ? atoi(getenv("FM_PL_VAR")) : 0;
  p.pvar = pvar_env;
  auto al = [](const void* q) { return (((uintptr_t)q) & 15) == 0; };
  // pre-split operands (gemm_pl.hip): the plane kernel whenever both operand planes are given and
  // the shape fits it (FM_F32_PLANES=0 disables it for A/B)
  static const bool planes_on = getenv("FM_F32_PLANES") == nullptr || atoi(getenv("FM_F32_PLANES")) != 0;
  if (planes_on && p.Ap && p.Bp && batch == 1 && K > 0 && K % 32 == 0 && M >= 64 && N >= 64 && al(p.Ap) && al(p.Bp) &&
      lda % 8 == 0 && ldb % 8 == 0 && p.psa % 8 == 0 && p.psb % 8 == 0 && (a_kcontig || M % 8 == 0) &&
      (b_kcontig || N % 8 == 0)) {
    int bm = 0, ks = 0;
    pl3_choose(M, N, K, act_y != nullptr || colsum != nullptr, ksplit_req, ws, ws_bytes, bm, ks);
    p.tiles_m = (M + bm - 1) / bm;
    p.tiles_n = (N + 127) / 128;
    p.ksplit = ks;
    if (ks > 1) fm_gemm_join(stream);
    if (fm_gemm_pl3_launch(&p, bm, a_kcontig, b_kcontig, upd != nullptr && ks == 1, stream) == 0) {
      if (ks > 1) {
        const int v4 = (N % 4 == 0) && (ldc % 4 == 0) && (sC % 4 == 0) && al(C);
        const long total = (long)M * N * batch / (v4 ? 4 : 1);
        launch_reduce_f32(p, v4, total, stream);
      }
      return ks;
    }
  }
  bool vec = al(A) && al(B) && (lda % 4 == 0) && (ldb % 4 == 0) && (sA % 4 == 0) && (sB % 4 == 0);
  vec = vec && (a_kcontig ? (K % 4 == 0) : (M % 4 == 0)) && (b_kcontig ? (K % 4 == 0) : (N % 4 == 0));
  // variant knob (tools/bench_gemm.py A/B): 1 = the LDS-DMA kernel where it applies, 2 = its
  // 4-wave 256x128 form.  OPT-IN: measured on the DLRM fp32 step (profiles/prof_r2_fp32b_*) it
  // ties the register-staged kernel on the 1024-wide layers (150.8 vs 150.7 us) and loses on the
  // small-grid ones (one 96 KiB block per CU: 22 -> 39 us, 29 -> 45 us), 1.72 vs 1.68 ms/step.
  const int variant = upd ? 0 : g_f32_variant;
  p.atomic = 0;
  // fp32 on the bf16 matrix cores (exact three-way operand split, fm_gemm_x3_kernel): FM_F32_SPLIT=1
  // or fm_gemm_f32_set_split(1)
  f32_split_mode();
  // second split form (gemm_x3.hip): split in the register staging pass, double-buffered planes,
  // 64x64 per wave.  FM_F32_SPLIT=2: every eligible GEMM; 3 (auto): only the big ones, where it
  // measured faster than the native kernel (min(M, N) >= FM_X3_MIN_MN and K >= FM_X3_MIN_K, both
  // 480 by default).  K-contiguous operands need 16-B rows; MN-contiguous ones are read per element.
  static const int x3_min_mn = getenv("FM_X3_MIN_MN") ? atoi(getenv("FM_X3_MIN_MN")) : 480;
  static const int x3_min_k = getenv("FM_X3_MIN_K") ? atoi(getenv("FM_X3_MIN_K")) : 480;
  // (an explicit A/B kernel variant, FM_GEMM_F32_VARIANT / fm_gemm_f32_set_variant, bypasses the auto policy)
  const bool x3_pick = g_f32_split == 2 || (g_f32_split == 3 && (upd || g_f32_variant == 0) &&
                                            std::min(M, N) >= x3_min_mn && K >= x3_min_k);
  if (x3_pick && K > 0 && K % 32 == 0 && M >= 64 && N >= 64) {
    auto opnd_ok = [&](const float* X, long ld, long sX, bool kc, int rows) {
      (void)rows;
      return kc ? (al(X) && ld % 4 == 0 && sX % 4 == 0) : true;   // MN-contiguous: 4-B loads
    };
    if (opnd_ok(A, lda, sA, a_kcontig, M) && opnd_ok(B, ldb, sB, b_kcontig, N)) {
      // 256x128 (8 waves, 2 per SIMD) whenever M fills it, split-K for the grid; FM_X3_BM=128 forces
      // the 4-wave 128x128 tile
      static const int bm_env = getenv("FM_X3_BM") ? atoi(getenv("FM_X3_BM")) : 0;
      const int bm = (bm_env == 128 || bm_env == 256) ? bm_env : (M >= 256 ? 256 : 128);
      p.tiles_m = (M + bm - 1) / bm;
      p.tiles_n = (N + 127) / 128;
      const long tiles = (long)p.tiles_m * p.tiles_n * batch;
      const int ktiles = K / 32;
      const bool fused = act_y != nullptr || colsum != nullptr;
      int ks = 1;
      if (ksplit_req > 0) ks = ksplit_req;
      else if (ws != nullptr && !fused)
        while (tiles * ks < 256 && ks * 2 <= ktiles / 4 && ks < 16) ks *= 2;
      if (fused) ks = 1;
      while (ks > 1 && (ws == nullptr || (long)batch * ks * M * (long)N * 4 > ws_bytes)) ks /= 2;
      p.ksplit = ks;
      if (ks > 1) fm_gemm_join(stream);
      if (fm_gemm_x3v2_launch(&p, bm, a_kcontig, b_kcontig, upd != nullptr && ks == 1, stream) == 0) {
        if (ks > 1) {
          const int v4 = (N % 4 == 0) && (ldc % 4 == 0) && (sC % 4 == 0) && al(C);
          const long total = (long)M * N * batch / (v4 ? 4 : 1);
          launch_reduce_f32(p, v4, total, stream);
        }
        return ks;
      }
    }
  }
  if (g_f32_split == 1 && !upd && K >= 64 && M >= 64 && N >= 64) {
    const bool fused = act_y != nullptr || colsum != nullptr;
    p.tiles_m = (M + 127) / 128;
    p.tiles_n = (N + 127) / 128;
    const long tiles = (long)p.tiles_m * p.tiles_n * batch;
    const int ktiles = (K + X3_BK - 1) / X3_BK;
    int ks = 1;
    if (ksplit_req > 0) ks = ksplit_req;
    else if (ws != nullptr && !fused)   // one 96 KB block per CU: split until the grid covers 256 CUs
      while (tiles * ks < 256 && ks * 2 <= ktiles / 2 && ks < 16) ks *= 2;
    if (fused) ks = 1;
    if (ks > 1 && (ws == nullptr || (long)batch * ks * M * (long)N * 4 > ws_bytes)) ks = 1;
    p.ksplit = ks;
    if (ks > 1) fm_gemm_join(stream);
    const int lds = 6 * 128 * X3_BK * 2;
    dim3 grid(p.tiles_m * p.tiles_n, batch, ks);
    // per-operand 16-B load permission (bit 0: A, bit 1: B); k / m / n tails take element loads
    const int vmask = ((al(A) && lda % 4 == 0 && sA % 4 == 0) ? 1 : 0) | ((al(B) && ldb % 4 == 0 && sB % 4 == 0) ? 2 : 0);
#define FM_X3_GO(AKv, BKv)                                                                                     \
    do {                                                                                                       \
      static bool attr = false;                                                                                \
      if (!attr) {                                                                                             \
        (void)hipFuncSetAttribute((const void*)fm_gemm_x3_kernel<AKv, BKv>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                  lds);                                                                        \
        attr = true;                                                                                           \
      }                                                                                                        \
      hipLaunchKernelGGL((fm_gemm_x3_kernel<AKv, BKv>), grid, dim3(512), lds, stream, p, vmask);               \
    } while (0)
    if (a_kcontig && b_kcontig) FM_X3_GO(true, true);
    else if (a_kcontig) FM_X3_GO(true, false);
    else if (b_kcontig) FM_X3_GO(false, true);
    else FM_X3_GO(false, false);
#undef FM_X3_GO
    if (ks > 1) {
      const int v4 = (N % 4 == 0) && (ldc % 4 == 0) && (sC % 4 == 0) && al(C);
      const long total = (long)M * N * batch / (v4 ? 4 : 1);
      launch_reduce_f32(p, v4, total, stream);
    }
    return ks;
  }
  if (vec && variant >= 20000 && variant < 20100 && K > 0) {
    const int rc = (variant - 20000) % fm_gemm_f32_ring_cfg(0, nullptr);
    int geo[5];
    fm_gemm_f32_ring_cfg(rc, geo);
    const struct { int bm, bn, bk, mode; } c = {geo[0], geo[1], geo[2], geo[4]};
    const bool pers_ok = c.mode == 0 || batch == 1;
    if (K % c.bk == 0 && (a_kcontig || M % 4 == 0) && (b_kcontig || N % 4 == 0) && M >= 4 && N >= 4 && pers_ok) {
      p.tiles_m = (M + c.bm - 1) / c.bm;
      p.tiles_n = (N + c.bn - 1) / c.bn;
      const long tiles = (long)p.tiles_m * p.tiles_n * batch;
      const int ktiles = K / c.bk;
      int ks = 1;
      if (ksplit_req > 0) ks = ksplit_req;
      else if (ws != nullptr)
        while (tiles * ks < 256 && ks * 2 <= ktiles / 4 && ks < 16) ks *= 2;
      if (act_y != nullptr || colsum != nullptr) ks = 1;
      while (ks > 1 && (ws == nullptr || (long)batch * ks * M * (long)N * 4 > ws_bytes)) ks /= 2;
      while (ks > 1 && c.mode != 0 && ktiles % ks != 0) ks /= 2;   // persistent: equal stages per unit
      p.ksplit = ks;
      if (ks > 1) fm_gemm_join(stream);
      fm_gemm_f32_ring_launch(&p, rc, a_kcontig, b_kcontig, 0, stream);
      if (ks > 1) {
        const int v4 = (N % 4 == 0) && (ldc % 4 == 0) && (sC % 4 == 0) && al(C);
        const long total = (long)M * N * batch / (v4 ? 4 : 1);
        launch_reduce_f32(p, v4, total, stream);
      }
      return ks;
    }
  }
  if (vec && variant >= 1000 && variant < 1200 && K > 0) {
    const XCfg c = kXCfgs[((variant - 1000) % 100) % kNumXCfgs];
    const bool atomic_ok = ((variant - 1000) / 100 == 1) && beta && bias == nullptr && act == ACT_NONE &&
                           act_y == nullptr && colsum == nullptr;
    p.tiles_m = (M + c.bm - 1) / c.bm;
    p.tiles_n = (N + c.bn - 1) / c.bn;
    const long tiles = (long)p.tiles_m * p.tiles_n * batch;
    const int ktiles = (K + c.bk - 1) / c.bk;
    int ks = 1;
    if (ksplit_req > 0) ks = ksplit_req;
    else if (ws != nullptr || atomic_ok) {
      const long target = (c.bm * c.bn >= 256 * 128) ? 256L : 512L;
      while (tiles * ks < target && ks * 2 <= ktiles / 4 && ks < 32) ks *= 2;
    }
    if (act_y != nullptr || colsum != nullptr) ks = 1;
    if (ks > 1 && !atomic_ok && (ws == nullptr || (long)batch * ks * M * (long)N * 4 > ws_bytes)) ks = 1;
    p.ksplit = ks;
    p.atomic = (ks > 1 && atomic_ok) ? 1 : 0;
    if (ks > 1) fm_gemm_join(stream);  // the slab workspace is shared
    launch_x_cfg((variant - 1000) % 100, p, a_kcontig, b_kcontig, stream);
    if (ks > 1 && !p.atomic) {
      const int v4 = (N % 4 == 0) && (ldc % 4 == 0) && (sC % 4 == 0) && al(C);
      const long total = (long)M * N * batch / (v4 ? 4 : 1);
      launch_reduce_f32(p, v4, total, stream);
    }
    return ks;
  }
  const long t256 = (long)((M + 255) / 256) * ((N + 127) / 128) * batch;
  const long t128g = (long)((M + 127) / 128) * ((N + 127) / 128) * batch;
  const bool mn_ok = (a_kcontig || M >= 4) && (b_kcontig || N >= 4);
  if (vec && (variant & 1) && K > 0 && K % BKF == 0 && M >= 8 && N >= 8 && mn_ok && K >= 4 * BKF) {
    const bool big = t256 >= 192;
    const int bm = big ? 256 : 128;
    p.tiles_m = (M + bm - 1) / bm;
    p.tiles_n = (N + 127) / 128;
    const long tiles = big ? t256 : t128g;
    const int ktiles = K / BKF;
    int ks = 1;
    if (ksplit_req > 0) ks = ksplit_req;
    else if (ws != nullptr) {
      while (tiles * ks < 256 && ks * 2 <= ktiles / 4 && ks < 16) ks *= 2;
    }
    if (act_y != nullptr || colsum != nullptr) ks = 1;
    if (ks > 1 && (ws == nullptr || (long)batch * ks * M * (long)N * 4 > ws_bytes)) ks = 1;
    p.ksplit = ks;
    if (ks > 1) fm_gemm_join(stream);
    if (big) {
      if (variant & 2) launch_f_glds<256, 128, 2, 2>(p, a_kcontig, b_kcontig, stream);
      else launch_f_glds<256, 128, 4, 2>(p, a_kcontig, b_kcontig, stream);
    } else {
      launch_f_glds<128, 128, 2, 2>(p, a_kcontig, b_kcontig, stream);
    }
    if (ks > 1) {
      const int v4 = (N % 4 == 0) && (ldc % 4 == 0) && (sC % 4 == 0) && al(C);
      const long total = (long)M * N * batch / (v4 ? 4 : 1);
      launch_reduce_f32(p, v4, total, stream);
    }
    return ks;
  }
  // tiles: 128x128 when that gives >= 2 blocks per CU; narrower N / smaller tiles for small grids
  int BMv = 128, BNv = 128;
  const long t128 = (long)((M + 127) / 128) * ((N + 127) / 128) * batch;
  if (t128 < 512 && N <= 64 * 8) BNv = 64;
  // 64x64 tiles (no split-K, 4 blocks per CU) up to one wave of 128x128 tiles: the 8192x512->256
  // forward runs unsplit instead of split-K 2 + reduce (step -0.2..0.9 %: profiles/ab_f32_t64.txt)
  static const long t64_below = getenv("FM_GEMM_F32_T64") ? atol(getenv("FM_GEMM_F32_T64")) : 129L;
  if (t128 < t64_below && K <= 2048) { BMv = 64; BNv = 64; }
  // a fused backward epilogue (act-bwd of the layer below / bias-grad column sums) cannot split K:
  // small grids take 64x64 tiles for 4x the blocks (summit_large dX, 256 x 4096 x 4096: 64 -> 256
  // blocks on 256 CUs)
  // ... unless K is long enough to split it: then 128x128 tiles split K and the fused epilogue runs in
  // the reduce (fm_gemm_f32_reduce_bwd)
  const bool fused_ep = act_y != nullptr || colsum != nullptr;
  const bool fused_split = fused_ep && t128 < 256 && K >= 1024 && ws != nullptr && batch == 1 && ksplit_req <= 0 &&
                           (long)M * N * 4 * 2 <= ws_bytes;
  if (fused_ep && t128 < 256 && !fused_split) { BMv = 64; BNv = 64; }
  // variant bit 4096 (A/B): 256x128 tiles, one 4-wave block per CU, when they fill >= 3/4 of the chip
  if ((variant & 4096) && vec && (long)((M + 255) / 256) * ((N + 127) / 128) * batch >= 192) { BMv = 256; BNv = 128; }
  p.tiles_m = (M + BMv - 1) / BMv;
  p.tiles_n = (N + BNv - 1) / BNv;
  const long tiles = (long)p.tiles_m * p.tiles_n * batch;
  const int ktiles = (K + BKF - 1) / BKF;
  int ks = 1;
  if (ksplit_req > 0) ks = ksplit_req;
  else if (ws != nullptr) {
    static const long env_target = getenv("FM_GEMM_F32_SPLIT_BLOCKS") ? std::max(1L, atol(getenv("FM_GEMM_F32_SPLIT_BLOCKS"))) : 0L;
    const long target = env_target > 0 ? env_target : 512L;   // 2 resident blocks per CU
    // up to 16-way, or 64-way for a handful of tiles (the bottom-MLP dW GEMMs: 128 x 256 x 8192
    // made 64 blocks at 16-way, 30 us)
    const int ks_max = tiles <= 8 ? 64 : 16;
    while (tiles * ks < target && ks * 2 <= ktiles / 4 && ks < ks_max) ks *= 2;
  }
  if (fused_ep && !fused_split) ks = 1;   // fused bwd epilogue in the tile: needs the full K sum
  while (ks > 1 && (ws == nullptr || (long)batch * ks * M * (long)N * 4 > ws_bytes)) ks /= 2;
  if (K <= 0) ks = 1;
  p.ksplit = ks;
  if (ks > 1) fm_gemm_join(stream);
  const int opt = (variant >> 2) & 63;
  if (vec && BMv == 256) launch_fbm<256, 128>(p, a_kcontig, b_kcontig, vec, stream, opt);
  else if (BNv == 128) launch_fbm<128, 128>(p, a_kcontig, b_kcontig, vec, stream, opt);
  else if (BMv == 128) launch_fbm<128, 64>(p, a_kcontig, b_kcontig, vec, stream, opt);
  else launch_fbm<64, 64>(p, a_kcontig, b_kcontig, vec, stream, 0);
  if (ks > 1 && fused_ep) {
    const int bx = (N + 1023) / 1024;
    const int by = std::max(1, std::min(M, 1024 / bx));
    const int RB = (M + by - 1) / by;
    hipLaunchKernelGGL(fm_gemm_f32_reduce_bwd, dim3(bx, (M + RB - 1) / RB), dim3(256), 0, stream, p, RB);
  } else if (ks > 1) {
    const int v4 = (N % 4 == 0) && (ldc % 4 == 0) && (sC % 4 == 0) && al(C);
    const long total = (long)M * N * batch / (v4 ? 4 : 1);
    launch_reduce_f32(p, v4, total, stream);
  }
  return ks;
}

// ------------------------------------------------------------------------------------------
// fp32 skinny layers (out_features == 1): GEMV forward, fused act-bwd / dX / dW / db backward.
namespace {

__global__ void __launch_bounds__(256) fm_skinny_fwd_f32(const float* __restrict__ x, long ldx, const float* __restrict__ w,
                                                        const float* __restrict__ bias, float* __restrict__ y, long ldy,
                                                        long B, int K, int act) {
  const int lane = threadIdx.x & 63;
  const long waves = (long)gridDim.x * 4;
  const bool vec = (K % 4 == 0) && (ldx % 4 == 0);
  for (long b = blockIdx.x * 4 + (threadIdx.x >> 6); b < B; b += waves) {
    const float* xr = x + b * ldx;
    float s = 0.f;
    if (vec) {
      for (int k = lane * 4; k < K; k += 256) {
        const f32x4_t a = *reinterpret_cast<const f32x4_t*>(xr + k);
        const f32x4_t c = *reinterpret_cast<const f32x4_t*>(w + k);
        s += a[0] * c[0] + a[1] * c[1] + a[2] * c[2] + a[3] * c[3];
      }
    } else {
      for (int k = lane; k < K; k += 64) s += xr[k] * w[k];
    }
    s = wave_reduce_sum(s);
    if (lane == 0) y[b * ldy] = act_fwd(act, s + (bias ? bias[0] : 0.f));
  }
}

// thread = 4 consecutive columns of rows sub, sub+rpi, ...; per-block dW/db partials reduced in
// LDS, one atomic per column per block
__global__ void __launch_bounds__(256) fm_skinny_bwd_f32(int ROWS, const float* __restrict__ x, long ldx,
                                                        const float* __restrict__ w, const float* __restrict__ y, long ldy,
                                                        const float* __restrict__ dy, long lddy, float* __restrict__ dx,
                                                        long lddx, int dx_acc, float* __restrict__ dw,
                                                        float* __restrict__ db, long B, int K, int act, int bact) {
  // bact != ACT_NONE: the activation backward of the layer below (whose output is x) is applied to
  // dX here, so that layer's separate act-bwd / bias-gradient pass is skipped (its dW GEMM then
  // takes dX as its pre-activation gradient and sums the bias gradient itself)
  __shared__ float red[256 * 4];
  __shared__ float redb[256];
  // column block blockIdx.y covers [1024 y, 1024 y + 1024) of K (host: K % 4 == 0)
  const int cb = blockIdx.y * 1024;
  const int Kc = min(1024, K - cb);
  const int lpr = Kc / 4;
  const int rpi = 256 / lpr;
  const int sub = threadIdx.x / lpr, g = threadIdx.x - sub * lpr;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  float dbs = 0.f;
  const long r0 = (long)blockIdx.x * ROWS;
  const int c0 = cb + g * 4;
  if (blockIdx.y) db = nullptr;          // db accumulated once, by column block 0
  const f32x4_t wv = *reinterpret_cast<const f32x4_t*>(w + c0);
  if (sub < rpi) {
    const long rend = min(B, r0 + ROWS);
    // SU rows per iteration with every load issued first (8 measured no faster than 4 on the
    // MLPerf click layer: 13.5 vs 12.6 us, and 68 vs 40 VGPRs)
    constexpr int SU = 4;
    for (long r = r0 + sub; r < rend; r += (long)SU * rpi) {
      float yv[SU], gv[SU];
      f32x4_t xv[SU], old[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const long rr = min(r + u * rpi, rend - 1);
        yv[u] = y[rr * ldy];
        gv[u] = dy[rr * lddy];
        xv[u] = *reinterpret_cast<const f32x4_t*>(x + rr * ldx + c0);
        old[u] = (dx && dx_acc) ? *reinterpret_cast<const f32x4_t*>(dx + rr * lddx + c0) : f32x4_t{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const long rr = r + u * rpi;
        if (rr >= rend) break;
        const float d = act_bwd(act, yv[u], gv[u]);
        dbs += d;
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] += d * xv[u][j];
        if (dx) {
          f32x4_t v = d * wv + old[u];
          if (bact != ACT_NONE) {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = act_bwd(bact, xv[u][j], v[j]);
          }
          *reinterpret_cast<f32x4_t*>(dx + rr * lddx + c0) = v;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) red[threadIdx.x * 4 + j] = (sub < rpi) ? acc[j] : 0.f;
  redb[threadIdx.x] = (sub < rpi && g == 0) ? dbs : 0.f;
  __syncthreads();
  for (int c = threadIdx.x; c < Kc; c += 256) {
    const int gg = c / 4, j = c % 4;
    float t = 0.f;
    for (int q = 0; q < rpi; ++q) t += red[(q * lpr + gg) * 4 + j];
    atomicAdd(dw + cb + c, t);
  }
  if (db && threadIdx.x == 0) {
    float t = 0.f;
    for (int q = 0; q < rpi; ++q) t += redb[q * lpr];
    atomicAdd(db, t);
  }
}

}  // namespace

extern "C" void fm_skinny_fwd_f32_launch(const float* x, long ldx, const float* w, const float* bias, float* y, long ldy,
                                         long B, int K, int act, hipStream_t s) {
  if (B <= 0) return;
  hipLaunchKernelGGL(fm_skinny_fwd_f32, dim3((unsigned)std::min<long>((B + 3) / 4, 4096)), dim3(256), 0, s, x, ldx, w,
                     bias, y, ldy, B, K, act);
}

// dW (fp32 [K]) and db (fp32 [1]) ACCUMULATE; requires K % 4 == 0 and 16-B aligned rows
extern "C" void fm_skinny_bwd_f32_launch(const float* x, long ldx, const float* w, const float* y, long ldy,
                                         const float* dy, long lddy, float* dx, long lddx, int dx_acc, float* dw, float* db,
                                         long B, int K, int act, int bact, hipStream_t s) {
  if (B <= 0) return;
  int ROWS = 64;
  while (ROWS > 2 && (B + ROWS - 1) / ROWS < 128) ROWS /= 2;
  hipLaunchKernelGGL(fm_skinny_bwd_f32, dim3((unsigned)((B + ROWS - 1) / ROWS), (unsigned)((K + 1023) / 1024)), dim3(256), 0,
                     s, ROWS, x, ldx, w, y, ldy,
                     dy, lddy, dx, lddx, dx_acc, dw, db, B, K, act, bact);
}
