// flexmi fp32 GEMM on the bf16 matrix cores, second form: exact three-way operand split done in
// the register staging pass, double-buffered planes, 64x64 output per wave (gfx950 / MI355X).
//
//   C[M,N] (+)= epilogue( alpha * sum_k A(m,k) * B(k,n) )      fp32 in, fp32 accumulate, fp32 out
//
// Every fp32 operand x is split EXACTLY into three bf16 terms by truncation: h = x with the low 16
// bits cleared, r = x - h (exact: <= 16 significant bits), m = r truncated the same way, l = r - m
// (<= 8 significant bits: exactly a bf16).  x*y is then the sum of the six products with
// i + j <= 2 (hh, hm, mh, hl, mm, lh) on v_mfma_f32_16x16x32_bf16 with fp32 accumulation: each
// bf16 x bf16 product is exact in fp32, and the dropped terms (ml, lm, ll) are <= 2^-24 |x y|, the
// order of the fp32 product rounding itself -- native-fp32 accuracy (tests/test_gpu_fp32.py checks
// it against float64 at the native kernel's tolerance).  The reference computes these GEMMs with
// cublasSgemm (src/ops/linear.cu:424-447 forward, :592-635 backward).
//
// Cost per 16x16x32 block: 6 bf16 MFMA x 16 cycles against 8 fp32 MFMA x 32 cycles (2.7x the fp32
// MFMA rate).  The first split kernel (gemm_f32.hip fm_gemm_x3_kernel: 128x128 tile, one LDS
// buffer, 64x32 per wave, split at the LDS store between two barriers) measured at parity with the
// native fp32 kernel (profiles/gemm_f32_split_vs_native_r4c.jsonl): its waves read 18 b128
// fragments per 48 MFMAs and stalled on the store phase.  This form:
//   * 64x64 output per wave (4x4 tiles): 24 b128 fragment reads per 96 MFMAs;
//   * two LDS stages of three bf16 planes per operand, [row][32 k] images with 64-B rows and the
//     16-B chunk XOR-swizzled by (row >> 1) & 3 (conflict-free ds_read_b128 fragment reads);
//   * one barrier per 32-deep k step: after it, the staged registers of step t+1 are split into the
//     free stage, the loads of step t+2 are issued, and the MFMAs of step t run -- the global loads
//     have a whole step of MFMAs to land;
//   * MN-contiguous operands (dX's W, both dW operands) are transposed in registers: a staging
//     unit is one row x 8 k (eight 4-B loads, 256 contiguous bytes per wave-instruction).
// Measured and dropped: fp32 LDS images with the split done per fragment in registers (LDS stage
// 48 instead of 72 KiB) -- 119 vs 95 us on 8192x1024x1024, the per-wave split VALU work (8 floats
// per fragment, 24 fragments a step) outweighs the staging split it replaces (gpurun_out r5j).
// Tiles: 256x128 (8 waves, 144 KiB LDS) or 128x128 (4 waves, 96 KiB), one block per CU, or 128x64
// (2 waves, 72 KiB, two blocks per CU),
// XCD-aware tile order, split-K slabs / fused epilogues / fused SGD shared with the native kernel
// (gemm_f32_common.h epilogue_f32).
#include "gemm_f32_common.h"

#include <cstdlib>

namespace {

constexpr int XK = 32;   // k per stage

// byte offset of 16-B chunk c (8 bf16) of row r in a [row][32 bf16] plane; the chunk XOR
// (r >> 1) & 3 makes the 16x16x32 fragment reads (lane = 16 rows x 4 chunks) conflict-free
FM_DEVICE int x3_off(int r, int c) { return r * 64 + 16 * (c ^ ((r >> 1) & 3)); }

// the exact split of fp32 pairs into three bf16 planes: fm_split3_pair (common.h).  A non-finite
// operand gives m = l = NaN, so a GEMM with an inf operand returns NaN where the native fp32 kernel
// returns +-inf: documented, pinned by tests/test_gpu_fp32_split.py::test_split_nonfinite_operand
// (no per-element select in the staging pass, which is the kernel's VALU budget).  The 9-VALU
// packed form cut the 256x128 main loop from 3.4 to 2.4 VALU per MFMA (static count, no register
// moves left) and the DLRM step's split GEMMs 609.8 -> 599.9 us (profiles/x3_phase_lab_r6.txt).

// fp16 two-plane split of a scaled pair (F16 form): x = s * v (s an exact power of two putting the
// row's max |v| in [2^14, 2^15)), hi = f16(x) (RNE), lo = f16((x - hi) * 2^11) (RNE; the residual is
// exact in fp32 and scaled back into fp16's normal range).  v = (hi + lo * 2^-11) / s to 2^-22 |v|.
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
FM_DEVICE void fm_split2h_pair(float a, float b, float sc, unsigned& hi, unsigned& lo) {
  typedef float f2_t __attribute__((ext_vector_type(2)));
  const f2_t x = f2_t{a, b} * sc;
  const f16x2_t h = __builtin_convertvector(x, f16x2_t);
  const f2_t r = (x - __builtin_convertvector(h, f2_t)) * 2048.f;
  const f16x2_t l = __builtin_convertvector(r, f16x2_t);
  hi = __builtin_bit_cast(unsigned, h);
  lo = __builtin_bit_cast(unsigned, l);
}

// One operand's k step (R rows x 32 k) staged through registers; unit = (row, k-octet): the 8 k
// values of one row, split and written as one 16-B chunk per plane.  K-contiguous: two 16-B loads
// per unit, consecutive lanes take consecutive octets.  MN-contiguous (global [k][rows]): eight
// 4-B loads per unit (one per k row), consecutive lanes take consecutive rows, so each load
// instruction reads 256 contiguous bytes and the LDS writes land exactly like the K-contiguous
// ones (an earlier row-pair x k-quad unit wrote 8-B halves 4-way bank-conflicted: 14 M conflicts
// per 8192x1024x1024 dW, gpurun_out r5k).  Rows past the edge load a clamped (valid) row and are
// NOT zeroed: row r of A only reaches output row r (and B row n output column n), which the
// epilogue never stores, and the row sums are stored for in-range rows only.  The loaded values
// are kept as they arrive -- no select on them -- so the wait for a load lands at its use in the
// next step's split, a whole step of MFMAs later (a select right after the load made hipcc wait
// for every load as soon as it was issued).
template <bool KC, int R, int NTH>
struct X3Stage {
  static constexpr int UNITS = R * 4;
  static constexpr int PER_T = (UNITS + NTH - 1) / NTH;
  f32x4_t a[PER_T], b[PER_T];        // k 0..3 / 4..7 of the unit's row

  FM_DEVICE static void unit(int ci, int& r, int& c) {
    if constexpr (KC) {
      r = ci >> 2;
      c = ci & 3;
    } else {
      r = ci % R;
      c = ci / R;
    }
  }

  FM_DEVICE void load(const float* __restrict__ p, long ld, int row0, int rows, int k0, int tid) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int ci = tid + NTH * i;
      if (UNITS % NTH != 0 && ci >= UNITS) continue;
      int r, c;
      unit(ci, r, c);
      const int gr = min(row0 + r, rows - 1);
      if constexpr (KC) {
        const float* src = p + (long)gr * ld + k0 + 8 * c;
        a[i] = *reinterpret_cast<const f32x4_t*>(src);
        b[i] = *reinterpret_cast<const f32x4_t*>(src + 4);
      } else {
        const float* src = p + (long)(k0 + 8 * c) * ld + gr;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          a[i][kk] = src[kk * ld];
          b[i][kk] = src[(kk + 4) * ld];
        }
      }
    }
  }

  // F16 form: two fp16 planes of the unit's row scaled by sc[i]
  FM_DEVICE void store_h(char* pl0, char* pl1, const float (&sc)[PER_T], int tid) const {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int ci = tid + NTH * i;
      if (UNITS % NTH != 0 && ci >= UNITS) continue;
      int r, c;
      unit(ci, r, c);
      u32x4_t h, l;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const f32x4_t& v = u < 2 ? a[i] : b[i];
        unsigned hh, ll;
        fm_split2h_pair(v[2 * (u & 1)], v[2 * (u & 1) + 1], sc[i], hh, ll);
        h[u] = hh;
        l[u] = ll;
      }
      const int off = x3_off(r, c);
      *reinterpret_cast<u32x4_t*>(pl0 + off) = h;
      *reinterpret_cast<u32x4_t*>(pl1 + off) = l;
    }
  }

  // the scales of this thread's units (rows fixed per thread and unit slot): 2^sig of the row's max
  FM_DEVICE static void scales(const unsigned* amax, int np, int row0, int rows, int tid, float (&sc)[PER_T]) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      int r, c;
      unit(min(tid + NTH * i, UNITS - 1), r, c);
      sc[i] = pow2f(f16_sig(amax_of(amax, np, rows, min(row0 + r, rows - 1))));
    }
  }

  FM_DEVICE void store(char* pl0, char* pl1, char* pl2, int tid) const {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int ci = tid + NTH * i;
      if (UNITS % NTH != 0 && ci >= UNITS) continue;
      int r, c;
      unit(ci, r, c);
      u32x4_t h, m, l;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const f32x4_t& v = u < 2 ? a[i] : b[i];
        unsigned hh, mm, ll;
        fm_split3_pair(v[2 * (u & 1)], v[2 * (u & 1) + 1], hh, mm, ll);
        h[u] = hh;
        m[u] = mm;
        l[u] = ll;
      }
      const int off = x3_off(r, c);
      *reinterpret_cast<u32x4_t*>(pl0 + off) = h;
      *reinterpret_cast<u32x4_t*>(pl1 + off) = m;
      *reinterpret_cast<u32x4_t*>(pl2 + off) = l;
    }
  }

  // MN-contiguous A (dW): per-thread sums of its row (tid % R, every unit) over the staged k
  FM_DEVICE void rowsum(float& s, int tid) const {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int ci = tid + NTH * i;
      if (UNITS % NTH != 0 && ci >= UNITS) continue;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) s += a[i][kk] + b[i][kk];
    }
  }
};

template <int BM, int BN, bool AK, bool BKC, bool SGD, int SCHED, bool F16 = false>
__global__ void __launch_bounds__((BM / 64) * (BN / 64) * 64, 1) fm_gemm_x3v2_kernel(GemmF p) {
  constexpr int WM = BM / 64, WN = BN / 64, NTH = WM * WN * 64;
  constexpr int MR = 4, NR = 4;
  constexpr int NPL = F16 ? 2 : 3;                     // planes per operand
  constexpr int PA_ = BM * 64, PB_ = BN * 64;          // bytes of one 16-bit plane per operand
  constexpr int STG = NPL * (PA_ + PB_);
  extern __shared__ __attribute__((aligned(16))) char smem[];
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
  const int ktiles = p.K / XK;
  const int kt_per = (ktiles + p.ksplit - 1) / p.ksplit;
  const int kt0 = split * kt_per, kt1 = min(ktiles, kt0 + kt_per);
  const int nst = kt1 - kt0;

  // F16: acc = the hi*hi products, acc2 = the two cross products (scaled by 2^11)
  f32x4_t acc[MR][NR], acc2[MR][F16 ? NR : 1];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      if constexpr (F16) acc2[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    }

  // staging register sets: SCHED 3 keeps two (loads two steps ahead), the others one
  X3Stage<AK, BM, NTH> sa, sa1;
  X3Stage<BKC, BN, NTH> sb, sb1;
  float sca[X3Stage<AK, BM, NTH>::PER_T], scb[X3Stage<BKC, BN, NTH>::PER_T];
  if constexpr (F16) {
    X3Stage<AK, BM, NTH>::scales(p.amax_a, p.amax_na, m0, p.M, tid, sca);
    X3Stage<BKC, BN, NTH>::scales(p.amax_b, p.amax_nb, n0, p.N, tid, scb);
  }
  const bool dorow = (!AK) && p.rowsum_a != nullptr && tn == 0;
  float rs = 0.f;
  auto stage = [&](int s) { return smem + s * STG; };
  auto put_from = [&](int s, auto& SA, auto& SB) {
    char* b = stage(s);
    if constexpr (F16) {
      SA.store_h(b, b + PA_, sca, tid);
      SB.store_h(b + 2 * PA_, b + 2 * PA_ + PB_, scb, tid);
    } else {
      SA.store(b, b + PA_, b + 2 * PA_, tid);
      SB.store(b + 3 * PA_, b + 3 * PA_ + PB_, b + 3 * PA_ + 2 * PB_, tid);
    }
    if constexpr (!AK) {
      if (dorow) SA.rowsum(rs, tid);
    }
  };
  auto get_into = [&](int kt, auto& SA, auto& SB) {
    SA.load(A, p.lda, m0, p.M, kt * XK, tid);
    SB.load(B, p.ldb, n0, p.N, kt * XK, tid);
  };
  const int q = lane & 15, g = lane >> 4;
  constexpr int TA[6] = {2, 1, 0, 1, 0, 0};    // small terms first, the dominant h*h product last
  constexpr int TB[6] = {0, 1, 2, 0, 1, 0};
  auto load_b = [&](const char* lb, bf16x8_t (&bf)[NPL][NR]) {
#pragma unroll
    for (int pl = 0; pl < NPL; ++pl)
#pragma unroll
      for (int j = 0; j < NR; ++j)
        bf[pl][j] = *reinterpret_cast<const bf16x8_t*>(lb + pl * PB_ + x3_off(wn * 64 + 16 * j + q, g));
  };
  // MFMAs of one step, A fragments read per tile row (NR independent accumulator chains per term);
  // reading row i + 1 ahead of row i's MFMAs, or the fragments in first-use order, measured the same
  // (profiles/x3_phase_lab_r6.txt)
  auto mfma_rows = [&](const char* la, const bf16x8_t (&bf)[NPL][NR]) {
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      bf16x8_t af[NPL];
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl)
        af[pl] = *reinterpret_cast<const bf16x8_t*>(la + pl * PA_ + x3_off(wm * 64 + 16 * i + q, g));
      if constexpr (F16) {
        // cross terms first (hi_b lo_a, lo_b hi_a into acc2), then hi_b hi_a
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(*reinterpret_cast<const f16x8_t*>(&bf[0][j]),
                                                              *reinterpret_cast<const f16x8_t*>(&af[1]), acc2[i][j],
                                                              0, 0, 0);
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(*reinterpret_cast<const f16x8_t*>(&bf[1][j]),
                                                              *reinterpret_cast<const f16x8_t*>(&af[0]), acc2[i][j],
                                                              0, 0, 0);
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(*reinterpret_cast<const f16x8_t*>(&bf[0][j]),
                                                             *reinterpret_cast<const f16x8_t*>(&af[0]), acc[i][j],
                                                             0, 0, 0);
        continue;
      }
#pragma unroll
      for (int s = 0; s < 6; ++s)
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8v_t*>(&bf[TB[s]][j]),
                                                              *reinterpret_cast<const bf16x8v_t*>(&af[TA[s]]), acc[i][j],
                                                              0, 0, 0);
    }
  };
  if constexpr (SCHED == 3) {
    // de-phased waves (as SCHED 2) with the global loads two steps ahead: step t splits the
    // registers of step t+1 (set (t+1)&1) into stage (t+1)&1 and reloads that set with step t+3
    if (nst > 0) {
      get_into(kt0, sa, sb);
      put_from(0, sa, sb);
      if (nst > 1) get_into(kt0 + 1, sa1, sb1);
      if (nst > 2) get_into(kt0 + 2, sa, sb);
    }
    const bool mfma_first = (wave >> 2) & 1;
    auto body = [&](int t, auto& SA, auto& SB) {
      __syncthreads();               // stage t&1 complete; stage (t+1)&1 no longer read
      const char* b = stage(t & 1);
      bf16x8_t bf[NPL][NR];
      load_b(b + NPL * PA_, bf);
      if (!mfma_first && t + 1 < nst) {
        put_from((t + 1) & 1, SA, SB);
        if (t + 3 < nst) get_into(kt0 + t + 3, SA, SB);
      }
      mfma_rows(b, bf);
      if (mfma_first && t + 1 < nst) {
        put_from((t + 1) & 1, SA, SB);
        if (t + 3 < nst) get_into(kt0 + t + 3, SA, SB);
      }
    };
    for (int t = 0; t < nst; t += 2) {
      body(t, sa1, sb1);             // step t stages step t+1 from set 1
      if (t + 1 < nst) body(t + 1, sa, sb);
    }
  } else {
    if (nst > 0) {
      get_into(kt0, sa, sb);
      put_from(0, sa, sb);
      if (nst > 1) get_into(kt0 + 1, sa, sb);
    }
    for (int t = 0; t < nst; ++t) {
      __syncthreads();               // stage t&1 complete; stage (t+1)&1 no longer read
      const char* b = stage(t & 1);
      bf16x8_t bf[NPL][NR];
      load_b(b + NPL * PA_, bf);
      if (t + 1 < nst) {
        put_from((t + 1) & 1, sa, sb);
        if (t + 2 < nst) get_into(kt0 + t + 2, sa, sb);
      }
      mfma_rows(b, bf);
    }
  }
  if constexpr (!AK) {
    if (dorow) {   // the NTH / BM threads of each row: reduce through LDS, one atomic per row
      static_assert(NTH % BM == 0, "every thread's A units share one row");
      __syncthreads();
      float* red = reinterpret_cast<float*>(smem);
      red[tid] = rs;
      __syncthreads();
      if (tid < BM) {
        float x = 0.f;
        for (int s = tid; s < NTH; s += BM) x += red[s];
        if (m0 + tid < p.M) atomicAdd(p.rowsum_a + m0 + tid, x);
      }
    }
  }
  if constexpr (F16) {   // acc = (hi*hi + 2^-11 cross) / (s_m s_n)
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      const int m = min(m0 + wm * 64 + 16 * i + q, p.M - 1);
      const float dm = pow2f(-f16_sig(amax_of(p.amax_a, p.amax_na, p.M, m)));
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        f32x4_t v = acc[i][j] + acc2[i][j] * (1.f / 2048.f);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = min(n0 + wn * 64 + 16 * j + 4 * g + r, p.N - 1);
          v[r] = v[r] * dm * pow2f(-f16_sig(amax_of(p.amax_b, p.amax_nb, p.N, n)));
        }
        acc[i][j] = v;
      }
    }
  }
  epilogue_f32<MR, NR, false, false, SGD>(p, acc, zb, split, m0 + wm * 64, n0 + wn * 64, lane);
}

template <int BM, int BN, bool SGD, int SCHED, bool F16 = false>
void launch_x3v2_s(const GemmF& p, bool ak, bool bk, hipStream_t s) {
  constexpr int NTH = (BM / 64) * (BN / 64) * 64;
  constexpr int LDS = 2 * (F16 ? 2 : 3) * (BM + BN) * 64;
  dim3 grid(p.tiles_m * p.tiles_n, p.batch, p.ksplit);
#define FM_X3V2(AKv, BKv)                                                                                        \
  do {                                                                                                           \
    static bool attr = false;                                                                                    \
    if (!attr) {                                                                                                 \
      (void)hipFuncSetAttribute((const void*)fm_gemm_x3v2_kernel<BM, BN, AKv, BKv, SGD, SCHED, F16>,              \
                                hipFuncAttributeMaxDynamicSharedMemorySize, LDS);                                \
      attr = true;                                                                                               \
    }                                                                                                            \
    hipLaunchKernelGGL((fm_gemm_x3v2_kernel<BM, BN, AKv, BKv, SGD, SCHED, F16>), grid, dim3(NTH), LDS, s, p);    \
  } while (0)
  if (ak && bk) FM_X3V2(true, true);
  else if (ak) FM_X3V2(true, false);
  else if (bk) FM_X3V2(false, true);
  else FM_X3V2(false, false);
#undef FM_X3V2
}

// Schedules: 256x128 tiles (8 waves, two per SIMD) run schedule 3 -- the two waves of a SIMD do
// the staging split and the MFMAs of a step in opposite order, global loads two steps ahead
// (972.6 vs 975.6 us for schedule 2 and more for the one-register-set forms over the DLRM lab
// shapes, profiles/bench_ab_x3_sched_embgrid_r5n.txt; schedules 1 / 2 deleted in r6); 128x128
// tiles (4 waves) the plain one-set schedule 0.  The same schedule on 32x32x16 MFMAs (each leaving
// 24 of its 32 issue cycles to the staging split) measured slower: 1.236 vs 1.185 ms per DLRM fp32
// step (profiles/gemm_x3_mfma_form_bench_r5p3.txt), deleted.

template <int BM, int BN, bool SGD>
void launch_x3v2(const GemmF& p, bool ak, bool bk, hipStream_t s) {
  const bool f16 = p.amax_a != nullptr;
  if constexpr (BM == 256) {
    // no F16 form at 256x128: its second accumulator set spills at the 256 VGPRs of two waves per
    // SIMD in either schedule (tests/test_kernel_resources.py); the caller takes 128-row tiles for it
    (void)f16;
    launch_x3v2_s<BM, BN, SGD, 3>(p, ak, bk, s);
  } else {
    if (f16) launch_x3v2_s<BM, BN, SGD, 0, true>(p, ak, bk, s);
    else launch_x3v2_s<BM, BN, SGD, 0>(p, ak, bk, s);
  }
}

}  // namespace

// Launch on a prepared parameter block (tiles_m / tiles_n / ksplit filled for the bm x 128 tile).
// Caller guarantees: K % 32 == 0 (per split: whole steps); K-contiguous operands 16-B aligned with
// ld % 4 == 0 (MN-contiguous ones: no constraint).
// sgd: the fused-SGD epilogue (unsplit tiles only).  Returns -1 for an unsupported tile.
// bn = 128, or 64 with bm = 128: the 128x64 tile (2 waves, 72 KiB LDS, two blocks per CU) for the
// narrow layers (N = 256 / 512 at batch 8192: 256 / 512 tiles where 128x128 gives half a wave)
extern "C" int fm_gemm_x3v2_launch(const void* params, int bm, int bn, int a_kcontig, int b_kcontig, int sgd,
                                   hipStream_t s) {
  const GemmF& p = *static_cast<const GemmF*>(params);
  if (sgd && p.ksplit > 1) return -1;
  if (bm == 256 && bn == 128) {
    if (sgd) launch_x3v2<256, 128, true>(p, a_kcontig, b_kcontig, s);
    else launch_x3v2<256, 128, false>(p, a_kcontig, b_kcontig, s);
  } else if (bm == 128 && bn == 128) {
    if (sgd) launch_x3v2<128, 128, true>(p, a_kcontig, b_kcontig, s);
    else launch_x3v2<128, 128, false>(p, a_kcontig, b_kcontig, s);
  } else if (bm == 128 && bn == 64) {
    if (sgd) launch_x3v2<128, 64, true>(p, a_kcontig, b_kcontig, s);
    else launch_x3v2<128, 64, false>(p, a_kcontig, b_kcontig, s);
  } else {
    return -1;
  }
  return 0;
}
