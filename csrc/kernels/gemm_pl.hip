// flexmi fp32 GEMM on the bf16 matrix cores from PRE-SPLIT operands (gfx950 / MI355X).
//
//   C[M,N] (+)= epilogue( alpha * sum_k A(m,k) * B(k,n) )      fp32 values, fp32 accumulate / out
//
// Every fp32 operand arrives as three exact bf16 planes x = h + m + l (gemm_f32_common.h
// split3_bits), written once by its producer -- the epilogue of the GEMM that computed it
// (GemmF::Cp), or fm_split3 for weights / inputs -- instead of being re-split in registers by every
// block that reads it (gemm_x3.hip: each operand tile is split by all N/BN resp. M/BM blocks that
// share it; 3.4 VALU per MFMA and the staging pass on the critical path, VERDICT r4 "What's weak" #1).
// x*y is the sum of the six products with i + j <= 2 (hh, hm, mh, hl, mm, lh) on
// v_mfma_f32_16x16x32_bf16 with fp32 accumulation; the dropped terms are <= 2^-24 |x y| (fp32-class:
// tests/test_gpu_planes.py against float64).  The reference runs these GEMMs as cublasSgemm
// (src/ops/linear.cu:424-447 forward, :592-635 backward).
//
// Main loop: no VALU besides addressing.  Operand planes go global -> LDS with
// global_load_lds_dwordx4 (no staging registers, no ds_write pass) into an NS-stage ring:
//
//   iteration t:  s_waitcnt vmcnt((NS-2) * per-wave loads of a stage)   -- stage t landed
//                 s_waitcnt lgkmcnt(0); s_barrier   (every wave: stage t landed, stage t-1 read)
//                 issue stage t+NS-1 into the slot stage t-1 used
//                 fragments + 6 x 16 MFMAs per 16 x 16 output tile on stage t
//
// The barrier is the raw s_barrier (a __syncthreads() would drain the LDS-DMA queue with
// vmcnt(0)); all LDS is the one extern array.  LDS images: K-contiguous planes [row][32 k] (64-B
// rows, 16-B chunks XOR-swizzled by (row >> 1) & 3: conflict-free ds_read_b128 fragments);
// MN-contiguous planes [k][R] read with the transposing ds_read_b64_tr_b16 (gemm_common.h frag).
// The global_load_lds destination is lane-linear, so both swizzles are applied to the per-lane
// SOURCE address and to the fragment reads (same involution).
// Tiles: 256x128 (8 waves of 64x64, two 72 KiB stages) or 128x128 (4 waves, three 48 KiB stages);
// one block per CU, XCD-aware tile order; split-K slabs / fused epilogues / plane emission of C are
// the shared gemm_f32_common.h epilogue.
#include "gemm_f32_common.h"

namespace {

constexpr int PKS = 32;             // k per stage
constexpr int PCPR = PKS / 8;       // 16-B chunks per K-contiguous row

FM_DEVICE int pk_off(int r, int c) { return r * (PKS * 2) + 16 * (c ^ ((r >> 1) & (PCPR - 1))); }

// one plane of one operand tile (R rows x 32 k) into its LDS image, 1 KiB per wave-instruction
template <bool KC, int R, int NW>
struct PlIssue {
  static constexpr int INSTR = R * PKS * 2 / 1024;
  static constexpr int PER_W = INSTR / NW;
  static_assert(INSTR % NW == 0, "plane image must split evenly over the waves");

  FM_DEVICE static void run(const unsigned short* __restrict__ src, long ld, int row0, int rows, int k0, char* lds,
                            int wave, int lane) {
#pragma unroll
    for (int i = 0; i < PER_W; ++i) {
      const int j = wave + NW * i;
      const unsigned short* s;
      if constexpr (KC) {            // [row][32 k]: 16 rows of 64 B per instruction
        constexpr int RPI = 1024 / (PKS * 2);
        const int row = RPI * j + lane / PCPR;
        const int c = (lane % PCPR) ^ ((row >> 1) & (PCPR - 1));
        const int gr = min(row0 + row, rows - 1);          // rows past the edge: never stored
        s = src + (long)gr * ld + k0 + 8 * c;
      } else {                       // [k][R]: 1024 / (2R) k-rows per instruction
        constexpr int CPR = R / 8;
        constexpr int KPI = 1024 / (2 * R);
        const int krow = KPI * j + lane / CPR;
        const int c = (lane % CPR) ^ MNSwz<R>::f(krow);
        const int gr = min(row0 + 8 * c, rows - 8);         // host: rows % 8 == 0
        s = src + (long)(k0 + krow) * ld + gr;
      }
      __builtin_amdgcn_global_load_lds((gptr_f)s, (lptr_f)(lds + j * 1024), 16, 0, 0);
    }
  }
};

template <bool KC, int R>
FM_DEVICE bf16x8_t pl_frag(const char* lds, int base, int lane) {
  if constexpr (KC) {
    return *reinterpret_cast<const bf16x8_t*>(lds + pk_off(base + (lane & 15), lane >> 4));
  } else {
    return frag<false, R>(lds, base, 0, lane);
  }
}

template <int N>
FM_DEVICE void wait_vm() {
  wait_vmcnt_f<N>();
}

template <int BM, int BN, int NS, bool AK, bool BKC, bool SGD>
__global__ void __launch_bounds__((BM / 64) * (BN / 64) * 64, 1) fm_gemm_pl3_kernel(GemmF p) {
  constexpr int WM = BM / 64, WN = BN / 64, NW = WM * WN, NTH = NW * 64;
  constexpr int MR = 4, NR = 4;
  constexpr int PA = BM * PKS * 2, PB = BN * PKS * 2;   // bytes of one plane image
  constexpr int STG = 3 * (PA + PB);
  constexpr int LPT = 3 * (PlIssue<AK, BM, NW>::PER_W + PlIssue<BKC, BN, NW>::PER_W);   // loads / wave / stage
  static_assert((NS - 2) * LPT < 64, "vmcnt range");
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
  const int split = blockIdx.z;
  const int m0 = tm * BM, n0 = tn * BN;
  const int ktiles = p.K / PKS;
  const int kt_per = (ktiles + p.ksplit - 1) / p.ksplit;
  const int kt0 = split * kt_per, kt1 = min(ktiles, kt0 + kt_per);
  const int nst = max(kt1 - kt0, 0);

  auto issue = [&](int t, int slot) {
    char* b = smem + slot * STG;
    const int k0 = (kt0 + t) * PKS;
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
      PlIssue<AK, BM, NW>::run(p.Ap + pl * p.psa, p.lda, m0, p.M, k0, b + pl * PA, wave, lane);
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
      PlIssue<BKC, BN, NW>::run(p.Bp + pl * p.psb, p.ldb, n0, p.N, k0, b + 3 * PA + pl * PB, wave, lane);
  };

  f32x4_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // bias gradient of dW GEMMs: row sums of the MN-contiguous A (h + m + l = x exactly), tn == 0 only
  const bool dorow = (!AK) && p.rowsum_a != nullptr && tn == 0;
  constexpr int RCH = BM / 8;                          // 16-B column chunks of an A k-row
  float rs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

  constexpr int TA[6] = {2, 1, 0, 1, 0, 0};            // small terms first, the dominant h*h last
  constexpr int TB[6] = {0, 1, 2, 0, 1, 0};

  if (p.pvar == 1 && __builtin_amdgcn_readfirstlane(tid) >= NTH / 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nst) issue(s, s);
  for (int t = 0; t < nst; ++t) {
    if (t + NS - 2 < nst) wait_vm<(NS - 2) * LPT>();
    else wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + NS - 1 < nst) issue(t + NS - 1, (t + NS - 1) % NS);
    const char* la = smem + (t % NS) * STG;
    const char* lb = la + 3 * PA;
    if constexpr (!AK) {
      if (dorow) {
        for (int kr = tid / RCH; kr < PKS; kr += NTH / RCH) {
#pragma unroll
          for (int pl = 0; pl < 3; ++pl) {
            const bf16x8_t v = *reinterpret_cast<const bf16x8_t*>(la + pl * PA + lds_off<false, BM>(kr, tid % RCH));
#pragma unroll
            for (int e = 0; e < 8; ++e) rs[e] += bf2f((unsigned short)v[e]);
          }
        }
      }
    }
    bf16x8_t bf[3][NR];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
      for (int j = 0; j < NR; ++j) bf[pl][j] = pl_frag<BKC, BN>(lb + pl * PB, wn * 64 + 16 * j, lane);
    if (p.pvar == 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < MR; ++i) {
      bf16x8_t af[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) af[pl] = pl_frag<AK, BM>(la + pl * PA, wm * 64 + 16 * i, lane);
#pragma unroll
      for (int s = 0; s < 6; ++s)
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8v_t*>(&bf[TB[s]][j]),
                                                              *reinterpret_cast<const bf16x8v_t*>(&af[TA[s]]), acc[i][j],
                                                              0, 0, 0);
    }
    if (p.pvar == 2) __builtin_amdgcn_s_setprio(0);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();           // every wave is done with the operand LDS (nothing in flight)
  if constexpr (!AK) {
    if (dorow) {   // the threads sharing each 8-column chunk: reduce through LDS, one atomic per row
      float* red = reinterpret_cast<float*>(smem);
      constexpr int G = NTH / RCH;
#pragma unroll
      for (int e = 0; e < 8; ++e) red[(tid / RCH) * BM + (tid % RCH) * 8 + e] = rs[e];
      __syncthreads();
      for (int r = tid; r < BM; r += NTH) {
        float x = 0.f;
        for (int g = 0; g < G; ++g) x += red[g * BM + r];
        if (m0 + r < p.M) atomicAdd(p.rowsum_a + m0 + r, x);
      }
    }
  }
  epilogue_f32<MR, NR, false, false, SGD>(p, acc, 0, split, m0 + wm * 64, n0 + wn * 64, lane);
}

template <int BM, int BN, int NS, bool SGD>
void launch_pl3(const GemmF& p, bool ak, bool bk, hipStream_t s) {
  constexpr int NTH = (BM / 64) * (BN / 64) * 64;
  constexpr int LDS = NS * 3 * (BM + BN) * PKS * 2;
  dim3 grid(p.tiles_m * p.tiles_n, 1, p.ksplit);
#define FM_PL3(AKv, BKv)                                                                                            \
  do {                                                                                                              \
    static bool attr = false;                                                                                       \
    if (!attr) {                                                                                                    \
      (void)hipFuncSetAttribute((const void*)fm_gemm_pl3_kernel<BM, BN, NS, AKv, BKv, SGD>,                         \
                                hipFuncAttributeMaxDynamicSharedMemorySize, LDS);                                   \
      attr = true;                                                                                                  \
    }                                                                                                               \
    hipLaunchKernelGGL((fm_gemm_pl3_kernel<BM, BN, NS, AKv, BKv, SGD>), grid, dim3(NTH), LDS, s, p);                \
  } while (0)
  if (ak && bk) FM_PL3(true, true);
  else if (ak) FM_PL3(true, false);
  else if (bk) FM_PL3(false, true);
  else FM_PL3(false, false);
#undef FM_PL3
}

// fp32 [rows][ld] -> three bf16 planes [3][rows][ldd] (plane stride ps), 4 values per thread
__global__ void __launch_bounds__(256) fm_split3_kernel(const float* __restrict__ src, long rows, int cols, long lds,
                                                        unsigned short* __restrict__ dst, long ldd, long ps) {
  const int c4 = (cols + 3) / 4;
  const long total = rows * c4;
  const bool vec = (cols & 3) == 0 && (lds & 3) == 0 && (ldd & 3) == 0 && (((uintptr_t)src) & 15) == 0 &&
                   (((uintptr_t)dst) & 7) == 0 && (ps & 3) == 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / c4;
    const int c = (int)(i % c4) * 4;
    const float* s = src + r * lds + c;
    const long o = r * ldd + c;
    if (vec) {
      const f32x4_t v = *reinterpret_cast<const f32x4_t*>(s);
      const float fv[4] = {v[0], v[1], v[2], v[3]};
      store_planes4(dst, ps, o, fv);
    } else {
      for (int e = 0; e < 4 && c + e < cols; ++e) store_planes1(dst, ps, o + e, s[e]);
    }
  }
}

}  // namespace

// Launch the plane kernel on a prepared parameter block (Ap / Bp / psa / psb, tiles and ksplit for
// the bm x 128 tile).  Caller guarantees: batch 1, K % 32 == 0 (whole stages per split), 16-B aligned
// planes with ld % 8 == 0 and ps % 8 == 0, MN-contiguous operands with rows % 8 == 0, M, N >= 64.
// sgd: the fused-SGD epilogue (unsplit tiles only).  Returns -1 for an unsupported configuration.
extern "C" int fm_gemm_pl3_launch(const void* params, int bm, int a_kcontig, int b_kcontig, int sgd, hipStream_t s) {
  const GemmF& p = *static_cast<const GemmF*>(params);
  if (sgd && p.ksplit > 1) return -1;
  if (bm == 256) {
    if (sgd) launch_pl3<256, 128, 2, true>(p, a_kcontig, b_kcontig, s);
    else launch_pl3<256, 128, 2, false>(p, a_kcontig, b_kcontig, s);
  } else if (bm == 128) {
    if (sgd) launch_pl3<128, 128, 3, true>(p, a_kcontig, b_kcontig, s);
    else launch_pl3<128, 128, 3, false>(p, a_kcontig, b_kcontig, s);
  } else {
    return -1;
  }
  return 0;
}

// planes of an fp32 matrix: dst[p][r][c] (plane stride ps elements) for the exact split x = h + m + l
extern "C" void fm_split3(const float* src, long rows, int cols, long lds, unsigned short* dst, long ldd, long ps,
                          hipStream_t s) {
  if (rows <= 0 || cols <= 0) return;
  hipLaunchKernelGGL(fm_split3_kernel, dim3(fm_grid(rows * ((cols + 3) / 4))), dim3(256), 0, s, src, rows, cols, lds, dst,
                     ldd, ps);
}
