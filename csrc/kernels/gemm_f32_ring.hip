// flexmi fp32 GEMM, ring form, for gfx950 (MI355X / CDNA4): see the comment block below.  Shares the
// parameter block and the fused epilogues with gemm_f32.hip (gemm_f32_common.h); gemm_f32.hip's
// dispatcher (gemm_f32_run) selects it through fm_gemm_f32_ring_cfg / fm_gemm_f32_ring_launch.
#include "gemm_f32_common.h"

#include <algorithm>

namespace {

// ---- ring kernel: NS-stage LDS-DMA ring, one barrier per K-stage, fragment double buffer -------
// The register-staged kernels above keep one K-tile in flight and pay a full barrier + first-
// fragment latency per 32-deep tile; at one or two waves per SIMD that is the ~15 % they lose to a
// saturated f32 MFMA pipe.  Here (src/ops/linear.cu:424-447 fwd, :592-635 bwd):
//   * operands go global -> LDS by global_load_lds_dwordx4 into an NS-deep ring (no staging VGPRs,
//     no ds_write pass); NS-1 K-stages are in flight behind the one being multiplied;
//   * ONE s_barrier per K-stage, placed after the stage's second-to-last fragment chunk has been
//     multiplied: by then the last chunk's fragments are in registers, so the barrier and the next
//     stage's first fragment reads overlap the last chunk's MFMAs (no pipe bubble per stage);
//   * the ring slot freed by that barrier is refilled at the top of the next stage.
// LDS images: K-contiguous operand [row][BK] with XOR-swizzled 16-B chunks (conflict-free b128
// fragment reads: one read = 4 k-steps of one 16x16 tile); MN-contiguous operand [k][R] with the
// wave's rows interleaved over its T tiles (one b128 / b64 read at a fixed k = T fragments).  The
// DMA destination is lane-linear, so every swizzle is applied to the per-lane SOURCE address.
// Requires K % BK == 0 (whole stages per split), 16-B aligned operands, M % 4 / N % 4 == 0 for
// MN-contiguous operands; rows past the M / N edge are clamped re-reads whose outputs are never
// stored.
template <int BK>
FM_DEVICE int rk_swz(int row) {   // K-contiguous image: chunk swizzle of a row (CPR = BK/4 chunks)
  constexpr int CPR = BK / 4;
  constexpr int RPL = (256 / (BK * 4)) > 0 ? 256 / (BK * 4) : 1;
  return (row / RPL) & (CPR - 1);
}
template <int T>
FM_DEVICE int rm_swz(int k) {     // MN-contiguous image: T = 2 (b64 reads) separates k-groups g, g+1
  return T == 2 ? (((k >> 2) & 1) << 3) : 0;
}

template <bool KC, int R, int BK, int T, int NTH>
struct RingLd {
  static constexpr int INSTR = R * BK * 4 / 1024;
  static constexpr int NWAVES = NTH / 64;
  static constexpr int PER_W = INSTR / NWAVES;
  static_assert(INSTR % NWAVES == 0 && PER_W >= 1, "stage bytes must split evenly over the waves");
  FM_DEVICE static void issue(const float* __restrict__ p, long ld, int row0, int rows, int k0, char* lds, int wave,
                              int lane) {
#pragma unroll
    for (int i = 0; i < PER_W; ++i) {
      const int j = wave * PER_W + i;
      const int o = j * 1024 + 16 * lane;
      const float* src;
      if constexpr (KC) {
        const int row = o / (BK * 4);
        const int c = (o % (BK * 4)) / 16;
        const int gr = min(row0 + row, rows - 1);
        src = p + (long)gr * ld + k0 + 4 * (c ^ rk_swz<BK>(row));
      } else {
        const int k = o / (R * 4);
        const int c = (o % (R * 4)) / 16;
        const int gr = min(row0 + 4 * (c ^ rm_swz<T>(k)), rows - 4);
        src = p + (long)(k0 + k) * ld + gr;
      }
      __builtin_amdgcn_global_load_lds((gptr_f)src, (lptr_f)(lds + j * 1024), 16, 0, 0);
    }
  }
};

// fragments of one operand for one 16-wide k-chunk kk: f[t][s] = element (tile t, k-step s)
template <bool KC, int R, int BK, int T>
FM_DEVICE void ring_frags(const char* lds, int base, int kk, int lane, float (&f)[T][4]) {
  const int q = lane & 15, g = lane >> 4;
  if constexpr (KC) {
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int row = base + 16 * t + q;
      const f32x4_t x = *reinterpret_cast<const f32x4_t*>(lds + row * (BK * 4) + 16 * ((4 * kk + g) ^ rk_swz<BK>(row)));
#pragma unroll
      for (int s = 0; s < 4; ++s) f[t][s] = x[s];
    }
  } else {
    static_assert(T == 2 || T == 4, "interleaved MN reads are b64 / b128");
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int k = 16 * kk + 4 * g + s;
      const int e = base + T * q;                       // first float of the lane's T rows
      const int off = k * (R * 4) + 16 * ((e >> 2) ^ rm_swz<T>(k)) + 4 * (e & 3);
      const fvec<T> x = *reinterpret_cast<const fvec<T>*>(lds + off);
#pragma unroll
      for (int t = 0; t < T; ++t) f[t][s] = x[t];
    }
  }
}

template <int N>
FM_DEVICE void ring_wait(int n_out) {   // s_waitcnt vmcnt(n_out * N) for n_out in {0, 1, 2}
  if (n_out >= 2) wait_vmcnt_f<(2 * N < 63 ? 2 * N : 63)>();
  else if (n_out == 1) wait_vmcnt_f<N>();
  else wait_vmcnt_f<0>();
}

template <int BM, int BN, int WM, int WN, int BK, int NS, bool AK, bool BKC, bool SGD = false>
__global__ void __launch_bounds__(WM * WN * 64, 1) fm_gemm_f32_ring_kernel(GemmF p) {
  constexpr int NTH = WM * WN * 64;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MR = TM / 16, NR = TN / 16;
  constexpr int CH = BK / 16;
  constexpr int A_BYTES = BM * BK * 4;
  constexpr int B_BYTES = BN * BK * 4;
  constexpr int STG = A_BYTES + B_BYTES;
  using LA = RingLd<AK, BM, BK, MR, NTH>;
  using LB = RingLd<BKC, BN, BK, NR, NTH>;
  constexpr int LPS = LA::PER_W + LB::PER_W;   // DMA instructions per wave per stage
  static_assert(NS >= 2 && NS <= 4 && 2 * LPS < 64, "ring depth / vmcnt range");
  static_assert(CH >= 2 && CH % 2 == 0, "fragment double buffer needs an even chunk count");
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

  const int ktiles_total = p.K / BK;
  const int kt_per = (ktiles_total + p.ksplit - 1) / p.ksplit;
  const int kt0 = split * kt_per;
  const int nkt = max(min(ktiles_total, kt0 + kt_per) - kt0, 0);

  auto issue = [&](int t) {
    char* base = smem + (t % NS) * STG;
    LA::issue(A, p.lda, m0, p.M, (kt0 + t) * BK, base, wave, lane);
    LB::issue(B, p.ldb, n0, p.N, (kt0 + t) * BK, base + A_BYTES, wave, lane);
  };

  f32x4_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const bool rowsum = (!AK) && (p.rowsum_a != nullptr) && (tn == 0);
  constexpr int CPR = BM / 4;
  float rs[4] = {0.f, 0.f, 0.f, 0.f};

  float af[2][MR][4], bfr[2][NR][4];
  if (nkt > 0) {
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
      if (s < nkt) issue(s);
    ring_wait<LPS>(min(NS - 2, nkt - 1));
    __builtin_amdgcn_s_barrier();
    ring_frags<AK, BM, BK, MR>(smem, wm * TM, 0, lane, af[0]);
    ring_frags<BKC, BN, BK, NR>(smem + A_BYTES, wn * TN, 0, lane, bfr[0]);
  }
  for (int t = 0; t < nkt; ++t) {
    const char* la = smem + (t % NS) * STG;
    const char* lb = la + A_BYTES;
    if (t + NS - 1 < nkt) issue(t + NS - 1);   // refills the slot every wave left at the last barrier
    if constexpr (!AK) {
      if (rowsum) {
        for (int kr = tid / CPR; kr < BK; kr += NTH / CPR) {
          const int e = 4 * (tid % CPR);
          const f32x4_t v = *reinterpret_cast<const f32x4_t*>(la + kr * (BM * 4) + 16 * ((e >> 2) ^ rm_swz<MR>(kr)));
#pragma unroll
          for (int x = 0; x < 4; ++x) rs[x] += v[x];
        }
      }
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int cur = c & 1, nxt = cur ^ 1;
      if (c + 1 < CH) {
        ring_frags<AK, BM, BK, MR>(la, wm * TM, c + 1, lane, af[nxt]);
        ring_frags<BKC, BN, BK, NR>(lb, wn * TN, c + 1, lane, bfr[nxt]);
      } else if (t + 1 < nkt) {
        // stage t+1: this wave's DMAs landed (later stages may stay in flight), every wave's
        // fragment reads of stage t are done, then all waves' DMAs of t+1 are visible
        ring_wait<LPS>(min(NS - 2, nkt - 2 - t));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        const char* na = smem + ((t + 1) % NS) * STG;
        ring_frags<AK, BM, BK, MR>(na, wm * TM, 0, lane, af[nxt]);
        ring_frags<BKC, BN, BK, NR>(na + A_BYTES, wn * TN, 0, lane, bfr[nxt]);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < MR; ++i)
#pragma unroll
          for (int j = 0; j < NR; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(bfr[cur][j][s], af[cur][i][s], acc[i][j], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();   // every wave is done with the ring before the epilogue reuses LDS
  if constexpr (!AK) {
    if (rowsum) {
      float* red = reinterpret_cast<float*>(smem);
      constexpr int G = NTH / CPR;
#pragma unroll
      for (int e = 0; e < 4; ++e) red[(tid / CPR) * BM + (tid % CPR) * 4 + e] = rs[e];
      __syncthreads();
      for (int r = tid; r < BM; r += NTH) {
        float x = 0.f;
        for (int g2 = 0; g2 < G; ++g2) x += red[g2 * BM + r];
        if (m0 + r < p.M) atomicAdd(p.rowsum_a + m0 + r, x);
      }
      __syncthreads();
    }
  }
  if constexpr (SGD && BM * BN * 4 <= NS * STG) {
    if (p.ksplit == 1 && p.ulds) {
      sgd_epilogue_lds_f32<BM, BN, NTH, MR, NR, !AK, !BKC, NS * STG>(p, acc, smem, m0, n0, m0 + wm * TM, n0 + wn * TN,
                                                                      lane, tid);
      return;
    }
  }
  epilogue_f32<MR, NR, !AK, !BKC, SGD>(p, acc, zb, split, m0 + wm * TM, n0 + wn * TN, lane);
}

template <int BM, int BN, int WM, int WN, int BK, int NS, bool SGD>
void launch_ring(const GemmF& p, bool ak, bool bk, hipStream_t s) {
  constexpr int NTH = WM * WN * 64;
  constexpr int LDS = NS * (BM + BN) * BK * 4;
  static bool attr_set = false;
  if (!attr_set) {
    auto set = [](const void* f) { (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS); };
    set((const void*)fm_gemm_f32_ring_kernel<BM, BN, WM, WN, BK, NS, true, true, SGD>);
    set((const void*)fm_gemm_f32_ring_kernel<BM, BN, WM, WN, BK, NS, true, false, SGD>);
    set((const void*)fm_gemm_f32_ring_kernel<BM, BN, WM, WN, BK, NS, false, true, SGD>);
    set((const void*)fm_gemm_f32_ring_kernel<BM, BN, WM, WN, BK, NS, false, false, SGD>);
    attr_set = true;
  }
  dim3 grid(p.tiles_m * p.tiles_n, p.batch, p.ksplit);
  if (ak && bk) hipLaunchKernelGGL((fm_gemm_f32_ring_kernel<BM, BN, WM, WN, BK, NS, true, true, SGD>), grid, dim3(NTH), LDS, s, p);
  else if (ak) hipLaunchKernelGGL((fm_gemm_f32_ring_kernel<BM, BN, WM, WN, BK, NS, true, false, SGD>), grid, dim3(NTH), LDS, s, p);
  else if (bk) hipLaunchKernelGGL((fm_gemm_f32_ring_kernel<BM, BN, WM, WN, BK, NS, false, true, SGD>), grid, dim3(NTH), LDS, s, p);
  else hipLaunchKernelGGL((fm_gemm_f32_ring_kernel<BM, BN, WM, WN, BK, NS, false, false, SGD>), grid, dim3(NTH), LDS, s, p);
}

// ---- persistent ring kernel ------------------------------------------------------------------
// One block per CU slot loops over work units (tile, K-split) u = blockIdx.x + j * gridDim.x,
// and the K-stage sequence runs ACROSS units: the prefetch (LDS-DMA ring, or register-staged
// loads) of the next unit's first stages is in flight while this unit's last stage multiplies,
// and its fragments are in registers before this unit's epilogue issues its stores -- so the
// per-tile prologue (first loads) and epilogue (C stores) overlap MFMA work instead of bracketing
// every tile of a one-tile-per-CU launch (measured on the fp32 MFMA probe, tools/mfma_probe.hip:
// ~8-10 % of a 1024-wide DLRM GEMM).  Units of one block share an XCD (u % 8 fixed), and
// xcd_remap_f hands each XCD contiguous tiles (shared A / B panels in its L2).
//   MODE 1: LDS-DMA NS-stage ring (as the ring kernel);
//   MODE 2: register-staged -- the stage after next is loaded into VGPRs (global_load_dwordx4)
//           during this stage and written to the free LDS slot (ds_write_b128, swizzled) right
//           before the stage's barrier: two LDS slots, no M0 / DMA issue cost.
// Epilogues: the direct forms of epilogue_f32 (bias / act / act-bwd + column sums / beta / split-K
// slabs / fused SGD, all from registers); no LDS epilogue (the ring is live across units).  The
// dW GEMMs' folded bias gradient (row sums of the MN-contiguous A tiles, tn == 0 units) is summed
// from the staged A image per stage, reduced across the lanes of a wave that share rows and
// added with one float atomic per (row, wave) at the end of the unit.
template <bool KC, int R, int BK, int NTH>
struct RegLd {
  static constexpr int CH = R * BK / 4;          // 16-B chunks of the operand tile
  static constexpr int PER_T = CH / NTH;
  static_assert(PER_T >= 1 && CH % NTH == 0, "stage chunks must split evenly over the threads");
  f32x4_t v[PER_T];
  template <int T>
  FM_DEVICE void load(const float* __restrict__ p, long ld, int row0, int rows, int k0, int tid) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int ci = tid + NTH * i;
      const float* src;
      if constexpr (KC) {
        const int row = ci / (BK / 4), kc = ci % (BK / 4);
        src = p + (long)min(row0 + row, rows - 1) * ld + k0 + 4 * kc;
      } else {
        const int k = ci / (R / 4), c = ci % (R / 4);
        src = p + (long)(k0 + k) * ld + min(row0 + 4 * c, rows - 4);
      }
      v[i] = *reinterpret_cast<const f32x4_t*>(src);
    }
  }
  template <int T>
  FM_DEVICE void store(char* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int ci = tid + NTH * i;
      int off;
      if constexpr (KC) {
        const int row = ci / (BK / 4), kc = ci % (BK / 4);
        off = row * (BK * 4) + 16 * (kc ^ rk_swz<BK>(row));
      } else {
        const int k = ci / (R / 4), c = ci % (R / 4);
        off = k * (R * 4) + 16 * (c ^ rm_swz<T>(k));
      }
      *reinterpret_cast<f32x4_t*>(lds + off) = v[i];
    }
  }
};

template <int BM, int BN, int WM, int WN, int BK, int NS, int MODE, bool AK, bool BKC, bool SGD>
__global__ void __launch_bounds__(WM * WN * 64, 1) fm_gemm_f32_pring_kernel(GemmF p, int units, int nkt) {
  constexpr int NTH = WM * WN * 64;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MR = TM / 16, NR = TN / 16;
  constexpr int CH = BK / 16;
  constexpr int A_BYTES = BM * BK * 4;
  constexpr int B_BYTES = BN * BK * 4;
  constexpr int STG = A_BYTES + B_BYTES;
  constexpr int SLOTS = MODE == 1 ? NS : 2;
  using LA = RingLd<AK, BM, BK, MR, NTH>;
  using LB = RingLd<BKC, BN, BK, NR, NTH>;
  constexpr int LPS = LA::PER_W + LB::PER_W;
  static_assert(MODE == 1 || MODE == 2, "mode");
  static_assert(MODE == 2 || (NS >= 2 && NS <= 4 && 2 * LPS < 64), "ring depth / vmcnt range");
  static_assert(CH >= 2 && CH % 2 == 0, "fragment double buffer needs an even chunk count");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles = p.tiles_m * p.tiles_n;
  const int nmy = units > (int)blockIdx.x ? (units - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x : 0;
  const int S = nmy * nkt;                          // this block's K-stages over all its units

  // unit j of this block -> (m0, n0, first k-tile)
  auto unit_geo = [&](int j, int& m0, int& n0, int& kt0, int& split) {
    const int u = (int)blockIdx.x + j * (int)gridDim.x;
    const int r = xcd_remap_f(u, units);
    split = r / tiles;
    const int tl = r % tiles;
    int tm, tn;
    if (p.n_fast) { tn = tl % p.tiles_n; tm = tl / p.tiles_n; }
    else { tm = tl % p.tiles_m; tn = tl / p.tiles_m; }
    m0 = tm * BM;
    n0 = tn * BN;
    kt0 = split * nkt;
  };

  RegLd<AK, BM, BK, NTH> ra;
  RegLd<BKC, BN, BK, NTH> rb;
  auto issue = [&](int g) {                         // MODE 1: DMA stage g into its ring slot
    int m0, n0, kt0, sp;
    unit_geo(g / nkt, m0, n0, kt0, sp);
    char* base = smem + (g % SLOTS) * STG;
    const int k0 = (kt0 + g % nkt) * BK;
    LA::issue(p.A, p.lda, m0, p.M, k0, base, wave, lane);
    LB::issue(p.B, p.ldb, n0, p.N, k0, base + A_BYTES, wave, lane);
  };
  auto reg_load = [&](int g) {                      // MODE 2: stage g into registers
    int m0, n0, kt0, sp;
    unit_geo(g / nkt, m0, n0, kt0, sp);
    const int k0 = (kt0 + g % nkt) * BK;
    ra.template load<MR>(p.A, p.lda, m0, p.M, k0, tid);
    rb.template load<NR>(p.B, p.ldb, n0, p.N, k0, tid);
  };
  auto reg_store = [&](int g) {
    char* base = smem + (g % SLOTS) * STG;
    ra.template store<MR>(base, tid);
    rb.template store<NR>(base + A_BYTES, tid);
  };

  f32x4_t acc[MR][NR];
  float af[2][MR][4], bfr[2][NR][4];
  constexpr int CPR = BM / 4;                       // 16-B chunks per k-row of an MN-contiguous A image
  float rs[4] = {0.f, 0.f, 0.f, 0.f};
  bool rowsum = false;
  if (S > 0) {
    if constexpr (MODE == 1) {
#pragma unroll
      for (int s = 0; s < NS - 1; ++s)
        if (s < S) issue(s);
      ring_wait<LPS>(min(NS - 2, S - 1));
    } else {
      reg_load(0);
      reg_store(0);
      if (S > 1) reg_load(1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    ring_frags<AK, BM, BK, MR>(smem, wm * TM, 0, lane, af[0]);
    ring_frags<BKC, BN, BK, NR>(smem + A_BYTES, wn * TN, 0, lane, bfr[0]);
  }
  int m0 = 0, n0 = 0, kt0 = 0, split = 0;
  for (int g = 0; g < S; ++g) {
    const int t = g % nkt;
    if (t == 0) {
      unit_geo(g / nkt, m0, n0, kt0, split);
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      rowsum = (!AK) && p.rowsum_a != nullptr && n0 == 0;
    }
    const char* la = smem + (g % SLOTS) * STG;
    const char* lb = la + A_BYTES;
    if constexpr (MODE == 1) {
      if (g + NS - 1 < S) issue(g + NS - 1);
    }
    if constexpr (!AK) {
      if (rowsum) {   // this stage's k-rows of the A image, 4 rows (one 16-B chunk) per thread
        for (int kr = tid / CPR; kr < BK; kr += NTH / CPR) {
          const int cc = tid % CPR;
          const f32x4_t v = *reinterpret_cast<const f32x4_t*>(la + kr * (BM * 4) + 16 * (cc ^ rm_swz<MR>(kr)));
#pragma unroll
          for (int x = 0; x < 4; ++x) rs[x] += v[x];
        }
      }
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int cur = c & 1, nxt = cur ^ 1;
      if (c + 1 < CH) {
        ring_frags<AK, BM, BK, MR>(la, wm * TM, c + 1, lane, af[nxt]);
        ring_frags<BKC, BN, BK, NR>(lb, wn * TN, c + 1, lane, bfr[nxt]);
      } else if (g + 1 < S) {
        if constexpr (MODE == 1) {
          ring_wait<LPS>(min(NS - 2, S - 2 - g));
        } else {
          // stage g+1 (in registers since stage g-1) -> the slot stage g-1 used; then the
          // stage after next into registers
          reg_store(g + 1);
          if (g + 2 < S) reg_load(g + 2);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        const char* na = smem + ((g + 1) % SLOTS) * STG;
        ring_frags<AK, BM, BK, MR>(na, wm * TM, 0, lane, af[nxt]);
        ring_frags<BKC, BN, BK, NR>(na + A_BYTES, wn * TN, 0, lane, bfr[nxt]);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < MR; ++i)
#pragma unroll
          for (int j = 0; j < NR; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(bfr[cur][j][s], af[cur][i][s], acc[i][j], 0, 0, 0);
    }
    if (t == nkt - 1) {
      if constexpr (!AK) {
        if (rowsum) {   // lanes l, l + CPR, ... of a wave hold the same 4 rows
#pragma unroll
          for (int x = 0; x < 4; ++x) {
            float v = rs[x];
#pragma unroll
            for (int o = CPR; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
            rs[x] = v;
          }
          const int r = m0 + 4 * (tid % CPR);
          if (lane < CPR || CPR >= 64) {
#pragma unroll
            for (int x = 0; x < 4; ++x)
              if (r + x < p.M) atomicAdd(p.rowsum_a + r + x, rs[x]);
          }
#pragma unroll
          for (int x = 0; x < 4; ++x) rs[x] = 0.f;
        }
      }
      epilogue_f32<MR, NR, !AK, !BKC, SGD>(p, acc, 0, split, m0 + wm * TM, n0 + wn * TN, lane);
    }
  }
  if constexpr (MODE == 1) wait_vmcnt_f<0>();
}

template <int BM, int BN, int WM, int WN, int BK, int NS, int MODE, bool SGD>
void launch_pring(const GemmF& p, bool ak, bool bk, hipStream_t s) {
  constexpr int NTH = WM * WN * 64;
  constexpr int LDS = (MODE == 1 ? NS : 2) * (BM + BN) * BK * 4;
  static bool attr_set = false;
  if (!attr_set) {
    auto set = [](const void* f) { (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS); };
    set((const void*)fm_gemm_f32_pring_kernel<BM, BN, WM, WN, BK, NS, MODE, true, true, SGD>);
    set((const void*)fm_gemm_f32_pring_kernel<BM, BN, WM, WN, BK, NS, MODE, true, false, SGD>);
    set((const void*)fm_gemm_f32_pring_kernel<BM, BN, WM, WN, BK, NS, MODE, false, true, SGD>);
    set((const void*)fm_gemm_f32_pring_kernel<BM, BN, WM, WN, BK, NS, MODE, false, false, SGD>);
    attr_set = true;
  }
  const int units = p.tiles_m * p.tiles_n * p.ksplit;
  const int nkt = p.K / BK / p.ksplit;
  // persistent grid = the blocks that are RESIDENT at once (occupancy API: VGPRs, LDS, waves);
  // a statically assigned unit list on a block that only starts after another retired would
  // serialise the launch
  static int resident = 0;
  if (resident == 0) {
    int dev = 0, cus = 0, occ = 1 << 20;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const void* ks[4] = {(const void*)fm_gemm_f32_pring_kernel<BM, BN, WM, WN, BK, NS, MODE, true, true, SGD>,
                         (const void*)fm_gemm_f32_pring_kernel<BM, BN, WM, WN, BK, NS, MODE, true, false, SGD>,
                         (const void*)fm_gemm_f32_pring_kernel<BM, BN, WM, WN, BK, NS, MODE, false, true, SGD>,
                         (const void*)fm_gemm_f32_pring_kernel<BM, BN, WM, WN, BK, NS, MODE, false, false, SGD>};
    for (const void* k : ks) {   // the lowest occupancy of the four operand orientations
      int o = 0;
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, k, NTH, LDS);
      occ = std::min(occ, std::max(1, o));
    }
    resident = std::max(1, cus) * occ;
  }
  const int grid = std::max(1, std::min(units, resident));
  if (ak && bk) hipLaunchKernelGGL((fm_gemm_f32_pring_kernel<BM, BN, WM, WN, BK, NS, MODE, true, true, SGD>), dim3(grid), dim3(NTH), LDS, s, p, units, nkt);
  else if (ak) hipLaunchKernelGGL((fm_gemm_f32_pring_kernel<BM, BN, WM, WN, BK, NS, MODE, true, false, SGD>), dim3(grid), dim3(NTH), LDS, s, p, units, nkt);
  else if (bk) hipLaunchKernelGGL((fm_gemm_f32_pring_kernel<BM, BN, WM, WN, BK, NS, MODE, false, true, SGD>), dim3(grid), dim3(NTH), LDS, s, p, units, nkt);
  else hipLaunchKernelGGL((fm_gemm_f32_pring_kernel<BM, BN, WM, WN, BK, NS, MODE, false, false, SGD>), dim3(grid), dim3(NTH), LDS, s, p, units, nkt);
}

// ring tile configurations (A/B index = FM_GEMM_F32_VARIANT - 20000); mode 0 = one tile per
// block (ring kernel), 1 = persistent LDS-DMA ring, 2 = persistent register-staged
struct RCfg { int bm, bn, wm, wn, bk, ns, mode; };
constexpr RCfg kRCfgs[] = {
    {128, 128, 2, 4, 32, 4, 0},   // 0: 8 waves of 64x32 (2 per SIMD), 4 x 32 KB ring
    {128, 128, 2, 4, 32, 4, 1},   // 1: persistent, same tile and ring
    {128, 128, 2, 4, 32, 2, 2},   // 2: persistent, register-staged, 64 KB (2 blocks / CU)
    {256, 128, 4, 2, 32, 2, 2},   // 3: persistent, register-staged, 8 waves of 64x64, 96 KB
    {256, 128, 4, 2, 32, 3, 1},   // 4: persistent, 3 x 48 KB ring, 8 waves of 64x64
    {128, 64, 2, 2, 32, 2, 2},    // 5: persistent, register-staged, 4 waves of 64x32, 48 KB (3 blocks / CU)
    {64, 64, 2, 2, 64, 2, 2},     // 6: persistent, register-staged, 4 waves of 32x32, BK 64 (hipBLASLt's tile)
    {64, 64, 2, 2, 64, 4, 1},     // 7: persistent, 4 x 32 KB ring, 4 waves of 32x32
};
constexpr int kNumRCfgs = sizeof(kRCfgs) / sizeof(kRCfgs[0]);

template <bool SGD>
void launch_ring_cfg(int c, const GemmF& p, bool ak, bool bk, hipStream_t s) {
  switch (c) {
    case 0: launch_ring<128, 128, 2, 4, 32, 4, SGD>(p, ak, bk, s); break;
    case 1: launch_pring<128, 128, 2, 4, 32, 4, 1, SGD>(p, ak, bk, s); break;
    case 2: launch_pring<128, 128, 2, 4, 32, 2, 2, SGD>(p, ak, bk, s); break;
    case 3: launch_pring<256, 128, 4, 2, 32, 2, 2, SGD>(p, ak, bk, s); break;
    case 4: launch_pring<256, 128, 4, 2, 32, 3, 1, SGD>(p, ak, bk, s); break;
    case 5: launch_pring<128, 64, 2, 2, 32, 2, 2, SGD>(p, ak, bk, s); break;
    case 6: launch_pring<64, 64, 2, 2, 64, 2, 2, SGD>(p, ak, bk, s); break;
    default: launch_pring<64, 64, 2, 2, 64, 4, 1, SGD>(p, ak, bk, s); break;
  }
}

}  // namespace

// tile geometry of ring configuration c: {bm, bn, bk, ns, mode}; returns the number of configurations
extern "C" int fm_gemm_f32_ring_cfg(int c, int* geo) {
  if (c >= 0 && c < kNumRCfgs && geo) {
    geo[0] = kRCfgs[c].bm; geo[1] = kRCfgs[c].bn; geo[2] = kRCfgs[c].bk; geo[3] = kRCfgs[c].ns;
    geo[4] = kRCfgs[c].mode;
  }
  return kNumRCfgs;
}

// launch ring configuration c for a prepared GemmF (tiles_m / tiles_n / ksplit filled in for it)
extern "C" void fm_gemm_f32_ring_launch(const void* params, int c, int a_kcontig, int b_kcontig, int sgd,
                                        hipStream_t stream) {
  const GemmF& p = *reinterpret_cast<const GemmF*>(params);
  if (sgd) launch_ring_cfg<true>(c, p, a_kcontig, b_kcontig, stream);
  else launch_ring_cfg<false>(c, p, a_kcontig, b_kcontig, stream);
}
