// flexmi MFMA GEMM, LDS-DMA pipelined variant for gfx950 (MI355X): the hot path for every GEMM
// whose K-tiles are whole (K % 64 == 0) and whose operands allow 16-B vector access.
//
// Why a second kernel: the register-staged kernel (gemm.hip) keeps one K-tile in flight and
// measured 19 % MFMA-busy at the DLRM shapes (rocprofv3 PMC, profiles/): every K-step waited a
// full HBM round trip.  Here operands go global -> LDS directly with global_load_lds_dwordx4
// (no staging VGPRs, no ds_write pass) into a 3-stage LDS ring, so two K-tiles are in flight
// behind the one being multiplied:
//
//   iteration t:  s_waitcnt vmcnt(L)   (this wave's loads of tile t landed; t+1 may be in flight)
//                 s_waitcnt lgkmcnt(0); s_barrier   (all waves: tile t landed, tile t-1 consumed)
//                 issue tile t+2 -> stage (t+2)%3   (the stage tile t-1 used)
//                 MFMAs on stage t%3
//
// The barrier is the raw s_barrier (a __syncthreads() would drain the DMA queue with vmcnt(0)),
// all LDS is one extern array, and prefetches past the last tile re-read the last tile so the
// vmcnt bookkeeping is the same on every iteration.  LDS images: the global_load_lds destination
// is lane-linear (wave base + 16*lane), so the XOR swizzles of gemm_common.h are applied to the
// per-lane SOURCE address and to the fragment reads (both sides, same involution).
// Tiles: BM x BN with 64x64 per wave (4x4 v_mfma_f32_16x16x32_bf16 tiles): 256x128 (8 waves,
// 144 KiB LDS) or 128x128 (4 waves, 96 KiB); one block per CU, XCD-aware tile order; split-K
// slabs and the fused epilogue are shared with gemm.hip.
#include "gemm_common.h"

namespace {

typedef __attribute__((address_space(1))) const void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

// one operand tile (R rows x BK) into a swizzled LDS image with wave-instructions of 1 KiB
template <bool KC, int R, int NTH>
struct Glds {
  static constexpr int INSTR = R * BK * 2 / 1024;
  static constexpr int NWAVES = NTH / 64;
  static constexpr int PER_W = INSTR / NWAVES;
  static_assert(INSTR % NWAVES == 0, "tile bytes must split evenly over waves");

  FM_DEVICE static void issue(const unsigned short* __restrict__ p, long ld, int row0, int rows, int k0, char* lds,
                              int wave, int lane) {
#pragma unroll
    for (int i = 0; i < PER_W; ++i) {
      const int j = wave + NWAVES * i;
      const unsigned short* src;
      if constexpr (KC) {           // image [row][64 k]: 8 rows of 128 B per instruction
        const int row = 8 * j + (lane >> 3);
        const int chunk = (lane & 7) ^ ((row >> 1) & 7);
        const int gr = min(row0 + row, rows - 1);          // rows past the edge: never stored
        src = p + (long)gr * ld + k0 + 8 * chunk;
      } else {                      // image [k][R rows]: 1024/(2R) k-rows per instruction
        constexpr int CPR = R / 8;
        constexpr int KPI = 1024 / (2 * R);
        const int krow = KPI * j + lane / CPR;
        const int chunk = (lane % CPR) ^ MNSwz<R>::f(krow);
        const int gr = min(row0 + 8 * chunk, rows - 8);
        src = p + (long)(k0 + krow) * ld + gr;
      }
      __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)(lds + j * 1024), 16, 0, 0);
    }
  }
};

// s_waitcnt with only the vector-memory counter constrained (gfx9 encoding: vmcnt[3:0] |
// expcnt[6:4] | lgkmcnt[11:8] | vmcnt[5:4] << 14)
template <int N>
FM_DEVICE void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

template <int BM, int BN, int WM, int WN, bool AK, bool BKC, bool PRIO>
__global__ void __launch_bounds__(WM * WN * 64, 1) fm_gemm_glds_kernel(GemmP p) {
  constexpr int NW = WM * WN;
  constexpr int NTH = NW * 64;
  constexpr int TM = BM / WM, TN = BN / WN;     // per-wave output tile
  constexpr int MR = TM / 16, NR = TN / 16;
  constexpr int A_BYTES = BM * BK * 2;
  constexpr int B_BYTES = BN * BK * 2;
  constexpr int STG = A_BYTES + B_BYTES;
  constexpr int NS = 3;
  constexpr int LPT = Glds<AK, BM, NTH>::PER_W + Glds<BKC, BN, NTH>::PER_W;   // glds per wave per tile
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  const int bid = xcd_remap(blockIdx.x, p.tiles_m * p.tiles_n);
  int tm, tn;
  tile_coords(p, bid, tm, tn);
  const int zb = blockIdx.y;
  const int split = blockIdx.z;
  const int m0 = tm * BM, n0 = tn * BN;
  const unsigned short* A = p.A + (long)zb * p.sA;
  const unsigned short* B = p.B + (long)zb * p.sB;

  const int ktiles_total = p.K / BK;
  const int kt_per = (ktiles_total + p.ksplit - 1) / p.ksplit;
  const int kt0 = split * kt_per;
  const int kt1 = min(ktiles_total, kt0 + kt_per);
  const int nkt = max(kt1 - kt0, 0);
  const int klast = max(min(kt1, ktiles_total) - 1, 0);

  auto issue = [&](int t, int stage) {
    const int kt = min(kt0 + t, klast);
    char* base = smem + stage * STG;
    Glds<AK, BM, NTH>::issue(A, p.lda, m0, p.M, kt * BK, base, wave, lane);
    Glds<BKC, BN, NTH>::issue(B, p.ldb, n0, p.N, kt * BK, base + A_BYTES, wave, lane);
  };

  f32x4_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // bias gradient folded into dW GEMMs: row sums of the MN-contiguous A image (tn == 0 only)
  const bool rowsum = (!AK) && (p.rowsum_a != nullptr) && (tn == 0);
  constexpr int CPR = BM / 8;
  float rs[8] = {0, 0, 0, 0, 0, 0, 0, 0};

  issue(0, 0);
  issue(1, 1);
  for (int t = 0; t < nkt; ++t) {
    const int stage = t % NS;
    wait_vmcnt<LPT>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    issue(t + 2, (t + 2) % NS);
    const char* la = smem + stage * STG;
    const char* lb = la + A_BYTES;
    if constexpr (!AK) {
      if (rowsum) {
        for (int kr = tid / CPR; kr < BK; kr += NTH / CPR) {
          const bf16x8_t v = *reinterpret_cast<const bf16x8_t*>(la + lds_off<false, BM>(kr, tid % CPR));
#pragma unroll
          for (int e = 0; e < 8; ++e) rs[e] += bf2f((unsigned short)v[e]);
        }
      }
    }
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8_t af[MR], bfr[NR];
#pragma unroll
      for (int i = 0; i < MR; ++i) af[i] = frag<AK, BM>(la, wm * TM + 16 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < NR; ++j) bfr[j] = frag<BKC, BN>(lb, wn * TN + 16 * j, kk, lane);
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);   // MFMA issue ahead of the other waves' loads
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<bf16x8v_t*>(&bfr[j]),
                                                              *reinterpret_cast<bf16x8v_t*>(&af[i]),
                                                              acc[i][j], 0, 0, 0);
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    }
  }
  // drain the (dummy) prefetches before the LDS is reused or the block exits
  wait_vmcnt<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if constexpr (!AK) {
    if (rowsum) {   // reduce the threads sharing each 8-row chunk, one atomic per row
      float* red = reinterpret_cast<float*>(smem);
      constexpr int G = NTH / CPR;
#pragma unroll
      for (int e = 0; e < 8; ++e) red[(tid / CPR) * BM + (tid % CPR) * 8 + e] = rs[e];
      __syncthreads();
      for (int r = tid; r < BM; r += NTH) {
        float x = 0.f;
        for (int g = 0; g < G; ++g) x += red[g * BM + r];
        if (m0 + r < p.M) atomicAdd(p.rowsum_a + m0 + r, x);
      }
    }
  }
  gemm_epilogue<MR, NR>(p, acc, zb, split, m0 + wm * TM, n0 + wn * TN, lane);
}

template <int BM, int BN, int WM, int WN, bool PRIO>
void launch_glds(const GemmP& p, bool ak, bool bk, hipStream_t s) {
  constexpr int NTH = WM * WN * 64;
  constexpr int LDS = 3 * (BM + BN) * BK * 2;
  static bool attr_set = false;
  if (!attr_set) {   // >64 KiB dynamic LDS needs the opt-in attribute
    auto set = [](const void* f) { (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS); };
    set((const void*)fm_gemm_glds_kernel<BM, BN, WM, WN, true, true, PRIO>);
    set((const void*)fm_gemm_glds_kernel<BM, BN, WM, WN, true, false, PRIO>);
    set((const void*)fm_gemm_glds_kernel<BM, BN, WM, WN, false, true, PRIO>);
    set((const void*)fm_gemm_glds_kernel<BM, BN, WM, WN, false, false, PRIO>);
    attr_set = true;
  }
  dim3 grid(p.tiles_m * p.tiles_n, p.batch, p.ksplit);
  if (ak && bk) hipLaunchKernelGGL((fm_gemm_glds_kernel<BM, BN, WM, WN, true, true, PRIO>), grid, dim3(NTH), LDS, s, p);
  else if (ak && !bk) hipLaunchKernelGGL((fm_gemm_glds_kernel<BM, BN, WM, WN, true, false, PRIO>), grid, dim3(NTH), LDS, s, p);
  else if (!ak && bk) hipLaunchKernelGGL((fm_gemm_glds_kernel<BM, BN, WM, WN, false, true, PRIO>), grid, dim3(NTH), LDS, s, p);
  else hipLaunchKernelGGL((fm_gemm_glds_kernel<BM, BN, WM, WN, false, false, PRIO>), grid, dim3(NTH), LDS, s, p);
}

}  // namespace

// Launch the pipelined kernel for a prepared parameter block (tiles_m/n and ksplit filled in
// for the chosen tile).  Caller guarantees: K % 64 == 0 (per split: whole tiles), 16-B aligned
// operands with leading dims % 8 == 0, and M % 8 == 0 / N % 8 == 0 for MN-contiguous operands.
// wide: 4 waves with 128x64 wave tiles (fewer LDS fragment reads per MFMA) instead of 8 waves
// of 64x64 for the 256x128 tile.
extern "C" void fm_gemm_glds_launch(const void* params, int bm, int bn, int a_kcontig, int b_kcontig, int prio,
                                    int wide, hipStream_t stream) {
  const GemmP& p = *reinterpret_cast<const GemmP*>(params);
  if (bm == 256) {
    if (wide) launch_glds<256, 128, 2, 2, false>(p, a_kcontig, b_kcontig, stream);
    else if (prio) launch_glds<256, 128, 4, 2, true>(p, a_kcontig, b_kcontig, stream);
    else launch_glds<256, 128, 4, 2, false>(p, a_kcontig, b_kcontig, stream);
  } else {
    launch_glds<128, 128, 2, 2, false>(p, a_kcontig, b_kcontig, stream);
  }
}
