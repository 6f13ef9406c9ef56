// flexmi multi-plane MFMA GEMM main loop for gfx950 (MI355X / CDNA4).
//
//   acc[m][n] = sum_k sum_{(pa,pb) in products} A_pa(m,k) * B_pb(k,n)        bf16 planes, fp32 accumulate
//
// NP = 1: a plain bf16 GEMM (one plane, one product).  NP = 3: fp32 operands held as their EXACT bf16
// triplets x = h + m + l (fm_split3_pair, common.h) stored plane by plane in global memory, and the six
// products with pa + pb <= 2 -- the fp32 GEMM of gemm_x3.hip without any split work in the loop: the
// planes are produced once by whoever writes the operand (a GEMM epilogue, the fused SGD's weight
// mirror, fm_split3_planes) and every consumer streams them straight into LDS.
//
// Structure (one block = BM x BN output, WM x WN waves of (BM/WM) x (BN/WN), 16x16x32 MFMAs):
//   * operands staged global -> LDS by LDS-DMA only (global_load_lds_dwordx4, 1 KiB per wave
//     instruction): no VGPR round trip, no ds_write, no staging registers.  The LDS images are the
//     swizzled K-contiguous [row][BK] (ds_read_b128 fragments) and MN-contiguous [BK][row]
//     (ds_read_b64_tr_b16 fragments) images of gemm_common.h, written lane-linearly with the
//     inverse swizzle applied to the per-lane GLOBAL address;
//   * STAGES LDS stages; the DMA of step t + STAGES - 1 is issued at the top of step t, into the
//     stage step t - 1 just finished reading, so STAGES - 1 steps of loads are in flight while step
//     t's MFMAs run.  STAGES > 2 waits with a COUNTED vmcnt and a raw s_barrier (a __syncthreads()
//     fence would drain every DMA in flight);
//   * the MFMA operands are swapped (B fragment as the MFMA "A"), so each lane ends up owning 4
//     consecutive output columns: acc[i][j][r] = C[mb + 16 i + (lane & 15)][nb + 16 j + 4 (lane >> 4) + r]
//     -- the layout every flexmi GEMM epilogue takes (gemm_common.h, gemm_f32_common.h).
// Full tiles only: the host guarantees M % BM == 0, N % BN == 0, (K per split) % BK == 0, 16-B aligned
// rows (ld % 8 == 0 elements) and plane strides.
#pragma once
#include "gemm_common.h"

namespace {
namespace mp {

typedef __attribute__((address_space(1))) const void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

template <int N>
FM_DEVICE void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// K-contiguous image [R][BK]: BK*2-byte rows of 16-B chunks, chunk XOR (row >> 1) & (CPR - 1): the
// 16x16x32 fragment reads (16 rows x 4 chunks per lane group) hit every 16-B slot of a bank row once
template <int BK>
FM_DEVICE int kc_off(int row, int chunk) {
  constexpr int CPR = BK / 8;
  return row * (BK * 2) + 16 * (chunk ^ ((row >> 1) & (CPR - 1)));
}

template <int BK>
FM_DEVICE bf16x8_t frag_kc(const char* lds, int base, int kk, int lane) {
  return *reinterpret_cast<const bf16x8_t*>(lds + kc_off<BK>(base + (lane & 15), 4 * kk + (lane >> 4)));
}

// one operand, one plane, one k step: R rows x BK k into its LDS image (lane-linear 1-KiB pieces)
template <bool KC, int R, int BK, int NW>
struct Dma {
  static constexpr int BYTES = R * BK * 2;
  static constexpr int PIECES = BYTES / 1024;
  static constexpr int PER_W = PIECES / NW;
  static_assert(PIECES % NW == 0 && PER_W >= 1, "whole 1-KiB pieces per wave");
  FM_DEVICE static void issue(const unsigned short* __restrict__ p, long ld, int row0, int k0, char* lds, int wave,
                              int lane) {
#pragma unroll
    for (int i = 0; i < PER_W; ++i) {
      const int piece = wave * PER_W + i;
      const int o = piece * 1024 + 16 * lane;
      const unsigned short* src;
      if constexpr (KC) {
        const int row = o / (BK * 2), slot = (o % (BK * 2)) / 16;
        const int c = slot ^ ((row >> 1) & (BK / 8 - 1));
        src = p + (long)(row0 + row) * ld + k0 + 8 * c;
      } else {
        const int kr = o / (R * 2), slot = (o % (R * 2)) / 16;
        const int c = slot ^ MNSwz<R>::f(kr);
        src = p + (long)(k0 + kr) * ld + row0 + 8 * c;
      }
      __builtin_amdgcn_global_load_lds((gptr_t)(const void*)src, (lptr_t)(void*)(lds + piece * 1024), 16, 0, 0);
    }
  }
};

// operands of one GEMM: NP planes each, plane p at X + p * sXp (elements); batch stride sX
struct Opnds {
  const unsigned short* A; long lda; long sA; long sAp;
  const unsigned short* B; long ldb; long sB; long sBp;
};

// LAB (tools/gemm_mp_lab.hip only): 1 = no DMA inside the K loop (MFMA + fragment reads on stage 0),
// 2 = no MFMAs (DMA, waits and barriers only)
template <int BM, int BN, int NP, bool AK, bool BKC, int WM, int WN, int STAGES, int LAB = 0>
struct Loop {
  static constexpr int BK = NP == 1 ? 64 : 32;
  static constexpr int NW = WM * WN;
  static constexpr int NTH = NW * 64;
  static constexpr int TM = BM / WM, TN = BN / WN;
  static constexpr int MR = TM / 16, NR = TN / 16;
  static constexpr int PA = BM * BK * 2, PB = BN * BK * 2;   // bytes of one plane image
  static constexpr int STG = NP * (PA + PB);
  static constexpr int LDS = STAGES * STG;
  static constexpr int GLDS = NP * (Dma<AK, BM, BK, NW>::PER_W + Dma<BKC, BN, BK, NW>::PER_W);   // per wave and step
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static_assert(STAGES >= 2 && STAGES <= 4, "stages");
  static constexpr int NPROD = NP == 1 ? 1 : 6;

  // step kt of operands (A rows m0.., B rows n0..) into stage s
  FM_DEVICE static void stage(const Opnds& o, int m0, int n0, int kt, char* smem, int s, int wave, int lane) {
    char* base = smem + s * STG;
#pragma unroll
    for (int pl = 0; pl < NP; ++pl) {
      Dma<AK, BM, BK, NW>::issue(o.A + pl * o.sAp, o.lda, m0, kt * BK, base + pl * PA, wave, lane);
      Dma<BKC, BN, BK, NW>::issue(o.B + pl * o.sBp, o.ldb, n0, kt * BK, base + NP * PA + pl * PB, wave, lane);
    }
  }

  FM_DEVICE static void compute(const char* st, int wm, int wn, int lane, f32x4_t (&acc)[MR][NR]) {
    // products pa + pb <= 2, smallest terms first so the dominant h*h product is added last
    constexpr int TA[6] = {2, 1, 0, 1, 0, 0};
    constexpr int TB[6] = {0, 1, 2, 0, 1, 0};
    const char* la = st;
    const char* lb = st + NP * PA;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8_t bfr[NP][NR];
#pragma unroll
      for (int pl = 0; pl < NP; ++pl)
#pragma unroll
        for (int j = 0; j < NR; ++j) {
          if constexpr (BKC) bfr[pl][j] = frag_kc<BK>(lb + pl * PB, wn * TN + 16 * j, kk, lane);
          else bfr[pl][j] = frag<false, BN>(lb + pl * PB, wn * TN + 16 * j, kk, lane);
        }
#pragma unroll
      for (int i = 0; i < MR; ++i) {
        bf16x8_t af[NP];
#pragma unroll
        for (int pl = 0; pl < NP; ++pl) {
          if constexpr (AK) af[pl] = frag_kc<BK>(la + pl * PA, wm * TM + 16 * i, kk, lane);
          else af[pl] = frag<false, BM>(la + pl * PA, wm * TM + 16 * i, kk, lane);
        }
#pragma unroll
        for (int s = 0; s < NPROD; ++s) {
          const int pa = NP == 1 ? 0 : TA[s], pb = NP == 1 ? 0 : TB[s];
#pragma unroll
          for (int j = 0; j < NR; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8v_t*>(&bfr[pb][j]),
                                                                *reinterpret_cast<const bf16x8v_t*>(&af[pa]),
                                                                acc[i][j], 0, 0, 0);
        }
      }
    }
  }

  // raw s_barrier (no vmcnt drain) between compiler memory fences; the lgkmcnt(0) retires this
  // wave's fragment reads of the stage the next DMA overwrites (WAR)
  FM_DEVICE static void barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  // the whole K loop of k steps [kt0, kt1) for output tile (m0, n0); every wave of the block calls it
  FM_DEVICE static void run(const Opnds& o, int m0, int n0, int kt0, int kt1, char* smem, f32x4_t (&acc)[MR][NR],
                            long long* stamps = nullptr) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const int nst = kt1 - kt0;
    if (nst <= 0) return;
    // prologue: steps 0 .. STAGES-2 in flight, wait for step 0
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s)
      if (s < nst) stage(o, m0, n0, kt0 + s, smem, s, wave, lane);
    if (nst >= STAGES - 1) wait_vm<GLDS * (STAGES - 2)>();
    else wait_vm<0>();
    barrier();
    long long tw = 0, t_in = 0;
    if (stamps) t_in = __builtin_amdgcn_s_memtime();
    int cur = 0;
    for (int t = 0; t < nst; ++t) {
      const int ahead = t + STAGES - 1;
      int nxt = cur + STAGES - 1;
      if (nxt >= STAGES) nxt -= STAGES;
      if (LAB != 1 && ahead < nst) stage(o, m0, n0, kt0 + ahead, smem, nxt, wave, lane);
      if constexpr (LAB == 2) {
#pragma unroll
        for (int i = 0; i < MR; ++i)
#pragma unroll
          for (int j = 0; j < NR; ++j) asm volatile("" : "+v"(acc[i][j]));
      } else {
        compute(smem + (LAB == 1 ? 0 : cur) * STG, wm, wn, lane, acc);
      }
      long long tb = 0;
      if (stamps) tb = __builtin_amdgcn_s_memtime();
      // step t+1 must have landed: the DMAs younger than it (steps t+2 .. t+STAGES-1 issued so far)
      // may stay in flight
      const int younger = min(nst - 1, ahead) - (t + 1);   // steps issued after step t+1
      if constexpr (STAGES == 2) {
        wait_vm<0>();
      } else if constexpr (STAGES == 3) {
        if (younger >= 1) wait_vm<GLDS>();
        else wait_vm<0>();
      } else {
        if (younger >= 2) wait_vm<2 * GLDS>();
        else if (younger == 1) wait_vm<GLDS>();
        else wait_vm<0>();
      }
      barrier();
      if (stamps) tw += __builtin_amdgcn_s_memtime() - tb;
      cur = cur + 1 == STAGES ? 0 : cur + 1;
    }
    if (stamps && (threadIdx.x & 63) == 0) {
      stamps[0] = t_in;
      stamps[1] = __builtin_amdgcn_s_memtime();
      stamps[2] = tw;
    }
  }
};

}  // namespace mp
}  // namespace
