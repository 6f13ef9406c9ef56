// flexmi bf16 GEMM, big-tile form (gfx950 / MI355X): the split-bf16 fp32 kernel's pipeline
// (gemm_x3.hip) with one operand plane.
//
//   C[M,N] (+)= epilogue( alpha * sum_k A(m,k) * B(k,n) )      bf16 in, fp32 accumulate
//
// Why a second bf16 kernel: the register-staged kernel (gemm.hip fm_gemm_kernel, 128x128 tiles,
// 8 waves of 64x32, two blocks per CU) is LDS-bound on the 1024-wide DLRM layers -- per 64-deep k
// tile a CU writes 64 KiB of operand images (ds_write_b128 moves ~79 B/clk) and reads 192 KiB of
// fragments (256 B/clk) against 1024 MFMA cycles per SIMD: ~1.5x the MFMA time in LDS traffic
// alone (26.5 us / 648 TF on 8192x1024x1024, profiles/gemm_variants_probe.txt).  Here:
//   * 256x128 tile, 8 waves of 64x64 (4x4 16x16x32 tiles): 8 fragment reads per 16 MFMAs;
//   * [row][64 k] images with 128-B rows and the 16-B chunk XOR-swizzled by (row >> 1) & 7
//     (conflict-free ds_read_b128), two 48 KiB stages, one block per CU;
//   * one barrier per 64-deep k step (two MFMA sub-steps; a 32-deep step measured slower than
//     the register-staged kernel: 35 vs 30 us on 8192x1024x1024, gpurun_out r5w); the global
//     loads run two steps ahead in two register sets
//     and the two waves of a SIMD run the staging pass and the MFMAs in opposite order (x3v2
//     schedule 3);
//   * K-contiguous operands: one 16-B load per (row, k-octet) unit; MN-contiguous operands (dX's
//     W, both dW operands): eight 2-B loads per unit (consecutive lanes = consecutive rows, 128 B
//     per wave-instruction), packed into the same 16-B chunk;
//   * the shared epilogue (gemm_common.h gemm_epilogue: bias, activation, fused activation
//     backward + column sums, beta, bf16 / fp32 C, split-K slabs, fused SGD).
// Reference call sites: src/ops/linear.cu:424-447 (forward), :592-635 (backward); SURVEY V1 / V4.
#include "gemm_common.h"

#include <cstdlib>

namespace {

constexpr int X1K = 64;   // k per stage (two 32-deep MFMA sub-steps per barrier)

// byte offset of 16-B chunk c (8 bf16) of row r in a [row][64 k] image (128-B rows, chunk XOR (r>>1)&7)
FM_DEVICE int x1_off(int r, int c) { return r * 128 + 16 * (c ^ ((r >> 1) & 7)); }

template <bool KC, int R, int NTH>
struct X1Stage {
  static constexpr int UNITS = R * (X1K / 8);
  static constexpr int PER_T = (UNITS + NTH - 1) / NTH;
  // KC: the unit's 16 B; MN: eight k values (low half of each word), packed at store time
  unsigned v[PER_T][KC ? 4 : 8];

  FM_DEVICE static void unit(int ci, int& r, int& c) {
    if constexpr (KC) {
      r = ci / (X1K / 8);
      c = ci % (X1K / 8);
    } else {
      r = ci % R;
      c = ci / R;
    }
  }

  // rows past the edge load a clamped (valid) row and are not zeroed: row r of A only reaches
  // output row r, which the epilogue never stores (as gemm_x3.hip); loads stay raw (no select)
  FM_DEVICE void load(const unsigned short* __restrict__ p, long ld, int row0, int rows, int k0, int tid) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int ci = tid + NTH * i;
      if (UNITS % NTH != 0 && ci >= UNITS) continue;
      int r, c;
      unit(ci, r, c);
      const int gr = min(row0 + r, rows - 1);
      if constexpr (KC) {
        const u32x4_t t = *reinterpret_cast<const u32x4_t*>(p + (long)gr * ld + k0 + 8 * c);
        v[i][0] = t[0];
        v[i][1] = t[1];
        v[i][2] = t[2];
        v[i][3] = t[3];
      } else {
        const unsigned short* src = p + (long)(k0 + 8 * c) * ld + gr;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) v[i][kk] = src[kk * ld];
      }
    }
  }

  FM_DEVICE void store(char* pl, int tid) const {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const int ci = tid + NTH * i;
      if (UNITS % NTH != 0 && ci >= UNITS) continue;
      int r, c;
      unit(ci, r, c);
      u32x4_t w;
      if constexpr (KC) {
        w = u32x4_t{v[i][0], v[i][1], v[i][2], v[i][3]};
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) w[u] = (v[i][2 * u] & 0xffffu) | (v[i][2 * u + 1] << 16);
      }
      *reinterpret_cast<u32x4_t*>(pl + x1_off(r, c)) = w;
    }
  }

  // MN-contiguous A (dW): per-thread sums of its row over the staged k (the bias gradient)
  FM_DEVICE void rowsum(float& s, int tid) const {
    if constexpr (!KC) {
#pragma unroll
      for (int i = 0; i < PER_T; ++i) {
        const int ci = tid + NTH * i;
        if (UNITS % NTH != 0 && ci >= UNITS) continue;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) s += bf2f((unsigned short)(v[i][kk] & 0xffffu));
      }
    }
  }
};

template <int BM, int BN, bool AK, bool BKC, bool SGD>
__global__ void __launch_bounds__((BM / 64) * (BN / 64) * 64, 1) fm_gemm_x1_kernel(GemmP p) {
  constexpr int WN = BN / 64, NTH = (BM / 64) * WN * 64;
  constexpr int MR = 4, NR = 4;
  constexpr int PA_ = BM * X1K * 2, PB_ = BN * X1K * 2;   // bytes of one operand image
  constexpr int STG = PA_ + PB_;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int bid = xcd_remap(blockIdx.x, p.tiles_m * p.tiles_n);
  int tm, tn;
  tile_coords(p, bid, tm, tn);
  const int zb = blockIdx.y, split = blockIdx.z;
  const int m0 = tm * BM, n0 = tn * BN;
  const unsigned short* A = p.A + (long)zb * p.sA;
  const unsigned short* B = p.B + (long)zb * p.sB;
  const int ktiles = p.K / X1K;
  const int kt_per = (ktiles + p.ksplit - 1) / p.ksplit;
  const int kt0 = split * kt_per, kt1 = min(ktiles, kt0 + kt_per);
  const int nst = kt1 - kt0;

  f32x4_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  X1Stage<AK, BM, NTH> sa, sa1;
  X1Stage<BKC, BN, NTH> sb, sb1;
  const bool dorow = (!AK) && p.rowsum_a != nullptr && tn == 0;
  float rs = 0.f;
  auto stage = [&](int s) { return smem + s * STG; };
  auto put_from = [&](int s, auto& SA, auto& SB) {
    char* b = stage(s);
    SA.store(b, tid);
    SB.store(b + PA_, tid);
    if constexpr (!AK) {
      if (dorow) SA.rowsum(rs, tid);
    }
  };
  auto get_into = [&](int kt, auto& SA, auto& SB) {
    SA.load(A, p.lda, m0, p.M, kt * X1K, tid);
    SB.load(B, p.ldb, n0, p.N, kt * X1K, tid);
  };
  const int q = lane & 15, g = lane >> 4;
  // loads two steps ahead: step t stores the registers of step t+1 (set (t+1)&1) into stage
  // (t+1)&1 and reloads that set with step t+3; waves w and w+4 (one SIMD) run the staging pass
  // and the MFMAs in opposite order
  if (nst > 0) {
    get_into(kt0, sa, sb);
    put_from(0, sa, sb);
    if (nst > 1) get_into(kt0 + 1, sa1, sb1);
    if (nst > 2) get_into(kt0 + 2, sa, sb);
  }
  const bool mfma_first = (wave >> 2) & 1;
  auto body = [&](int t, auto& SA, auto& SB) {
    __syncthreads();                 // stage t&1 complete; stage (t+1)&1 no longer read
    const char* la = stage(t & 1);
    const char* lb = la + PA_;
    if (!mfma_first && t + 1 < nst) {
      put_from((t + 1) & 1, SA, SB);
      if (t + 3 < nst) get_into(kt0 + t + 3, SA, SB);
    }
#pragma unroll
    for (int ss = 0; ss < X1K / 32; ++ss) {
      bf16x8_t bf[NR];
#pragma unroll
      for (int j = 0; j < NR; ++j)
        bf[j] = *reinterpret_cast<const bf16x8_t*>(lb + x1_off(wn * 64 + 16 * j + q, 4 * ss + g));
#pragma unroll
      for (int i = 0; i < MR; ++i) {
        const bf16x8_t af = *reinterpret_cast<const bf16x8_t*>(la + x1_off(wm * 64 + 16 * i + q, 4 * ss + g));
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8v_t*>(&bf[j]),
                                                              *reinterpret_cast<const bf16x8v_t*>(&af), acc[i][j], 0, 0, 0);
      }
    }
    if (mfma_first && t + 1 < nst) {
      put_from((t + 1) & 1, SA, SB);
      if (t + 3 < nst) get_into(kt0 + t + 3, SA, SB);
    }
  };
  for (int t = 0; t < nst; t += 2) {
    body(t, sa1, sb1);
    if (t + 1 < nst) body(t + 1, sa, sb);
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
  gemm_epilogue<MR, NR, SGD>(p, acc, zb, split, m0 + wm * 64, n0 + wn * 64, lane);
}

template <int BM, int BN, bool SGD>
void launch_x1(const GemmP& p, bool ak, bool bk, hipStream_t s) {
  constexpr int NTH = (BM / 64) * (BN / 64) * 64;
  constexpr int LDS = 2 * (BM + BN) * X1K * 2;
  dim3 grid(p.tiles_m * p.tiles_n, p.batch, p.ksplit);
  if (ak && bk) hipLaunchKernelGGL((fm_gemm_x1_kernel<BM, BN, true, true, SGD>), grid, dim3(NTH), LDS, s, p);
  else if (ak) hipLaunchKernelGGL((fm_gemm_x1_kernel<BM, BN, true, false, SGD>), grid, dim3(NTH), LDS, s, p);
  else if (bk) hipLaunchKernelGGL((fm_gemm_x1_kernel<BM, BN, false, true, SGD>), grid, dim3(NTH), LDS, s, p);
  else hipLaunchKernelGGL((fm_gemm_x1_kernel<BM, BN, false, false, SGD>), grid, dim3(NTH), LDS, s, p);
}

}  // namespace

// Launch on a prepared parameter block (tiles_m / tiles_n / ksplit filled for the bm x 128 tile).
// Caller guarantees: K % 64 == 0 (per split: whole steps); K-contiguous operands 16-B aligned
// with ld % 8 == 0 (MN-contiguous: no constraint); no in-launch split-K combine (tile_cnt null).
// sgd: the fused-SGD epilogue (unsplit tiles only).  Returns -1 for an unsupported tile.
extern "C" int fm_gemm_x1_launch(const void* params, int bm, int a_kcontig, int b_kcontig, int sgd, hipStream_t s) {
  const GemmP& p = *static_cast<const GemmP*>(params);
  if ((sgd && p.ksplit > 1) || p.tile_cnt != nullptr) return -1;
  if (bm == 256) {
    if (sgd) launch_x1<256, 128, true>(p, a_kcontig, b_kcontig, s);
    else launch_x1<256, 128, false>(p, a_kcontig, b_kcontig, s);
  } else if (bm == 128) {
    if (sgd) launch_x1<128, 128, true>(p, a_kcontig, b_kcontig, s);
    else launch_x1<128, 128, false>(p, a_kcontig, b_kcontig, s);
  } else {
    return -1;
  }
  return 0;
}
