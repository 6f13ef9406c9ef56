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

  // OPT & 4: LDS-DMA staging (full tiles, row sums read back from the image; as gemm.hip): step kt+1's pieces issued into
  // the free stage before step kt's MFMAs, vmcnt(0) before the barrier that publishes them
  constexpr bool DMA = (OPT & 4) != 0;
  StageF<AK, BM, VEC, NT> sa;
  StageF<BKC, BN, VEC, NT> sb;
  const bool rowsum = (!AK) && (p.rowsum_a != nullptr) && (tn == 0);
  float rs[4] = {0.f, 0.f, 0.f, 0.f};
#define LDSF_A(b) (smem + (b) * (A_BYTES + B_BYTES))
#define LDSF_B(b) (smem + (b) * (A_BYTES + B_BYTES) + A_BYTES)
  auto stage_dma = [&](int kt, int b) {
    DmaStageF<AK, BM, NT>::issue(A, p.lda, m0, kt * BKF, LDSF_A(b), wave, lane);
    DmaStageF<BKC, BN, NT>::issue(B, p.ldb, n0, kt * BKF, LDSF_B(b), wave, lane);
  };
  if (kt0 < kt1) {
    if constexpr (DMA) {
      stage_dma(kt0, 0);
      __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    } else {
      sa.load(A, p.lda, m0, p.M, kt0 * BKF, p.K, tid);
      sb.load(B, p.ldb, n0, p.N, kt0 * BKF, p.K, tid);
      sa.store(LDSF_A(0), tid);
      sb.store(LDSF_B(0), tid);
      if (rowsum) sa.accumulate_rows(rs);
    }
  }
  __syncthreads();
  for (int kt = kt0; kt < kt1; ++kt) {
    const int cur = (kt - kt0) & 1;
    const bool more = kt + 1 < kt1;
    if (more) {
      if constexpr (DMA) {
        stage_dma(kt + 1, cur ^ 1);
      } else {
        sa.load(A, p.lda, m0, p.M, (kt + 1) * BKF, p.K, tid);
        sb.load(B, p.ldb, n0, p.N, (kt + 1) * BKF, p.K, tid);
      }
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
    if constexpr (DMA) {
      if constexpr (!AK) {   // bias-gradient row sums from the DMA-staged image (the register form's chunks)
        if (rowsum) {
#pragma unroll
          for (int i = 0; i < StageF<AK, BM, VEC, NT>::PER_T; ++i) {
            const int ci = tid + NT * i;
            const f32x4_t v = *reinterpret_cast<const f32x4_t*>(LDSF_A(cur) + (ci / (BM / 4)) * (BM * 4) + 16 * (ci % (BM / 4)));
#pragma unroll
            for (int j = 0; j < 4; ++j) rs[j] += v[j];
          }
        }
      }
      __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): this wave's pieces of step kt+1 landed
    } else if (more) {
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
    } else {
      float s = slab_sum1(src, MN, p.ksplit);
      if constexpr (SGD) {
        sgd_apply1(p, (long)m * p.ldc + n, s * p.alpha);
        continue;
      }
      s = act_fwd(p.act, s * p.alpha + (p.bias ? p.bias[n] : 0.f));
      *d = s + (p.beta ? *d : 0.f);
    }
  }
}

// split-K reduce for DEEP splits (ks >= 16, N % 4 == 0; the small-output dW GEMMs: 128 x 256 x 8192
// runs 64-way): the one-thread-per-4-outputs reduce above leaves a 32-block grid with 64 dependent
// slab reads per thread (21 us for 8 MB, profiles/prof_r5final_step_fp32.txt).  Here G = 8 threads
// share each 4-output group -- thread g sums slabs g, g + 8, ... in order -- and the G partial sums are
// added through LDS in g order (deterministic): 8x the blocks and the loads in flight.
constexpr int RD_G = 8;
template <bool SGD>
__global__ void __launch_bounds__(256) fm_gemm_f32_reduce_deep(GemmF p) {
  __shared__ f32x4_t part[RD_G][256 / RD_G];
  constexpr int O = 256 / RD_G;
  const long MN = (long)p.M * p.N;
  const long total = MN * p.batch / 4;
  const int o = threadIdx.x % O, g = threadIdx.x / O;
  const long i = blockIdx.x * (long)O + o;
  const long e0 = (i < total ? i : total - 1) * 4;
  const long zb = e0 / MN, e = e0 % MN;
  const float* src = p.ws + zb * p.ksplit * MN + e;
  f32x4_t s = {0.f, 0.f, 0.f, 0.f};
  int k = g;
  for (; k + 3 * RD_G < p.ksplit; k += 4 * RD_G) {
    f32x4_t v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const f32x4_t*>(src + (long)(k + u * RD_G) * MN);
#pragma unroll
    for (int u = 0; u < 4; ++u) s += v[u];
  }
  for (; k < p.ksplit; k += RD_G) s += *reinterpret_cast<const f32x4_t*>(src + (long)k * MN);
  part[g][o] = s;
  __syncthreads();
  if (g != 0 || i >= total) return;
  s = part[0][o];
#pragma unroll
  for (int t = 1; t < RD_G; ++t) s += part[t][o];
  const int m = (int)(e / p.N), n = (int)(e % p.N);
  if constexpr (SGD) {
    sgd_apply4(p, (long)m * p.ldc + n, s * p.alpha);
    return;
  }
  float* d = p.C + zb * p.sC + (long)m * p.ldc + n;
#pragma unroll
  for (int r = 0; r < 4; ++r) s[r] = act_fwd(p.act, s[r] * p.alpha + (p.bias ? p.bias[n + r] : 0.f));
  if (p.beta) s += *reinterpret_cast<const f32x4_t*>(d);
  *reinterpret_cast<f32x4_t*>(d) = s;
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
extern "C" int fm_gemm_x3v2_launch(const void* params, int bm, int bn, int a_kcontig, int b_kcontig, int sgd,
                                   hipStream_t s);


namespace {

void launch_reduce_f32(const GemmF& p, int v4, long total, hipStream_t stream) {
  if (v4 && p.ksplit >= 16) {
    const dim3 grid((unsigned)((total + 256 / RD_G - 1) / (256 / RD_G)));
    if (p.uw) hipLaunchKernelGGL(fm_gemm_f32_reduce_deep<true>, grid, dim3(256), 0, stream, p);
    else hipLaunchKernelGGL(fm_gemm_f32_reduce_deep<false>, grid, dim3(256), 0, stream, p);
    return;
  }
  if (p.uw) hipLaunchKernelGGL(fm_gemm_f32_reduce<true>, dim3(fm_grid(total)), dim3(256), 0, stream, p, v4);
  else hipLaunchKernelGGL(fm_gemm_f32_reduce<false>, dim3(fm_grid(total)), dim3(256), 0, stream, p, v4);
}

template <int BM, int BN, bool AK, bool BKC, bool VEC>
void launch_f(const GemmF& p, hipStream_t s) {
  constexpr int LDS = 2 * (BM + BN) * BKF * 4;
  dim3 grid(p.tiles_m * p.tiles_n, p.batch, p.ksplit);
  if constexpr (!AK && !BKC && BM <= 128) {   // fused-SGD dW GEMMs: own instantiation of the default forms
    if (p.uw) {
      if constexpr (VEC && BM == 128) {
        if (p.dma) hipLaunchKernelGGL((fm_gemm_f32_kernel<BM, BN, AK, BKC, VEC, 6, 512, 2, true>), grid, dim3(512), LDS, s, p);
        else hipLaunchKernelGGL((fm_gemm_f32_kernel<BM, BN, AK, BKC, VEC, 2, 512, 2, true>), grid, dim3(512), LDS, s, p);
      } else {
        hipLaunchKernelGGL((fm_gemm_f32_kernel<BM, BN, AK, BKC, VEC, 0, NTF, 2, true>), grid, dim3(NTF), LDS, s, p);
      }
      return;
    }
  }
  if constexpr (VEC && BM == 128) {
    // 8 waves with the fragment double buffer: 4 waves per SIMD hide the per-K-tile barrier and
    // first-fragment latency (DLRM fp32 GEMMs -3.7 %, the 1024-wide layers -5..8 %, the 512/256-wide
    // layers' dX/dW -5..14 % against the 4-wave kernel: profiles/gemm_f32_variants_ab.jsonl,
    // gemm_f32_8wave_ab.jsonl; the 4-wave / s_setprio / 256x128 A/B variants deleted in r6)
    if (p.dma) hipLaunchKernelGGL((fm_gemm_f32_kernel<BM, BN, AK, BKC, VEC, 6, 512>), grid, dim3(512), LDS, s, p);
    else hipLaunchKernelGGL((fm_gemm_f32_kernel<BM, BN, AK, BKC, VEC, 2, 512>), grid, dim3(512), LDS, s, p);
    return;
  }
  if constexpr (VEC) {
    if (p.dma) {
      hipLaunchKernelGGL((fm_gemm_f32_kernel<BM, BN, AK, BKC, VEC, 4>), grid, dim3(NTF), LDS, s, p);
      return;
    }
  }
  hipLaunchKernelGGL((fm_gemm_f32_kernel<BM, BN, AK, BKC, VEC>), grid, dim3(NTF), LDS, s, p);
}

template <int BM, int BN>
void launch_fbm(const GemmF& p, bool ak, bool bk, bool vec, hipStream_t s) {
  if (vec) {
    if (ak && bk) launch_f<BM, BN, true, true, true>(p, s);
    else if (ak) launch_f<BM, BN, true, false, true>(p, s);
    else if (bk) launch_f<BM, BN, false, true, true>(p, s);
    else launch_f<BM, BN, false, false, true>(p, s);
  } else {
    if (ak && bk) launch_f<BM, BN, true, true, false>(p, s);
    else if (ak) launch_f<BM, BN, true, false, false>(p, s);
    else if (bk) launch_f<BM, BN, false, true, false>(p, s);
    else launch_f<BM, BN, false, false, false>(p, s);
  }
}

}  // namespace

// ---- per-row / per-column max |x| (the F16 split form's operand scales) ----------------------------
// max |x| as a bit pattern (non-negative floats order like their bits).  One launch serves both
// operands of a GEMM (two jobs; blocks [0, nb0) job 0, the rest job 1).  A job reduces either along
// the rows of a [R][C] array (ROWS: one wave per row, out[r]) or down its columns (COLS: a block covers
// 256 columns x rpb rows, folded through LDS, one PARTIAL per block row: out[by * C + c], by < np --
// no atomics, no zeroing; the consumer takes the max over the np partials).
struct AmaxJob {
  const float* X;
  long ld;
  int R, C, cols, rpb, nbx;   // cols: 0 = ROWS, 1 = COLS (nbx column blocks)
  unsigned* out;
};

__global__ void __launch_bounds__(256) fm_f32_amax2(AmaxJob j0, AmaxJob j1, int nb0) {
  __shared__ unsigned red[4][256];
  const bool second = (int)blockIdx.x >= nb0;
  const AmaxJob& j = second ? j1 : j0;
  const int b = second ? blockIdx.x - nb0 : blockIdx.x;
  const int nb = second ? gridDim.x - nb0 : nb0;
  const bool vec = (j.ld % 4 == 0) && ((((uintptr_t)j.X) & 15) == 0);
  if (!j.cols) {
    const int lane = threadIdx.x & 63;
    for (long r = b * 4L + (threadIdx.x >> 6); r < j.R; r += nb * 4L) {
      const float* x = j.X + r * j.ld;
      unsigned m = 0;
      if (vec && j.C % 4 == 0) {
        for (int c = lane * 4; c < j.C; c += 256) {
          const u32x4_t v = *reinterpret_cast<const u32x4_t*>(x + c);
          m = max(max(m, max(v[0] & 0x7fffffffu, v[1] & 0x7fffffffu)), max(v[2] & 0x7fffffffu, v[3] & 0x7fffffffu));
        }
      } else {
        for (int c = lane; c < j.C; c += 64) m = max(m, __float_as_uint(x[c]) & 0x7fffffffu);
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o, 64));
      if (lane == 0) j.out[r] = m;
    }
    return;
  }
  const int bx = b % j.nbx, by = b / j.nbx;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = bx * 256 + tx * 4;
  const int r0 = by * j.rpb, r1 = min(j.R, r0 + j.rpb);
  const bool v4 = vec && c + 3 < j.C;
  unsigned m[4] = {0u, 0u, 0u, 0u};
  if (c < j.C) {
    for (int r = r0 + ty; r < r1; r += 4) {
      const float* x = j.X + (long)r * j.ld + c;
      if (v4) {
        const u32x4_t v = *reinterpret_cast<const u32x4_t*>(x);
#pragma unroll
        for (int e = 0; e < 4; ++e) m[e] = max(m[e], v[e] & 0x7fffffffu);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (c + e < j.C) m[e] = max(m[e], __float_as_uint(x[e]) & 0x7fffffffu);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) red[ty][tx * 4 + e] = m[e];
  __syncthreads();
  if (ty == 0) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (c + e < j.C)
        j.out[(long)by * j.C + c + e] =
            max(max(red[0][tx * 4 + e], red[1][tx * 4 + e]), max(red[2][tx * 4 + e], red[3][tx * 4 + e]));
  }
}

// the job computing the max |x| of every M row of A / N column of B over K; np = partial count
static AmaxJob amax_job(const float* X, long ld, bool kcontig, int rows_mn, int K, unsigned* out, int& nblocks, int& np) {
  AmaxJob j{X, ld, 0, 0, 0, 0, 1, out};
  if (kcontig) {   // [rows_mn][K]: a row reduction
    j.R = rows_mn; j.C = K; j.cols = 0;
    nblocks = (int)std::min<long>((rows_mn + 3) / 4, 1024);
    np = 1;
  } else {         // [K][rows_mn]: partial column reductions, <= 16 partials of >= 64 rows
    j.R = K; j.C = rows_mn; j.cols = 1;
    j.nbx = (rows_mn + 255) / 256;
    int by = std::max(1, std::min(16, (K + 63) / 64));
    j.rpb = (K + by - 1) / by;
    by = (K + j.rpb - 1) / j.rpb;
    nblocks = j.nbx * by;
    np = by;
  }
  return j;
}

// Same contract as fm_gemm (gemm.hip) with fp32 operands and output:
//   A_kcontig: A stored [M][K] (lda >= K) else [K][M] (lda >= M)
//   B_kcontig: B stored [N][K] (ldb >= K) else [K][N] (ldb >= N)
static int g_f32_split = -1;   // -1: from FM_F32_SPLIT at the first call
extern "C" void fm_gemm_f32_set_split(int on) { g_f32_split = on < 0 ? 0 : on; }

// LDS-DMA operand staging of the GEMM / convolution kernels for eligible shapes (full tiles; dW row
// sums read back from the image): FM_GEMM_DMA (default 1) or fm_gemm_set_dma; 0 = register staging (A/B, tests)
static int g_gemm_dma = -1;
extern "C" void fm_gemm_set_dma(int on) { g_gemm_dma = on ? 1 : 0; }
extern "C" int fm_gemm_dma_enabled() {
  if (g_gemm_dma < 0) g_gemm_dma = !getenv("FM_GEMM_DMA") || atoi(getenv("FM_GEMM_DMA")) != 0;
  return g_gemm_dma;
}
// default 3: the split kernel (gemm_x3.hip) for the big GEMMs, where it beat both the native
// fp32 MFMA kernel and hipBLASLt on every DLRM shape and orientation (profiles/gemm_f32_lab_r5i_*);
// 1 (the first split kernel, deleted in r6) reads as 2.  4 / 5: as 3 / 2 with the F16 form of the
// split kernel (two scaled fp16 planes, three products instead of six bf16 ones)
static int f32_split_mode() {
  if (g_f32_split < 0) g_f32_split = getenv("FM_F32_SPLIT") != nullptr ? std::max(0, atoi(getenv("FM_F32_SPLIT"))) : 3;
  if (g_f32_split == 1) g_f32_split = 2;
  return g_f32_split;
}
extern "C" int fm_gemm_f32_get_split() { return f32_split_mode(); }

// the form (see gemm_f32_run) the last fp32 GEMM issued from this thread ran with (tuner check)
static thread_local int g_last_form = 0;
extern "C" int fm_gemm_f32_last_form() { return g_last_form; }

struct SgdUpdF {
  float* w; unsigned short* wc; float* v; const float* lr; float wd, mom; int nest;
};

static int gemm_f32_run(const float* A, long lda, long sA, int a_kcontig, const float* B, long ldb, long sB,
                        int b_kcontig, float* C, long ldc, long sC, const float* bias, int M, int N, int K, int batch,
                        float alpha, int beta, int act, float* ws, long ws_bytes, int ksplit_req, const float* act_y,
                        long lday, int bwd_act, float* colsum, float* rowsum_a, const SgdUpdF* upd,
                        hipStream_t stream);

extern "C" int fm_gemm_f32(const float* A, long lda, long sA, int a_kcontig, const float* B, long ldb, long sB,
                           int b_kcontig, float* C, long ldc, long sC, const float* bias, int M, int N, int K, int batch,
                           float alpha, int beta, int act, float* ws, long ws_bytes, int ksplit_req, const float* act_y,
                           long lday, int bwd_act, float* colsum, float* rowsum_a, hipStream_t stream) {
  return gemm_f32_run(A, lda, sA, a_kcontig, B, ldb, sB, b_kcontig, C, ldc, sC, bias, M, N, K, batch, alpha, beta, act, ws,
                      ws_bytes, ksplit_req, act_y, lday, bwd_act, colsum, rowsum_a, nullptr, stream);
}

// fp32 weight-gradient GEMM with the SGD update fused in (same contract as gemm.hip fm_gemm_dw_sgd):
// A = dpre [K][M], B = x [K][N], W [M][ldw] updated in place, the gradient never stored; -1 when
// the fused form does not apply (the caller falls back to GEMM + optimizer kernel).  Always the
// split kernel (gemm_x3.hip) or the default register-staged kernel, the update in its epilogue.
extern "C" int fm_gemm_f32_dw_sgd(const float* A, long lda, const float* B, long ldb, float* W, long ldw,
                                  unsigned short* Wc, float* V, const float* lr, float wd, float mom, int nesterov,
                                  int M, int N, int K, float* ws, long ws_bytes, float* rowsum_a, int cfg,
                                  hipStream_t stream) {
  SgdUpdF u{W, Wc, V, lr, wd, mom, nesterov};
  return gemm_f32_run(A, lda, 0, 0, B, ldb, 0, 0, W, ldw, 0, nullptr, M, N, K, 1, 1.f, 0, 10, ws, ws_bytes, cfg, nullptr,
                      0, 10, nullptr, rowsum_a, &u, stream);
}

static int gemm_f32_run(const float* A, long lda, long sA, int a_kcontig, const float* B, long ldb, long sB,
                        int b_kcontig, float* C, long ldc, long sC, const float* bias, int M, int N, int K, int batch,
                        float alpha, int beta, int act, float* ws, long ws_bytes, int ksplit_req, const float* act_y,
                        long lday, int bwd_act, float* colsum, float* rowsum_a, const SgdUpdF* upd,
                        hipStream_t stream) {
  if (M <= 0 || N <= 0 || batch <= 0) return 0;
  if (upd && (K <= 0 || ldc % 4 != 0 || (((uintptr_t)upd->w | (uintptr_t)(upd->v ? upd->v : upd->w)) & 15) ||
              (((uintptr_t)(upd->wc ? (void*)upd->wc : (void*)upd->w)) & 7)))
    return -1;
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
  p.ulds = upd != nullptr;   // the update staged through LDS (whole-row W accesses)
  p.dma = 0;
  p.amax_a = p.amax_b = nullptr;
  p.amax_na = p.amax_nb = 1;
  auto al = [](const void* q) { return (((uintptr_t)q) & 15) == 0; };
  bool vec = al(A) && al(B) && (lda % 4 == 0) && (ldb % 4 == 0) && (sA % 4 == 0) && (sB % 4 == 0);
  vec = vec && (a_kcontig ? (K % 4 == 0) : (M % 4 == 0)) && (b_kcontig ? (K % 4 == 0) : (N % 4 == 0));
  // ksplit_req = ks | form << 8: a measured configuration (flexmi/ops/gemm_tune.py) -- form 1/2/3 the
  // native kernel with 128x128 / 128x64 / 64x64 tiles, 4/5/6 the split kernel with 256x128 / 128x128 /
  // 128x64,
  // ks the split-K depth (0: the heuristic's); form 0 = the heuristic tile.  A form that does not
  // apply to the operands falls back to the heuristic.
  int form = ksplit_req >> 8;
  ksplit_req &= 255;
  const bool fused_ok_split = ws != nullptr && batch == 1 && (long)M * N * 4 * 2 <= ws_bytes;
  // fp32 on the bf16 matrix cores (gemm_x3.hip: exact three-way operand split in the register
  // staging pass).  Split mode (FM_F32_SPLIT / fm_gemm_f32_set_split): 0 = the native fp32 MFMA
  // kernel only, 2 = the split kernel for every eligible GEMM, 3 (default) = only the big ones,
  // where it measured faster than the native kernel (min(M, N) >= 480 and K >= 480,
  // profiles/gemm_f32_lab_r5i_*).  K-contiguous operands need 16-B rows; MN-contiguous ones are
  // read per element.
  const int split_mode = f32_split_mode();
  const bool big = std::min(M, N) >= 480 && K >= 480;
  const bool x3_pick = form ? (form >= 4 && split_mode != 0)
                            : split_mode == 2 || split_mode == 5 || ((split_mode == 3 || split_mode == 4) && big);
  const bool f16_form = split_mode >= 4 && batch == 1;
  if (x3_pick && K > 0 && K % 32 == 0 && M >= 64 && N >= 64) {
    auto opnd_ok = [&](const float* X, long ld, long sX, bool kc) {
      return kc ? (al(X) && ld % 4 == 0 && sX % 4 == 0) : true;   // MN-contiguous: 4-B loads
    };
    if (opnd_ok(A, lda, sA, a_kcontig) && opnd_ok(B, ldb, sB, b_kcontig)) {
      // 256x128 (8 waves, 2 per SIMD) whenever M fills it, split-K for the grid
      // the F16 form runs on 128-row tiles (4 or 2 waves per block: room for its second accumulator set)
      const bool f16_pick = f16_form && ws != nullptr && (a_kcontig || split_mode == 5);
      const int bm = (form == 4 && !f16_pick) ? 256 : (form == 4 || form == 5 || form == 6) ? 128
                                                     : (M >= 256 && !f16_pick) ? 256 : 128;
      const int bn = form == 6 ? 64 : 128;
      p.tiles_m = (M + bm - 1) / bm;
      p.tiles_n = (N + bn - 1) / bn;
      const long tiles = (long)p.tiles_m * p.tiles_n * batch;
      const int ktiles = K / 32;
      const bool fused = act_y != nullptr || colsum != nullptr;
      int ks = 1;
      if (ksplit_req > 0) ks = ksplit_req;
      else if (ws != nullptr && !fused)
        while (tiles * ks < 256 && ks * 2 <= ktiles / 4 && ks < 16) ks *= 2;
      if (fused) ks = 1;
      ks = std::min(ks, std::max(1, ktiles));
      while (ks > 1 && (ws == nullptr || (long)batch * ks * M * (long)N * 4 > ws_bytes)) ks /= 2;
      p.ksplit = ks;
      p.amax_a = p.amax_b = nullptr;
      // F16 form for the GEMMs with a K-contiguous A (forward, dX): measured faster than the bf16
      // six-product split there, slower on the dW orientation whose two column scans read both
      // batch-long operands (profiles/f16_split_ab_r7.txt)
      if (f16_pick) {
        // per-row / per-column scales from the tail of the workspace (the slabs use the front)
        const long abytes = (((long)M + N) * 16 * 4 + 255) & ~255L;
        const long slab = (long)batch * ks * M * (long)N * 4;
        if (slab + abytes <= ws_bytes) {
          unsigned* am = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(ws) + ws_bytes - abytes);
          int nba, nbb, npa, npb;
          const AmaxJob ja = amax_job(A, lda, a_kcontig, M, K, am, nba, npa);
          const AmaxJob jb = amax_job(B, ldb, b_kcontig, N, K, am + (long)M * 16, nbb, npb);
          hipLaunchKernelGGL(fm_f32_amax2, dim3(nba + nbb), dim3(256), 0, stream, ja, jb, nba);
          p.amax_a = am;
          p.amax_b = am + (long)M * 16;
          p.amax_na = npa;
          p.amax_nb = npb;
        }
      }
      g_last_form = bm == 256 ? 4 : bn == 64 ? 6 : 5;
      if (fm_gemm_x3v2_launch(&p, bm, bn, a_kcontig, b_kcontig, upd != nullptr && ks == 1, stream) == 0) {
        if (ks > 1) {
          const int v4 = (N % 4 == 0) && (ldc % 4 == 0) && (sC % 4 == 0) && al(C);
          const long total = (long)M * N * batch / (v4 ? 4 : 1);
          launch_reduce_f32(p, v4, total, stream);
        }
        return ks;
      }
    }
  }
  // tiles: 128x128 when that gives >= 2 blocks per CU; narrower N / smaller tiles for small grids
  int BMv = 128, BNv = 128;
  const long t128 = (long)((M + 127) / 128) * ((N + 127) / 128) * batch;
  if (t128 < 512 && N <= 64 * 8) BNv = 64;
  // 64x64 tiles (no split-K, 4 blocks per CU) up to one wave of 128x128 tiles: the 8192x512->256
  // forward runs unsplit instead of split-K 2 + reduce (step -0.2..0.9 %: profiles/ab_f32_t64.txt)
  if (t128 < 129 && K <= 2048) { BMv = 64; BNv = 64; }
  // a fused backward epilogue (act-bwd of the layer below / bias-grad column sums) cannot split K:
  // small grids take 64x64 tiles for 4x the blocks (summit_large dX, 256 x 4096 x 4096: 64 -> 256
  // blocks on 256 CUs)
  // ... unless K is long enough to split it: then 128x128 tiles split K and the fused epilogue runs in
  // the reduce (fm_gemm_f32_reduce_bwd)
  const bool fused_ep = act_y != nullptr || colsum != nullptr;
  const bool fused_split = fused_ep && t128 < 256 && K >= 1024 && ws != nullptr && batch == 1 && ksplit_req <= 0 &&
                           (long)M * N * 4 * 2 <= ws_bytes;
  if (fused_ep && t128 < 256 && !fused_split) { BMv = 64; BNv = 64; }
  if (form >= 4) form = 0;   // the split kernel did not apply
  if (form == 1) { BMv = 128; BNv = 128; }
  if (form == 2) { BMv = 128; BNv = 64; }
  if (form == 3) { BMv = 64; BNv = 64; }
  p.tiles_m = (M + BMv - 1) / BMv;
  p.tiles_n = (N + BNv - 1) / BNv;
  const long tiles = (long)p.tiles_m * p.tiles_n * batch;
  const int ktiles = (K + BKF - 1) / BKF;
  int ks = 1;
  if (ksplit_req > 0) ks = ksplit_req;
  else if (ws != nullptr) {
    const long target = 512L;   // 2 resident blocks per CU (profiles/ab_f32_split_blocks.txt)
    // up to 16-way, or 64-way for a handful of tiles (the bottom-MLP dW GEMMs: 128 x 256 x 8192
    // made 64 blocks at 16-way, 30 us)
    const int ks_max = tiles <= 8 ? 64 : 16;
    while (tiles * ks < target && ks * 2 <= ktiles / 4 && ks < ks_max) ks *= 2;
  }
  // fused bwd epilogue in the tile needs the full K sum (split: the epilogue runs in the reduce)
  if (fused_ep && !(form ? fused_ok_split : fused_split)) ks = 1;
  ks = std::min(ks, std::max(1, ktiles));
  while (ks > 1 && (ws == nullptr || (long)batch * ks * M * (long)N * 4 > ws_bytes)) ks /= 2;
  if (K <= 0) ks = 1;
  p.ksplit = ks;
  {   // LDS-DMA operand staging for full tiles (FM_GEMM_DMA=0: register staging)
    p.dma = fm_gemm_dma_enabled() && vec && M % BMv == 0 && N % BNv == 0 && K % BKF == 0 && K > 0;
  }
  g_last_form = BNv == 128 ? 1 : BMv == 128 ? 2 : 3;
  if (BNv == 128) launch_fbm<128, 128>(p, a_kcontig, b_kcontig, vec, stream);
  else if (BMv == 128) launch_fbm<128, 64>(p, a_kcontig, b_kcontig, vec, stream);
  else launch_fbm<64, 64>(p, a_kcontig, b_kcontig, vec, stream);
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
