// flexmi MFMA GEMM for gfx950 (MI355X / CDNA4).
//
//   C[M,N] (+)= epilogue( alpha * sum_k A(m,k) * B(k,n) )      bf16 inputs, fp32 accumulate
//
// Replaces the reference's cuBLAS Sgemm call sites (src/ops/linear.cu:432-441 fwd + bias,
// :616-634 dW/dX, src/ops/batch_matmul.cu:199-201, :349-354).  One kernel template covers every
// operand orientation the framework needs WITHOUT transposed copies:
//   * K-contiguous operand (A stored [M][K], B stored [N][K])  -> LDS image [row][k] (128-B rows,
//     16-B chunks XOR-swizzled by (row>>1)&7, conflict-free ds_read_b128 fragment reads);
//   * MN-contiguous operand (A stored [K][M], B stored [K][N]) -> LDS image [k][row], fragments
//     read with the CDNA4 transposing ds_read_b64_tr_b16 (chunk pairs XOR-swizzled per k-row so
//     each 32-lane half hits all 64 banks once).
// Tile: BM x BN x 64, 256 threads = 4 waves (2x2), each wave (BM/2)x(BN/2) of 16x16 tiles of
// v_mfma_f32_16x16x32_bf16.  LDS is double-buffered with register staging: the global loads of
// tile t+1 are issued before the MFMAs of tile t and written to the other LDS buffer after them
// (one barrier per K-tile).  The MFMA operands are swapped (B fragment as the MFMA "A") so each
// lane ends up owning 4 consecutive output COLUMNS -> 8-B/16-B vector stores in the epilogue.
// Epilogue: alpha, fp32 bias[n], activation (relu/sigmoid/tanh), beta=1 accumulate, bf16 or
// fp32 output.  Split-K writes fp32 slabs reduced by fm_gemm_splitk_reduce (same epilogue).
// Blocks are remapped so consecutive tiles share an XCD (private 4 MB L2 per XCD).
#include "gemm_common.h"

#include <algorithm>
#include <cstdlib>

extern "C" int fm_gemm_dma_enabled();   // gemm_f32.hip

namespace {

constexpr int NT = 256;

// ---- global -> registers (one tile of an operand) --------------------------------------
template <bool KC, int R, bool VEC, int NTH = NT>
struct Stage {
  static constexpr int CHUNKS = R * BK / 8;
  static constexpr int PER_T = CHUNKS / NTH;
  u32x4_t v[PER_T];

  FM_DEVICE void load(const unsigned short* __restrict__ p, long ld, int row0, int rows, int k0, int K, int tid) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      int ci = tid + NTH * i;
      int r, c, gr, gk;
      if constexpr (KC) {
        r = ci >> 3; c = ci & 7;
        gr = row0 + r; gk = k0 + 8 * c;
      } else {
        r = ci / (R / 8); c = ci % (R / 8);   // r = k row, c = chunk along rows
        gk = k0 + r; gr = row0 + 8 * c;
      }
      if constexpr (VEC) {
        bool ok = KC ? (gr < rows && gk < K) : (gk < K && gr < rows);
        if (ok) {
          const unsigned short* src = KC ? (p + (long)gr * ld + gk) : (p + (long)gk * ld + gr);
          v[i] = *reinterpret_cast<const u32x4_t*>(src);
        } else {
          v[i] = u32x4_t{0u, 0u, 0u, 0u};
        }
      } else {
        unsigned short e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          int rr = KC ? gr : gr + j;
          int kk = KC ? gk + j : gk;
          e[j] = (rr < rows && kk < K) ? (KC ? p[(long)rr * ld + kk] : p[(long)kk * ld + rr]) : (unsigned short)0;
        }
        v[i] = u32x4_t{(unsigned)e[0] | ((unsigned)e[1] << 16), (unsigned)e[2] | ((unsigned)e[3] << 16),
                       (unsigned)e[4] | ((unsigned)e[5] << 16), (unsigned)e[6] | ((unsigned)e[7] << 16)};
      }
    }
  }

  FM_DEVICE void store(char* lds, int tid) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      int ci = tid + NTH * i;
      int a, c;
      if constexpr (KC) { a = ci >> 3; c = ci & 7; }
      else { a = ci / (R / 8); c = ci % (R / 8); }
      *reinterpret_cast<u32x4_t*>(lds + lds_off<KC, R>(a, c)) = v[i];
    }
  }

  // MN-contiguous operand: every chunk a thread loads covers the SAME 8 rows (tid % (R/8)),
  // so summing the staged chunks over k gives per-row partial sums for free (bias gradient
  // db[n] = sum_b dpre[b][n] computed inside the dW GEMM, no extra pass over dpre).
  FM_DEVICE void accumulate_rows(float (&s)[8]) const {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      const unsigned w[4] = {v[i][0], v[i][1], v[i][2], v[i][3]};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s[2 * j] += bf2f((unsigned short)(w[j] & 0xFFFF));
        s[2 * j + 1] += bf2f((unsigned short)(w[j] >> 16));
      }
    }
  }
};

typedef __attribute__((address_space(1))) const void* gptr_b;
typedef __attribute__((address_space(3))) void* lptr_b;

// ---- global -> LDS by LDS-DMA (global_load_lds: no VGPR round trip, no ds_write) ------------
// One wave-instruction fills 1 KiB of the operand image: lane L's 16 B land at base + 16 L, so each
// lane loads the global chunk that the image's swizzle puts there (the inverse of lds_off).  Full
// tiles only (the caller guarantees M, N multiples of the tile, K of BK): no edge predication.
template <bool KC, int R, int NTH>
struct DmaStage {
  static constexpr int BYTES = R * BK * 2;
  static constexpr int PER_W = BYTES / 1024 / (NTH / 64);   // wave-instructions per wave
  static_assert(PER_W >= 1 && BYTES % (1024 * (NTH / 64)) == 0, "whole 1-KiB pieces per wave");
  FM_DEVICE static void issue(const unsigned short* __restrict__ p, long ld, int row0, int k0, char* lds, int wave,
                              int lane) {
#pragma unroll
    for (int i = 0; i < PER_W; ++i) {
      const int piece = wave * PER_W + i;
      const int o = piece * 1024 + 16 * lane;
      const unsigned short* src;
      if constexpr (KC) {
        const int row = o / (BK * 2), slot = (o % (BK * 2)) / 16;
        const int c = slot ^ ((row >> 1) & 7);
        src = p + (long)(row0 + row) * ld + k0 + 8 * c;
      } else {
        const int kr = o / (R * 2), slot = (o % (R * 2)) / 16;
        const int c = slot ^ MNSwz<R>::f(kr);
        src = p + (long)(k0 + kr) * ld + row0 + 8 * c;
      }
      __builtin_amdgcn_global_load_lds((gptr_b)(const void*)src, (lptr_b)(void*)(lds + piece * 1024), 16, 0, 0);
    }
  }
};

// NTH = 256: 4 waves (2x2, wave tile BM/2 x BN/2); 512: 8 waves (2x4 for BN >= 128, else 4x2).
// Fused-SGD epilogue of an unsplit dW tile, staged through LDS: the accumulator layout gives each
// lane 4 columns of one row, i.e. 64-B row pieces per 16x16 tile -- a scattered pattern that held the
// W read-modify-write (fp32 master + bf16 mirror, ~10 B per element) at ~2.8 TB/s.  The waves first
// park the BM x BN fp32 tile in the (free) operand LDS, 16-B chunks XOR-swizzled by row so both the
// accumulator writes and the row reads stay conflict-light, then every wave updates whole rows:
// BN*4 contiguous bytes of W per row (512 B for BN = 128).  The tile fits the K-loop LDS exactly
// (BM*BN*4 <= 2*(BM+BN)*BK*2).
template <int BM, int BN, int NTH, int MR, int NR>
FM_DEVICE void sgd_epilogue_lds(const GemmP& p, const f32x4_t (&acc)[MR][NR], char* smem, int m0, int n0, int mb,
                                int nb, int lane, int tid) {
  constexpr int CPR = BN / 4;                       // 16-B chunks per tile row
  static_assert(BM * BN * 4 <= 2 * (BM + BN) * BK * 2, "fp32 tile must fit the K-loop LDS");
  static_assert(CPR >= 8, "row XOR swizzle (r & 7) needs >= 8 chunks per row");
  f32x4_t* t = reinterpret_cast<f32x4_t*>(smem);
  __syncthreads();                                  // every wave is done with the operand tiles
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int r = mb + 16 * i + (lane & 15);
      const int c = (nb + 16 * j + 4 * (lane >> 4)) >> 2;
      t[r * CPR + (c ^ (r & 7))] = acc[i][j] * p.alpha;
    }
  __syncthreads();
  const bool n4 = (p.N & 3) == 0;
#pragma unroll 4
  for (int q = tid; q < BM * CPR; q += NTH) {
    const int r = q / CPR, c = q % CPR;
    const int m = m0 + r, n = n0 + 4 * c;
    if (m >= p.M || n >= p.N) continue;
    const f32x4_t g = t[r * CPR + (c ^ (r & 7))];
    const long o = (long)m * p.ldc + n;
    if (n4 && n + 3 < p.N) {
      sgd_apply4(p, o, g);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (n + e < p.N) sgd_apply1(p, o + e, g[e]);
    }
  }
}

template <int BM, int BN, bool AK, bool BKC, bool VEC, int NTH = NT, bool SGD = false, bool DMA = false>
__global__ void __launch_bounds__(NTH, 2) fm_gemm_kernel(GemmP p) {
  constexpr int A_BYTES = BM * BK * 2;
  constexpr int B_BYTES = BN * BK * 2;
  constexpr int WN = (NTH == 512 && BN >= 128) ? 4 : 2;
  constexpr int WM = NTH / 64 / WN;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MR = TM / 16;  // 16-row subtiles per wave
  constexpr int NR = TN / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // buffer b of operand X at smem + b*(A_BYTES+B_BYTES) (+A_BYTES for B)
#define LDS_A(b) (smem + (b) * (A_BYTES + B_BYTES))
#define LDS_B(b) (smem + (b) * (A_BYTES + B_BYTES) + A_BYTES)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  // XCD-aware bijective remap of the tile id (blocks b and b+8 share an XCD)
  const int bid = xcd_remap(blockIdx.x, p.tiles_m * p.tiles_n);
  int tm, tn;
  tile_coords(p, bid, tm, tn);
  const int zb = blockIdx.y;           // batch
  const int split = blockIdx.z;
  const int m0 = tm * BM, n0 = tn * BN;

  const unsigned short* A = p.A + (long)zb * p.sA;
  const unsigned short* B = p.B + (long)zb * p.sB;

  const int ktiles_total = (p.K + BK - 1) / BK;
  const int kt_per = (ktiles_total + p.ksplit - 1) / p.ksplit;
  const int kt0 = split * kt_per;
  const int kt1 = min(ktiles_total, kt0 + kt_per);

  f32x4_t acc[MR][NR];
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  Stage<AK, BM, VEC, NTH> sa;
  Stage<BKC, BN, VEC, NTH> sb;
  const bool rowsum = (!AK) && (p.rowsum_a != nullptr) && (tn == 0);
  float rs[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // DMA: LDS-DMA staging (full tiles; row sums read back from the image): step kt+1's 1-KiB pieces are issued into the
  // free stage before step kt's MFMAs and waited for (vmcnt 0) before the barrier that publishes
  // them -- no VGPR round trip, no ds_write (the register-staged form's 64 KiB of ds_write_b128 per
  // CU and k-step run at ~79 B/clk beside 192 KiB of fragment reads: the LDS, not the MFMA, set
  // its step time).  8192x1024x1024: fwd 30.7 -> 24.5, dX 31.9 -> 27.8, dW 35.3 -> 30.6 us
  // (profiles/gemm_bf16_dma_ab_r6.txt).
  auto stage_dma = [&](int kt, int b) {
    DmaStage<AK, BM, NTH>::issue(A, p.lda, m0, kt * BK, LDS_A(b), wave, lane);
    DmaStage<BKC, BN, NTH>::issue(B, p.ldb, n0, kt * BK, LDS_B(b), wave, lane);
  };
  if (kt0 < kt1) {
    if constexpr (DMA) {
      stage_dma(kt0, 0);
      __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    } else {
      sa.load(A, p.lda, m0, p.M, kt0 * BK, p.K, tid);
      sb.load(B, p.ldb, n0, p.N, kt0 * BK, p.K, tid);
      sa.store(LDS_A(0), tid);
      sb.store(LDS_B(0), tid);
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
        sa.load(A, p.lda, m0, p.M, (kt + 1) * BK, p.K, tid);
        sb.load(B, p.ldb, n0, p.N, (kt + 1) * BK, p.K, tid);
      }
    }
    const char* la = LDS_A(cur);
    const char* lb = LDS_B(cur);
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8_t af[MR], bfr[NR];
#pragma unroll
      for (int i = 0; i < MR; ++i) af[i] = frag<AK, BM>(la, wm * TM + 16 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < NR; ++j) bfr[j] = frag<BKC, BN>(lb, wn * TN + 16 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<bf16x8v_t*>(&bfr[j]),
                                                              *reinterpret_cast<bf16x8v_t*>(&af[i]),
                                                              acc[i][j], 0, 0, 0);
    }
    if constexpr (DMA) {
      if constexpr (!AK) {   // bias-gradient row sums from the DMA-staged image (the register form's chunks)
        if (rowsum) {
#pragma unroll
          for (int i = 0; i < Stage<AK, BM, VEC, NTH>::PER_T; ++i) {
            const int ci = tid + NTH * i;
            const u32x4_t w = *reinterpret_cast<const u32x4_t*>(la + lds_off<false, BM>(ci / (BM / 8), ci % (BM / 8)));
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              rs[2 * j] += bf2f((unsigned short)(w[j] & 0xFFFF));
              rs[2 * j + 1] += bf2f((unsigned short)(w[j] >> 16));
            }
          }
        }
      }
      __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): this wave's pieces of step kt+1 landed
    } else if (more) {
      sa.store(LDS_A(cur ^ 1), tid);
      sb.store(LDS_B(cur ^ 1), tid);
      if (rowsum) sa.accumulate_rows(rs);
    }
    __syncthreads();
  }
  if constexpr (!AK) {
    if (rowsum) {  // reduce the NT/(BM/8) threads that share each 8-row group, then 1 atomic per row
      float* red = reinterpret_cast<float*>(smem);   // LDS is free after the K loop
      constexpr int G = BM / 8;                      // row groups
#pragma unroll
      for (int j = 0; j < 8; ++j) red[(tid / G) * BM + (tid % G) * 8 + j] = rs[j];
      __syncthreads();
      if (tid < BM) {
        float x = 0.f;
        for (int t = 0; t < NTH / G; ++t) x += red[t * BM + tid];
        if (m0 + tid < p.M) atomicAdd(p.rowsum_a + m0 + tid, x);
      }
      __syncthreads();
    }
  }

#undef LDS_A
#undef LDS_B
  if constexpr (SGD) {
    if (p.ksplit == 1 && p.ulds) {
      sgd_epilogue_lds<BM, BN, NTH, MR, NR>(p, acc, smem, m0, n0, wm * TM, wn * TN, lane, tid);
      return;
    }
  }
  gemm_epilogue<MR, NR, SGD>(p, acc, zb, split, m0 + wm * TM, n0 + wn * TN, lane);
}

template <bool SGD>
__global__ void fm_gemm_splitk_reduce(GemmP p);

// 4 consecutive outputs per thread (16-B slab loads): N % 4 == 0, fp32 C with ldc % 4 == 0
template <bool SGD>
__global__ void fm_gemm_splitk_reduce4(GemmP p) {
  const long MN = (long)p.M * p.N;
  const long total4 = MN * p.batch / 4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total4; i += (long)gridDim.x * blockDim.x) {
    const long e4 = i * 4;
    const long zb = e4 / MN, e = e4 % MN;
    const int m = (int)(e / p.N), n = (int)(e % p.N);
    const float* src = p.ws + zb * p.ksplit * MN + e;
    f32x4_t s = slab_sum4(src, MN, p.ksplit);
    s *= p.alpha;
    if constexpr (SGD) {
      sgd_apply4(p, (long)m * p.ldc + n, s);
      continue;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) s[r] = act_fwd(p.act, s[r] + (p.bias ? p.bias[n + r] : 0.f));
    f32x4_t* d = reinterpret_cast<f32x4_t*>(reinterpret_cast<float*>(p.C) + zb * p.sC + (long)m * p.ldc + n);
    if (p.beta) s += *d;
    *d = s;
  }
}

}  // namespace


namespace {

void launch_splitk_reduce(const GemmP& p, hipStream_t stream) {
  const long total = (long)p.M * p.N * p.batch;
  const bool v4 = p.c_fp32 && (p.N % 4 == 0) && (p.ldc % 4 == 0) && (p.sC % 4 == 0) &&
                  ((((uintptr_t)p.C) & 15) == 0);
  if (p.uw) {
    if (v4) hipLaunchKernelGGL(fm_gemm_splitk_reduce4<true>, dim3(fm_grid(total / 4)), dim3(256), 0, stream, p);
    else hipLaunchKernelGGL(fm_gemm_splitk_reduce<true>, dim3(fm_grid(total)), dim3(256), 0, stream, p);
  } else {
    if (v4) hipLaunchKernelGGL(fm_gemm_splitk_reduce4<false>, dim3(fm_grid(total / 4)), dim3(256), 0, stream, p);
    else hipLaunchKernelGGL(fm_gemm_splitk_reduce<false>, dim3(fm_grid(total)), dim3(256), 0, stream, p);
  }
}

template <bool SGD>
__global__ void fm_gemm_splitk_reduce(GemmP p) {
  const long MN = (long)p.M * p.N;
  const long total = MN * p.batch;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    long zb = i / MN, e = i % MN;
    int m = (int)(e / p.N), n = (int)(e % p.N);
    const float* src = p.ws + zb * p.ksplit * MN + e;
    float s = slab_sum1(src, MN, p.ksplit);
    float v = s * p.alpha;
    if constexpr (SGD) {
      sgd_apply1(p, (long)m * p.ldc + n, v);
      continue;
    }
    if (p.bias) v += p.bias[n];
    v = act_fwd(p.act, v);
    long ci = zb * p.sC + (long)m * p.ldc + n;
    if (p.c_fp32) {
      float* d = reinterpret_cast<float*>(p.C) + ci;
      *d = v + (p.beta ? *d : 0.f);
    } else {
      unsigned short* d = reinterpret_cast<unsigned short*>(p.C) + ci;
      *d = f2bf(v + (p.beta ? bf2f(*d) : 0.f));
    }
  }
}

// split-K reduce with the FUSED BACKWARD epilogue (bf16 act_y): v = act_bwd(bact, ay, act(alpha*sum +
// bias)), colsum[n] += column sums of v.  Thread = 4 columns x RB rows (one atomic per column and
// block); lets small-batch dX GEMMs split K (summit_large 256 x 4096 x 4096).
__global__ void __launch_bounds__(256) fm_gemm_splitk_reduce_bwd(GemmP p, int RB) {
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
    const long ci = (long)m * p.ldc + n;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (n + r >= p.N) break;
      float v = act_fwd(p.act, sv[r] * p.alpha + (p.bias ? p.bias[n + r] : 0.f));
      if (p.ay) v = act_bwd(p.bact, bf2f(p.ay[(long)m * p.lday + n + r]), v);
      cs[r] += v;                               // as the in-tile epilogue: the unrounded value
      if (p.c_fp32) {
        float* d = reinterpret_cast<float*>(p.C) + ci + r;
        *d = v + (p.beta ? *d : 0.f);
      } else {
        unsigned short* d = reinterpret_cast<unsigned short*>(p.C) + ci + r;
        *d = f2bf(v + (p.beta ? bf2f(*d) : 0.f));
      }
    }
  }
  if (p.colsum) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (n + r < p.N) atomicAdd(p.colsum + n + r, cs[r]);
  }
}

template <int BM, int BN, bool AK, bool BKC, bool VEC>
void launch_t(const GemmP& p, hipStream_t s) {
  constexpr int LDS = 2 * (BM + BN) * BK * 2;
  dim3 grid(p.tiles_m * p.tiles_n, p.batch, p.ksplit);
  if constexpr (!AK && !BKC) {   // fused-SGD dW GEMMs (both operands MN-contiguous): own instantiation
    if (p.uw) {
      if constexpr (VEC && BM == 128) {
        if (p.dma) hipLaunchKernelGGL((fm_gemm_kernel<BM, BN, AK, BKC, VEC, 512, true, true>), grid, dim3(512), LDS, s, p);
        else hipLaunchKernelGGL((fm_gemm_kernel<BM, BN, AK, BKC, VEC, 512, true>), grid, dim3(512), LDS, s, p);
        return;
      }
      hipLaunchKernelGGL((fm_gemm_kernel<BM, BN, AK, BKC, VEC, NT, true>), grid, dim3(NT), LDS, s, p);
      return;
    }
  }
  // the 8-wave form of the 128-row tiles (4 waves per SIMD hide the per-K-tile barrier and
  // fragment latency: DLRM GEMMs -6 %, bf16 step 0.673 -> 0.626 ms, profiles/gemm_bf16_8wave_ab.jsonl)
  if constexpr (VEC && BM == 128) {
    if (p.dma) hipLaunchKernelGGL((fm_gemm_kernel<BM, BN, AK, BKC, VEC, 512, false, true>), grid, dim3(512), LDS, s, p);
    else hipLaunchKernelGGL((fm_gemm_kernel<BM, BN, AK, BKC, VEC, 512>), grid, dim3(512), LDS, s, p);
    return;
  }
  if constexpr (VEC) {
    if (p.dma) {
      hipLaunchKernelGGL((fm_gemm_kernel<BM, BN, AK, BKC, VEC, NT, false, true>), grid, dim3(NT), LDS, s, p);
      return;
    }
  }
  hipLaunchKernelGGL((fm_gemm_kernel<BM, BN, AK, BKC, VEC>), grid, dim3(NT), LDS, s, p);
}

template <int BM, int BN>
void launch_bm(const GemmP& p, bool ak, bool bk, bool vec, hipStream_t s) {
  if (vec) {
    if (ak && bk) launch_t<BM, BN, true, true, true>(p, s);
    else if (ak && !bk) launch_t<BM, BN, true, false, true>(p, s);
    else if (!ak && bk) launch_t<BM, BN, false, true, true>(p, s);
    else launch_t<BM, BN, false, false, true>(p, s);
  } else {
    if (ak && bk) launch_t<BM, BN, true, true, false>(p, s);
    else if (ak && !bk) launch_t<BM, BN, true, false, false>(p, s);
    else if (!ak && bk) launch_t<BM, BN, false, true, false>(p, s);
    else launch_t<BM, BN, false, false, false>(p, s);
  }
}

}  // namespace

// A_kcontig: A stored [M][K] (lda >= K) else [K][M] (lda >= M)
// B_kcontig: B stored [N][K] (ldb >= K) else [K][N] (ldb >= N)
struct SgdUpd {
  float* w; unsigned short* wc; float* v; const float* lr; float wd, mom; int nest;
};

static int gemm_run(const void* A, long lda, long sA, int a_kcontig,
                    const void* B, long ldb, long sB, int b_kcontig,
                    void* C, long ldc, long sC, int c_fp32,
                    const float* bias, int M, int N, int K, int batch,
                    float alpha, int beta, int act, float* ws, long ws_bytes, int ksplit_req,
                    const void* act_y, long lday, int bwd_act, float* colsum, float* rowsum_a,
                    const SgdUpd* upd, hipStream_t stream);

extern "C" int fm_gemm(const void* A, long lda, long sA, int a_kcontig,
                       const void* B, long ldb, long sB, int b_kcontig,
                       void* C, long ldc, long sC, int c_fp32,
                       const float* bias, int M, int N, int K, int batch,
                       float alpha, int beta, int act, float* ws, long ws_bytes, int ksplit_req,
                       const void* act_y, long lday, int bwd_act, float* colsum, float* rowsum_a,
                       hipStream_t stream) {
  return gemm_run(A, lda, sA, a_kcontig, B, ldb, sB, b_kcontig, C, ldc, sC, c_fp32, bias, M, N, K, batch, alpha, beta,
                  act, ws, ws_bytes, ksplit_req, act_y, lday, bwd_act, colsum, rowsum_a, nullptr, stream);
}

// Weight-gradient GEMM with the SGD update fused into its epilogue (or its split-K reduce):
// W[M][ldw] -= lr * (A^T B + wd W) (momentum / Nesterov as fm_sgd_update), bf16 mirror Wc
// rewritten; the gradient itself is never stored.  A = dpre [K][M], B = x [K][N] (MN-contiguous,
// the dW orientation), rowsum_a += column sums of dpre (the bias gradient).  Returns the split.
extern "C" int fm_gemm_dw_sgd(const void* A, long lda, const void* B, long ldb, float* W, long ldw,
                              unsigned short* Wc, float* V, const float* lr, float wd, float mom, int nesterov,
                              int M, int N, int K, float* ws, long ws_bytes, float* rowsum_a, int cfg,
                              hipStream_t stream) {
  SgdUpd u{W, Wc, V, lr, wd, mom, nesterov};
  return gemm_run(A, lda, 0, 0, B, ldb, 0, 0, W, ldw, 0, 1, nullptr, M, N, K, 1, 1.f, 0, 10, ws, ws_bytes, cfg, nullptr,
                  0, 10, nullptr, rowsum_a, &u, stream);
}

static int gemm_run(const void* A, long lda, long sA, int a_kcontig,
                    const void* B, long ldb, long sB, int b_kcontig,
                    void* C, long ldc, long sC, int c_fp32,
                    const float* bias, int M, int N, int K, int batch,
                    float alpha, int beta, int act, float* ws, long ws_bytes, int ksplit_req,
                    const void* act_y, long lday, int bwd_act, float* colsum, float* rowsum_a,
                    const SgdUpd* upd, hipStream_t stream) {
  if (M <= 0 || N <= 0 || batch <= 0) return 0;
  if (upd && (K <= 0 || ldc % 4 != 0 || (((uintptr_t)upd->w | (uintptr_t)(upd->v ? upd->v : upd->w)) & 15) ||
              (((uintptr_t)(upd->wc ? (void*)upd->wc : (void*)upd->w)) & 7)))
    return -1;                         // the caller computes the gradient and runs the update itself
  GemmP p;
  p.A = (const unsigned short*)A; p.lda = lda; p.sA = sA;
  p.B = (const unsigned short*)B; p.ldb = ldb; p.sB = sB;
  p.C = C; p.ldc = ldc; p.sC = sC;
  p.bias = bias; p.M = M; p.N = N; p.K = K; p.act = act; p.beta = beta; p.c_fp32 = c_fp32;
  p.alpha = alpha; p.batch = batch; p.ws = ws;
  p.ay = (const unsigned short*)act_y; p.lday = lday; p.bact = bwd_act; p.colsum = colsum; p.rowsum_a = rowsum_a;
  p.n_fast = M >= N;
  p.uw = upd ? upd->w : nullptr;
  p.uwc = upd ? upd->wc : nullptr;
  p.uv = upd ? upd->v : nullptr;
  p.ulr = upd ? upd->lr : nullptr;
  p.uwd = upd ? upd->wd : 0.f;
  p.umom = upd ? upd->mom : 0.f;
  p.unest = upd ? upd->nest : 0;
  p.ulds = upd != nullptr;   // the update staged through LDS (whole-row W accesses, gemm.hip sgd_epilogue_lds)
  // vector (16-B) loads need the contiguous extent and leading dims to be multiples of 8
  auto al = [](const void* q) { return (((uintptr_t)q) & 15) == 0; };
  bool vec = al(A) && al(B) && (lda % 8 == 0) && (ldb % 8 == 0) && (sA % 8 == 0) && (sB % 8 == 0);
  vec = vec && (a_kcontig ? (K % 8 == 0) : (M % 8 == 0)) && (b_kcontig ? (K % 8 == 0) : (N % 8 == 0));
  // ksplit_req = ks | form << 8: a measured configuration (flexmi/ops/gemm_tune.py), form 1/2/3 =
  // 128x128 / 128x64 / 64x64 tiles, ks the split-K depth (0: the heuristic's); form 0: heuristic tile
  const int form = ksplit_req >> 8;
  ksplit_req &= 255;
  const bool fused_ok_split = ws != nullptr && batch == 1 && (long)M * N * 4 * 2 <= ws_bytes;
  // tile choice: 128x128 when it yields >= 2 waves of blocks on 256 CUs, else narrower N
  int BMv = 128, BNv = 128;
  long t128 = (long)((M + 127) / 128) * ((N + 127) / 128) * batch;
  if (t128 < 512 && N <= 64 * 8) BNv = 64;
  {   // small grids with short K (measured, tools/gemm_probe.py): 64x64 tiles keep >= 2 blocks
      // resident per CU where 128x64 gives at most one wave of blocks; long-K GEMMs (dW, K =
      // batch) keep the bigger tile and split K instead
    long t12864 = (long)((M + 127) / 128) * ((N + 63) / 64) * batch;
    if (BNv == 64 && t12864 <= 256 && K <= 1024) BMv = 64;
  }
  // few 128x128 tiles and a short K (small-batch layers, e.g. DLRM run_random at 256 samples
  // per GPU): 64x64 tiles give 4x the blocks without split-K slabs (measured +26 % step rate)
  if (t128 < 128 && K <= 2048) { BMv = 64; BNv = 64; }
  // a fused backward epilogue in the tile cannot split K: small grids with a long K split it and run
  // the epilogue in the reduce (fm_gemm_splitk_reduce_bwd), short ones take 64x64 tiles for 4x the
  // blocks (summit_large dX, 256 x 4096 x 4096)
  const bool fused_ep = act_y != nullptr || colsum != nullptr;
  const bool fused_split = fused_ep && t128 < 256 && K >= 1024 && ws != nullptr && batch == 1 && ksplit_req <= 0 &&
                           (long)M * N * 4 * 2 <= ws_bytes;
  if (fused_ep && t128 < 256 && !fused_split) { BMv = 64; BNv = 64; }
  if (form == 1) { BMv = 128; BNv = 128; }
  if (form == 2) { BMv = 128; BNv = 64; }
  if (form == 3) { BMv = 64; BNv = 64; }
  p.tiles_m = (M + BMv - 1) / BMv;
  p.tiles_n = (N + BNv - 1) / BNv;
  long tiles = (long)p.tiles_m * p.tiles_n * batch;
  int ktiles = (K + BK - 1) / BK;
  int ks = 1;
  if (ksplit_req > 0) ks = ksplit_req;
  else if (ws != nullptr) {
    // split until the grid reaches ~1.5 blocks per CU (measured on the DLRM step, 200-step runs:
    // target 256 -> 11.05, 384 -> 11.32, 512 -> 11.27, 1024 -> 9.81 M samples/s)
    // -- long-K (dW at large batch) only: short-K small-batch GEMMs keep 256 (DLRM run_random at
    // 256/GPU: 1.10 M samples/s at 256 vs 1.04 M at 384)
    const long target = K >= 4096 ? 384L : 256L;
    while (tiles * ks < target && ks * 2 <= ktiles / 2 && ks < 16) ks *= 2;
  }
  if (fused_ep && !(form ? fused_ok_split : fused_split)) ks = 1;  // fused bwd epilogue needs the full K sum
  ks = std::min(ks, std::max(1, ktiles));
  while (ks > 1 && (ws == nullptr || (long)batch * ks * M * (long)N * 4 > ws_bytes)) ks /= 2;
  p.ksplit = ks;
  if (K <= 0) {  // degenerate: C = epilogue(0)
    p.ksplit = 1;
  }
  {   // LDS-DMA staging for full tiles (FM_GEMM_DMA=0: register staging everywhere)
    p.dma = fm_gemm_dma_enabled() && vec && M % BMv == 0 && N % BNv == 0 && K % BK == 0 && K > 0;
  }
  const bool reduce_bwd = p.ksplit > 1 && fused_ep;
  if (BNv == 128) launch_bm<128, 128>(p, a_kcontig, b_kcontig, vec, stream);
  else if (BMv == 128) launch_bm<128, 64>(p, a_kcontig, b_kcontig, vec, stream);
  else launch_bm<64, 64>(p, a_kcontig, b_kcontig, vec, stream);
  if (reduce_bwd) {
    const int bx = (N + 1023) / 1024;
    const int by = std::max(1, std::min(M, 1024 / bx));
    const int RB = (M + by - 1) / by;
    hipLaunchKernelGGL(fm_gemm_splitk_reduce_bwd, dim3(bx, (M + RB - 1) / RB), dim3(256), 0, stream, p, RB);
  } else if (p.ksplit > 1) {
    launch_splitk_reduce(p, stream);
  }
  return p.ksplit;
}

// ------------------------------------------------------------------------------------------
// Skinny layers (out_features == 1, e.g. the DLRM click-probability layer): an MFMA tile would be
// 1/128 utilised and the transposed dW path degenerates to scalar loads, so these run as
// bandwidth-bound GEMV / outer-product / column-reduction kernels instead.
namespace {

__global__ void __launch_bounds__(256) fm_skinny_fwd_kernel(const unsigned short* __restrict__ x, long ldx,
                                                           const unsigned short* __restrict__ w,
                                                           const float* __restrict__ bias, unsigned short* __restrict__ y,
                                                           long ldy, long B, int K, int act) {
  const int lane = threadIdx.x & 63;
  const long waves = (long)gridDim.x * 4;
  const bool vec = (K % 4 == 0) && (ldx % 4 == 0);
  for (long b = blockIdx.x * 4 + (threadIdx.x >> 6); b < B; b += waves) {
    const unsigned short* xr = x + b * ldx;
    float s = 0.f;
    if (vec) {
      for (int k = lane * 4; k < K; k += 256) {
        bf16x4_t a = *reinterpret_cast<const bf16x4_t*>(xr + k);
        bf16x4_t c = *reinterpret_cast<const bf16x4_t*>(w + k);
#pragma unroll
        for (int j = 0; j < 4; ++j) s += bf2f((unsigned short)a[j]) * bf2f((unsigned short)c[j]);
      }
    } else {
      for (int k = lane; k < K; k += 64) s += bf2f(xr[k]) * bf2f(w[k]);
    }
    s = wave_reduce_sum(s);
    if (lane == 0) y[b * ldy] = f2bf(act_fwd(act, s + (bias ? bias[0] : 0.f)));
  }
}

__global__ void __launch_bounds__(256) fm_skinny_bwd_kernel(int ROWS, const unsigned short* __restrict__ x, long ldx,
                                                           const unsigned short* __restrict__ w,
                                                           const unsigned short* __restrict__ y, long ldy,
                                                           const unsigned short* __restrict__ dy, long lddy,
                                                           unsigned short* __restrict__ dx, long lddx, int dx_acc,
                                                           float* __restrict__ dw, float* __restrict__ db, long B, int K,
                                                           int act, int bact) {
  // bact: activation backward of the layer below applied to dX (see the fp32 kernel)
  // thread = 8 consecutive columns (16-B loads/stores) of rows sub, sub+rpi, ...; per-block
  // partial dW/db reduced in LDS -> one atomic per column per block (B/ROWS adders per address)
  __shared__ float red[256 * 8];
  __shared__ float redb[256];
  // column block blockIdx.y covers [2048 y, 2048 y + 2048) of K (host: K % 8 == 0)
  const int cb = blockIdx.y * 2048;
  const int Kc = min(2048, K - cb);
  const int lpr = Kc / 8;                         // threads per row
  const int rpi = 256 / lpr;
  const int sub = threadIdx.x / lpr, g = threadIdx.x - sub * lpr;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float dbs = 0.f;
  const long r0 = (long)blockIdx.x * ROWS;
  const int c0 = cb + g * 8;
  if (blockIdx.y) db = nullptr;                   // db accumulated once, by column block 0
  bf16x8_t wv = *reinterpret_cast<const bf16x8_t*>(w + c0);
  if (sub < rpi) {
    // 4 rows per iteration with every load issued first (clamped, unconditional): the per-row
    // y -> d -> FMA chain no longer pays one HBM round trip per row
    const long rend = min(B, r0 + ROWS);
    for (long r = r0 + sub; r < rend; r += 4L * rpi) {
      float yv[4], gv[4];
      bf16x8_t xv[4], old[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long rr = min(r + u * rpi, rend - 1);
        yv[u] = bf2f(y[rr * ldy]);
        gv[u] = bf2f(dy[rr * lddy]);
        xv[u] = *reinterpret_cast<const bf16x8_t*>(x + rr * ldx + c0);
        old[u] = (dx && dx_acc) ? *reinterpret_cast<const bf16x8_t*>(dx + rr * lddx + c0)
                                : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long rr = r + u * rpi;
        if (rr >= rend) break;
        const float d = act_bwd(act, yv[u], gv[u]);
        dbs += d;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += d * bf2f((unsigned short)xv[u][j]);
        if (dx) {
          bf16x8_t o;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float v = d * bf2f((unsigned short)wv[j]);
            if (dx_acc) v += bf2f((unsigned short)old[u][j]);
            if (bact != ACT_NONE) v = act_bwd(bact, bf2f((unsigned short)xv[u][j]), v);
            o[j] = (short)f2bf(v);
          }
          *reinterpret_cast<bf16x8_t*>(dx + rr * lddx + c0) = o;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[threadIdx.x * 8 + j] = (sub < rpi) ? acc[j] : 0.f;
  redb[threadIdx.x] = (sub < rpi && g == 0) ? dbs : 0.f;
  __syncthreads();
  for (int c = threadIdx.x; c < Kc; c += 256) {
    const int gg = c / 8, j = c % 8;
    float t = 0.f;
    for (int q = 0; q < rpi; ++q) t += red[(q * lpr + gg) * 8 + j];
    atomicAdd(dw + cb + c, t);
  }
  if (db && threadIdx.x == 0) {
    float t = 0.f;
    for (int q = 0; q < rpi; ++q) t += redb[q * lpr];
    atomicAdd(db, t);
  }
}

}  // namespace

extern "C" void fm_skinny_fwd(const void* x, long ldx, const void* w, const float* bias, void* y, long ldy, long B, int K,
                              int act, hipStream_t s) {
  if (B <= 0) return;
  hipLaunchKernelGGL(fm_skinny_fwd_kernel, dim3((unsigned)std::min<long>((B + 3) / 4, 4096)), dim3(256), 0, s,
                     (const unsigned short*)x, ldx, (const unsigned short*)w, bias, (unsigned short*)y, ldy, B, K, act);
}

// dW (fp32 [K]) and db (fp32 [1]) are ACCUMULATED (callers zero them); requires K % 8 == 0
extern "C" void fm_skinny_bwd(const void* x, long ldx, const void* w, const void* y, long ldy, const void* dy, long lddy,
                              void* dx, long lddx, int dx_acc, float* dw, float* db, long B, int K, int act, int bact,
                              hipStream_t s) {
  if (B <= 0) return;
  // rows per block: 64 gives 128 blocks at B=8192 (fills the chip, 128 adders per dW column);
  // small batches shrink it so there are still >= 128 blocks (B=256 -> 2 rows per block)
  int ROWS = 64;
  while (ROWS > 2 && (B + ROWS - 1) / ROWS < 128) ROWS /= 2;
  hipLaunchKernelGGL(fm_skinny_bwd_kernel, dim3((unsigned)((B + ROWS - 1) / ROWS), (unsigned)((K + 2047) / 2048)), dim3(256),
                     0, s, ROWS,
                     (const unsigned short*)x, ldx, (const unsigned short*)w, (const unsigned short*)y, ldy,
                     (const unsigned short*)dy, lddy, (unsigned short*)dx, lddx, dx_acc, dw, db, B, K, act, bact);
}
