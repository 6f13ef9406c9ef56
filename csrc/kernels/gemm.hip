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
#include "common.h"

namespace {

constexpr int BK = 64;
constexpr int NT = 256;

typedef __attribute__((address_space(3))) bf16x4_t lds_v4_t;

template <int R>
struct MNSwz;
template <>
struct MNSwz<128> {  // 256-B rows, 16 chunks
  static FM_DEVICE int f(int k) { return 2 * ((k & 3) | (((k >> 3) & 1) << 2)); }
};
template <>
struct MNSwz<64> {  // 128-B rows, 8 chunks
  static FM_DEVICE int f(int k) { return 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1)); }
};

// byte offset inside an operand LDS image
template <bool KC, int R>
FM_DEVICE int lds_off(int row_or_k, int chunk) {
  if constexpr (KC) {
    return row_or_k * (BK * 2) + 16 * (chunk ^ ((row_or_k >> 1) & 7));
  } else {
    return row_or_k * (R * 2) + 16 * (chunk ^ MNSwz<R>::f(row_or_k));
  }
}

// ---- global -> registers (one tile of an operand) --------------------------------------
template <bool KC, int R, bool VEC>
struct Stage {
  static constexpr int CHUNKS = R * BK / 8;
  static constexpr int PER_T = CHUNKS / NT;
  u32x4_t v[PER_T];

  FM_DEVICE void load(const unsigned short* __restrict__ p, long ld, int row0, int rows, int k0, int K, int tid) {
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
      int ci = tid + NT * i;
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
      int ci = tid + NT * i;
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

// ---- LDS -> MFMA fragment (8 bf16: k = 8*(lane>>4)+j for row/col lane&15) -------------
template <bool KC, int R>
FM_DEVICE bf16x8_t frag(const char* lds, int base, int kk, int lane) {
  if constexpr (KC) {
    int row = base + (lane & 15);
    int chunk = 4 * kk + (lane >> 4);
    return *reinterpret_cast<const bf16x8_t*>(lds + lds_off<true, R>(row, chunk));
  } else {
    int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    int chunk = (base >> 3) + (p >> 1);
    int k0 = 32 * kk + 8 * g + q;
    int o0 = lds_off<false, R>(k0, chunk) + 8 * (p & 1);
    int o1 = lds_off<false, R>(k0 + 4, chunk) + 8 * (p & 1);
    bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4_t*)(lds + o0));
    bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4_t*)(lds + o1));
    bf16x8_t r;
    r.lo = lo;
    r.hi = hi;
    return r;
  }
}

struct GemmP {
  const unsigned short* A; long lda; long sA;
  const unsigned short* B; long ldb; long sB;
  void* C; long ldc; long sC;
  const float* bias;
  float* ws;          // split-K slabs [batch][split][M][N]
  // fused backward epilogue of the producing layer below: v = act'(ay) * v ; colsum[n] += sum_m v
  const unsigned short* ay;
  long lday;
  float* colsum;
  float* rowsum_a;   // += sum_k A(m,k)  (MN-contiguous A only; used for bias grads in dW GEMMs)
  int bact;
  int M, N, K, act, beta, c_fp32, ksplit, batch;
  float alpha;
  int tiles_m, tiles_n;
};

template <int BM, int BN, bool AK, bool BKC, bool VEC>
__global__ void __launch_bounds__(NT, 2) fm_gemm_kernel(GemmP p) {
  constexpr int A_BYTES = BM * BK * 2;
  constexpr int B_BYTES = BN * BK * 2;
  constexpr int MR = BM / 32;  // 16-row subtiles per wave (wave covers BM/2)
  constexpr int NR = BN / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // buffer b of operand X at smem + b*(A_BYTES+B_BYTES) (+A_BYTES for B)
#define LDS_A(b) (smem + (b) * (A_BYTES + B_BYTES))
#define LDS_B(b) (smem + (b) * (A_BYTES + B_BYTES) + A_BYTES)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-aware bijective remap of the tile id (blocks b and b+8 share an XCD)
  const int ntiles = p.tiles_m * p.tiles_n;
  int bid = blockIdx.x;
  {
    int q = ntiles / 8, r = ntiles % 8, x = bid % 8;
    if (ntiles >= 8) bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
  }
  const int tm = bid % p.tiles_m, tn = bid / p.tiles_m;
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

  Stage<AK, BM, VEC> sa;
  Stage<BKC, BN, VEC> sb;
  const bool rowsum = (!AK) && (p.rowsum_a != nullptr) && (tn == 0);
  float rs[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (kt0 < kt1) {
    sa.load(A, p.lda, m0, p.M, kt0 * BK, p.K, tid);
    sb.load(B, p.ldb, n0, p.N, kt0 * BK, p.K, tid);
    sa.store(LDS_A(0), tid);
    sb.store(LDS_B(0), tid);
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
    const char* la = LDS_A(cur);
    const char* lb = LDS_B(cur);
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8_t af[MR], bfr[NR];
#pragma unroll
      for (int i = 0; i < MR; ++i) af[i] = frag<AK, BM>(la, wm * (BM / 2) + 16 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < NR; ++j) bfr[j] = frag<BKC, BN>(lb, wn * (BN / 2) + 16 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < MR; ++i)
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<bf16x8v_t*>(&bfr[j]),
                                                              *reinterpret_cast<bf16x8v_t*>(&af[i]),
                                                              acc[i][j], 0, 0, 0);
    }
    if (more) {
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
        for (int t = 0; t < NT / G; ++t) x += red[t * BM + tid];
        if (m0 + tid < p.M) atomicAdd(p.rowsum_a + m0 + tid, x);
      }
      __syncthreads();
    }
  }

#undef LDS_A
#undef LDS_B
  // ---- epilogue: lane owns C[m][n..n+3], m = lane&15, n = 4*(lane>>4) ------------------
  const int mrow = lane & 15;
  const int ncol = 4 * (lane >> 4);
  if (p.ksplit > 1) {
    float* ws = p.ws + ((long)zb * p.ksplit + split) * (long)p.M * p.N;
#pragma unroll
    for (int i = 0; i < MR; ++i)
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        int m = m0 + wm * (BM / 2) + 16 * i + mrow;
        int n = n0 + wn * (BN / 2) + 16 * j + ncol;
        if (m >= p.M) continue;
        float* dst = ws + (long)m * p.N + n;
        if (n + 3 < p.N && (p.N & 3) == 0) {
          *reinterpret_cast<f32x4_t*>(dst) = acc[i][j];
        } else {
          for (int r = 0; r < 4; ++r)
            if (n + r < p.N) dst[r] = acc[i][j][r];
        }
      }
    return;
  }
  float csum[NR][4];
#pragma unroll
  for (int j = 0; j < NR; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) csum[j][r] = 0.f;
#pragma unroll
  for (int i = 0; i < MR; ++i)
#pragma unroll
    for (int j = 0; j < NR; ++j) {
      const int m = m0 + wm * (BM / 2) + 16 * i + mrow;
      const int n = n0 + wn * (BN / 2) + 16 * j + ncol;
      const bool mok = m < p.M;
      const bool full = (n + 3 < p.N);
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] * p.alpha;
      if (p.bias) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += (n + r < p.N) ? p.bias[n + r] : 0.f;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = act_fwd(p.act, v[r]);
      if (p.ay) {  // fused activation backward of the layer below (dX -> dpre)
        float yv[4] = {0.f, 0.f, 0.f, 0.f};
        if (mok) {
          const unsigned short* yp = p.ay + (long)m * p.lday + n;
          if (full && ((p.lday & 3) == 0)) {
            bf16x4_t t = *reinterpret_cast<const bf16x4_t*>(yp);
#pragma unroll
            for (int r = 0; r < 4; ++r) yv[r] = bf2f((unsigned short)t[r]);
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) yv[r] = (n + r < p.N) ? bf2f(yp[r]) : 0.f;
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = act_bwd(p.bact, yv[r], v[r]);
      }
      if (p.colsum && mok) {
#pragma unroll
        for (int r = 0; r < 4; ++r) csum[j][r] += (n + r < p.N) ? v[r] : 0.f;
      }
      if (!mok) continue;
      if (p.c_fp32) {
        float* dst = reinterpret_cast<float*>(p.C) + (long)zb * p.sC + (long)m * p.ldc + n;
        if (full && ((p.ldc & 3) == 0) && ((((uintptr_t)dst) & 15) == 0)) {
          f32x4_t o = {v[0], v[1], v[2], v[3]};
          if (p.beta) o += *reinterpret_cast<f32x4_t*>(dst);
          *reinterpret_cast<f32x4_t*>(dst) = o;
        } else {
          for (int r = 0; r < 4; ++r)
            if (n + r < p.N) dst[r] = v[r] + (p.beta ? dst[r] : 0.f);
        }
      } else {
        unsigned short* dst = reinterpret_cast<unsigned short*>(p.C) + (long)zb * p.sC + (long)m * p.ldc + n;
        if (full && ((p.ldc & 3) == 0) && ((((uintptr_t)dst) & 7) == 0)) {
          if (p.beta) {
            bf16x4_t old = *reinterpret_cast<bf16x4_t*>(dst);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += bf2f((unsigned short)old[r]);
          }
          bf16x4_t o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(v[r]);
          *reinterpret_cast<bf16x4_t*>(dst) = o;
        } else {
          for (int r = 0; r < 4; ++r)
            if (n + r < p.N) dst[r] = f2bf(v[r] + (p.beta ? bf2f(dst[r]) : 0.f));
        }
      }
    }
  if (p.colsum) {  // bias gradient of the layer below: reduce the 16 rows of each lane group, 1 atomic/col
#pragma unroll
    for (int j = 0; j < NR; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float x = csum[j][r];
        x += __shfl_xor(x, 1, 64);
        x += __shfl_xor(x, 2, 64);
        x += __shfl_xor(x, 4, 64);
        x += __shfl_xor(x, 8, 64);
        const int n = n0 + wn * (BN / 2) + 16 * j + ncol + r;
        if (mrow == 0 && n < p.N) atomicAdd(p.colsum + n, x);
      }
  }
}

__global__ void fm_gemm_splitk_reduce(GemmP p) {
  const long MN = (long)p.M * p.N;
  const long total = MN * p.batch;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    long zb = i / MN, e = i % MN;
    int m = (int)(e / p.N), n = (int)(e % p.N);
    const float* src = p.ws + zb * p.ksplit * MN + e;
    float s = 0.f;
    for (int k = 0; k < p.ksplit; ++k) s += src[k * MN];
    float v = s * p.alpha;
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

template <int BM, int BN, bool AK, bool BKC, bool VEC>
void launch_t(const GemmP& p, hipStream_t s) {
  constexpr int LDS = 2 * (BM + BN) * BK * 2;
  dim3 grid(p.tiles_m * p.tiles_n, p.batch, p.ksplit);
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
extern "C" int fm_gemm(const void* A, long lda, long sA, int a_kcontig,
                       const void* B, long ldb, long sB, int b_kcontig,
                       void* C, long ldc, long sC, int c_fp32,
                       const float* bias, int M, int N, int K, int batch,
                       float alpha, int beta, int act, float* ws, long ws_bytes, int ksplit_req,
                       const void* act_y, long lday, int bwd_act, float* colsum, float* rowsum_a,
                       hipStream_t stream) {
  if (M <= 0 || N <= 0 || batch <= 0) return 0;
  GemmP p;
  p.A = (const unsigned short*)A; p.lda = lda; p.sA = sA;
  p.B = (const unsigned short*)B; p.ldb = ldb; p.sB = sB;
  p.C = C; p.ldc = ldc; p.sC = sC;
  p.bias = bias; p.M = M; p.N = N; p.K = K; p.act = act; p.beta = beta; p.c_fp32 = c_fp32;
  p.alpha = alpha; p.batch = batch; p.ws = ws;
  p.ay = (const unsigned short*)act_y; p.lday = lday; p.bact = bwd_act; p.colsum = colsum; p.rowsum_a = rowsum_a;
  // vector (16-B) loads need the contiguous extent and leading dims to be multiples of 8
  auto al = [](const void* q) { return (((uintptr_t)q) & 15) == 0; };
  bool vec = al(A) && al(B) && (lda % 8 == 0) && (ldb % 8 == 0) && (sA % 8 == 0) && (sB % 8 == 0);
  vec = vec && (a_kcontig ? (K % 8 == 0) : (M % 8 == 0)) && (b_kcontig ? (K % 8 == 0) : (N % 8 == 0));
  // tile choice: 128x128 when it yields >= 2 waves of blocks on 256 CUs, else narrower N
  int BMv = 128, BNv = 128;
  long t128 = (long)((M + 127) / 128) * ((N + 127) / 128) * batch;
  if (t128 < 512 && N <= 64 * 8) BNv = 64;
  p.tiles_m = (M + BMv - 1) / BMv;
  p.tiles_n = (N + BNv - 1) / BNv;
  long tiles = (long)p.tiles_m * p.tiles_n * batch;
  int ktiles = (K + BK - 1) / BK;
  int ks = 1;
  if (ksplit_req > 0) ks = ksplit_req;
  else if (ws != nullptr) {
    while (tiles * ks < 256 && ks * 2 <= ktiles / 2 && ks < 16) ks *= 2;
  }
  if (act_y != nullptr || colsum != nullptr) ks = 1;  // fused bwd epilogue needs the full K sum
  if (ks > 1) {
    long need = (long)batch * ks * M * (long)N * 4;
    if (ws == nullptr || need > ws_bytes) ks = 1;
  }
  p.ksplit = ks;
  if (K <= 0) {  // degenerate: C = epilogue(0)
    p.ksplit = 1;
  }
  if (BNv == 128) launch_bm<128, 128>(p, a_kcontig, b_kcontig, vec, stream);
  else launch_bm<128, 64>(p, a_kcontig, b_kcontig, vec, stream);
  if (p.ksplit > 1) {
    long total = (long)M * N * batch;
    hipLaunchKernelGGL(fm_gemm_splitk_reduce, dim3(fm_grid(total)), dim3(256), 0, stream, p);
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

template <int ROWS>
__global__ void __launch_bounds__(256) fm_skinny_bwd_kernel(const unsigned short* __restrict__ x, long ldx,
                                                           const unsigned short* __restrict__ w,
                                                           const unsigned short* __restrict__ y, long ldy,
                                                           const unsigned short* __restrict__ dy, long lddy,
                                                           unsigned short* __restrict__ dx, long lddx, int dx_acc,
                                                           float* __restrict__ dw, float* __restrict__ db, long B, int K,
                                                           int act) {
  // thread = 8 consecutive columns (16-B loads/stores) of rows sub, sub+rpi, ...; per-block
  // partial dW/db reduced in LDS -> one atomic per column per block (B/ROWS adders per address)
  __shared__ float red[256 * 8];
  __shared__ float redb[256];
  const int groups = K / 8;                       // host guarantees K % 8 == 0, K <= 2048
  const int lpr = groups;                         // threads per row
  const int rpi = 256 / lpr;
  const int sub = threadIdx.x / lpr, g = threadIdx.x - sub * lpr;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float dbs = 0.f;
  const long r0 = (long)blockIdx.x * ROWS;
  const int c0 = g * 8;
  bf16x8_t wv = *reinterpret_cast<const bf16x8_t*>(w + c0);
  if (sub < rpi) {
    for (long r = r0 + sub; r < min(B, r0 + ROWS); r += rpi) {
      const float d = act_bwd(act, bf2f(y[r * ldy]), bf2f(dy[r * lddy]));
      dbs += d;
      bf16x8_t xv = *reinterpret_cast<const bf16x8_t*>(x + r * ldx + c0);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += d * bf2f((unsigned short)xv[j]);
      if (dx) {
        unsigned short* dp = dx + r * lddx + c0;
        bf16x8_t o;
        bf16x8_t old = dx_acc ? *reinterpret_cast<const bf16x8_t*>(dp) : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float v = d * bf2f((unsigned short)wv[j]);
          if (dx_acc) v += bf2f((unsigned short)old[j]);
          o[j] = (short)f2bf(v);
        }
        *reinterpret_cast<bf16x8_t*>(dp) = o;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[threadIdx.x * 8 + j] = (sub < rpi) ? acc[j] : 0.f;
  redb[threadIdx.x] = (sub < rpi && g == 0) ? dbs : 0.f;
  __syncthreads();
  for (int c = threadIdx.x; c < K; c += 256) {
    const int gg = c / 8, j = c % 8;
    float t = 0.f;
    for (int q = 0; q < rpi; ++q) t += red[(q * lpr + gg) * 8 + j];
    atomicAdd(dw + c, t);
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

// dW (fp32 [K]) and db (fp32 [1]) are ACCUMULATED (callers zero them); requires K <= 2048
extern "C" void fm_skinny_bwd(const void* x, long ldx, const void* w, const void* y, long ldy, const void* dy, long lddy,
                              void* dx, long lddx, int dx_acc, float* dw, float* db, long B, int K, int act, hipStream_t s) {
  if (B <= 0) return;
  constexpr int ROWS = 256;
  hipLaunchKernelGGL((fm_skinny_bwd_kernel<ROWS>), dim3((unsigned)((B + ROWS - 1) / ROWS)), dim3(256), 0, s,
                     (const unsigned short*)x, ldx, (const unsigned short*)w, (const unsigned short*)y, ldy,
                     (const unsigned short*)dy, lddy, (unsigned short*)dx, lddx, dx_acc, dw, db, B, K, act);
}
