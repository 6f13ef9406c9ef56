// flexmi thin-input Linear layers for gfx950 (MI355X): in_features K <= 32 (the DLRM bottom MLP's
// first layer, 13 dense features padded to 16).  A K-deep GEMM tile wastes the MFMA pipeline on a
// 1-2 step K loop and the split-K dW on slab traffic; these layers are bound by the activation
// bytes (8192 x 512 x 4 B = 16 MB written forward, read backward), so both passes are VALU kernels
// at the store / load rate (reference: the same Linear, cublasSgemm, src/ops/linear.cu:424-447,
// :592-635).
//
//   forward   y[m][n..n+3] = act(x[m][:] . W[n..n+3][:] + b): a block stages its 32 x rows in
//             LDS, a thread keeps its 4 weight rows (4K floats) in registers, reads x rows as LDS
//             broadcasts and stores 16 B per row -- no global load inside the row loop.
//   dW / db   dW[n][k] += sum_m dpre[m][n] x[m][k], db[n] += sum_m dpre[m][n]: one block per 64
//             rows (x rows in LDS) reduces them into per-thread partials (thread = 4 output rows n
//             x all K + bias, its 8 dpre loads in flight together), sums them through LDS into one
//             partial per block, and a second small launch adds the partials in a fixed order
//             (deterministic, no atomics) -- optionally applying the SGD step right there (the
//             gradient of the weight is never stored).
// The first version kept x in global memory and looped rows one load at a time: latency-bound at
// 1 wave per SIMD (dW 20 + 12 us on the MLPerf step, gpurun_out r5e); measured again in r5f.
#include "common.h"

#include <algorithm>
#include <cstdlib>

namespace {

// 4 consecutive operands -> fp32 (T = float or bf16 bits), and back
template <typename T>
FM_DEVICE f32x4_t ld4(const T* p) {
  if constexpr (sizeof(T) == 4) {
    return *reinterpret_cast<const f32x4_t*>(p);
  } else {
    const bf16x4_t v = *reinterpret_cast<const bf16x4_t*>(p);
    return f32x4_t{bf2f((unsigned short)v[0]), bf2f((unsigned short)v[1]), bf2f((unsigned short)v[2]),
                   bf2f((unsigned short)v[3])};
  }
}
template <typename T>
FM_DEVICE void st4(T* p, const f32x4_t& v) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<f32x4_t*>(p) = v;
  } else {
    bf16x4_t o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (short)f2bf(v[e]);
    *reinterpret_cast<bf16x4_t*>(p) = o;
  }
}

constexpr int SK_ROWS_FWD = 32;   // rows per forward block (x rows staged in LDS)
constexpr int SK_ROWS_DW = 64;    // rows per dW partial block
constexpr int SK_DW_NT = 512;     // dW partial block size

// x rows [m0, m0 + rows) -> LDS (rows * K floats, 16-B chunks), zero past M
template <int K, int NT, typename T>
FM_DEVICE void stage_x(const T* __restrict__ x, long ldx, long m0, long M, int rows, float* xs) {
  constexpr int C = K / 4;
  for (int i = threadIdx.x; i < rows * C; i += NT) {
    const int r = i / C, c = i % C;
    const long m = m0 + r;
    f32x4_t v = {0.f, 0.f, 0.f, 0.f};
    if (m < M) v = ld4<T>(x + m * ldx + 4 * c);
    *reinterpret_cast<f32x4_t*>(xs + r * K + 4 * c) = v;
  }
}

// forward: block = SK_ROWS_FWD rows x (4 G) columns; thread = 4 columns (weight rows in registers)
// x (sub-row, rows sub, sub + R, ...); x rows are LDS broadcast reads, y one 16-B store per row
template <int K, typename T>
__global__ void __launch_bounds__(256) fm_smallk_fwd(const T* __restrict__ x, long ldx, const T* __restrict__ w,
                                                    const float* __restrict__ bias, T* __restrict__ y, long ldy, long M,
                                                    int N, int G, int act) {
  __shared__ __attribute__((aligned(16))) float xs[SK_ROWS_FWD * K];
  const int R = 256 / G;
  const int sub = threadIdx.x / G, cg = threadIdx.x % G;
  const int g = blockIdx.y * G + cg;
  const long m0 = (long)blockIdx.x * SK_ROWS_FWD;
  stage_x<K, 256, T>(x, ldx, m0, M, SK_ROWS_FWD, xs);
  __syncthreads();
  if (sub >= R || 4 * g >= N) return;
  const int n0 = 4 * g;
  float wr[4][K];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < K; k += 4) {
      const f32x4_t v = ld4<T>(w + (long)(n0 + j) * K + k);
#pragma unroll
      for (int e = 0; e < 4; ++e) wr[j][k + e] = v[e];
    }
  float bv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bv[j] = bias ? bias[n0 + j] : 0.f;
  const int rows = (int)min((long)SK_ROWS_FWD, M - m0);
#pragma unroll 2
  for (int r = sub; r < rows; r += R) {
    float xr[K];
#pragma unroll
    for (int k = 0; k < K; k += 4) {
      const f32x4_t v = *reinterpret_cast<const f32x4_t*>(xs + r * K + k);
#pragma unroll
      for (int e = 0; e < 4; ++e) xr[k + e] = v[e];
    }
    f32x4_t o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float acc = bv[j];
#pragma unroll
      for (int k = 0; k < K; ++k) acc = fmaf(xr[k], wr[j][k], acc);
      o[j] = act_fwd(act, acc);
    }
    st4<T>(y + (m0 + r) * ldy + n0, o);
  }
}

// dW partials: block (p, c) reduces rows [p*SK_ROWS_DW, +SK_ROWS_DW) for the column groups
// [c*G, (c+1)*G) (G groups of 4 output rows n); thread = (sub-row, group) with its rows' dpre
// loads all in flight at once; x rows come from LDS.  The R = NT/G sub-rows of a group are summed
// through LDS into ws[p][k][j][g] (n = 4g + j, k = K: the bias)
template <int K, typename T, int ROWS = SK_ROWS_DW>
__global__ void __launch_bounds__(SK_DW_NT) fm_smallk_dw_part(const T* __restrict__ dpre, long ldd, const T* __restrict__ x,
                                                             long ldx, float* __restrict__ ws, long M, int N, int G) {
  constexpr int NT = SK_DW_NT;
  constexpr int PER = 8;                          // rows per thread in flight
  __shared__ __attribute__((aligned(16))) float xs[ROWS * K];
  constexpr int KCH = 17;                         // partial sums staged per LDS pass (k chunk)
  __shared__ float red[KCH * NT];
  const int R = NT / G;
  const int NG = N / 4;
  const int sub = threadIdx.x / G, cg = threadIdx.x % G;
  const int g = blockIdx.y * G + cg;
  const bool live = sub < R && g < NG;
  const long m0 = (long)blockIdx.x * ROWS;
  stage_x<K, NT, T>(x, ldx, m0, M, ROWS, xs);
  __syncthreads();
  float acc[4][K + 1];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int k = 0; k <= K; ++k) acc[j][k] = 0.f;
  if (live) {
    const int rows = (int)min((long)ROWS, M - m0);
    for (int r0 = sub; r0 < rows; r0 += PER * R) {
      f32x4_t d[PER];
#pragma unroll
      for (int u = 0; u < PER; ++u) {              // clamped row: every load unconditional
        const int r = min(r0 + u * R, rows - 1);
        d[u] = ld4<T>(dpre + (m0 + r) * ldd + 4 * g);
      }
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int r = r0 + u * R;
        if (r >= rows) break;
        float xr[K];
#pragma unroll
        for (int k = 0; k < K; k += 4) {
          const f32x4_t v = *reinterpret_cast<const f32x4_t*>(xs + r * K + k);
#pragma unroll
          for (int e = 0; e < 4; ++e) xr[k + e] = v[e];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
          for (int k = 0; k < K; ++k) acc[j][k] = fmaf(d[u][j], xr[k], acc[j][k]);
          acc[j][K] += d[u][j];
        }
      }
    }
  }
  float* out = ws + (long)blockIdx.x * (K + 1) * N;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
#pragma unroll
    for (int k0 = 0; k0 <= K; k0 += KCH) {
#pragma unroll
      for (int kk = 0; kk < KCH; ++kk)
        if (k0 + kk <= K) red[kk * NT + threadIdx.x] = acc[j][k0 + kk];
      __syncthreads();
      const int nk = min(KCH, K + 1 - k0);
      for (int o = threadIdx.x; o < nk * G; o += NT) {
        const int kk = o / G, c = o % G;
        const int gg = blockIdx.y * G + c;
        float s = 0.f;
        for (int r = 0; r < R; ++r) s += red[kk * NT + r * G + c];
        if (gg < NG) out[((long)(k0 + kk) * 4 + j) * NG + gg] = s;
      }
      __syncthreads();
    }
  }
}

// dW / db from the P partials in a fixed order (deterministic): block = 64 outputs x 4 slices of
// the partials, the slices combined through LDS; dw[n][k] += sum, db[n] += sum; with lr != null
// the SGD step of optim.hip fm_sgd_kernel is applied to W = dw instead (the gradient is never
// stored; momentum V and the bf16 mirror Wc optional)
__global__ void __launch_bounds__(256) fm_smallk_dw_reduce(const float* __restrict__ ws, int P, int K, int N,
                                                          float* __restrict__ dw, float* __restrict__ db,
                                                          float* __restrict__ V, unsigned short* __restrict__ Wc,
                                                          const float* __restrict__ lr_p, float wd, float mom,
                                                          int nesterov) {
  __shared__ float part[4][64];
  const long per = (long)(K + 1) * N;
  const int oi = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const long o = blockIdx.x * 64L + oi;
  const long oc = o < per ? o : per - 1;
  const int p0 = (int)((long)P * sl / 4), p1 = (int)((long)P * (sl + 1) / 4);
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  int p = p0;
  for (; p + 4 <= p1; p += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) s[u] += ws[(long)(p + u) * per + oc];
  }
  for (; p < p1; ++p) s[0] += ws[(long)p * per + oc];
  part[sl][oi] = (s[0] + s[1]) + (s[2] + s[3]);
  __syncthreads();
  if (sl != 0 || o >= per) return;
  const float sum = (part[0][oi] + part[1][oi]) + (part[2][oi] + part[3][oi]);
  const int NG = N / 4;
  const int g = (int)(o % NG), j = (int)((o / NG) % 4), k = (int)(o / (4L * NG));
  const int n = 4 * g + j;
  if (k == K) {
    if (db) db[n] += sum;
    return;
  }
  const long i = (long)n * K + k;
  if (!lr_p) {
    dw[i] += sum;
    return;
  }
  float gi = sum + wd * dw[i];
  if (mom > 0.f) {
    const float vi = V[i] * mom + gi;
    V[i] = vi;
    gi = nesterov ? gi + mom * vi : vi;
  }
  const float wi = dw[i] - lr_p[0] * gi;
  dw[i] = wi;
  if (Wc) Wc[i] = f2bf(wi);
}

}  // namespace

// y = act(x W^T + b) for K in {4, 8, ..., 32}, N % 4 == 0, rows aligned to 4 elements (x, w, y
// all fp32 or all bf16: bf16 = 1); returns -1 (nothing launched) otherwise
extern "C" int fm_smallk_fwd_launch(const void* x, long ldx, const void* w, const float* bias, void* y, long ldy, long M,
                                    int K, int N, int act, int bf16, hipStream_t s) {
  if (M <= 0) return 0;
  const uintptr_t amask = bf16 ? 7 : 15;
  if (K % 4 || K < 4 || K > 32 || N % 4 || N < 4 || ldx % 4 || ldy % 4 ||
      (((uintptr_t)x | (uintptr_t)w | (uintptr_t)y) & amask))
    return -1;
  const int NG = N / 4;
  const int G = NG < 64 ? NG : 64;
  const dim3 grid((unsigned)((M + SK_ROWS_FWD - 1) / SK_ROWS_FWD), (unsigned)((NG + G - 1) / G));
#define FM_SK(KK)                                                                                                 \
  case KK:                                                                                                        \
    if (bf16)                                                                                                     \
      hipLaunchKernelGGL((fm_smallk_fwd<KK, unsigned short>), grid, dim3(256), 0, s, (const unsigned short*)x, ldx,  \
                         (const unsigned short*)w, bias, (unsigned short*)y, ldy, M, N, G, act);                 \
    else                                                                                                          \
      hipLaunchKernelGGL((fm_smallk_fwd<KK, float>), grid, dim3(256), 0, s, (const float*)x, ldx, (const float*)w, bias, \
                         (float*)y, ldy, M, N, G, act);                                                           \
    break;
  switch (K) {
    FM_SK(4) FM_SK(8) FM_SK(12) FM_SK(16) FM_SK(20) FM_SK(24) FM_SK(28) FM_SK(32)
  }
#undef FM_SK
  return 0;
}

// dW[N][K] += dpre^T x, db[N] += colsum(dpre) (db may be null); with lr the SGD step is applied to
// the weight dw = W instead (V / Wc optional).  ws: (K + 1) * N * ceil(M / 64) floats; returns -1
// (nothing launched) outside the shape limits of the forward or with too small a workspace.
extern "C" int fm_smallk_dw_launch(const void* dpre, long ldd, const void* x, long ldx, float* dw, float* db, long M, int K,
                                   int N, float* ws, long ws_bytes, float* V, unsigned short* Wc, const float* lr, float wd,
                                   float mom, int nesterov, int bf16, hipStream_t s) {
  if (M <= 0) return 0;
  const uintptr_t amask = bf16 ? 7 : 15;
  if (K % 4 || K < 4 || K > 32 || N % 4 || N < 4 || ldd % 4 || ldx % 4 || (((uintptr_t)dpre | (uintptr_t)x) & amask))
    return -1;
  const int NG = N / 4;
  const int G = NG < 64 ? NG : 64;               // column groups per block
  // 64 rows per partial block: fewer, longer blocks leave fewer partials for the deterministic
  // reduce, 64 measured best on the step (1.161-1.163 vs 1.164-1.170 ms, profiles/smallk_dw_rows_ab_r5sk.txt)
  constexpr int RW = SK_ROWS_DW;
  const long P = (M + RW - 1) / RW;
  const long per = (long)(K + 1) * N;
  if (P * per * 4 > ws_bytes || P > (1L << 30)) return -1;
  const dim3 grid((unsigned)P, (unsigned)((NG + G - 1) / G));
#define FM_SD(KK)                                                                                              \
  case KK:                                                                                                     \
    if (bf16)                                                                                                  \
      hipLaunchKernelGGL((fm_smallk_dw_part<KK, unsigned short>), grid, dim3(SK_DW_NT), 0, s,                  \
                         (const unsigned short*)dpre, ldd, (const unsigned short*)x, ldx, ws, M, N, G);         \
    else                                                                                                       \
      hipLaunchKernelGGL((fm_smallk_dw_part<KK, float>), grid, dim3(SK_DW_NT), 0, s, (const float*)dpre, ldd,  \
                         (const float*)x, ldx, ws, M, N, G);                                                    \
    break;
  switch (K) {
    FM_SD(4) FM_SD(8) FM_SD(12) FM_SD(16) FM_SD(20) FM_SD(24) FM_SD(28) FM_SD(32)
  }
#undef FM_SD
  hipLaunchKernelGGL(fm_smallk_dw_reduce, dim3((unsigned)((per + 63) / 64)), dim3(256), 0, s, ws, (int)P, K, N, dw, db, V,
                     Wc, lr, wd, mom, nesterov);
  return 0;
}
