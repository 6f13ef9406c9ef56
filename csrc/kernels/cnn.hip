// CNN kernels for gfx950: the data-movement halves of GEMM-based convolution, pooling and
// batch normalisation (replace the reference's cuDNN calls: src/ops/conv_2d.cu:405-565,
// src/ops/pool_2d.cu:256-357, src/ops/batch_norm.cu:348-503).
//
// Convolution runs on the MFMA GEMM (gemm.hip / gemm_glds.hip):
//   forward   out[NPQ, K]   = col[NPQ, CRS] . W[K, CRS]^T   (+bias, activation in the epilogue)
//   dW, db    dW[K, CRS]    = g[NPQ, K]^T . col               (db from the A-tile row sums)
//   dX        dcol[NPQ, CRS] = g . W                          -> col2im gather
// with the kernels below: im2col (zero-filled halos, per-side pads so spatially sharded
// shards with halo rows use the same code), col2im as a GATHER over the kernel taps (no
// atomics), and batched 32x32 LDS-tiled transposes between the GEMM's NHWC rows and the
// framework's NCHW tensors (the backward one fuses the activation derivative).
// Pooling: one thread per output (forward) / per input (backward, gather form: each input
// re-derives which windows it is the max of -- no atomics, no argmax buffer).  Batch norm:
// per-channel block partial sums + atomics into a [2C] fp32 buffer, then an elementwise pass.
#include "common.h"

#include <algorithm>

namespace {

// ---- im2col / col2im -------------------------------------------------------------------
__global__ void __launch_bounds__(256) fm_im2col_kernel(const unsigned short* __restrict__ x, unsigned short* __restrict__ col,
                                                        int C, int H, int W, int R, int S, int P, int Q, int sh, int sw,
                                                        int pt, int pl, int CRS, int ldcol, long rows) {
  for (long row = blockIdx.x; row < rows; row += gridDim.x) {
    const int q = (int)(row % Q);
    const long t = row / Q;
    const int p = (int)(t % P);
    const int n = (int)(t / P);
    const int h0 = p * sh - pt, w0 = q * sw - pl;
    const unsigned short* xn = x + (long)n * C * H * W;
    unsigned short* dst = col + row * ldcol;
    for (int k = threadIdx.x; k < ldcol; k += blockDim.x) {
      unsigned short v = 0;
      if (k < CRS) {
        const int s = k % S;
        const int r = (k / S) % R;
        const int c = k / (R * S);
        const int h = h0 + r, w = w0 + s;
        if (h >= 0 && h < H && w >= 0 && w < W) v = xn[((long)c * H + h) * W + w];
      }
      dst[k] = v;
    }
  }
}

__global__ void __launch_bounds__(256) fm_col2im_kernel(const unsigned short* __restrict__ dcol, unsigned short* __restrict__ dx,
                                                        int N, int C, int H, int W, int R, int S, int P, int Q, int sh,
                                                        int sw, int pt, int pl, int ldcol, int acc) {
  const long total = (long)N * C * H * W;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int w = (int)(i % W);
    long t = i / W;
    const int h = (int)(t % H);
    t /= H;
    const int c = (int)(t % C);
    const int n = (int)(t / C);
    float s_ = 0.f;
    for (int r = 0; r < R; ++r) {
      const int hp = h + pt - r;
      if (hp < 0 || hp % sh) continue;
      const int p = hp / sh;
      if (p >= P) continue;
      for (int s = 0; s < S; ++s) {
        const int wq = w + pl - s;
        if (wq < 0 || wq % sw) continue;
        const int q = wq / sw;
        if (q >= Q) continue;
        s_ += bf2f(dcol[((long)(n * P + p) * Q + q) * ldcol + (c * R + r) * S + s]);
      }
    }
    if (acc) s_ += bf2f(dx[i]);
    dx[i] = f2bf(s_);
  }
}

// ---- NHWC <-> NCHW (batched [N][A][B] -> [N][B][A] 32x32 LDS tiles) ----------------------
// mode 0: plain copy; mode 1: out = act_bwd(act, y_in[same index as in], in) (backward: dy, y NCHW)
__global__ void __launch_bounds__(256) fm_transpose_kernel(const unsigned short* __restrict__ in, const unsigned short* __restrict__ yin,
                                                           unsigned short* __restrict__ out, int A, int B, int act, int mode) {
  __shared__ float tile[32][33];
  const long base = (long)blockIdx.z * A * B;
  const int a0 = blockIdx.y * 32, b0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 x 8
  for (int j = ty; j < 32; j += 8) {
    const int a = a0 + j, b = b0 + tx;
    float v = 0.f;
    if (a < A && b < B) {
      const long idx = base + (long)a * B + b;
      v = bf2f(in[idx]);
      if (mode == 1) v = act_bwd(act, bf2f(yin[idx]), v);
    }
    tile[j][tx] = v;
  }
  __syncthreads();
  for (int j = ty; j < 32; j += 8) {
    const int b = b0 + j, a = a0 + tx;
    if (a < A && b < B) out[base + (long)b * A + a] = f2bf(tile[tx][j]);
  }
}

// ---- pooling ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) fm_pool_fwd_kernel(const unsigned short* __restrict__ x, unsigned short* __restrict__ y,
                                                          int N, int C, int H, int W, int P, int Q, int kh, int kw, int sh,
                                                          int sw, int pt, int pl, int is_max, int act) {
  const long total = (long)N * C * P * Q;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int q = (int)(i % Q);
    long t = i / Q;
    const int p = (int)(t % P);
    const long nc = t / P;
    const unsigned short* xp = x + nc * H * W;
    const int h0 = p * sh - pt, w0 = q * sw - pl;
    float m = -INFINITY, s = 0.f;
    int cnt = 0;
    for (int r = 0; r < kh; ++r) {
      const int h = h0 + r;
      if (h < 0 || h >= H) continue;
      for (int c = 0; c < kw; ++c) {
        const int w = w0 + c;
        if (w < 0 || w >= W) continue;
        const float v = bf2f(xp[h * W + w]);
        m = fmaxf(m, v);
        s += v;
        ++cnt;
      }
    }
    const float o = is_max ? m : (cnt ? s / cnt : 0.f);
    y[i] = f2bf(act_fwd(act, o));
  }
}

__global__ void __launch_bounds__(256) fm_pool_bwd_kernel(const unsigned short* __restrict__ x, const unsigned short* __restrict__ y,
                                                          const unsigned short* __restrict__ dy, unsigned short* __restrict__ dx,
                                                          int N, int C, int H, int W, int P, int Q, int kh, int kw, int sh,
                                                          int sw, int pt, int pl, int is_max, int act, int acc) {
  const long total = (long)N * C * H * W;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int w = (int)(i % W);
    long t = i / W;
    const int h = (int)(t % H);
    const long nc = t / H;
    const unsigned short* xp = x + nc * H * W;
    float g = 0.f;
    // windows (p, q) containing (h, w): p*sh - pt <= h < p*sh - pt + kh
    const int pmin = max(0, (h + pt - kh + sh) / sh), pmax = min(P - 1, (h + pt) / sh);
    const int qmin = max(0, (w + pl - kw + sw) / sw), qmax = min(Q - 1, (w + pl) / sw);
    for (int p = pmin; p <= pmax; ++p) {
      const int h0 = p * sh - pt;
      if (h < h0 || h >= h0 + kh) continue;
      for (int q = qmin; q <= qmax; ++q) {
        const int w0 = q * sw - pl;
        if (w < w0 || w >= w0 + kw) continue;
        const long o = (nc * P + p) * Q + q;
        const float go = act_bwd(act, bf2f(y[o]), bf2f(dy[o]));
        if (is_max) {   // gradient goes to the window's first maximum (row-major scan, like PyTorch)
          float best = -INFINITY;
          int bh = -1, bw = -1;
          for (int r = 0; r < kh; ++r) {
            const int hh = h0 + r;
            if (hh < 0 || hh >= H) continue;
            for (int c = 0; c < kw; ++c) {
              const int ww = w0 + c;
              if (ww < 0 || ww >= W) continue;
              const float v = bf2f(xp[hh * W + ww]);
              if (v > best) { best = v; bh = hh; bw = ww; }
            }
          }
          if (bh == h && bw == w) g += go;
        } else {
          const int hs = max(h0, 0), he = min(h0 + kh, H), ws = max(w0, 0), we = min(w0 + kw, W);
          g += go / (float)((he - hs) * (we - ws));
        }
      }
    }
    if (acc) g += bf2f(dx[i]);
    dx[i] = f2bf(g);
  }
}

// ---- batch norm (training mode, per-channel statistics over N*H*W) -----------------------
// stats[0:C] = sum, stats[C:2C] = sum of squares   (zeroed by the caller)
__global__ void __launch_bounds__(256) fm_bn_stats_kernel(const unsigned short* __restrict__ x, float* __restrict__ stats,
                                                          int N, int C, int HW) {
  const int c = blockIdx.y;
  float s = 0.f, s2 = 0.f;
  const long per_c = (long)N * HW;
  for (long j = blockIdx.x * (long)blockDim.x + threadIdx.x; j < per_c; j += (long)gridDim.x * blockDim.x) {
    const long n = j / HW, hw = j % HW;
    const float v = bf2f(x[(n * C + c) * HW + hw]);
    s += v;
    s2 += v * v;
  }
  __shared__ float red[2][4];
  s = wave_reduce_sum(s);
  s2 = wave_reduce_sum(s2);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s;
    red[1][threadIdx.x >> 6] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(stats + c, red[0][0] + red[0][1] + red[0][2] + red[0][3]);
    atomicAdd(stats + C + c, red[1][0] + red[1][1] + red[1][2] + red[1][3]);
  }
}

// y = relu?((x - mean) * inv * gamma + beta); meaninv[0:C] = mean, [C:2C] = inv (saved for bwd)
__global__ void __launch_bounds__(256) fm_bn_apply_kernel(const unsigned short* __restrict__ x, unsigned short* __restrict__ y,
                                                          const float* __restrict__ stats, const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float* __restrict__ meaninv,
                                                          int N, int C, int HW, float eps, int relu) {
  const long total = (long)N * C * HW;
  const float m = (float)N * HW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)((i / HW) % C);
    const float mean = stats[c] / m;
    const float var = fmaxf(stats[C + c] / m - mean * mean, 0.f);
    const float inv = rsqrtf(var + eps);
    if (i < C) {   // one thread per channel records the statistics
      const float mc = stats[i] / m;
      meaninv[i] = mc;
      meaninv[C + i] = rsqrtf(fmaxf(stats[C + i] / m - mc * mc, 0.f) + eps);
    }
    float v = (bf2f(x[i]) - mean) * inv * gamma[c] + beta[c];
    if (relu) v = fmaxf(v, 0.f);
    y[i] = f2bf(v);
  }
}

// gsum[0:C] += sum g ; gsum[C:2C] += sum g * xhat   (g = relu-masked dy), zeroed by the caller
__global__ void __launch_bounds__(256) fm_bn_bwd_stats_kernel(const unsigned short* __restrict__ x, const unsigned short* __restrict__ y,
                                                              const unsigned short* __restrict__ dy, const float* __restrict__ meaninv,
                                                              float* __restrict__ gsum, int N, int C, int HW, int relu) {
  const int c = blockIdx.y;
  const float mean = meaninv[c], inv = meaninv[C + c];
  float s = 0.f, s2 = 0.f;
  const long per_c = (long)N * HW;
  for (long j = blockIdx.x * (long)blockDim.x + threadIdx.x; j < per_c; j += (long)gridDim.x * blockDim.x) {
    const long n = j / HW, hw = j % HW;
    const long idx = (n * C + c) * HW + hw;
    float g = bf2f(dy[idx]);
    if (relu && bf2f(y[idx]) <= 0.f) g = 0.f;
    s += g;
    s2 += g * (bf2f(x[idx]) - mean) * inv;
  }
  __shared__ float red[2][4];
  s = wave_reduce_sum(s);
  s2 = wave_reduce_sum(s2);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s;
    red[1][threadIdx.x >> 6] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(gsum + c, red[0][0] + red[0][1] + red[0][2] + red[0][3]);
    atomicAdd(gsum + C + c, red[1][0] + red[1][1] + red[1][2] + red[1][3]);
  }
}

__global__ void __launch_bounds__(256) fm_bn_bwd_apply_kernel(const unsigned short* __restrict__ x, const unsigned short* __restrict__ y,
                                                              const unsigned short* __restrict__ dy, const float* __restrict__ meaninv,
                                                              const float* __restrict__ gsum, const float* __restrict__ gamma,
                                                              unsigned short* __restrict__ dx, int N, int C, int HW, int relu,
                                                              int acc) {
  const long total = (long)N * C * HW;
  const float m = (float)N * HW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)((i / HW) % C);
    const float mean = meaninv[c], inv = meaninv[C + c];
    float g = bf2f(dy[i]);
    if (relu && bf2f(y[i]) <= 0.f) g = 0.f;
    const float xhat = (bf2f(x[i]) - mean) * inv;
    float v = gamma[c] * inv / m * (m * g - gsum[c] - xhat * gsum[C + c]);
    if (acc) v += bf2f(dx[i]);
    dx[i] = f2bf(v);
  }
}

// compact a padded [K][ldp] fp32 matrix into [K][n] (+= when acc)
__global__ void __launch_bounds__(256) fm_compact_kernel(const float* __restrict__ src, float* __restrict__ dst, int K, int n,
                                                         int ldp, int acc) {
  const long total = (long)K * n;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long k = i / n, j = i % n;
    const float v = src[k * ldp + j];
    dst[i] = acc ? dst[i] + v : v;
  }
}

// pad [K][n] bf16/fp32 weights into [K][ldp] bf16 with zero columns
__global__ void __launch_bounds__(256) fm_pad_rows_kernel(const unsigned short* __restrict__ src, unsigned short* __restrict__ dst,
                                                          int K, int n, int ldp) {
  const long total = (long)K * ldp;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long k = i / ldp, j = i % ldp;
    dst[i] = j < n ? src[k * n + j] : (unsigned short)0;
  }
}

}  // namespace

extern "C" {

void fm_im2col(const void* x, void* col, int N, int C, int H, int W, int R, int S, int P, int Q, int sh, int sw, int pt,
               int pl, int ldcol, hipStream_t st) {
  const long rows = (long)N * P * Q;
  if (rows <= 0) return;
  const int blocks = (int)std::min<long>(rows, 65536);
  hipLaunchKernelGGL(fm_im2col_kernel, dim3(blocks), dim3(ldcol >= 256 ? 256 : 128), 0, st, (const unsigned short*)x,
                     (unsigned short*)col, C, H, W, R, S, P, Q, sh, sw, pt, pl, C * R * S, ldcol, rows);
}

void fm_col2im(const void* dcol, void* dx, int N, int C, int H, int W, int R, int S, int P, int Q, int sh, int sw, int pt,
               int pl, int ldcol, int acc, hipStream_t st) {
  const long total = (long)N * C * H * W;
  if (total <= 0) return;
  hipLaunchKernelGGL(fm_col2im_kernel, dim3(fm_grid(total)), dim3(256), 0, st, (const unsigned short*)dcol,
                     (unsigned short*)dx, N, C, H, W, R, S, P, Q, sh, sw, pt, pl, ldcol, acc);
}

// batched [N][A][B] -> [N][B][A]; mode 1 applies act_bwd(act, yin, in) first
void fm_transpose_batched(const void* in, const void* yin, void* out, int N, int A, int B, int act, int mode, hipStream_t st) {
  if ((long)N * A * B <= 0) return;
  dim3 grid((B + 31) / 32, (A + 31) / 32, N);
  hipLaunchKernelGGL(fm_transpose_kernel, grid, dim3(256), 0, st, (const unsigned short*)in, (const unsigned short*)yin,
                     (unsigned short*)out, A, B, act, mode);
}

void fm_pool_fwd(const void* x, void* y, int N, int C, int H, int W, int P, int Q, int kh, int kw, int sh, int sw, int pt,
                 int pl, int is_max, int act, hipStream_t st) {
  const long total = (long)N * C * P * Q;
  if (total <= 0) return;
  hipLaunchKernelGGL(fm_pool_fwd_kernel, dim3(fm_grid(total)), dim3(256), 0, st, (const unsigned short*)x, (unsigned short*)y,
                     N, C, H, W, P, Q, kh, kw, sh, sw, pt, pl, is_max, act);
}

void fm_pool_bwd(const void* x, const void* y, const void* dy, void* dx, int N, int C, int H, int W, int P, int Q, int kh,
                 int kw, int sh, int sw, int pt, int pl, int is_max, int act, int acc, hipStream_t st) {
  const long total = (long)N * C * H * W;
  if (total <= 0) return;
  hipLaunchKernelGGL(fm_pool_bwd_kernel, dim3(fm_grid(total)), dim3(256), 0, st, (const unsigned short*)x,
                     (const unsigned short*)y, (const unsigned short*)dy, (unsigned short*)dx, N, C, H, W, P, Q, kh, kw, sh,
                     sw, pt, pl, is_max, act, acc);
}

// stats / meaninv: fp32 [2C] device buffers owned by the op
void fm_bn_fwd(const void* x, void* y, const float* gamma, const float* beta, float* stats, float* meaninv, int N, int C,
               int HW, float eps, int relu, hipStream_t st) {
  (void)hipMemsetAsync(stats, 0, sizeof(float) * 2 * C, st);
  const long per_c = (long)N * HW;
  dim3 g1((unsigned)std::max<long>(1, std::min<long>((per_c + 255) / 256, 64)), C);
  hipLaunchKernelGGL(fm_bn_stats_kernel, g1, dim3(256), 0, st, (const unsigned short*)x, stats, N, C, HW);
  const long total = (long)N * C * HW;
  hipLaunchKernelGGL(fm_bn_apply_kernel, dim3(fm_grid(total)), dim3(256), 0, st, (const unsigned short*)x,
                     (unsigned short*)y, stats, gamma, beta, meaninv, N, C, HW, eps, relu);
}

// dgamma/dbeta: fp32 [C] outputs (overwritten); gsum fp32 [2C] scratch
void fm_bn_bwd(const void* x, const void* y, const void* dy, const float* meaninv, const float* gamma, float* gsum,
               float* dgamma, float* dbeta, void* dx, int N, int C, int HW, int relu, int acc, hipStream_t st) {
  (void)hipMemsetAsync(gsum, 0, sizeof(float) * 2 * C, st);
  const long per_c = (long)N * HW;
  dim3 g1((unsigned)std::max<long>(1, std::min<long>((per_c + 255) / 256, 64)), C);
  hipLaunchKernelGGL(fm_bn_bwd_stats_kernel, g1, dim3(256), 0, st, (const unsigned short*)x, (const unsigned short*)y,
                     (const unsigned short*)dy, meaninv, gsum, N, C, HW, relu);
  (void)hipMemcpyAsync(dbeta, gsum, sizeof(float) * C, hipMemcpyDeviceToDevice, st);
  (void)hipMemcpyAsync(dgamma, gsum + C, sizeof(float) * C, hipMemcpyDeviceToDevice, st);
  if (dx) {
    const long total = (long)N * C * HW;
    hipLaunchKernelGGL(fm_bn_bwd_apply_kernel, dim3(fm_grid(total)), dim3(256), 0, st, (const unsigned short*)x,
                       (const unsigned short*)y, (const unsigned short*)dy, meaninv, gsum, gamma, (unsigned short*)dx, N, C,
                       HW, relu, acc);
  }
}

void fm_compact_rows(const float* src, float* dst, int K, int n, int ldp, int acc, hipStream_t st) {
  const long total = (long)K * n;
  if (total <= 0) return;
  hipLaunchKernelGGL(fm_compact_kernel, dim3(fm_grid(total)), dim3(256), 0, st, src, dst, K, n, ldp, acc);
}

void fm_pad_rows(const void* src, void* dst, int K, int n, int ldp, hipStream_t st) {
  const long total = (long)K * ldp;
  if (total <= 0) return;
  hipLaunchKernelGGL(fm_pad_rows_kernel, dim3(fm_grid(total)), dim3(256), 0, st, (const unsigned short*)src,
                     (unsigned short*)dst, K, n, ldp);
}

}  // extern "C"
