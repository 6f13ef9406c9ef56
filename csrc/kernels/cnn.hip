// CNN kernels for gfx950: the data-movement halves of GEMM-based convolution, pooling and
// batch normalisation (replace the reference's cuDNN calls: src/ops/conv_2d.cu:405-565,
// src/ops/pool_2d.cu:256-357, src/ops/batch_norm.cu:348-503).
//
// Convolution runs on the MFMA GEMM (gemm.hip):
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

#include <cstdlib>

#include <algorithm>

namespace {

// ---- im2col / col2im -------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) fm_im2col_kernel(const T* __restrict__ x, T* __restrict__ col,
                                                        int C, int H, int W, int R, int S, int P, int Q, int sh, int sw,
                                                        int pt, int pl, int CRS, int ldcol, long rows) {
  for (long row = blockIdx.x; row < rows; row += gridDim.x) {
    const int q = (int)(row % Q);
    const long t = row / Q;
    const int p = (int)(t % P);
    const int n = (int)(t / P);
    const int h0 = p * sh - pt, w0 = q * sw - pl;
    const T* xn = x + (long)n * C * H * W;
    T* dst = col + row * ldcol;
    for (int k = threadIdx.x; k < ldcol; k += blockDim.x) {
      T v = fromf<T>(0.f);
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

template <typename T>
__global__ void __launch_bounds__(256) fm_col2im_kernel(const T* __restrict__ dcol, T* __restrict__ dx,
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
        s_ += tof(dcol[((long)(n * P + p) * Q + q) * ldcol + (c * R + r) * S + s]);
      }
    }
    if (acc) s_ += tof(dx[i]);
    dx[i] = fromf<T>(s_);
  }
}

// ---- NHWC <-> NCHW (batched [N][A][B] -> [N][B][A] 32x32 LDS tiles) ----------------------
// mode 0: plain copy; mode 1: out = act_bwd(act, y_in[same index as in], in) (backward: dy, y NCHW)
template <typename T>
__global__ void __launch_bounds__(256) fm_transpose_kernel(const T* __restrict__ in, const T* __restrict__ yin,
                                                           T* __restrict__ out, int A, int B, int act, int mode) {
  __shared__ float tile[32][33];
  const long base = (long)blockIdx.z * A * B;
  const int a0 = blockIdx.y * 32, b0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 x 8
  for (int j = ty; j < 32; j += 8) {
    const int a = a0 + j, b = b0 + tx;
    float v = 0.f;
    if (a < A && b < B) {
      const long idx = base + (long)a * B + b;
      v = tof(in[idx]);
      if (mode == 1) v = act_bwd(act, tof(yin[idx]), v);
    }
    tile[j][tx] = v;
  }
  __syncthreads();
  for (int j = ty; j < 32; j += 8) {
    const int b = b0 + j, a = a0 + tx;
    if (a < A && b < B) out[base + (long)b * A + a] = fromf<T>(tile[tx][j]);
  }
}

// ---- pooling ---------------------------------------------------------------------------
// pooling forward: one thread per output (32-bit index math, magic-number division); max pooling
// also records the row-major position of the window's FIRST maximum (PyTorch's tie rule) as a byte
// code r*kw + c (255: empty window) for the backward pass when ``code`` is given
template <typename T>
__global__ void __launch_bounds__(256) fm_pool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                          unsigned char* __restrict__ code, int total, FastDiv dQ,
                                                          FastDiv dP, int H, int W, int P, int Q, int kh, int kw, int sh,
                                                          int sw, int pt, int pl, int is_max, int act) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int t = fdiv(i, dQ), q = i - t * Q;
  const int nc = fdiv(t, dP), p = t - nc * P;
  const T* xp = x + (long)nc * H * W;
  const int h0 = p * sh - pt, w0 = q * sw - pl;
  float m = -INFINITY, s = 0.f;
  int cnt = 0, bc = 255;
  for (int r = 0; r < kh; ++r) {
    const int h = h0 + r;
    if (h < 0 || h >= H) continue;
    for (int c = 0; c < kw; ++c) {
      const int w = w0 + c;
      if (w < 0 || w >= W) continue;
      const float v = tof(xp[h * W + w]);
      if (v > m || bc == 255) bc = r * kw + c;
      m = fmaxf(m, v);
      s += v;
      ++cnt;
    }
  }
  const float o = is_max ? m : (cnt ? s / cnt : 0.f);
  y[i] = fromf<T>(act_fwd(act, o));
  if (code) code[i] = (unsigned char)bc;
}

// max pooling backward without a forward-recorded code: the argmax bytes per output window
template <typename T>
__global__ void __launch_bounds__(256) fm_pool_argmax_kernel(const T* __restrict__ x, unsigned char* __restrict__ code,
                                                             int total, int H, int W, int P, int Q, int kh, int kw, int sh,
                                                             int sw, int pt, int pl) {
  const int o = blockIdx.x * 256 + threadIdx.x;
  if (o >= total) return;
  const int q = o % Q, t = o / Q, p = t % P, nc = t / P;
  const T* xp = x + (long)nc * H * W;
  const int h0 = p * sh - pt, w0 = q * sw - pl;
  float best = -INFINITY;
  int bc = 255;
  for (int r = 0; r < kh; ++r) {
    const int hh = h0 + r;
    if (hh < 0 || hh >= H) continue;
    for (int c = 0; c < kw; ++c) {
      const int ww = w0 + c;
      if (ww < 0 || ww >= W) continue;
      const float v = tof(xp[hh * W + ww]);
      if (v > best || bc == 255) { best = v; bc = r * kw + c; }
    }
  }
  code[o] = (unsigned char)bc;
}

// pooling backward, per input element (32-bit index math, one thread per element): sum the
// gradients of the <= ceil(k/s)^2 windows that route to it (max: the window's argmax code is this
// element; avg: 1 / clipped window size)

// pooling backward, row segments: one thread = VW consecutive input columns of one (n, c, h) row.
// The windows that route to the segment are the same rows p for all VW columns and a short run of
// columns q, so each window's argmax code / output gradient is loaded ONCE per thread instead of
// once per element (the per-element kernel above re-derived and re-loaded them for every input
// element: 572 us/step of AlexNet b256 bf16, profiles/prof_r2_alexnet_b256_bf16_kernels.txt);
// the VW results leave as one 16-B (bf16) / two 16-B (fp32) store when the row allows it.
template <typename T, int VW>
__global__ void __launch_bounds__(256) fm_pool_bwd_rows(const T* __restrict__ y, const T* __restrict__ dy,
                                                        const unsigned char* __restrict__ code, T* __restrict__ dx,
                                                        int total, FastDiv dWS, FastDiv dH, FastDiv dsh, FastDiv dsw,
                                                        int WS, int H, int W, int P, int Q, int kh, int kw, int sh, int sw,
                                                        int pt, int pl, int is_max, int act, int acc) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int t = fdiv(i, dWS), ws = i - t * WS;
  const int nc = fdiv(t, dH), h = t - nc * H;
  const int wb = ws * VW;
  const int we = min(W, wb + VW) - 1;                  // last column of the segment
  float g[VW];
#pragma unroll
  for (int e = 0; e < VW; ++e) g[e] = 0.f;
  const int pmin = h + pt + 1 >= kh ? fdiv(h + pt - kh + sh, dsh) : 0;
  const int pmax = h + pt >= 0 ? min(P - 1, fdiv(h + pt, dsh)) : -1;
  const int qmin = wb + pl + 1 >= kw ? fdiv(wb + pl - kw + sw, dsw) : 0;
  const int qmax = we + pl >= 0 ? min(Q - 1, fdiv(we + pl, dsw)) : -1;
  for (int p = pmin; p <= pmax; ++p) {
    const int h0 = p * sh - pt;
    if (h < h0 || h >= h0 + kh) continue;
    const int orow = (nc * P + p) * Q;
    for (int q = qmin; q <= qmax; ++q) {
      const int w0 = q * sw - pl;
      const int o = orow + q;
      const float gd = tof(dy[o]);
      const float go = act == ACT_NONE ? gd : act_bwd(act, tof(y[o]), gd);
      if (is_max) {
        const int cd = code[o];
        if (cd == 255) continue;
        const int ch = cd / kw, cw = cd - ch * kw;
        if (h0 + ch != h) continue;                    // the window's max is on another row
        const int w = w0 + cw - wb;
#pragma unroll
        for (int e = 0; e < VW; ++e)
          if (e == w) g[e] += go;
      } else {
        const int hs = max(h0, 0), hend = min(h0 + kh, H), wsx = max(w0, 0), wend = min(w0 + kw, W);
        const float v = go / (float)((hend - hs) * (wend - wsx));
#pragma unroll
        for (int e = 0; e < VW; ++e) {
          const int w = wb + e;
          if (w >= w0 && w < w0 + kw) g[e] += v;
        }
      }
    }
  }
  T* dp = dx + (long)t * W + wb;
  const bool vec = (we - wb + 1 == VW) && ((((uintptr_t)dp) & 15) == 0);
  if (vec) {
    if (acc) {
      float old[VW];
      if constexpr (VW == 8) ld8<T>(dp, old);
#pragma unroll
      for (int e = 0; e < VW; ++e) g[e] += old[e];
    }
    if constexpr (VW == 8) st8<T>(dp, g);
  } else {
    for (int e = 0; e <= we - wb; ++e) dp[e] = fromf<T>(g[e] + (acc ? tof(dp[e]) : 0.f));
  }
}

// ---- pooling on row bands (one block per (n, c, band) staged in LDS) ----------------------
// The forward block reads the input rows its band of output rows needs as ONE contiguous chunk
// of the plane (coalesced 2-B loads, each input element loaded once instead of once per window
// that covers it), computes the band's outputs from LDS and writes them contiguously.  The
// backward block stages the output-gradient rows (act'(y)*dy as fp32, plus max pooling's argmax
// bytes) that reach its band of input rows, then every input element gathers its <= ceil(k/s)^2
// windows from LDS.  Bands are sized to ~4 K staged elements so a layer launches thousands of
// blocks (the whole-plane kernels below ran one block per plane: too few waves).
// G > 1 (whole-plane bands only): one block takes G consecutive (n, c) planes -- a contiguous chunk
// too -- so 17x17 / 8x8 Inception planes do not pay a block per 289 / 64 elements.
template <typename T>
__global__ void __launch_bounds__(256) fm_pool_fwd_band(const T* __restrict__ x, T* __restrict__ y,
                                                        unsigned char* __restrict__ code, int NC, int H, int W, int P, int Q,
                                                        int kh, int kw, int sh, int sw, int pt, int pl, int is_max, int act,
                                                        int PB, int nbands, int G, FastDiv dQ, FastDiv dPQ) {
  extern __shared__ float sx[];
  int nc0, band, planes;
  if (G > 1) {
    nc0 = blockIdx.x * G;
    band = 0;
    planes = min(G, NC - nc0);
  } else {
    nc0 = blockIdx.x / nbands;
    band = blockIdx.x - nc0 * nbands;
    planes = 1;
  }
  const int p0 = band * PB, p1 = min(P, p0 + PB);
  const int hlo = G > 1 ? 0 : max(0, p0 * sh - pt);
  const int hhi = G > 1 ? H : min(H, (p1 - 1) * sh - pt + kh);
  const int rows = max(0, hhi - hlo);
  const T* xp = x + ((long)nc0 * H + hlo) * W;
  // 8 loads in flight per thread before the LDS stores (a load -> store loop waits on every load)
  const int nst = planes * rows * W;
  for (int b0 = 0; b0 < nst; b0 += 256 * 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = b0 + u * 256 + (int)threadIdx.x;
      v[u] = tof(xp[min(e, nst - 1)]);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = b0 + u * 256 + (int)threadIdx.x;
      if (e < nst) sx[e] = v[u];
    }
  }
  __syncthreads();
  const int nout1 = (p1 - p0) * Q;
  const int nout = planes * nout1;
  for (int o = threadIdx.x; o < nout; o += 256) {
    int gi = 0, r = o;
    if (G > 1) {
      gi = fdiv(o, dPQ);
      r = o - gi * nout1;
    }
    const int pr = fdiv(r, dQ), q = r - pr * Q;
    const int p = p0 + pr;
    const int h0 = p * sh - pt, w0 = q * sw - pl;
    // the window clipped to the plane: no per-tap bounds tests
    const int r0 = max(0, -h0), r1 = min(kh, H - h0), c0 = max(0, -w0), c1 = min(kw, W - w0);
    const float* plane = sx + gi * rows * W;
    float m = -INFINITY, sacc = 0.f;
    int bc = 255;
    for (int rr = r0; rr < r1; ++rr) {
      const float* row = plane + (h0 + rr - hlo) * W + w0;
      for (int c = c0; c < c1; ++c) {
        const float v = row[c];
        if (v > m || bc == 255) bc = rr * kw + c;
        m = fmaxf(m, v);
        sacc += v;
      }
    }
    const int cnt = max(0, r1 - r0) * max(0, c1 - c0);
    const long oi = ((long)(nc0 + gi) * P + p) * Q + q;
    y[oi] = fromf<T>(act_fwd(act, is_max ? m : (cnt ? sacc / cnt : 0.f)));
    if (code) code[oi] = (unsigned char)bc;
  }
}

// bf16 form of fm_pool_fwd_band: the block's input chunk is staged with 16-B loads aligned down from
// its first element (all of a thread's loads in flight at once) into a bf16 LDS image that starts at
// that aligned element; the windows read it with 2-B LDS loads.  (The 2-B staging loads of the band
// kernel needed two or more dependent load rounds per block.)
__global__ void __launch_bounds__(256) fm_pool_fwd_band_v8(const unsigned short* __restrict__ x, unsigned short* __restrict__ y,
                                                           unsigned char* __restrict__ code, int NC, int H, int W, int P, int Q,
                                                           int kh, int kw, int sh, int sw, int pt, int pl, int is_max, int act,
                                                           int PB, int nbands, int G, FastDiv dQ, FastDiv dPQ, long total) {
  extern __shared__ __attribute__((aligned(16))) unsigned short sxb[];
  int nc0, band, planes;
  if (G > 1) {
    nc0 = blockIdx.x * G;
    band = 0;
    planes = min(G, NC - nc0);
  } else {
    nc0 = blockIdx.x / nbands;
    band = blockIdx.x - nc0 * nbands;
    planes = 1;
  }
  const int p0 = band * PB, p1 = min(P, p0 + PB);
  const int hlo = G > 1 ? 0 : max(0, p0 * sh - pt);
  const int hhi = G > 1 ? H : min(H, (p1 - 1) * sh - pt + kh);
  const int rows = max(0, hhi - hlo);
  const long start = ((long)nc0 * H + hlo) * W;
  const long a0 = start & ~7L;
  const int off = (int)(start - a0);
  const int nst = planes * rows * W;
  const int nvec = (off + nst + 7) >> 3;
  for (int v0 = 0; v0 < nvec; v0 += 256 * 4) {
    u32x4_t vv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int v = min(v0 + u * 256 + (int)threadIdx.x, nvec - 1);
      const long g = a0 + 8L * v;
      if (g + 8 <= total) {
        vv[u] = *reinterpret_cast<const u32x4_t*>(x + g);
      } else {                                         // the tensor's last partial vector
        unsigned e16[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) e16[e] = g + e < total ? x[g + e] : 0u;
#pragma unroll
        for (int i = 0; i < 4; ++i) vv[u][i] = e16[2 * i] | (e16[2 * i + 1] << 16);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int v = v0 + u * 256 + (int)threadIdx.x;
      if (v < nvec) *reinterpret_cast<u32x4_t*>(sxb + 8 * v) = vv[u];
    }
  }
  __syncthreads();
  const int nout1 = (p1 - p0) * Q;
  const int nout = planes * nout1;
  for (int o = threadIdx.x; o < nout; o += 256) {
    int gi = 0, r = o;
    if (G > 1) {
      gi = fdiv(o, dPQ);
      r = o - gi * nout1;
    }
    const int pr = fdiv(r, dQ), q = r - pr * Q;
    const int p = p0 + pr;
    const int h0 = p * sh - pt, w0 = q * sw - pl;
    const int r0 = max(0, -h0), r1 = min(kh, H - h0), c0 = max(0, -w0), c1 = min(kw, W - w0);
    const unsigned short* plane = sxb + off + gi * rows * W;
    float m = -INFINITY, sacc = 0.f;
    int bc = 255;
    for (int rr = r0; rr < r1; ++rr) {
      const unsigned short* row = plane + (h0 + rr - hlo) * W + w0;
      for (int c = c0; c < c1; ++c) {
        const float v = bf2f(row[c]);
        if (v > m || bc == 255) bc = rr * kw + c;
        m = fmaxf(m, v);
        sacc += v;
      }
    }
    const int cnt = max(0, r1 - r0) * max(0, c1 - c0);
    const long oi = ((long)(nc0 + gi) * P + p) * Q + q;
    y[oi] = f2bf(act_fwd(act, is_max ? m : (cnt ? sacc / cnt : 0.f)));
    if (code) code[oi] = (unsigned char)bc;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) fm_pool_bwd_band(const T* __restrict__ y, const T* __restrict__ dy,
                                                        const unsigned char* __restrict__ code, T* __restrict__ dx, int NC,
                                                        int H, int W, int P, int Q, int kh, int kw, int sh, int sw, int pt,
                                                        int pl, int is_max, int act, int acc, int HB, int nbands, int maxprows,
                                                        int G, FastDiv dW, FastDiv dQ, FastDiv dsh, FastDiv dsw, FastDiv dPQ,
                                                        FastDiv dHW) {
  extern __shared__ float sg[];                       // [planes][prows][Q] gradients, then the argmax bytes
  unsigned char* sc = reinterpret_cast<unsigned char*>(sg + G * maxprows * Q);
  int nc0, band, planes;
  if (G > 1) {
    nc0 = blockIdx.x * G;
    band = 0;
    planes = min(G, NC - nc0);
  } else {
    nc0 = blockIdx.x / nbands;
    band = blockIdx.x - nc0 * nbands;
    planes = 1;
  }
  const int h0b = band * HB, h1b = min(H, h0b + HB);
  // output rows whose windows reach input rows [h0b, h1b): p*sh - pt <= h1b-1 and p*sh - pt + kh > h0b
  const int plo = G > 1 ? 0 : ((h0b + pt - kh + 1) > 0 ? fdiv(h0b + pt - kh + sh, dsh) : 0);
  const int phi = G > 1 ? P : min(P, (h1b - 1 + pt) >= 0 ? fdiv(h1b - 1 + pt, dsh) + 1 : 0);
  const int prows = max(0, phi - plo);
  const int nst1 = prows * Q;
  const long obase = ((long)nc0 * P + plo) * Q;
  const int nst = planes * nst1;                      // planes > 1: prows == P, contiguous
  // stage g = act'(y) * dy per output window; average pooling divides by the window's clipped size
  // here, once per window instead of once per (input element, window) pair
  for (int b0 = 0; b0 < nst; b0 += 256 * 4) {
    float gd[4], yv[4];
    unsigned char cd[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {           // 4 (dy, y, code) loads in flight per thread
      const long oi = obase + min(b0 + u * 256 + (int)threadIdx.x, max(nst - 1, 0));
      gd[u] = tof(dy[oi]);
      yv[u] = act == ACT_NONE ? 0.f : tof(y[oi]);
      cd[u] = is_max ? code[oi] : (unsigned char)0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = b0 + u * 256 + (int)threadIdx.x;
      if (e >= nst) continue;
      float g = act == ACT_NONE ? gd[u] : act_bwd(act, yv[u], gd[u]);
      if (is_max) {
        sc[e] = cd[u];
      } else {
        const int r = G > 1 ? e - fdiv(e, dPQ) * nst1 : e;
        const int pr = fdiv(r, dQ), q = r - pr * Q;
        const int hw0 = (plo + pr) * sh - pt, ww0 = q * sw - pl;
        g /= (float)((min(hw0 + kh, H) - max(hw0, 0)) * (min(ww0 + kw, W) - max(ww0, 0)));
      }
      sg[e] = g;
    }
  }
  __syncthreads();
  const int nin1 = (h1b - h0b) * W;
  const int nin = planes * nin1;
  T* dxp = dx + ((long)nc0 * H + h0b) * W;
  for (int e = threadIdx.x; e < nin; e += 256) {
    int gi = 0, r = e;
    if (G > 1) {
      gi = fdiv(e, dHW);
      r = e - gi * nin1;
    }
    const int hr = fdiv(r, dW), w = r - hr * W;
    const int h = h0b + hr;
    // windows holding (h, w): p in [ceil((h+pt-kh+1)/sh), floor((h+pt)/sh)], q likewise
    const int pmin = max(plo, h + pt + 1 > kh ? fdiv(h + pt - kh + sh, dsh) : 0);
    const int pmax = min(phi - 1, h + pt >= 0 ? fdiv(h + pt, dsh) : -1);
    const int qmin = w + pl + 1 > kw ? fdiv(w + pl - kw + sw, dsw) : 0;
    const int qmax = min(Q - 1, w + pl >= 0 ? fdiv(w + pl, dsw) : -1);
    const float* gp = sg + gi * nst1;
    const unsigned char* cp = sc + gi * nst1;
    float g = 0.f;
    for (int p = pmin; p <= pmax; ++p) {
      const float* gr = gp + (p - plo) * Q;
      if (is_max) {
        const unsigned char* cr = cp + (p - plo) * Q;
        const int rr = (h - (p * sh - pt)) * kw;
        for (int q = qmin; q <= qmax; ++q)
          if (cr[q] == (unsigned char)(rr + w - (q * sw - pl))) g += gr[q];
      } else {
        for (int q = qmin; q <= qmax; ++q) g += gr[q];
      }
    }
    if (acc) g += tof(dxp[e]);
    dxp[e] = fromf<T>(g);
  }
}

// Max pooling backward as a SCATTER: every output window routes its gradient to exactly one input
// (its recorded argmax), so a block zeroes its dx band (or plane group) in LDS, adds each window's
// gradient at the argmax with an LDS float atomic (overlapping windows can share an argmax), and
// writes the band out once -- ~1/4 of the per-element gather's VALU work at stride 2, where the
// gather re-derived each input's <= 4 candidate windows.
template <typename T>
__global__ void __launch_bounds__(256) fm_pool_bwd_max_scatter(const T* __restrict__ y, const T* __restrict__ dy,
                                                               const unsigned char* __restrict__ code, T* __restrict__ dx,
                                                               int NC, int H, int W, int P, int Q, int kh, int kw, int sh,
                                                               int pt, int pl, int sw, int act, int acc, int HB, int nbands,
                                                               int G, FastDiv dQ, FastDiv dPQ, FastDiv dkw, FastDiv dsh) {
  extern __shared__ float sdx[];
  int nc0, band, planes;
  if (G > 1) {
    nc0 = blockIdx.x * G;
    band = 0;
    planes = min(G, NC - nc0);
  } else {
    nc0 = blockIdx.x / nbands;
    band = blockIdx.x - nc0 * nbands;
    planes = 1;
  }
  const int h0b = band * HB, h1b = min(H, h0b + HB);
  const int rows = h1b - h0b;
  const int nin = planes * rows * W;
  for (int e = threadIdx.x; e < nin; e += 256) sdx[e] = 0.f;
  __syncthreads();
  const int plo = G > 1 ? 0 : ((h0b + pt - kh + 1) > 0 ? fdiv(h0b + pt - kh + sh, dsh) : 0);
  const int phi = G > 1 ? P : min(P, (h1b - 1 + pt) >= 0 ? fdiv(h1b - 1 + pt, dsh) + 1 : 0);
  const int nwin1 = max(0, phi - plo) * Q;
  const int nwin = planes * nwin1;
  // (measured and deleted in r6: running the (p mod ceil(kh/sh), q mod ceil(kw/sw)) window classes one
  // after another with plain LDS read-add-writes instead of LDS float atomics -- 82.5 k vs 84.1 k
  // img/s on AlexNet b256, profiles/pool_scatter_phases_ab_r5z.txt)
  // 4 windows per thread per pass with every (code, dy, y) load issued up front: the code -> dy
  // dependency was a second memory round trip per window
  for (int e0 = 0; e0 < nwin; e0 += 256 * 4) {
    long oi[4];
    int cdv[4];
    float gdv[4], yvv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = min(e0 + u * 256 + (int)threadIdx.x, nwin - 1);
      int gi = 0, r = e;
      if (G > 1) {
        gi = fdiv(e, dPQ);
        r = e - gi * nwin1;
      }
      const int pr = fdiv(r, dQ), q = r - pr * Q;
      oi[u] = ((long)(nc0 + gi) * P + plo + pr) * Q + q;
      cdv[u] = code[oi[u]];
      gdv[u] = tof(dy[oi[u]]);
      yvv[u] = act == ACT_NONE ? 0.f : tof(y[oi[u]]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * 256 + (int)threadIdx.x;
      if (e >= nwin || cdv[u] == 255) continue;
      int gi = 0, r = e;
      if (G > 1) {
        gi = fdiv(e, dPQ);
        r = e - gi * nwin1;
      }
      const int pr = fdiv(r, dQ), q = r - pr * Q;
      const int p = plo + pr;
      const int rr = fdiv(cdv[u], dkw), cc = cdv[u] - rr * kw;
      const int h = p * sh - pt + rr;
      if (h < h0b || h >= h1b) continue;           // this window's max lies in another band
      const int w = q * sw - pl + cc;
      const float v = act == ACT_NONE ? gdv[u] : act_bwd(act, yvv[u], gdv[u]);
      atomicAdd(&sdx[(gi * rows + h - h0b) * W + w], v);
    }
  }
  __syncthreads();
  // (a 16-B vector-store form of this loop -- 8 bf16 per lane between scalar head / tail -- measured
  // SLOWER on AlexNet b256: 177 -> 200 us/step, profiles/prof_r4m_alexnet_b256_kernels.txt: its
  // 8-float-per-lane LDS reads conflict 8 ways); bf16 pairs per lane (4-B stores) measured neutral
  // (176.7 us/step, profiles/prof_r4j_alexnet_b256_kernels.txt).
  T* dxp = dx + ((long)nc0 * H + h0b) * W;
  for (int e = threadIdx.x; e < nin; e += 256) {
    float g = sdx[e];
    if (acc) g += tof(dxp[e]);
    dxp[e] = fromf<T>(g);
  }
}

// (Pooling on whole planes -- one block per (n, c) plane staged in LDS -- measured slower than the
// row / band kernels: AlexNet b256 pool bwd 479 vs 286 us/step, ResNet-50 b64 fwd 335 vs 137;
// one block per plane leaves too few waves in flight.  Deleted in r6.)


// ---- generic 4-D strided copy (stride-phase convolutions) ----------------------------------
// dst[o_d + sum i_k t_k] (+)= src[o_s + sum i_k s_k] over the box d0 x d1 x d2 x d3 (innermost
// d3): gathers an input phase x[:, :, a::s, b::s], scatters a phase gradient back, and moves the
// taps of a sub-kernel w[:, :, r0::s, t0::s] in both directions.  Consecutive threads walk d3.
struct Strided4 {
  int d[4];
  long ss[4], ts[4];
  long so, to;
};
template <typename T>
__global__ void __launch_bounds__(256) fm_strided_copy4(const T* __restrict__ src, T* __restrict__ dst, Strided4 g,
                                                        long total, int acc) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    long r = i;
    const int i3 = (int)(r % g.d[3]); r /= g.d[3];
    const int i2 = (int)(r % g.d[2]); r /= g.d[2];
    const int i1 = (int)(r % g.d[1]);
    const int i0 = (int)(r / g.d[1]);
    const long si = g.so + i0 * g.ss[0] + i1 * g.ss[1] + i2 * g.ss[2] + i3 * g.ss[3];
    const long ti = g.to + i0 * g.ts[0] + i1 * g.ts[1] + i2 * g.ts[2] + i3 * g.ts[3];
    float v = tof(src[si]);
    if (acc) v += tof(dst[ti]);
    dst[ti] = fromf<T>(v);
  }
}

// ---- batch norm (training mode, per-channel statistics over N*H*W) -----------------------
// stats[0:C] = sum, stats[C:2C] = sum of squares   (zeroed by the caller)
template <typename T>
__global__ void __launch_bounds__(256) fm_bn_stats_kernel(const T* __restrict__ x, float* __restrict__ stats,
                                                          int N, int C, int HW) {
  const int c = blockIdx.y;
  float s = 0.f, s2 = 0.f;
  const long per_c = (long)N * HW;
  for (long j = blockIdx.x * (long)blockDim.x + threadIdx.x; j < per_c; j += (long)gridDim.x * blockDim.x) {
    const long n = j / HW, hw = j % HW;
    const float v = tof(x[(n * C + c) * HW + hw]);
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
template <typename T>
__global__ void __launch_bounds__(256) fm_bn_apply_kernel(const T* __restrict__ x, T* __restrict__ y,
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
    float v = (tof(x[i]) - mean) * inv * gamma[c] + beta[c];
    if (relu) v = fmaxf(v, 0.f);
    y[i] = fromf<T>(v);
  }
}

// gsum[0:C] += sum g ; gsum[C:2C] += sum g * xhat   (g = relu-masked dy), zeroed by the caller
template <typename T>
__global__ void __launch_bounds__(256) fm_bn_bwd_stats_kernel(const T* __restrict__ x, const T* __restrict__ y,
                                                              const T* __restrict__ dy, const float* __restrict__ meaninv,
                                                              float* __restrict__ gsum, int N, int C, int HW, int relu) {
  const int c = blockIdx.y;
  const float mean = meaninv[c], inv = meaninv[C + c];
  float s = 0.f, s2 = 0.f;
  const long per_c = (long)N * HW;
  for (long j = blockIdx.x * (long)blockDim.x + threadIdx.x; j < per_c; j += (long)gridDim.x * blockDim.x) {
    const long n = j / HW, hw = j % HW;
    const long idx = (n * C + c) * HW + hw;
    float g = tof(dy[idx]);
    if (relu && tof(y[idx]) <= 0.f) g = 0.f;
    s += g;
    s2 += g * (tof(x[idx]) - mean) * inv;
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

template <typename T>
__global__ void __launch_bounds__(256) fm_bn_bwd_apply_kernel(const T* __restrict__ x, const T* __restrict__ y,
                                                              const T* __restrict__ dy, const float* __restrict__ meaninv,
                                                              const float* __restrict__ gsum, const float* __restrict__ gamma,
                                                              T* __restrict__ dx, int N, int C, int HW, int relu,
                                                              int acc) {
  const long total = (long)N * C * HW;
  const float m = (float)N * HW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)((i / HW) % C);
    const float mean = meaninv[c], inv = meaninv[C + c];
    float g = tof(dy[i]);
    if (relu && tof(y[i]) <= 0.f) g = 0.f;
    const float xhat = (tof(x[i]) - mean) * inv;
    float v = gamma[c] * inv / m * (m * g - gsum[c] - xhat * gsum[C + c]);
    if (acc) v += tof(dx[i]);
    dx[i] = fromf<T>(v);
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
template <typename T>
__global__ void __launch_bounds__(256) fm_pad_rows_kernel(const T* __restrict__ src, T* __restrict__ dst,
                                                          int K, int n, int ldp) {
  const long total = (long)K * ldp;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long k = i / ldp, j = i % ldp;
    dst[i] = j < n ? src[k * n + j] : fromf<T>(0.f);
  }
}

}  // namespace

namespace {

template <typename T>
static void fm_im2col_t(const void* x, void* col, int N, int C, int H, int W, int R, int S, int P, int Q, int sh, int sw, int pt,
               int pl, int ldcol, hipStream_t st) {
  const long rows = (long)N * P * Q;
  if (rows <= 0) return;
  const int blocks = (int)std::min<long>(rows, 65536);
  hipLaunchKernelGGL(fm_im2col_kernel<T>, dim3(blocks), dim3(ldcol >= 256 ? 256 : 128), 0, st, (const T*)x,
                     (T*)col, C, H, W, R, S, P, Q, sh, sw, pt, pl, C * R * S, ldcol, rows);
}

template <typename T>
static void fm_col2im_t(const void* dcol, void* dx, int N, int C, int H, int W, int R, int S, int P, int Q, int sh, int sw, int pt,
               int pl, int ldcol, int acc, hipStream_t st) {
  const long total = (long)N * C * H * W;
  if (total <= 0) return;
  hipLaunchKernelGGL(fm_col2im_kernel<T>, dim3(fm_grid(total)), dim3(256), 0, st, (const T*)dcol,
                     (T*)dx, N, C, H, W, R, S, P, Q, sh, sw, pt, pl, ldcol, acc);
}

// batched [N][A][B] -> [N][B][A]; mode 1 applies act_bwd(act, yin, in) first
template <typename T>
static void fm_transpose_batched_t(const void* in, const void* yin, void* out, int N, int A, int B, int act, int mode, hipStream_t st) {
  if ((long)N * A * B <= 0) return;
  dim3 grid((B + 31) / 32, (A + 31) / 32, N);
  hipLaunchKernelGGL(fm_transpose_kernel<T>, grid, dim3(256), 0, st, (const T*)in, (const T*)yin,
                     (T*)out, A, B, act, mode);
}

// the 16-B staged bf16 forward (fm_pool_fwd_band_v8) for bf16; the 2-B staging band kernel for fp32
constexpr bool POOL_FWD_V8 = true;

template <typename T>
static void fm_pool_fwd_t(const void* x, void* y, unsigned char* code, int N, int C, int H, int W, int P, int Q, int kh, int kw,
                          int sh, int sw, int pt, int pl, int is_max, int act, hipStream_t st) {
  const int total = N * C * P * Q;
  if (total <= 0) return;
  if ((long)kh * W <= 4096) {   // LDS row bands (the per-output kernel below past their limit)
    const int PB = std::max(1, std::min(P, ((4096 / W) - kh) / sh + 1));
    const int nbands = (P + PB - 1) / PB;
    const int NC = N * C;
    // whole planes that are small: several per block
    const int G = (nbands == 1 && (long)H * W <= 2048) ? std::max(1, std::min(NC, 4096 / (H * W))) : 1;
    const int rows = G > 1 ? H : std::min(H, (PB - 1) * sh + kh);
    const int blocks = G > 1 ? (NC + G - 1) / G : NC * nbands;
    if constexpr (sizeof(T) == 2) {
      if (POOL_FWD_V8) {
        const size_t lds = ((size_t)G * rows * W + 16) * 2;
        hipLaunchKernelGGL(fm_pool_fwd_band_v8, dim3(blocks), dim3(256), lds, st, (const unsigned short*)x, (unsigned short*)y,
                           is_max ? code : nullptr, NC, H, W, P, Q, kh, kw, sh, sw, pt, pl, is_max, act, PB, nbands, G,
                           make_fastdiv(Q), make_fastdiv(P * Q), (long)NC * H * W);
        return;
      }
    }
    hipLaunchKernelGGL(fm_pool_fwd_band<T>, dim3(blocks), dim3(256), (size_t)G * rows * W * sizeof(float), st, (const T*)x,
                       (T*)y, is_max ? code : nullptr, NC, H, W, P, Q, kh, kw, sh, sw, pt, pl, is_max, act, PB, nbands, G,
                       make_fastdiv(Q), make_fastdiv(P * Q));
    return;
  }
  hipLaunchKernelGGL(fm_pool_fwd_kernel<T>, dim3((total + 255) / 256), dim3(256), 0, st, (const T*)x, (T*)y,
                     is_max ? code : nullptr, total, make_fastdiv(Q), make_fastdiv(P), H, W, P, Q, kh, kw, sh, sw, pt, pl,
                     is_max, act);
}

// code: max pooling's argmax bytes -- filled by the forward when code_ready, else recomputed here
template <typename T>
static void fm_pool_bwd_t(const void* x, const void* y, const void* dy, void* dx, unsigned char* code, int code_ready, int N,
                          int C, int H, int W, int P, int Q, int kh, int kw, int sh, int sw, int pt, int pl, int is_max,
                          int act, int acc, hipStream_t st) {
  const int total = N * C * H * W, outs = N * C * P * Q;
  if (total <= 0) return;
  if (is_max && !code_ready)
    hipLaunchKernelGGL(fm_pool_argmax_kernel<T>, dim3((outs + 255) / 256), dim3(256), 0, st, (const T*)x, code, outs, H, W,
                       P, Q, kh, kw, sh, sw, pt, pl);
  {   // input-row band kernels (the per-input gather below only past their LDS limits; a one-plane
      // LDS kernel measured slower than these, profiles/prof_r3e_*, and was deleted in r6)
    // input-row band HB: ~4 K input elements; it needs <= (HB + kh - 1) / sh + 1 output rows staged
    const int HB = std::max(1, std::min(H, 4096 / W));
    const int nbands = (H + HB - 1) / HB;
    const int NC = N * C;
    const int G = (nbands == 1 && (long)H * W <= 2048) ? std::max(1, std::min(NC, 4096 / (H * W))) : 1;
    const int maxprows = G > 1 ? P : std::min(P, (HB + kh - 1) / sh + 2);
    const size_t lds = (size_t)G * maxprows * Q * 5;
    if (is_max) {                        // max pooling: scatter through the recorded argmax
      const int blocks = G > 1 ? (NC + G - 1) / G : NC * nbands;
      const size_t lds_s = (size_t)(G > 1 ? G * H : HB) * W * sizeof(float);
      hipLaunchKernelGGL(fm_pool_bwd_max_scatter<T>, dim3(blocks), dim3(256), lds_s, st, (const T*)y, (const T*)dy,
                         (const unsigned char*)code, (T*)dx, NC, H, W, P, Q, kh, kw, sh, pt, pl, sw, act, acc, HB, nbands, G,
                         make_fastdiv(Q), make_fastdiv(P * Q), make_fastdiv(kw), make_fastdiv(sh));
      return;
    }
    if (lds <= 48 * 1024) {
      const int blocks = G > 1 ? (NC + G - 1) / G : NC * nbands;
      hipLaunchKernelGGL(fm_pool_bwd_band<T>, dim3(blocks), dim3(256), lds, st, (const T*)y, (const T*)dy,
                         (const unsigned char*)code, (T*)dx, NC, H, W, P, Q, kh, kw, sh, sw, pt, pl, is_max, act, acc, HB,
                         nbands, maxprows, G, make_fastdiv(W), make_fastdiv(Q), make_fastdiv(sh), make_fastdiv(sw),
                         make_fastdiv(P * Q), make_fastdiv(H * W));
      return;
    }
  }
  {   // past the band kernels' LDS limits: 8-wide input row segments gather their windows
    constexpr int VW = 8;
    const int WS = (W + VW - 1) / VW;
    const int rows_total = N * C * H * WS;
    hipLaunchKernelGGL((fm_pool_bwd_rows<T, VW>), dim3((rows_total + 255) / 256), dim3(256), 0, st, (const T*)y,
                       (const T*)dy, (const unsigned char*)code, (T*)dx, rows_total, make_fastdiv(WS), make_fastdiv(H),
                       make_fastdiv(sh), make_fastdiv(sw), WS, H, W, P, Q, kh, kw, sh, sw, pt, pl, is_max, act, acc);
  }
}

// stats / meaninv: fp32 [2C] device buffers owned by the op
template <typename T>
static void fm_bn_fwd_t(const void* x, void* y, const float* gamma, const float* beta, float* stats, float* meaninv, int N, int C,
               int HW, float eps, int relu, hipStream_t st) {
  (void)hipMemsetAsync(stats, 0, sizeof(float) * 2 * C, st);
  const long per_c = (long)N * HW;
  dim3 g1((unsigned)std::max<long>(1, std::min<long>((per_c + 255) / 256, 64)), C);
  hipLaunchKernelGGL(fm_bn_stats_kernel<T>, g1, dim3(256), 0, st, (const T*)x, stats, N, C, HW);
  const long total = (long)N * C * HW;
  hipLaunchKernelGGL(fm_bn_apply_kernel<T>, dim3(fm_grid(total)), dim3(256), 0, st, (const T*)x,
                     (T*)y, stats, gamma, beta, meaninv, N, C, HW, eps, relu);
}

// dgamma/dbeta: fp32 [C] outputs (overwritten); gsum fp32 [2C] scratch
template <typename T>
static void fm_bn_bwd_t(const void* x, const void* y, const void* dy, const float* meaninv, const float* gamma, float* gsum,
               float* dgamma, float* dbeta, void* dx, int N, int C, int HW, int relu, int acc, hipStream_t st) {
  (void)hipMemsetAsync(gsum, 0, sizeof(float) * 2 * C, st);
  const long per_c = (long)N * HW;
  dim3 g1((unsigned)std::max<long>(1, std::min<long>((per_c + 255) / 256, 64)), C);
  hipLaunchKernelGGL(fm_bn_bwd_stats_kernel<T>, g1, dim3(256), 0, st, (const T*)x, (const T*)y,
                     (const T*)dy, meaninv, gsum, N, C, HW, relu);
  (void)hipMemcpyAsync(dbeta, gsum, sizeof(float) * C, hipMemcpyDeviceToDevice, st);
  (void)hipMemcpyAsync(dgamma, gsum + C, sizeof(float) * C, hipMemcpyDeviceToDevice, st);
  if (dx) {
    const long total = (long)N * C * HW;
    hipLaunchKernelGGL(fm_bn_bwd_apply_kernel<T>, dim3(fm_grid(total)), dim3(256), 0, st, (const T*)x,
                       (const T*)y, (const T*)dy, meaninv, gsum, gamma, (T*)dx, N, C,
                       HW, relu, acc);
  }
}

static void fm_compact_rows_t(const float* src, float* dst, int K, int n, int ldp, int acc, hipStream_t st) {
  const long total = (long)K * n;
  if (total <= 0) return;
  hipLaunchKernelGGL(fm_compact_kernel, dim3(fm_grid(total)), dim3(256), 0, st, src, dst, K, n, ldp, acc);
}

template <typename T>
static void fm_pad_rows_t(const void* src, void* dst, int K, int n, int ldp, hipStream_t st) {
  const long total = (long)K * ldp;
  if (total <= 0) return;
  hipLaunchKernelGGL(fm_pad_rows_kernel<T>, dim3(fm_grid(total)), dim3(256), 0, st, (const T*)src,
                     (T*)dst, K, n, ldp);
}

}  // namespace

extern "C" {
void fm_im2col(const void* x, void* col, int N, int C, int H, int W, int R, int S, int P, int Q, int sh, int sw, int pt, int pl, int ldcol, int bf16, hipStream_t st) {
  if (bf16) fm_im2col_t<unsigned short>(x, col, N, C, H, W, R, S, P, Q, sh, sw, pt, pl, ldcol, st);
  else fm_im2col_t<float>(x, col, N, C, H, W, R, S, P, Q, sh, sw, pt, pl, ldcol, st);
}
void fm_col2im(const void* dcol, void* dx, int N, int C, int H, int W, int R, int S, int P, int Q, int sh, int sw, int pt, int pl, int ldcol, int acc, int bf16, hipStream_t st) {
  if (bf16) fm_col2im_t<unsigned short>(dcol, dx, N, C, H, W, R, S, P, Q, sh, sw, pt, pl, ldcol, acc, st);
  else fm_col2im_t<float>(dcol, dx, N, C, H, W, R, S, P, Q, sh, sw, pt, pl, ldcol, acc, st);
}
void fm_transpose_batched(const void* in, const void* yin, void* out, int N, int A, int B, int act, int mode, int bf16, hipStream_t st) {
  if (bf16) fm_transpose_batched_t<unsigned short>(in, yin, out, N, A, B, act, mode, st);
  else fm_transpose_batched_t<float>(in, yin, out, N, A, B, act, mode, st);
}
void fm_pool_fwd(const void* x, void* y, unsigned char* code, int N, int C, int H, int W, int P, int Q, int kh, int kw, int sh, int sw, int pt, int pl, int is_max, int act, int bf16, hipStream_t st) {
  if (bf16) fm_pool_fwd_t<unsigned short>(x, y, code, N, C, H, W, P, Q, kh, kw, sh, sw, pt, pl, is_max, act, st);
  else fm_pool_fwd_t<float>(x, y, code, N, C, H, W, P, Q, kh, kw, sh, sw, pt, pl, is_max, act, st);
}
void fm_pool_bwd(const void* x, const void* y, const void* dy, void* dx, unsigned char* code, int code_ready, int N, int C, int H, int W, int P, int Q, int kh, int kw, int sh, int sw, int pt, int pl, int is_max, int act, int acc, int bf16, hipStream_t st) {
  if (bf16) fm_pool_bwd_t<unsigned short>(x, y, dy, dx, code, code_ready, N, C, H, W, P, Q, kh, kw, sh, sw, pt, pl, is_max, act, acc, st);
  else fm_pool_bwd_t<float>(x, y, dy, dx, code, code_ready, N, C, H, W, P, Q, kh, kw, sh, sw, pt, pl, is_max, act, acc, st);
}
void fm_bn_fwd(const void* x, void* y, const float* gamma, const float* beta, float* stats, float* meaninv, int N, int C, int HW, float eps, int relu, int bf16, hipStream_t st) {
  if (bf16) fm_bn_fwd_t<unsigned short>(x, y, gamma, beta, stats, meaninv, N, C, HW, eps, relu, st);
  else fm_bn_fwd_t<float>(x, y, gamma, beta, stats, meaninv, N, C, HW, eps, relu, st);
}
void fm_bn_bwd(const void* x, const void* y, const void* dy, const float* meaninv, const float* gamma, float* gsum, float* dgamma, float* dbeta, void* dx, int N, int C, int HW, int relu, int acc, int bf16, hipStream_t st) {
  if (bf16) fm_bn_bwd_t<unsigned short>(x, y, dy, meaninv, gamma, gsum, dgamma, dbeta, dx, N, C, HW, relu, acc, st);
  else fm_bn_bwd_t<float>(x, y, dy, meaninv, gamma, gsum, dgamma, dbeta, dx, N, C, HW, relu, acc, st);
}
void fm_pad_rows(const void* src, void* dst, int K, int n, int ldp, int bf16, hipStream_t st) {
  if (bf16) fm_pad_rows_t<unsigned short>(src, dst, K, n, ldp, st);
  else fm_pad_rows_t<float>(src, dst, K, n, ldp, st);
}

void fm_strided_copy4_run(const void* src, void* dst, int bf16, const int* d, const long* ss, const long* ts, long so,
                          long to, int acc, hipStream_t st) {
  Strided4 g;
  long total = 1;
  for (int k = 0; k < 4; ++k) {
    g.d[k] = d[k];
    g.ss[k] = ss[k];
    g.ts[k] = ts[k];
    total *= d[k];
  }
  g.so = so;
  g.to = to;
  if (total <= 0) return;
  if (bf16) hipLaunchKernelGGL(fm_strided_copy4<unsigned short>, dim3(fm_grid(total, 256, 8192)), dim3(256), 0, st,
                               (const unsigned short*)src, (unsigned short*)dst, g, total, acc);
  else hipLaunchKernelGGL(fm_strided_copy4<float>, dim3(fm_grid(total, 256, 8192)), dim3(256), 0, st, (const float*)src,
                          (float*)dst, g, total, acc);
}

void fm_compact_rows(const float* src, float* dst, int K, int n, int ldp, int acc, hipStream_t st) {
  fm_compact_rows_t(src, dst, K, n, ldp, acc, st);
}
}  // extern "C"
