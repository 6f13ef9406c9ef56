// Element-wise, data-movement and normalisation kernels:
//   unary fwd/bwd      (src/ops/element_unary.cu: cuDNN activations + exp kernel :283-404)
//   binary fwd/bwd     (src/ops/element_binary.cu: cuDNN OpTensor; DIV asserted there, C9 -- works here)
//   act-bwd + bias-grad column reduction for Linear (src/ops/linear.cu:583-627 reluBackward /
//                       sigmoid_backward + cublasSgemv db) fused in one pass
//   multi-copy         (concat/split fwd+bwd: copy_with_stride / add_with_stride, cuda_helper.cu:70-104;
//                       all pieces of an op in ONE launch from a descriptor table)
//   permute / reverse  (transpose.cu:135-159, reverse.cu:126-144)
//   softmax            (softmax.cu cuDNN softmax; wave per row)
//   dropout            (dropout.cu cuDNN; counter-based mask regenerated in backward: no mask buffer)
// Storage type T is bf16 (unsigned short) or fp32, selected at launch.
#include "common.h"

namespace {

// ---------------------------------------------------------------- unary
FM_DEVICE float un_f(int code, float x) {
  switch (code) {
    case 0: return x > 0.f ? x : 0.f;
    case 1: return 1.f / (1.f + __expf(-x));
    case 2: return tanhf(x);
    case 3: return x > 0.f ? x : (__expf(x) - 1.f);
    default: return __expf(x);
  }
}
FM_DEVICE float un_b(int code, float x, float y, float dy) {
  switch (code) {
    case 0: return x > 0.f ? dy : 0.f;
    case 1: return dy * y * (1.f - y);
    case 2: return dy * (1.f - y * y);
    case 3: return x > 0.f ? dy : dy * (y + 1.f);
    default: return dy * y;
  }
}

// All four kernels take 8 consecutive elements per thread-iteration (one 16-B access per bf16
// operand, two per fp32 operand) when every operand is 16-B aligned, plus a scalar tail: the
// scalar 2-B form ran at ~2.3 TB/s on the ResNet-50 residual adds / ReLUs.
template <typename T>
__global__ void fm_unary_fwd(int code, const T* __restrict__ x, T* __restrict__ y, long n, int vec) {
  const long stride = (long)gridDim.x * blockDim.x;
  long i0 = 0;
  if (vec) {
    const long n8 = n / 8;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += stride) {
      float v[8];
      ld8<T>(x + 8 * i, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = un_f(code, v[j]);
      st8<T>(y + 8 * i, v);
    }
    i0 = n8 * 8;
  }
  for (long i = i0 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) st<T>(y + i, un_f(code, ld<T>(x + i)));
}
template <typename T>
__global__ void fm_unary_bwd(int code, const T* __restrict__ x, const T* __restrict__ y, const T* __restrict__ dy,
                             T* __restrict__ dx, long n, int acc, int vec) {
  const long stride = (long)gridDim.x * blockDim.x;
  long i0 = 0;
  if (vec) {
    const long n8 = n / 8;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += stride) {
      float xv[8], yv[8], g[8];
      ld8<T>(x + 8 * i, xv);
      ld8<T>(y + 8 * i, yv);
      ld8<T>(dy + 8 * i, g);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = un_b(code, xv[j], yv[j], g[j]);
      if (acc) {
        float o[8];
        ld8<T>(dx + 8 * i, o);
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] += o[j];
      }
      st8<T>(dx + 8 * i, g);
    }
    i0 = n8 * 8;
  }
  for (long i = i0 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
    float g = un_b(code, ld<T>(x + i), ld<T>(y + i), ld<T>(dy + i));
    if (acc) g += ld<T>(dx + i);
    st<T>(dx + i, g);
  }
}

// ---------------------------------------------------------------- binary
// relu != 0: y = relu(a op b) (a residual add fused with the ReLU that consumes it); backward
// with ymask: the incoming gradient is masked by (y > 0) first
FM_DEVICE float bin_f(int code, float u, float v) { return code == 0 ? u + v : code == 1 ? u - v : code == 2 ? u * v : u / v; }
FM_DEVICE void bin_b(int code, float g, float u, float v, float& ga, float& gb) {
  if (code == 0) { ga = g; gb = g; }
  else if (code == 1) { ga = g; gb = -g; }
  else if (code == 2) { ga = g * v; gb = g * u; }
  else { ga = g / v; gb = -g * u / (v * v); }
}

template <typename T>
__global__ void fm_binary_fwd(int code, const T* __restrict__ a, const T* __restrict__ b, T* __restrict__ y, long n, int relu,
                              int vec) {
  const long stride = (long)gridDim.x * blockDim.x;
  long i0 = 0;
  if (vec) {
    const long n8 = n / 8;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += stride) {
      float u[8], v[8];
      ld8<T>(a + 8 * i, u);
      ld8<T>(b + 8 * i, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float r = bin_f(code, u[j], v[j]);
        u[j] = relu ? fmaxf(r, 0.f) : r;
      }
      st8<T>(y + 8 * i, u);
    }
    i0 = n8 * 8;
  }
  for (long i = i0 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
    const float r = bin_f(code, ld<T>(a + i), ld<T>(b + i));
    st<T>(y + i, relu ? fmaxf(r, 0.f) : r);
  }
}
template <typename T>
__global__ void fm_binary_bwd(int code, const T* __restrict__ a, const T* __restrict__ b, const T* __restrict__ dy,
                              const T* __restrict__ ymask, T* __restrict__ da, T* __restrict__ db, long n, int acca, int accb,
                              int vec) {
  const long stride = (long)gridDim.x * blockDim.x;
  const bool need_ab = code >= 2;
  long i0 = 0;
  if (vec) {
    const long n8 = n / 8;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += stride) {
      float g[8], u[8] = {0, 0, 0, 0, 0, 0, 0, 0}, v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      ld8<T>(dy + 8 * i, g);
      if (ymask) {
        float m[8];
        ld8<T>(ymask + 8 * i, m);
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = m[j] > 0.f ? g[j] : 0.f;
      }
      if (need_ab) {
        ld8<T>(a + 8 * i, u);
        ld8<T>(b + 8 * i, v);
      }
      float ga[8], gb[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) bin_b(code, g[j], u[j], v[j], ga[j], gb[j]);
      if (da) {
        if (acca) {
          float o[8];
          ld8<T>(da + 8 * i, o);
#pragma unroll
          for (int j = 0; j < 8; ++j) ga[j] += o[j];
        }
        st8<T>(da + 8 * i, ga);
      }
      if (db) {
        if (accb) {
          float o[8];
          ld8<T>(db + 8 * i, o);
#pragma unroll
          for (int j = 0; j < 8; ++j) gb[j] += o[j];
        }
        st8<T>(db + 8 * i, gb);
      }
    }
    i0 = n8 * 8;
  }
  for (long i = i0 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
    float g = ld<T>(dy + i);
    if (ymask && !(ld<T>(ymask + i) > 0.f)) g = 0.f;
    const float u = need_ab ? ld<T>(a + i) : 0.f, v = need_ab ? ld<T>(b + i) : 0.f;
    float ga, gb;
    bin_b(code, g, u, v, ga, gb);
    if (da) st<T>(da + i, ga + (acca ? ld<T>(da + i) : 0.f));
    if (db) st<T>(db + i, gb + (accb ? ld<T>(db + i) : 0.f));
  }
}

// ---------------------------------------------------------------- act bwd + bias grad
// dpre[b][n] = act'(y) * dy ; db[n] += sum_b dpre[b][n].
// A block covers a strip of tpr*8 columns (tpr threads per row, a power of two <= 64; a thread owns
// 8 consecutive columns, 16-B loads) and ROWS rows; its 256 threads take rpb = 256/tpr rows at a
// time -- so a 128-wide layer keeps every lane busy (16 lanes per row, 16 rows per pass) -- and
// each thread handles four such rows per iteration with all their loads issued first.  Partial
// column sums meet in LDS; one fp32 atomic per column per block.
// NY = false: act is the identity (bias gradient = plain column sums of dy): y is never read
template <typename T, bool NY>
__global__ void __launch_bounds__(256) fm_act_bwd_colsum(const T* __restrict__ y, const T* __restrict__ dy,
                                                        T* __restrict__ dpre, float* __restrict__ db,
                                                        long B, int N, int act, int tpr, int ROWS) {
  __shared__ float red[256 * 8];
  const int tid = threadIdx.x;
  const int rpb = 256 / tpr;
  const int sub = tid / tpr, g = tid - sub * tpr;
  const int c0 = blockIdx.x * tpr * 8 + g * 8;
  const long r0 = (long)blockIdx.y * ROWS;
  const long rend = min(B, r0 + ROWS);
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const bool vec = ((N & 7) == 0) && (c0 + 8 <= N);
  if (c0 < N) {
    for (long r = r0 + sub; r < rend; r += 4L * rpb) {
      if (vec) {
        float yy[4][8], gg[4][8];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const long o = min(r + u * rpb, rend - 1) * N + c0;    // clamped: unconditional loads
          if constexpr (NY) ld8<T>(y + o, yy[u]);
          ld8<T>(dy + o, gg[u]);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const long rr = r + u * rpb;
          if (rr >= rend) break;
          float out[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            out[j] = NY ? act_bwd(act, yy[u][j], gg[u][j]) : gg[u][j];
            s[j] += out[j];
          }
          if (dpre) st8<T>(dpre + rr * N + c0, out);
        }
      } else {
        for (int u = 0; u < 4; ++u) {
          const long rr = r + u * rpb;
          if (rr >= rend) break;
          const long o = rr * N + c0;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            if (c0 + j < N) {
              const float gv = NY ? act_bwd(act, ld<T>(y + o + j), ld<T>(dy + o + j)) : ld<T>(dy + o + j);
              s[j] += gv;
              if (dpre) st<T>(dpre + o + j, gv);
            }
          }
        }
      }
    }
  }
  if (!db) return;
#pragma unroll
  for (int j = 0; j < 8; ++j) red[tid * 8 + j] = s[j];
  __syncthreads();
  for (int c = tid; c < tpr * 8; c += 256) {
    const int col = blockIdx.x * tpr * 8 + c;
    if (col < N) {
      const int gc = c >> 3, j = c & 7;
      float v = 0.f;
      for (int q = 0; q < rpb; ++q) v += red[(q * tpr + gc) * 8 + j];
      atomicAdd(db + col, v);
    }
  }
}

// ---------------------------------------------------------------- multi 2-D copy
struct CopyDesc {
  const void* src;
  void* dst;
  long rows, cols, lds, ldd;
  int vec;   // 16-B units: pointers, row bytes and leading dims all multiples of 16 B
};
constexpr int MAXC = 32;   // one launch stages a DLRM batch's 27 inputs
struct CopyTab {
  CopyDesc d[MAXC];
  int n;
  unsigned add;  // bitmask: accumulate into dst
};

template <typename T>
__global__ void fm_multi_copy(CopyTab t) {
  const CopyDesc& d = t.d[blockIdx.y];
  const int add = (t.add >> blockIdx.y) & 1u;
  if (d.vec) {   // 16-B vector path: 8 bf16 / 4 fp32 per thread-iteration
    constexpr int E = 16 / sizeof(T);
    const long cu = d.cols / E, total = d.rows * cu;
    const char* s = reinterpret_cast<const char*>(d.src);
    char* o = reinterpret_cast<char*>(d.dst);
    for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
      const long r = e / cu, c = e - r * cu;
      const u32x4_t* sp = reinterpret_cast<const u32x4_t*>(s + (r * d.lds + c * E) * (long)sizeof(T));
      u32x4_t* op = reinterpret_cast<u32x4_t*>(o + (r * d.ldd + c * E) * (long)sizeof(T));
      u32x4_t v = *sp;
      if (add) {
        u32x4_t w = *op;
        if constexpr (sizeof(T) == 4) {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = __float_as_uint(__uint_as_float(v[j]) + __uint_as_float(w[j]));
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float lo = bf2f((unsigned short)(v[j] & 0xFFFF)) + bf2f((unsigned short)(w[j] & 0xFFFF));
            const float hi = bf2f((unsigned short)(v[j] >> 16)) + bf2f((unsigned short)(w[j] >> 16));
            v[j] = (unsigned)f2bf(lo) | ((unsigned)f2bf(hi) << 16);
          }
        }
      }
      *op = v;
    }
    return;
  }
  const long total = d.rows * d.cols;
  const T* s = reinterpret_cast<const T*>(d.src);
  T* o = reinterpret_cast<T*>(d.dst);
  const bool small = total < 0x7fffffffL;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    long r, c;
    if (small) {  // 32-bit division (64-bit div/mod is a ~100-instruction sequence on gfx950)
      unsigned ue = (unsigned)e, uc = (unsigned)d.cols;
      r = ue / uc;
      c = ue - (unsigned)r * uc;
    } else {
      r = e / d.cols;
      c = e % d.cols;
    }
    float v = ld<T>(s + r * d.lds + c);
    if (add) v += ld<T>(o + r * d.ldd + c);
    st<T>(o + r * d.ldd + c, v);
  }
}

// ---------------------------------------------------------------- permute (N-D <= 6)
struct PermArgs {
  long out_dims[6];
  long in_strides_perm[6];  // stride in the input of output dim i
  int nd;
  int acc;
};
template <typename T>
__global__ void fm_permute(const T* __restrict__ x, T* __restrict__ y, long n, PermArgs a) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    long rem = e, off = 0;
    for (int i = a.nd - 1; i >= 0; --i) {
      long c = rem % a.out_dims[i];
      rem /= a.out_dims[i];
      off += c * a.in_strides_perm[i];
    }
    float v = ld<T>(x + off);
    if (a.acc) v += ld<T>(y + e);
    st<T>(y + e, v);
  }
}

template <typename T>
__global__ void fm_reverse(const T* __restrict__ x, T* __restrict__ y, long outer, long len, long inner, int acc) {
  const long n = outer * len * inner;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    long i = e % inner, t = e / inner;
    long l = t % len, o = t / len;
    float v = ld<T>(x + (o * len + (len - 1 - l)) * inner + i);
    if (acc) v += ld<T>(y + e);
    st<T>(y + e, v);
  }
}

// ---------------------------------------------------------------- softmax (wave per row)
template <typename T>
__global__ void fm_softmax(const T* __restrict__ x, T* __restrict__ y, long rows, int C) {
  const int lane = threadIdx.x & 63;
  const long waves = (long)gridDim.x * (blockDim.x >> 6);
  for (long r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < rows; r += waves) {
    const T* xr = x + r * C;
    float m = -3.4e38f;
    for (int c = lane; c < C; c += 64) m = fmaxf(m, ld<T>(xr + c));
    m = wave_reduce_max(m);
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s += __expf(ld<T>(xr + c) - m);
    s = wave_reduce_sum(s);
    const float inv = 1.f / s;
    for (int c = lane; c < C; c += 64) st<T>(y + r * C + c, __expf(ld<T>(xr + c) - m) * inv);
  }
}

// ---------------------------------------------------------------- dropout (counter-based mask)
FM_DEVICE unsigned mix32(unsigned x) {
  x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
  return x;
}
template <typename T>
__global__ void fm_dropout(const T* __restrict__ x, T* __restrict__ y, long n, float rate, unsigned seed, unsigned step,
                           int acc) {
  const float keep = 1.f / (1.f - rate);
  const unsigned thr = (unsigned)(rate * 4294967295.0);
  const unsigned s2 = mix32(seed ^ mix32(step + 0x9E3779B9u));
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < n; e += (long)gridDim.x * blockDim.x) {
    unsigned h = mix32((unsigned)e ^ mix32(s2 ^ (unsigned)(e >> 32)));
    float v = (h >= thr) ? ld<T>(x + e) * keep : 0.f;
    if (acc) v += ld<T>(y + e);
    st<T>(y + e, v);
  }
}

}  // namespace

#define FM_DISPATCH_T(bf16, KERNEL, ...)                                   \
  do {                                                                      \
    if (bf16) hipLaunchKernelGGL((KERNEL<unsigned short>), __VA_ARGS__);    \
    else hipLaunchKernelGGL((KERNEL<float>), __VA_ARGS__);                  \
  } while (0)

static bool al16h(const void* p) { return p == nullptr || (((uintptr_t)p) & 15) == 0; }
static int vec_grid(long n) { return fm_grid((n + 7) / 8); }

extern "C" void fm_unary_forward(int code, const void* x, void* y, long n, int bf16, hipStream_t s) {
  if (n <= 0) return;
  const int vec = al16h(x) && al16h(y);
  if (bf16) hipLaunchKernelGGL((fm_unary_fwd<unsigned short>), dim3(vec_grid(n)), dim3(256), 0, s, code, (const unsigned short*)x, (unsigned short*)y, n, vec);
  else hipLaunchKernelGGL((fm_unary_fwd<float>), dim3(vec_grid(n)), dim3(256), 0, s, code, (const float*)x, (float*)y, n, vec);
}

extern "C" void fm_unary_backward(int code, const void* x, const void* y, const void* dy, void* dx, long n, int acc, int bf16,
                                  hipStream_t s) {
  if (n <= 0) return;
  const int vec = al16h(x) && al16h(y) && al16h(dy) && al16h(dx);
  if (bf16) hipLaunchKernelGGL((fm_unary_bwd<unsigned short>), dim3(vec_grid(n)), dim3(256), 0, s, code, (const unsigned short*)x,
                               (const unsigned short*)y, (const unsigned short*)dy, (unsigned short*)dx, n, acc, vec);
  else hipLaunchKernelGGL((fm_unary_bwd<float>), dim3(vec_grid(n)), dim3(256), 0, s, code, (const float*)x, (const float*)y,
                          (const float*)dy, (float*)dx, n, acc, vec);
}

extern "C" void fm_binary_forward(int code, const void* a, const void* b, void* y, long n, int relu, int bf16, hipStream_t s) {
  if (n <= 0) return;
  const int vec = al16h(a) && al16h(b) && al16h(y);
  if (bf16) hipLaunchKernelGGL((fm_binary_fwd<unsigned short>), dim3(vec_grid(n)), dim3(256), 0, s, code, (const unsigned short*)a,
                               (const unsigned short*)b, (unsigned short*)y, n, relu, vec);
  else hipLaunchKernelGGL((fm_binary_fwd<float>), dim3(vec_grid(n)), dim3(256), 0, s, code, (const float*)a, (const float*)b, (float*)y,
                          n, relu, vec);
}

extern "C" void fm_binary_backward(int code, const void* a, const void* b, const void* dy, const void* ymask, void* da, void* db,
                                   long n, int acca, int accb, int bf16, hipStream_t s) {
  if (n <= 0) return;
  const int vec = al16h(a) && al16h(b) && al16h(dy) && al16h(ymask) && al16h(da) && al16h(db);
  if (bf16) hipLaunchKernelGGL((fm_binary_bwd<unsigned short>), dim3(vec_grid(n)), dim3(256), 0, s, code, (const unsigned short*)a,
                               (const unsigned short*)b, (const unsigned short*)dy, (const unsigned short*)ymask, (unsigned short*)da,
                               (unsigned short*)db, n, acca, accb, vec);
  else hipLaunchKernelGGL((fm_binary_bwd<float>), dim3(vec_grid(n)), dim3(256), 0, s, code, (const float*)a, (const float*)b,
                          (const float*)dy, (const float*)ymask, (float*)da, (float*)db, n, acca, accb, vec);
}

extern "C" void fm_act_bwd_bias(const void* y, const void* dy, void* dpre, float* db, long B, int N, int act, int bf16,
                                hipStream_t s) {
  if (B <= 0 || N <= 0) return;
  int tpr = 1;
  while (tpr < 64 && tpr * 8 < N) tpr *= 2;                 // threads per row (power of two)
  const int rpb = 256 / tpr;
  const long strips = (N + tpr * 8 - 1) / (tpr * 8);
  // ~256 blocks: few column-sum atomics per address, every CU busy at DLRM sizes (512 blocks
  // measured slower: 12.4 -> 17.2 us at 8192 x 512, gpurun_out r5f)
  const long nrb = std::max<long>(1, 256 / strips);
  long ROWS = (B + nrb - 1) / nrb;
  ROWS = (ROWS + 4L * rpb - 1) / (4L * rpb) * (4L * rpb);
  dim3 grid((unsigned)strips, (unsigned)((B + ROWS - 1) / ROWS));
  const bool ny = act != 10;   // ACT_NONE: column sums of dy only
  if (bf16) {
    if (ny)
      hipLaunchKernelGGL((fm_act_bwd_colsum<unsigned short, true>), grid, dim3(256), 0, s, (const unsigned short*)y,
                         (const unsigned short*)dy, (unsigned short*)dpre, db, B, N, act, tpr, (int)ROWS);
    else
      hipLaunchKernelGGL((fm_act_bwd_colsum<unsigned short, false>), grid, dim3(256), 0, s, (const unsigned short*)y,
                         (const unsigned short*)dy, (unsigned short*)dpre, db, B, N, act, tpr, (int)ROWS);
  } else {
    if (ny)
      hipLaunchKernelGGL((fm_act_bwd_colsum<float, true>), grid, dim3(256), 0, s, (const float*)y, (const float*)dy,
                         (float*)dpre, db, B, N, act, tpr, (int)ROWS);
    else
      hipLaunchKernelGGL((fm_act_bwd_colsum<float, false>), grid, dim3(256), 0, s, (const float*)y, (const float*)dy,
                         (float*)dpre, db, B, N, act, tpr, (int)ROWS);
  }
}

extern "C" void fm_multi_copy2d(int n, const void* const* src, void* const* dst, const long* rows, const long* cols,
                                const long* lds, const long* ldd, int add_mask, int elem_bytes, hipStream_t s) {
  for (int base = 0; base < n; base += MAXC) {
    CopyTab t;
    int m = std::min(MAXC, n - base);
    long maxe = 1;
    for (int i = 0; i < m; ++i) {
      const long E = 16 / elem_bytes;
      const int vec = ((((uintptr_t)src[base + i]) | ((uintptr_t)dst[base + i])) & 15) == 0 && cols[base + i] % E == 0 &&
                      lds[base + i] % E == 0 && ldd[base + i] % E == 0;
      t.d[i] = CopyDesc{src[base + i], dst[base + i], rows[base + i], cols[base + i], lds[base + i], ldd[base + i], vec};
      maxe = std::max(maxe, rows[base + i] * cols[base + i] / (vec ? E : 1));
    }
    t.n = m;
    t.add = base < 32 ? ((unsigned)add_mask >> base) & (m >= 32 ? 0xffffffffu : ((1u << m) - 1u)) : 0u;
    dim3 grid(fm_grid(maxe, 256, 1024), m);
    if (elem_bytes == 2) hipLaunchKernelGGL((fm_multi_copy<unsigned short>), grid, dim3(256), 0, s, t);
    else hipLaunchKernelGGL((fm_multi_copy<float>), grid, dim3(256), 0, s, t);
  }
}

extern "C" void fm_permute_nd(const void* x, void* y, int nd, const long* out_dims, const long* in_strides_perm, int acc,
                              int bf16, hipStream_t s) {
  PermArgs a;
  long n = 1;
  for (int i = 0; i < nd; ++i) {
    a.out_dims[i] = out_dims[i];
    a.in_strides_perm[i] = in_strides_perm[i];
    n *= out_dims[i];
  }
  a.nd = nd;
  a.acc = acc;
  if (n <= 0) return;
  if (bf16) hipLaunchKernelGGL((fm_permute<unsigned short>), dim3(fm_grid(n)), dim3(256), 0, s, (const unsigned short*)x, (unsigned short*)y, n, a);
  else hipLaunchKernelGGL((fm_permute<float>), dim3(fm_grid(n)), dim3(256), 0, s, (const float*)x, (float*)y, n, a);
}

extern "C" void fm_reverse_axis(const void* x, void* y, long outer, long len, long inner, int acc, int bf16, hipStream_t s) {
  long n = outer * len * inner;
  if (n <= 0) return;
  if (bf16) hipLaunchKernelGGL((fm_reverse<unsigned short>), dim3(fm_grid(n)), dim3(256), 0, s, (const unsigned short*)x, (unsigned short*)y, outer, len, inner, acc);
  else hipLaunchKernelGGL((fm_reverse<float>), dim3(fm_grid(n)), dim3(256), 0, s, (const float*)x, (float*)y, outer, len, inner, acc);
}

extern "C" void fm_softmax_fwd(const void* x, void* y, long rows, int C, int bf16, hipStream_t s) {
  if (rows <= 0) return;
  dim3 g((unsigned)std::min<long>((rows + 3) / 4, 4096));
  if (bf16) hipLaunchKernelGGL((fm_softmax<unsigned short>), g, dim3(256), 0, s, (const unsigned short*)x, (unsigned short*)y, rows, C);
  else hipLaunchKernelGGL((fm_softmax<float>), g, dim3(256), 0, s, (const float*)x, (float*)y, rows, C);
}

extern "C" void fm_dropout_apply(const void* x, void* y, long n, float rate, unsigned seed, unsigned step, int acc, int bf16,
                                 hipStream_t s) {
  if (n <= 0) return;
  if (bf16) hipLaunchKernelGGL((fm_dropout<unsigned short>), dim3(fm_grid(n)), dim3(256), 0, s, (const unsigned short*)x, (unsigned short*)y, n, rate, seed, step, acc);
  else hipLaunchKernelGGL((fm_dropout<float>), dim3(fm_grid(n)), dim3(256), 0, s, (const float*)x, (float*)y, n, rate, seed, step, acc);
}
