// Common helpers for flexmi CDNA4 (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define FM_HOST_DEVICE __host__ __device__ __forceinline__
#define FM_DEVICE __device__ __forceinline__

typedef short bf16x4_t __attribute__((ext_vector_type(4)));
typedef short bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8v_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// bf16 <-> f32 (round-to-nearest-even via the compiler's cast: keeps NaNs, emits v_cvt_pk_bf16_f32)
FM_DEVICE float bf2f(unsigned short v) { return __uint_as_float(((unsigned)v) << 16); }
FM_DEVICE unsigned short f2bf(float f) {
  __bf16 b = (__bf16)f;
  return *reinterpret_cast<unsigned short*>(&b);
}

// Exact three-way bf16 split of two fp32 values x = h + m + l (truncation: h = x with the low 16
// bits cleared, r = x - h exact, m = r truncated, l = r - m: <= 8 significant bits, already a bf16),
// returned as one packed bf16 pair per plane (a in the low half).  9 VALU per pair: one v_perm_b32
// per plane packs the high halves (truncation needs no mask there), each residual subtraction is
// one v_pk_add_f32, only the fp32 images of h and m need masks.  The per-element form (mask every
// term, shift/or packing) compiled to 26 VALU per pair with SDWA ors and moves into the ds_write
// quads.  A non-finite x gives m = l = NaN (inf - inf): the split GEMMs document it.
FM_DEVICE unsigned fm_hi_pair(unsigned a, unsigned b) { return __builtin_amdgcn_perm(b, a, 0x07060302u); }

FM_DEVICE void fm_split3_pair(float a, float b, unsigned& h, unsigned& m, unsigned& l) {
  typedef float f2_t __attribute__((ext_vector_type(2)));
  const unsigned ua = __float_as_uint(a), ub = __float_as_uint(b);
  h = fm_hi_pair(ua, ub);
  const f2_t x = {a, b};
  const f2_t hf = {__uint_as_float(ua & 0xffff0000u), __uint_as_float(ub & 0xffff0000u)};
  const f2_t r = x - hf;
  const unsigned ra = __float_as_uint(r.x), rb = __float_as_uint(r.y);
  m = fm_hi_pair(ra, rb);
  const f2_t mf = {__uint_as_float(ra & 0xffff0000u), __uint_as_float(rb & 0xffff0000u)};
  const f2_t lf = r - mf;
  l = fm_hi_pair(__float_as_uint(lf.x), __float_as_uint(lf.y));
}

// value conversion generic over float / bf16 storage (tof: storage -> f32, fromf<T>: f32 -> storage)
FM_DEVICE float tof(float v) { return v; }
FM_DEVICE float tof(unsigned short v) { return bf2f(v); }
template <typename T> FM_DEVICE T fromf(float v);
template <> FM_DEVICE float fromf<float>(float v) { return v; }
template <> FM_DEVICE unsigned short fromf<unsigned short>(float v) { return f2bf(v); }

// element loads/stores generic over float / bf16 storage
template <typename T> FM_DEVICE float ld(const T* p);
template <> FM_DEVICE float ld<float>(const float* p) { return *p; }
template <> FM_DEVICE float ld<unsigned short>(const unsigned short* p) { return bf2f(*p); }
template <typename T> FM_DEVICE void st(T* p, float v);
template <> FM_DEVICE void st<float>(float* p, float v) { *p = v; }
template <> FM_DEVICE void st<unsigned short>(unsigned short* p, float v) { *p = f2bf(v); }

// 8 consecutive elements (16-B aligned) as floats: one b128 access for bf16, two for fp32
template <typename T> FM_DEVICE void ld8(const T* p, float (&v)[8]);
template <> FM_DEVICE void ld8<unsigned short>(const unsigned short* p, float (&v)[8]) {
  const bf16x8_t t = *reinterpret_cast<const bf16x8_t*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = bf2f((unsigned short)t[j]);
}
template <> FM_DEVICE void ld8<float>(const float* p, float (&v)[8]) {
  const f32x4_t a = *reinterpret_cast<const f32x4_t*>(p);
  const f32x4_t b = *reinterpret_cast<const f32x4_t*>(p + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[4 + j] = b[j]; }
}
template <typename T> FM_DEVICE void st8(T* p, const float (&v)[8]);
template <> FM_DEVICE void st8<unsigned short>(unsigned short* p, const float (&v)[8]) {
  bf16x8_t t;
#pragma unroll
  for (int j = 0; j < 8; ++j) t[j] = (short)f2bf(v[j]);
  *reinterpret_cast<bf16x8_t*>(p) = t;
}
template <> FM_DEVICE void st8<float>(float* p, const float (&v)[8]) {
  *reinterpret_cast<f32x4_t*>(p) = f32x4_t{v[0], v[1], v[2], v[3]};
  *reinterpret_cast<f32x4_t*>(p + 4) = f32x4_t{v[4], v[5], v[6], v[7]};
}

// activations (ActiMode values of include/ffconst.h)
enum { ACT_NONE = 10, ACT_RELU = 11, ACT_SIGMOID = 12, ACT_TANH = 13 };

FM_DEVICE float act_fwd(int act, float x) {
  if (act == ACT_RELU) return x > 0.f ? x : 0.f;
  if (act == ACT_SIGMOID) return 1.f / (1.f + __expf(-x));
  if (act == ACT_TANH) return tanhf(x);
  return x;
}
// derivative expressed through the activation OUTPUT y
FM_DEVICE float act_bwd(int act, float y, float dy) {
  if (act == ACT_RELU) return y > 0.f ? dy : 0.f;
  if (act == ACT_SIGMOID) return dy * y * (1.f - y);
  if (act == ACT_TANH) return dy * (1.f - y * y);
  return dy;
}

// n / d for 0 <= n < 2^31 by multiply-high (round-up magic; d >= 1): built on the host, passed
// by value in kernel arguments
struct FastDiv {
  unsigned m;
  int l;
};
static inline FastDiv make_fastdiv(int d) {
  FastDiv f;
  int l = 0;
  while ((1L << l) < d) ++l;
  f.l = l;
  f.m = (unsigned)((((1UL << 32) * ((1UL << l) - (unsigned long)d)) / (unsigned long)d) + 1);
  return f;
}
FM_DEVICE int fdiv(int n, FastDiv f) { return (int)((__umulhi((unsigned)n, f.m) + (unsigned)n) >> f.l); }

FM_DEVICE float wave_reduce_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

FM_DEVICE float wave_reduce_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// grid sizing for memory-bound kernels: ~8 blocks per CU on 256 CUs, grid-stride beyond
static inline int fm_grid(long long n, int block = 256, int cap = 2048) {
  long long g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

// order this wave's LDS writes before its later LDS reads (cross-lane) -- compiler + hw fence
#define FM_WAVE_LDS_SYNC() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")

#define FM_CHECK(x)                                                                   \
  do {                                                                                \
    hipError_t e__ = (x);                                                             \
    if (e__ != hipSuccess) {                                                          \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e__), __FILE__, __LINE__); \
    }                                                                                 \
  } while (0)
