// Counter-based parameter initialisation (replaces the cuRAND tasks of
// src/runtime/initializer_kernel.cu:24-295).  Element i of the LOGICAL tensor gets f(seed, i), so
// every GPU fills only its own shard (a 100 GB embedding table is initialised in place, in
// parallel) and any sharding reproduces the unsharded values bit-for-bit.  Same hash as
// flexmi/core/initializers.py (lowbias32 twice over the 64-bit element index).
#include "common.h"

namespace {

FM_DEVICE unsigned lowbias32(unsigned x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

FM_DEVICE unsigned hash64(unsigned seed, unsigned long long idx) {
  unsigned lo = (unsigned)(idx & 0xFFFFFFFFull), hi = (unsigned)(idx >> 32);
  unsigned h = lowbias32(hi ^ lowbias32(seed ^ 0x9E3779B9u));
  return lowbias32(lo ^ h);
}

FM_DEVICE double u01(unsigned seed, unsigned long long idx) {
  return (double)(hash64(seed, idx) >> 8) * (1.0 / 16777216.0);
}

// Fill a 2-D box [r0, r0+rows) x [c0, c0+cols) of a logical [*, ldg] tensor into a dense
// [rows, cols] shard.  kind: 0 zero, 1 constant a, 2 uniform[a,b), 3 normal(a, b)
__global__ void fm_init_kernel(float* out, long rows, long cols, long r0, long c0, long ldg,
                               int kind, unsigned seed, float a, float b) {
  const long total = rows * cols;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    long r = e / cols, c = e % cols;
    unsigned long long gi = (unsigned long long)((r0 + r) * ldg + (c0 + c));
    float v;
    if (kind == 0) v = 0.f;
    else if (kind == 1) v = a;
    else if (kind == 2) v = (float)(a + (b - a) * u01(seed, gi));
    else {
      double x1 = u01(seed, 2ull * gi), x2 = u01(seed, 2ull * gi + 1ull);
      double z = sqrt(-2.0 * log(1.0 - x1)) * cos(6.283185307179586 * x2);
      v = (float)(a + b * z);
    }
    out[e] = v;
  }
}

}  // namespace

extern "C" void fm_init_fill(float* out, long rows, long cols, long r0, long c0, long ldg, int kind,
                             unsigned seed, float a, float b, hipStream_t s) {
  long total = rows * cols;
  if (total <= 0) return;
  hipLaunchKernelGGL(fm_init_kernel, dim3(fm_grid(total, 256, 8192)), dim3(256), 0, s, out, rows, cols,
                     r0, c0, ldg, kind, seed, a, b);
}
