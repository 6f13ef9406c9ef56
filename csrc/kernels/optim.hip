// Fused optimizer updates over a rank's flat parameter buffer (replaces the per-parameter Legion
// tasks of src/runtime/optimizer_kernel.cu:23-41 sgd_update and :134-154 adam_update, and the
// gradient-replica sums of :96-101 / :220-225 which RCCL all-reduce now does).
// ONE launch updates every parameter shard of the rank: fp32 master weights, optional momentum /
// Adam state, and the bf16 compute mirror written in the same pass (no separate cast kernel).
// Vectorised 16-B loads/stores; lr is read from device memory so the step is graph-capturable.
#include "common.h"

namespace {

__global__ void fm_sgd_kernel(float* __restrict__ W, float* __restrict__ G, float* __restrict__ V,
                              unsigned short* __restrict__ Wc, const float* __restrict__ lr_p, long n, float wd,
                              float mom, int nesterov, int vec, int zero_g) {
  // zero_g: the gradient is consumed here -- write it back as 0 so the next step's backward
  // starts from a clean accumulator without a separate memset (Executor._optimizer_step)
  const float lr = lr_p[0];
  const long n4 = vec ? n / 4 : 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    f32x4_t w = reinterpret_cast<f32x4_t*>(W)[i];
    f32x4_t g = reinterpret_cast<f32x4_t*>(G)[i] + wd * w;
    if (zero_g) reinterpret_cast<f32x4_t*>(G)[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    if (mom > 0.f) {
      f32x4_t v = reinterpret_cast<f32x4_t*>(V)[i] * mom + g;
      reinterpret_cast<f32x4_t*>(V)[i] = v;
      g = nesterov ? g + mom * v : v;
    }
    w -= lr * g;
    reinterpret_cast<f32x4_t*>(W)[i] = w;
    if (Wc) {
      bf16x4_t o;
      o[0] = (short)f2bf(w[0]); o[1] = (short)f2bf(w[1]); o[2] = (short)f2bf(w[2]); o[3] = (short)f2bf(w[3]);
      reinterpret_cast<bf16x4_t*>(Wc)[i] = o;
    }
  }
  // tail
  for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float g = G[i] + wd * W[i];
    if (zero_g) G[i] = 0.f;
    if (mom > 0.f) {
      float v = V[i] * mom + g;
      V[i] = v;
      g = nesterov ? g + mom * v : v;
    }
    W[i] -= lr * g;
    if (Wc) Wc[i] = f2bf(W[i]);
  }
}

// The same update over up to 32 disjoint ranges of one flat buffer (blockIdx.y = range): the
// parameters left to the optimizer launch when most weights were updated inside their dW GEMMs
// (gemm.hip fm_gemm_dw_sgd) -- one launch instead of one per bias-sized gap.
struct SgdSegs {
  long off[32];
  long len[32];
};

__global__ void fm_sgd_segs_kernel(float* __restrict__ W, float* __restrict__ G, float* __restrict__ V,
                                   unsigned short* __restrict__ Wc, const float* __restrict__ lr_p, SgdSegs segs,
                                   float wd, float mom, int nesterov, int zero_g) {
  const float lr = lr_p[0];
  const long o = segs.off[blockIdx.y], n = segs.len[blockIdx.y];
  // scalar head up to a 4-element boundary of the flat buffers (16-B W / G / V, 8-B Wc), vector body
  const long head = min(n, (4 - (o & 3)) & 3L);
  const long n4 = (n - head) / 4;
  const long stride = (long)gridDim.x * blockDim.x, t0 = blockIdx.x * (long)blockDim.x + threadIdx.x;
  auto one = [&](long i) {
    float gi = G[i] + wd * W[i];
    if (zero_g) G[i] = 0.f;
    if (mom > 0.f) {
      const float vi = V[i] * mom + gi;
      V[i] = vi;
      gi = nesterov ? gi + mom * vi : vi;
    }
    const float wi = W[i] - lr * gi;
    W[i] = wi;
    if (Wc) Wc[i] = f2bf(wi);
  };
  for (long i = t0; i < head; i += stride) one(o + i);
  const long b = o + head;   // multiple of 4
  for (long i = t0; i < n4; i += stride) {
    const long e = b + 4 * i;
    f32x4_t w = *reinterpret_cast<const f32x4_t*>(W + e);
    f32x4_t g = *reinterpret_cast<const f32x4_t*>(G + e) + wd * w;
    if (zero_g) *reinterpret_cast<f32x4_t*>(G + e) = f32x4_t{0.f, 0.f, 0.f, 0.f};
    if (mom > 0.f) {
      const f32x4_t v = *reinterpret_cast<const f32x4_t*>(V + e) * mom + g;
      *reinterpret_cast<f32x4_t*>(V + e) = v;
      g = nesterov ? g + mom * v : v;
    }
    w -= lr * g;
    *reinterpret_cast<f32x4_t*>(W + e) = w;
    if (Wc) {
      bf16x4_t c;
      c[0] = (short)f2bf(w[0]); c[1] = (short)f2bf(w[1]); c[2] = (short)f2bf(w[2]); c[3] = (short)f2bf(w[3]);
      *reinterpret_cast<bf16x4_t*>(Wc + e) = c;
    }
  }
  for (long i = head + 4 * n4 + t0; i < n; i += stride) one(o + i);
}

__global__ void fm_adam_kernel(float* __restrict__ W, float* __restrict__ G, float* __restrict__ M,
                               float* __restrict__ V, unsigned short* __restrict__ Wc, long n,
                               const float* __restrict__ alpha_t_p, float b1, float b2, float wd, float eps,
                               int zero_g) {
  const float alpha_t = alpha_t_p[0];  // device-side bias-corrected step size (graph-capturable)
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float w = W[i];
    float g = G[i] + wd * w;
    if (zero_g) G[i] = 0.f;
    float m = b1 * M[i] + (1.f - b1) * g;
    float v = b2 * V[i] + (1.f - b2) * g * g;
    M[i] = m;
    V[i] = v;
    w -= alpha_t * m / (sqrtf(v) + eps);
    W[i] = w;
    if (Wc) Wc[i] = f2bf(w);
  }
}

__global__ void fm_cast_bf16_kernel(const float* __restrict__ src, unsigned short* __restrict__ dst, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) dst[i] = f2bf(src[i]);
}

}  // namespace

extern "C" void fm_sgd_update(float* W, float* G, float* V, unsigned short* Wc, const float* lr, long n, float wd,
                              float mom, int nesterov, int zero_g, hipStream_t s) {
  if (n <= 0) return;
  bool al = ((((uintptr_t)W) | ((uintptr_t)G) | ((uintptr_t)(V ? V : W))) & 15) == 0 && ((((uintptr_t)(Wc ? Wc : (unsigned short*)W)) & 7) == 0);
  hipLaunchKernelGGL(fm_sgd_kernel, dim3(fm_grid(al ? n / 4 + 1 : n)), dim3(256), 0, s, W, G, V, Wc, lr, n, wd, mom,
                     nesterov, al ? 1 : 0, zero_g);
}

extern "C" void fm_sgd_update_segs(float* W, float* G, float* V, unsigned short* Wc, const float* lr, const long* off,
                                   const long* len, int nseg, float wd, float mom, int nesterov, int zero_g,
                                   hipStream_t s) {
  for (int b = 0; b < nseg; b += 32) {
    SgdSegs sg;
    long mx = 0;
    const int k = nseg - b < 32 ? nseg - b : 32;
    for (int i = 0; i < 32; ++i) {
      sg.off[i] = i < k ? off[b + i] : 0;
      sg.len[i] = i < k ? len[b + i] : 0;
      mx = sg.len[i] > mx ? sg.len[i] : mx;
    }
    if (mx <= 0) continue;
    const long per = (mx + 3) / 4;   // one 4-element group per thread
    const int gx = (int)((per + 255) / 256 < 1024 ? (per + 255) / 256 : 1024);
    hipLaunchKernelGGL(fm_sgd_segs_kernel, dim3(gx, k), dim3(256), 0, s, W, G, V, Wc, lr, sg, wd, mom, nesterov, zero_g);
  }
}

extern "C" void fm_adam_update(float* W, float* G, float* M, float* V, unsigned short* Wc, long n,
                               const float* alpha_t, float b1, float b2, float wd, float eps, int zero_g,
                               hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(fm_adam_kernel, dim3(fm_grid(n)), dim3(256), 0, s, W, G, M, V, Wc, n, alpha_t, b1, b2, wd, eps,
                     zero_g);
}

extern "C" void fm_cast_bf16(const float* src, unsigned short* dst, long n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(fm_cast_bf16_kernel, dim3(fm_grid(n)), dim3(256), 0, s, src, dst, n);
}
