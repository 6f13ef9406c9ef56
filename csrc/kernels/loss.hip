// Fused loss gradient + training metrics (replaces src/loss_functions/loss_functions.cu:36-181 and
// src/metrics_functions/metrics_functions.cu:57-175, which were two separate passes with one
// atomicAdd per sample per metric).  One pass over the logits computes dL/dlogit = scale*(p - y)
// and accumulates all requested metrics; each block reduces in registers/LDS and issues 8 atomics.
// Slots: 0 all, 1 correct, 2 cce, 3 sparse cce, 4 mse, 5 rmse, 6 mae, 7 loss value.
// clamp_t in (0, 0.5): DLRM --loss-threshold -- predictions are clamped to [t, 1-t] before the
// loss and metrics, and clamped predictions pass no gradient (reference dlrm.cc:129 left it a TODO).
#include "common.h"

namespace {

enum { LOSS_CCE = 50, LOSS_SCCE = 51, LOSS_MSE_AVG = 52, LOSS_MSE_SUM = 53, LOSS_BCE = 54 };
constexpr float LOG_MIN = 1e-7f;

template <typename T>
FM_DEVICE void block_accumulate(float (&v)[8], float* acc) {
  __shared__ float red[8][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    float x = wave_reduce_sum(v[s]);
    if (lane == 0) red[s][wave] = x;
  }
  __syncthreads();
  if (threadIdx.x < 8) {
    float x = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) x += red[threadIdx.x][w];
    if (x != 0.f) atomicAdd(acc + threadIdx.x, x);
  }
}

// wave per row (any C)
template <typename LT, typename GT>
__global__ void __launch_bounds__(256) fm_loss_kernel(const LT* __restrict__ logits, const void* __restrict__ labels,
                                                     GT* __restrict__ grad, long B, int C, int loss_type, float scale,
                                                     float* __restrict__ acc, int mask, float clamp_t) {
  float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int lane = threadIdx.x & 63;
  const long waves = (long)gridDim.x * (blockDim.x >> 6);
  const bool sparse = loss_type == LOSS_SCCE;
  for (long b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); b < B; b += waves) {
    const LT* lp = logits + b * C;
    int lab = sparse ? reinterpret_cast<const int*>(labels)[b] : -1;
    const float* yp = sparse ? nullptr : reinterpret_cast<const float*>(labels) + b * C;
    float best = -3.4e38f, besty = -3.4e38f;
    int bi = 0x7fffffff, byi = 0x7fffffff;
    float se = 0.f, ae = 0.f, cce = 0.f, lossv = 0.f, plab = 1.f;
    for (int c = lane; c < C; c += 64) {
      float p = ld<LT>(lp + c);
      bool clipped = false;
      if (clamp_t > 0.f) {
        const float pc = fminf(fmaxf(p, clamp_t), 1.f - clamp_t);
        clipped = pc != p;
        p = pc;
      }
      float y = sparse ? (c == lab ? 1.f : 0.f) : yp[c];
      if (grad) st<GT>(grad + b * C + c, clipped ? 0.f : scale * (p - y));
      float d = p - y;
      se += d * d;
      ae += fabsf(d);
      if (y > 0.f) cce += -y * __logf(fmaxf(p, LOG_MIN));
      if (p > best || (p == best && c < bi)) { best = p; bi = c; }
      if (y > besty || (y == besty && c < byi)) { besty = y; byi = c; }
      if (c == lab) plab = p;
      if (loss_type == LOSS_BCE) {
        float pc = fminf(fmaxf(p, LOG_MIN), 1.f - LOG_MIN);
        lossv += -(y * __logf(pc) + (1.f - y) * __logf(1.f - pc));
      }
    }
    // wave reductions
    se = wave_reduce_sum(se);
    ae = wave_reduce_sum(ae);
    cce = wave_reduce_sum(cce);
    lossv = wave_reduce_sum(lossv);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      float ob = __shfl_xor(best, o, 64);
      int oi = __shfl_xor(bi, o, 64);
      if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
      float oy = __shfl_xor(besty, o, 64);
      int oyi = __shfl_xor(byi, o, 64);
      if (oy > besty || (oy == besty && oyi < byi)) { besty = oy; byi = oyi; }
      plab = fminf(plab, __shfl_xor(plab, o, 64));
    }
    if (lane == 0) {
      v[0] += 1.f;
      if (mask & 1) {
        bool ok;
        if (C == 1) ok = (ld<LT>(lp) >= 0.5f) == ((sparse ? (float)lab : yp[0]) >= 0.5f);
        else ok = sparse ? (bi == lab) : (bi == byi);
        v[1] += ok ? 1.f : 0.f;
      }
      v[2] += cce;
      if (sparse) v[3] += -__logf(fmaxf(plab, LOG_MIN));
      v[4] += se;
      v[5] += sqrtf(se);
      v[6] += ae;
      if (loss_type == LOSS_BCE) v[7] += lossv;
      else if (loss_type == LOSS_CCE || loss_type == LOSS_SCCE) v[7] += sparse ? -__logf(fmaxf(plab, LOG_MIN)) : cce;
      else v[7] += se;
    }
  }
  block_accumulate<float>(v, acc);
}

// thread per row (C == 1, e.g. DLRM click probability)
template <typename LT, typename GT>
__global__ void __launch_bounds__(256) fm_loss1_kernel(const LT* __restrict__ logits, const float* __restrict__ labels,
                                                      GT* __restrict__ grad, long B, int loss_type, float scale,
                                                      float* __restrict__ acc, int mask, float clamp_t) {
  float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (long b = blockIdx.x * (long)blockDim.x + threadIdx.x; b < B; b += (long)gridDim.x * blockDim.x) {
    float p = ld<LT>(logits + b);
    bool clipped = false;
    if (clamp_t > 0.f) {
      const float pc = fminf(fmaxf(p, clamp_t), 1.f - clamp_t);
      clipped = pc != p;
      p = pc;
    }
    float y = labels[b];
    if (grad) st<GT>(grad + b, clipped ? 0.f : scale * (p - y));
    float d = p - y;
    v[0] += 1.f;
    v[1] += ((p >= 0.5f) == (y >= 0.5f)) ? 1.f : 0.f;
    if (y > 0.f) v[2] += -y * __logf(fmaxf(p, LOG_MIN));
    v[4] += d * d;
    v[5] += fabsf(d);
    v[6] += fabsf(d);
    if (loss_type == LOSS_BCE) {
      float pc = fminf(fmaxf(p, LOG_MIN), 1.f - LOG_MIN);
      v[7] += -(y * __logf(pc) + (1.f - y) * __logf(1.f - pc));
    } else {
      v[7] += d * d;
    }
  }
  if (!(mask & 1)) v[1] = 0.f;
  block_accumulate<float>(v, acc);
}

}  // namespace

extern "C" void fm_loss_fwd_bwd(const void* logits, int logits_bf16, const void* labels, void* grad, int grad_bf16, long B,
                                int C, int loss_type, float scale, float* acc, int mask, float clamp_t, hipStream_t s) {
  if (B <= 0) return;
  if (C == 1 && loss_type != LOSS_SCCE) {
    dim3 g(fm_grid(B, 256, 1024));
#define L1(LT, GT) hipLaunchKernelGGL((fm_loss1_kernel<LT, GT>), g, dim3(256), 0, s, (const LT*)logits, (const float*)labels, (GT*)grad, B, loss_type, scale, acc, mask, clamp_t)
    if (logits_bf16) { if (grad_bf16) L1(unsigned short, unsigned short); else L1(unsigned short, float); }
    else { if (grad_bf16) L1(float, unsigned short); else L1(float, float); }
#undef L1
    return;
  }
  dim3 g((int)std::min<long>((B + 3) / 4, 2048));
#define LW(LT, GT) hipLaunchKernelGGL((fm_loss_kernel<LT, GT>), g, dim3(256), 0, s, (const LT*)logits, labels, (GT*)grad, B, C, loss_type, scale, acc, mask, clamp_t)
  if (logits_bf16) { if (grad_bf16) LW(unsigned short, unsigned short); else LW(unsigned short, float); }
  else { if (grad_bf16) LW(float, unsigned short); else LW(float, float); }
#undef LW
}
