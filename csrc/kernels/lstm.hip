// LSTM cell kernels for gfx950 (NMT workload; replaces cuDNN cudnnRNNForwardTraining /
// BackwardData / BackwardWeights in nmt/lstm.cu:323-498).
//
// The recurrence is split between the MFMA GEMM and these pointwise kernels:
//   forward   G = X.W_ih^T + b            (one GEMM over all B*T rows, fp32 gates)
//             per step t: G_t += h_{t-1}.W_hh^T (GEMM, beta=1) ; fm_lstm_cell_fwd
//   backward  per step t (reverse): fm_lstm_cell_bwd -> dG_t ; dh_{t-1} = dG_t.W_hh (GEMM)
//             then dW_ih = dG^T.X (+db row sums), dW_hh = dG^T.Hprev, dX = dG.W_ih (3 GEMMs)
// Gate order i, f, g, o (PyTorch).  Batch-major buffers: row b*T + t.  The forward kernel
// overwrites the pre-activations with the activations (what the backward needs), keeps the
// cell state in fp32, and writes h_t (activation dtype: bf16 or fp32) to the output y[b, t] and to Hprev[b, t+1] -- the
// A operand of the next step's recurrent GEMM and of the dW_hh GEMM.
#include "common.h"

namespace {

FM_DEVICE float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

// h0/c0 (bf16 [B,H], optional) -> Hprev[b, 0] (bf16) and c_init (fp32 [B,H])
template <typename T>
__global__ void fm_lstm_init_kernel(const T* __restrict__ h0, const T* __restrict__ c0,
                                    T* __restrict__ hprev, long ldhp, float* __restrict__ cinit, int B,
                                    int H) {
  const long total = (long)B * H;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long b = i / H, j = i % H;
    hprev[b * ldhp + j] = h0 ? h0[i] : fromf<T>(0.f);
    cinit[i] = c0 ? tof(c0[i]) : 0.f;
  }
}

// one time step.  G rows (ldg), c_prev/c_out fp32 (ldc), y bf16 (ldy), hprev_next bf16 (ldhp,
// null at the last step), hT/cT bf16 [B,H] written at the last step (optional)
template <typename T>
__global__ void fm_lstm_cell_fwd_kernel(float* __restrict__ G, long ldg, const float* __restrict__ c_prev, long ldcp,
                                        float* __restrict__ c_out, long ldc, T* __restrict__ y, long ldy,
                                        T* __restrict__ hprev_next, long ldhp, T* __restrict__ hT,
                                        T* __restrict__ cT, int B, int H) {
  const long total = (long)B * H;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long b = i / H, j = i % H;
    float* g = G + b * ldg;
    const float ig = sigm(g[j]), fg = sigm(g[H + j]), gg = tanhf(g[2 * H + j]), og = sigm(g[3 * H + j]);
    const float c = fg * c_prev[b * ldcp + j] + ig * gg;
    const float h = og * tanhf(c);
    g[j] = ig;
    g[H + j] = fg;
    g[2 * H + j] = gg;
    g[3 * H + j] = og;
    c_out[b * ldc + j] = c;
    const T hb = fromf<T>(h);
    y[b * ldy + j] = hb;
    if (hprev_next) hprev_next[b * ldhp + j] = hb;
    if (hT) hT[i] = hb;
    if (cT) cT[i] = fromf<T>(c);
  }
}

// backward of one step.  A (activations, fp32, lda), c_t / c_prev fp32, dy bf16 (ldy, may be
// null), dh/dc fp32 [B,H] carries (dh in: dL/dh_t from step t+1; dc in/out), dG bf16 (lddg)
template <typename T>
__global__ void fm_lstm_cell_bwd_kernel(const float* __restrict__ A, long lda, const float* __restrict__ c_t, long ldc,
                                        const float* __restrict__ c_prev, long ldcp, const T* __restrict__ dy,
                                        long ldy, const float* __restrict__ dh, float* __restrict__ dc,
                                        T* __restrict__ dG, long lddg, int B, int H) {
  const long total = (long)B * H;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long b = i / H, j = i % H;
    const float* a = A + b * lda;
    const float ig = a[j], fg = a[H + j], gg = a[2 * H + j], og = a[3 * H + j];
    const float c = c_t[b * ldc + j];
    const float tc = tanhf(c);
    const float dht = dh[i] + (dy ? tof(dy[b * ldy + j]) : 0.f);
    const float dct = dc[i] + dht * og * (1.f - tc * tc);
    const float cp = c_prev[b * ldcp + j];
    T* d = dG + b * lddg;
    d[j] = fromf<T>(dct * gg * ig * (1.f - ig));
    d[H + j] = fromf<T>(dct * cp * fg * (1.f - fg));
    d[2 * H + j] = fromf<T>(dct * ig * (1.f - gg * gg));
    d[3 * H + j] = fromf<T>(dht * tc * og * (1.f - og));
    dc[i] = dct * fg;
  }
}

}  // namespace

extern "C" {

// bf16 != 0: activation / gradient tensors (h0, c0, Hprev, y, hT, cT, dy, dG) are bf16, else fp32
void fm_lstm_init(const void* h0, const void* c0, void* hprev, long ldhp, float* cinit, int B, int H, int bf16, hipStream_t s) {
  const long total = (long)B * H;
  if (bf16)
    hipLaunchKernelGGL(fm_lstm_init_kernel<unsigned short>, dim3(fm_grid(total)), dim3(256), 0, s, (const unsigned short*)h0,
                       (const unsigned short*)c0, (unsigned short*)hprev, ldhp, cinit, B, H);
  else
    hipLaunchKernelGGL(fm_lstm_init_kernel<float>, dim3(fm_grid(total)), dim3(256), 0, s, (const float*)h0, (const float*)c0,
                       (float*)hprev, ldhp, cinit, B, H);
}

void fm_lstm_cell_fwd(float* G, long ldg, const float* c_prev, long ldcp, float* c_out, long ldc, void* y, long ldy,
                      void* hprev_next, long ldhp, void* hT, void* cT, int B, int H, int bf16, hipStream_t s) {
  const long total = (long)B * H;
  if (bf16)
    hipLaunchKernelGGL(fm_lstm_cell_fwd_kernel<unsigned short>, dim3(fm_grid(total)), dim3(256), 0, s, G, ldg, c_prev, ldcp,
                       c_out, ldc, (unsigned short*)y, ldy, (unsigned short*)hprev_next, ldhp, (unsigned short*)hT,
                       (unsigned short*)cT, B, H);
  else
    hipLaunchKernelGGL(fm_lstm_cell_fwd_kernel<float>, dim3(fm_grid(total)), dim3(256), 0, s, G, ldg, c_prev, ldcp, c_out,
                       ldc, (float*)y, ldy, (float*)hprev_next, ldhp, (float*)hT, (float*)cT, B, H);
}

void fm_lstm_cell_bwd(const float* A, long lda, const float* c_t, long ldc, const float* c_prev, long ldcp,
                      const void* dy, long ldy, const float* dh, float* dc, void* dG, long lddg, int B, int H, int bf16,
                      hipStream_t s) {
  const long total = (long)B * H;
  if (bf16)
    hipLaunchKernelGGL(fm_lstm_cell_bwd_kernel<unsigned short>, dim3(fm_grid(total)), dim3(256), 0, s, A, lda, c_t, ldc,
                       c_prev, ldcp, (const unsigned short*)dy, ldy, dh, dc, (unsigned short*)dG, lddg, B, H);
  else
    hipLaunchKernelGGL(fm_lstm_cell_bwd_kernel<float>, dim3(fm_grid(total)), dim3(256), 0, s, A, lda, c_t, ldc, c_prev, ldcp,
                       (const float*)dy, ldy, dh, dc, (float*)dG, lddg, B, H);
}

}  // extern "C"
