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
// cell state in fp32, and writes h_t (bf16) to the output y[b, t] and to Hprev[b, t+1] -- the
// A operand of the next step's recurrent GEMM and of the dW_hh GEMM.
#include "common.h"

namespace {

FM_DEVICE float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

// h0/c0 (bf16 [B,H], optional) -> Hprev[b, 0] (bf16) and c_init (fp32 [B,H])
__global__ void fm_lstm_init_kernel(const unsigned short* __restrict__ h0, const unsigned short* __restrict__ c0,
                                    unsigned short* __restrict__ hprev, long ldhp, float* __restrict__ cinit, int B,
                                    int H) {
  const long total = (long)B * H;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long b = i / H, j = i % H;
    hprev[b * ldhp + j] = h0 ? h0[i] : (unsigned short)0;
    cinit[i] = c0 ? bf2f(c0[i]) : 0.f;
  }
}

// one time step.  G rows (ldg), c_prev/c_out fp32 (ldc), y bf16 (ldy), hprev_next bf16 (ldhp,
// null at the last step), hT/cT bf16 [B,H] written at the last step (optional)
__global__ void fm_lstm_cell_fwd_kernel(float* __restrict__ G, long ldg, const float* __restrict__ c_prev, long ldcp,
                                        float* __restrict__ c_out, long ldc, unsigned short* __restrict__ y, long ldy,
                                        unsigned short* __restrict__ hprev_next, long ldhp, unsigned short* __restrict__ hT,
                                        unsigned short* __restrict__ cT, int B, int H) {
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
    const unsigned short hb = f2bf(h);
    y[b * ldy + j] = hb;
    if (hprev_next) hprev_next[b * ldhp + j] = hb;
    if (hT) hT[i] = hb;
    if (cT) cT[i] = f2bf(c);
  }
}

// backward of one step.  A (activations, fp32, lda), c_t / c_prev fp32, dy bf16 (ldy, may be
// null), dh/dc fp32 [B,H] carries (dh in: dL/dh_t from step t+1; dc in/out), dG bf16 (lddg)
__global__ void fm_lstm_cell_bwd_kernel(const float* __restrict__ A, long lda, const float* __restrict__ c_t, long ldc,
                                        const float* __restrict__ c_prev, long ldcp, const unsigned short* __restrict__ dy,
                                        long ldy, const float* __restrict__ dh, float* __restrict__ dc,
                                        unsigned short* __restrict__ dG, long lddg, int B, int H) {
  const long total = (long)B * H;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long b = i / H, j = i % H;
    const float* a = A + b * lda;
    const float ig = a[j], fg = a[H + j], gg = a[2 * H + j], og = a[3 * H + j];
    const float c = c_t[b * ldc + j];
    const float tc = tanhf(c);
    const float dht = dh[i] + (dy ? bf2f(dy[b * ldy + j]) : 0.f);
    const float dct = dc[i] + dht * og * (1.f - tc * tc);
    const float cp = c_prev[b * ldcp + j];
    unsigned short* d = dG + b * lddg;
    d[j] = f2bf(dct * gg * ig * (1.f - ig));
    d[H + j] = f2bf(dct * cp * fg * (1.f - fg));
    d[2 * H + j] = f2bf(dct * ig * (1.f - gg * gg));
    d[3 * H + j] = f2bf(dht * tc * og * (1.f - og));
    dc[i] = dct * fg;
  }
}

}  // namespace

extern "C" {

void fm_lstm_init(const void* h0, const void* c0, void* hprev, long ldhp, float* cinit, int B, int H, hipStream_t s) {
  const long total = (long)B * H;
  hipLaunchKernelGGL(fm_lstm_init_kernel, dim3(fm_grid(total)), dim3(256), 0, s, (const unsigned short*)h0,
                     (const unsigned short*)c0, (unsigned short*)hprev, ldhp, cinit, B, H);
}

void fm_lstm_cell_fwd(float* G, long ldg, const float* c_prev, long ldcp, float* c_out, long ldc, void* y, long ldy,
                      void* hprev_next, long ldhp, void* hT, void* cT, int B, int H, hipStream_t s) {
  const long total = (long)B * H;
  hipLaunchKernelGGL(fm_lstm_cell_fwd_kernel, dim3(fm_grid(total)), dim3(256), 0, s, G, ldg, c_prev, ldcp, c_out, ldc,
                     (unsigned short*)y, ldy, (unsigned short*)hprev_next, ldhp, (unsigned short*)hT,
                     (unsigned short*)cT, B, H);
}

void fm_lstm_cell_bwd(const float* A, long lda, const float* c_t, long ldc, const float* c_prev, long ldcp,
                      const void* dy, long ldy, const float* dh, float* dc, void* dG, long lddg, int B, int H,
                      hipStream_t s) {
  const long total = (long)B * H;
  hipLaunchKernelGGL(fm_lstm_cell_bwd_kernel, dim3(fm_grid(total)), dim3(256), 0, s, A, lda, c_t, ldc, c_prev, ldcp,
                     (const unsigned short*)dy, ldy, dh, dc, (unsigned short*)dG, lddg, B, H);
}

}  // extern "C"
