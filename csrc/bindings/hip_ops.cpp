// pybind11 bindings of the flexmi HIP kernels (module flexmi._C).
// Kernels live in csrc/kernels/*.hip behind extern "C" launchers (compiled with hipcc for gfx950
// only, no torch headers); this file only unpacks torch tensors into raw pointers and launches on
// PyTorch's current HIP stream, so kernels compose with torch's caching allocator, RCCL streams
// and hipGraph capture.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <cstring>
#include <vector>

extern "C" {
void fm_sgd_update_segs(float* W, float* G, float* V, unsigned short* Wc, const float* lr, const long* off,
                        const long* len, int nseg, float wd, float mom, int nesterov, int zero_g, hipStream_t s);
void fm_image_normalize(const unsigned char* src, void* dst, long N, int H, int W, const float* mean, const float* stdv,
                        int bf16, hipStream_t s);
int fm_gemm_dw_sgd(const void* A, long lda, const void* B, long ldb, float* W, long ldw, unsigned short* Wc, float* V,
                   const float* lr, float wd, float mom, int nesterov, int M, int N, int K, float* ws, long ws_bytes,
                   float* rowsum_a, int cfg, hipStream_t stream);
int fm_gemm_f32_dw_sgd(const float* A, long lda, const float* B, long ldb, float* W, long ldw, unsigned short* Wc,
                       float* V, const float* lr, float wd, float mom, int nesterov, int M, int N, int K, float* ws,
                       long ws_bytes, float* rowsum_a, int cfg, hipStream_t stream);
int fm_gemm(const void* A, long lda, long sA, int a_kcontig, const void* B, long ldb, long sB, int b_kcontig, void* C,
            long ldc, long sC, int c_fp32, const float* bias, int M, int N, int K, int batch, float alpha, int beta,
            int act, float* ws, long ws_bytes, int ksplit_req, const void* act_y, long lday, int bwd_act,
            float* colsum, float* rowsum_a, hipStream_t stream);
void fm_gemm_f32_set_split(int on);
void fm_gemm_set_dma(int on);
int fm_gemm_dma_enabled();
void fm_embedding_set_bwd_mode(int count);
int fm_gemm_f32_get_split();
int fm_gemm_f32_last_form();
int fm_gemm_f32(const float* A, long lda, long sA, int a_kcontig, const float* B, long ldb, long sB, int b_kcontig,
                float* C, long ldc, long sC, const float* bias, int M, int N, int K, int batch, float alpha, int beta,
                int act, float* ws, long ws_bytes, int ksplit_req, const float* act_y, long lday, int bwd_act,
                float* colsum, float* rowsum_a, hipStream_t stream);
int fm_smallk_fwd_launch(const void* x, long ldx, const void* w, const float* bias, void* y, long ldy, long M, int K, int N,
                         int act, int bf16, hipStream_t s);
int fm_smallk_dw_launch(const void* dpre, long ldd, const void* x, long ldx, float* dw, float* db, long M, int K, int N,
                        float* ws, long ws_bytes, float* V, unsigned short* Wc, const float* lr, float wd, float mom,
                        int nesterov, int bf16, hipStream_t s);
void fm_skinny_fwd_f32_launch(const float* x, long ldx, const float* w, const float* bias, float* y, long ldy, long B, int K,
                              int act, hipStream_t s);
void fm_skinny_bwd_f32_launch(const float* x, long ldx, const float* w, const float* y, long ldy, const float* dy, long lddy,
                              float* dx, long lddx, int dx_acc, float* dw, float* db, long B, int K, int act, int bact,
                              hipStream_t s);
void fm_skinny_fwd(const void* x, long ldx, const void* w, const float* bias, void* y, long ldy, long B, int K, int act,
                   hipStream_t s);
void fm_skinny_bwd(const void* x, long ldx, const void* w, const void* y, long ldy, const void* dy, long lddy, void* dx,
                   long lddx, int dx_acc, float* dw, float* db, long B, int K, int act, int bact, hipStream_t s);
void fm_init_fill(float* out, long rows, long cols, long r0, long c0, long ldg, int kind, unsigned seed, float a, float b,
                  hipStream_t s);
void fm_embedding_fwd(const void* idx, int idx64, const float* W, void* out, int out_bf16, long B, int bag, int rows, int D,
                      long ldo, float scale, hipStream_t s);
void fm_embedding_bwd(const void* idx, int idx64, const void* dy, int dy_bf16, float* W, const float* lr, long B, int bag,
                      int rows, int D, long ldg, float scale, hipStream_t s);
void fm_embedding_fwd_multi(int n, const float* const* W, const void* const* idx, const int* idx64, void* const* out,
                            const long* ldo, const long* lo, const int* rows, const int* D, const int* bag,
                            const float* scale, int out_bf16, long B, hipStream_t st);
void fm_embedding_bwd_multi(int n, float* const* W, const void* const* idx, const int* idx64, const void* const* dy,
                            const long* ldg, const long* lo, const int* rows, const int* D, const int* bag,
                            const float* scale, int dy_bf16, const float* lr, long B, int* const* owner,
                            int* const* dups, int* const* ndup, hipStream_t st);
void fm_sdp_coalesce(int n, const void* const* idx, const int* idx64, const void* const* dy, const long* ldg,
                     const long* lo, const int* rows, const int* D, const int* bag, const float* scale, int dy_bf16, long B,
                     int* const* slot, int* const* cid, int* const* ids, float* const* g, int* const* count, hipStream_t st);
void fm_sdp_apply_segments(int n, int segs, int own_seg, float* const* W, const int* D, const int* const* seg_ids,
                           const float* const* seg_g, const int* const* seg_count, int* const* slot, int* const* own_count,
                           const int* nmax, const float* lr, hipStream_t st);
void fm_strided_copy4_run(const void* src, void* dst, int bf16, const int* d, const long* ss, const long* ts, long so,
                          long to, int acc, hipStream_t st);
void fm_dot_interaction_fwd(const void* const* z, int F, long ldz, void* out, long ldo, long B, int D, int W, int self,
                            hipStream_t s);
void fm_dot_interaction_bwd(const void* const* z, int F, long ldz, const void* dout, long ldo, void* const* dz, long lddz,
                            unsigned acc_mask, long B, int D, int self, hipStream_t s);
void fm_dot_interaction_fwd_f32(const float* const* z, int F, long ldz, float* out, long ldo, long B, int D, int W, int self,
                                hipStream_t s);
void fm_dot_interaction_bwd_f32(const float* const* z, int F, long ldz, const float* dout, long ldo, float* const* dz,
                                long lddz, unsigned acc_mask, long B, int D, int self, int act0, hipStream_t s);
void fm_sgd_update(float* W, float* G, float* V, unsigned short* Wc, const float* lr, long n, float wd, float mom,
                   int nesterov, int zero_g, hipStream_t s);
void fm_adam_update(float* W, float* G, float* M, float* V, unsigned short* Wc, long n, const float* alpha_t,
                    float b1, float b2, float wd, float eps, int zero_g, hipStream_t s);
void fm_cast_bf16(const float* src, unsigned short* dst, long n, hipStream_t s);
void fm_loss_fwd_bwd(const void* logits, int logits_bf16, const void* labels, void* grad, int grad_bf16, long B, int C,
                     int loss_type, float scale, float* acc, int mask, float clamp_t, hipStream_t s);
void fm_unary_forward(int code, const void* x, void* y, long n, int bf16, hipStream_t s);
void fm_unary_backward(int code, const void* x, const void* y, const void* dy, void* dx, long n, int acc, int bf16,
                       hipStream_t s);
void fm_binary_forward(int code, const void* a, const void* b, void* y, long n, int relu, int bf16, hipStream_t s);
void fm_binary_backward(int code, const void* a, const void* b, const void* dy, const void* ymask, void* da, void* db,
                        long n, int acca, int accb, int bf16, hipStream_t s);
void fm_act_bwd_bias(const void* y, const void* dy, void* dpre, float* db, long B, int N, int act, int bf16, hipStream_t s);
void fm_multi_copy2d(int n, const void* const* src, void* const* dst, const long* rows, const long* cols, const long* lds,
                     const long* ldd, int add_mask, int elem_bytes, hipStream_t s);
void fm_permute_nd(const void* x, void* y, int nd, const long* out_dims, const long* in_strides_perm, int acc, int bf16,
                   hipStream_t s);
void fm_reverse_axis(const void* x, void* y, long outer, long len, long inner, int acc, int bf16, hipStream_t s);
void fm_softmax_fwd(const void* x, void* y, long rows, int C, int bf16, hipStream_t s);
void fm_dropout_apply(const void* x, void* y, long n, float rate, unsigned seed, unsigned step, int acc, int bf16,
                      hipStream_t s);
void fm_im2col(const void* x, void* col, int N, int C, int H, int W, int R, int S, int P, int Q, int sh, int sw, int pt,
               int pl, int ldcol, int bf16, hipStream_t st);
void fm_col2im(const void* dcol, void* dx, int N, int C, int H, int W, int R, int S, int P, int Q, int sh, int sw, int pt,
               int pl, int ldcol, int acc, int bf16, hipStream_t st);
void fm_transpose_batched(const void* in, const void* yin, void* out, int N, int A, int B, int act, int mode, int bf16,
                          hipStream_t st);
void fm_pool_fwd(const void* x, void* y, unsigned char* code, int N, int C, int H, int W, int P, int Q, int kh, int kw, int sh,
                 int sw, int pt, int pl, int is_max, int act, int bf16, hipStream_t st);
void fm_pool_bwd(const void* x, const void* y, const void* dy, void* dx, unsigned char* code, int code_ready, int N, int C,
                 int H, int W, int P, int Q, int kh, int kw, int sh, int sw, int pt, int pl, int is_max, int act, int acc,
                 int bf16, hipStream_t st);
void fm_bn_fwd(const void* x, void* y, const float* gamma, const float* beta, float* stats, float* meaninv, int N, int C,
               int HW, float eps, int relu, int bf16, hipStream_t st);
void fm_bn_bwd(const void* x, const void* y, const void* dy, const float* meaninv, const float* gamma, float* gsum,
               float* dgamma, float* dbeta, void* dx, int N, int C, int HW, int relu, int acc, int bf16, hipStream_t st);
void fm_compact_rows(const float* src, float* dst, int K, int n, int ldp, int acc, hipStream_t st);
int fm_conv_lda(int cols);
int fm_conv_fwd(const void* x, const void* w, void* wpad, const float* bias, void* y, int bf16, int N, int C, int H, int W,
                int K, int R, int S, int P, int Q, int sh, int sw, int pt, int pl, int act, hipStream_t s);
int fm_conv_dgrad(const void* g, const void* w, void* wt, void* dx, int accum, int bf16, int N, int C, int H, int W, int K,
                  int R, int S, int P, int Q, int sh, int sw, int pt, int pl, hipStream_t s);
int fm_conv_wgrad(const void* g, const void* x, float* dw, int bf16, int N, int C, int H, int W, int K, int R, int S, int P,
                  int Q, int sh, int sw, int pt, int pl, hipStream_t s);
void fm_conv_act_bwd(const void* dy, const void* y, void* g, float* db, int bf16, int N, int K, int PQ, int act,
                     hipStream_t s);
void fm_conv_s2d_run(const void* x, void* xs, int bf16, int N, int C, int H, int W, int s, int pt, int pl, int Hs, int Ws,
                     int inv, int acc, hipStream_t st);
void fm_conv_w_s2d_run(const void* w, void* ws, const float* dws, float* dw, int bf16, int K, int C, int R, int S, int s,
                       int Rs, int Ss, int inv, hipStream_t st);
void fm_pad_rows(const void* src, void* dst, int K, int n, int ldp, int bf16, hipStream_t st);
int fm_stem_supported(int C, int K, int R, int S, int sh, int sw);
long fm_stem_wgrad_ws(int C, int K, int R, int S, int s);
long fm_stem_wf_elems(int C, int K, int R, int S, int s);
int fm_stem_fwd_run(const void* x, const void* w, void* wf, const float* bias, void* y, int N, int C, int H, int W, int R, int S,
                    int P, int Q, int s, int pt, int pl, int act, hipStream_t st);
int fm_stem_wgrad_run(const void* x, const void* y, const void* dy, float* dw, float* db, float* ws, int N, int C, int H,
                      int W, int R, int S, int P, int Q, int s, int pt, int pl, int act, hipStream_t st);
void fm_nhwc_stage_run(const void* src, void* dst, int N, int C, int H, int W, int Cp, int Hp, int Wp, int top, int left,
                       int dh, int dw, hipStream_t s);
void fm_nhwc_stage_grad_run(const void* dy, const void* y, void* dst, int act, int N, int C, int H, int W, int Cp, int Hp,
                            int Wp, int top, int left, int dh, int dw, hipStream_t s);
void fm_conv_nhwc_dgrad_strided(const void* gs, long gs_bytes, const void* w, void* wsub, void* dx, int accum, int N, int C,
                                int H, int W, int K, int R, int S, int Kp, int Hg, int Wg, int gt, int gl, int sh, int sw,
                                void* out2, int H2, int W2, int C2, int t2, int l2, int d2h, int d2w, int write_nchw,
                                hipStream_t s);
long fm_conv_nhwc_wgrad_ws(int N, int K, int P, int Q, int R, int S, int Cp);
void fm_conv_nhwc_set_shape(int mode, int shape);
void fm_cnhwc_wprep_multi_run(int n, const void* const* w, void* const* out, void* const* out2, const int* K, const int* C,
                              const int* R, const int* S, const int* Cp, const int* Kp, hipStream_t s);
void fm_cnhwc_wprep_run(const void* w, void* out, void* out2, const float* g2, float* dw, int K, int C, int R, int S, int Cp,
                        int Kp, int mode, int nsplit, hipStream_t s);
void fm_conv_nhwc_fwd(const void* xs, long xs_bytes, const void* wf, const float* bias, void* y, int N, int K, int P, int Q,
                      int R, int S, int Cp, int Hp, int Wp, int sh, int sw, int act, void* out2, int H2, int W2, int C2, int t2,
                      int l2, int d2h, int d2w, int write_nchw, hipStream_t s);
void fm_conv_nhwc_dgrad(const void* gs, long gs_bytes, const void* wd, void* dx, int accum, int N, int C, int H, int W, int R,
                        int S, int Kp, int Hg, int Wg, void* out2, int H2, int W2, int C2, int t2, int l2, int d2h, int d2w,
                        int write_nchw, hipStream_t s);
int fm_conv_nhwc_wgrad(const void* gs, long gs_bytes, const void* xs, long xs_bytes, float* g2, float* db, int N, int K, int Kp, int P,
                        int Q, int Hg, int Wg, int gt, int gl, int gsh, int gsw, int R, int S, int Cp, int Hp, int Wp, int sh,
                        int sw, int* ptab, int build_tab, hipStream_t s);
void fm_lstm_init(const void* h0, const void* c0, void* hprev, long ldhp, float* cinit, int B, int H, int bf16, hipStream_t s);
void fm_lstm_cell_fwd(float* G, long ldg, const float* c_prev, long ldcp, float* c_out, long ldc, void* y, long ldy,
                      void* hprev_next, long ldhp, void* hT, void* cT, int B, int H, int bf16, hipStream_t s);
void fm_lstm_cell_bwd(const float* A, long lda, const float* c_t, long ldc, const float* c_prev, long ldcp,
                      const void* dy, long ldy, const float* dh, float* dc, void* dG, long lddg, int B, int H, int bf16,
                      hipStream_t s);
}

namespace {

hipStream_t cur() { return at::hip::getCurrentHIPStream().stream(); }

const void* cptr(const c10::optional<torch::Tensor>& t) { return (t.has_value() && t->defined()) ? t->data_ptr() : nullptr; }
void* mptr(const c10::optional<torch::Tensor>& t) { return (t.has_value() && t->defined()) ? t->data_ptr() : nullptr; }

void check_cuda(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a HIP device tensor");
}

int is_bf16(const torch::Tensor& t) { return t.scalar_type() == torch::kBFloat16 ? 1 : 0; }

// ----------------------------------------------------------------------------- GEMM
int gemm(torch::Tensor A, int64_t lda, int64_t sA, bool a_kcontig, torch::Tensor B, int64_t ldb, int64_t sB, bool b_kcontig,
         torch::Tensor C, int64_t ldc, int64_t sC, c10::optional<torch::Tensor> bias, int64_t M, int64_t N, int64_t K,
         int64_t batch, double alpha, bool beta, int64_t act, c10::optional<torch::Tensor> ws, int64_t ksplit,
         c10::optional<torch::Tensor> act_y, int64_t lday, int64_t bwd_act, c10::optional<torch::Tensor> colsum,
         c10::optional<torch::Tensor> rowsum_a) {
  check_cuda(A, "A");
  check_cuda(B, "B");
  check_cuda(C, "C");
  // bf16 operands (MFMA bf16, bf16 or fp32 C) or fp32 operands (reference-precision path:
  // v_mfma_f32_16x16x4_f32, fp32 C, gemm_f32.hip)
  const bool f32 = A.scalar_type() == torch::kFloat32;
  TORCH_CHECK((A.scalar_type() == torch::kBFloat16 && B.scalar_type() == torch::kBFloat16) ||
                  (f32 && B.scalar_type() == torch::kFloat32),
              "gemm operands must both be bf16 or both fp32");
  TORCH_CHECK(C.scalar_type() == torch::kBFloat16 || C.scalar_type() == torch::kFloat32, "gemm output bf16/fp32");
  TORCH_CHECK(!f32 || C.scalar_type() == torch::kFloat32, "fp32 gemm: fp32 output");
  // extent checks (the kernel trusts these): last element of each operand must be inside the storage
  auto lastA = a_kcontig ? (M - 1) * lda + (K - 1) : (K - 1) * lda + (M - 1);
  auto lastB = b_kcontig ? (N - 1) * ldb + (K - 1) : (K - 1) * ldb + (N - 1);
  if (K > 0) {
    TORCH_CHECK(lastA + (batch - 1) * sA < A.numel(), "gemm: A too small");
    TORCH_CHECK(lastB + (batch - 1) * sB < B.numel(), "gemm: B too small");
  }
  TORCH_CHECK((M - 1) * ldc + (N - 1) + (batch - 1) * sC < C.numel(), "gemm: C too small");
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == torch::kFloat32 && bias->numel() >= N, "bias must be fp32 [N]");
  }
  if (act_y.has_value() && act_y->defined()) {
    TORCH_CHECK(act_y->scalar_type() == A.scalar_type() && batch == 1 && (M - 1) * lday + N <= act_y->numel(),
                "gemm act_y: [M, >=N] of the operand dtype");
  }
  if (rowsum_a.has_value() && rowsum_a->defined()) {
    TORCH_CHECK(!a_kcontig && rowsum_a->scalar_type() == torch::kFloat32 && rowsum_a->numel() >= M && batch == 1,
                "gemm rowsum_a: fp32 [M], MN-contiguous A");
  }
  if (colsum.has_value() && colsum->defined()) {
    TORCH_CHECK(colsum->scalar_type() == torch::kFloat32 && colsum->numel() >= N && batch == 1, "gemm colsum: fp32 [N]");
  }
  float* w = nullptr;
  long wsb = 0;
  if (ws.has_value() && ws->defined()) {
    w = ws->data_ptr<float>();
    wsb = ws->numel() * 4;
  }
  int ks;
  if (f32)
    ks = fm_gemm_f32(A.data_ptr<float>(), lda, sA, a_kcontig, B.data_ptr<float>(), ldb, sB, b_kcontig, C.data_ptr<float>(),
                     ldc, sC, bias.has_value() && bias->defined() ? bias->data_ptr<float>() : nullptr, (int)M, (int)N,
                     (int)K, (int)batch, (float)alpha, beta ? 1 : 0, (int)act, w, wsb, (int)ksplit,
                     (const float*)cptr(act_y), lday, (int)bwd_act, (float*)mptr(colsum), (float*)mptr(rowsum_a), cur());
  else
    ks = fm_gemm(A.data_ptr(), lda, sA, a_kcontig, B.data_ptr(), ldb, sB, b_kcontig, C.data_ptr(), ldc, sC,
                 C.scalar_type() == torch::kFloat32, bias.has_value() && bias->defined() ? bias->data_ptr<float>() : nullptr,
                 (int)M, (int)N, (int)K, (int)batch, (float)alpha, beta ? 1 : 0, (int)act, w, wsb, (int)ksplit,
                 cptr(act_y), lday, (int)bwd_act, (float*)mptr(colsum), (float*)mptr(rowsum_a), cur());
  return ks;
}


// fm_sgd over disjoint [off, off + len) ranges of one flat master / grad / state / mirror set
void sgd_segs(torch::Tensor W, torch::Tensor G, c10::optional<torch::Tensor> V, c10::optional<torch::Tensor> Wc,
              torch::Tensor lr, std::vector<int64_t> off, std::vector<int64_t> len, double wd, double mom, bool nesterov,
              bool zero_g) {
  TORCH_CHECK(off.size() == len.size(), "sgd_segs: off/len");
  TORCH_CHECK(W.is_cuda() && W.scalar_type() == torch::kFloat32 && W.is_contiguous() && G.scalar_type() == torch::kFloat32 &&
                  G.is_contiguous() && G.numel() == W.numel(), "sgd_segs: fp32 W / G");
  TORCH_CHECK(mom <= 0.0 || (V.has_value() && V->defined() && V->numel() == W.numel()), "sgd_segs: momentum buffer");
  if (Wc.has_value() && Wc->defined())
    TORCH_CHECK(Wc->scalar_type() == torch::kBFloat16 && Wc->numel() == W.numel(), "sgd_segs: bf16 mirror");
  for (size_t i = 0; i < off.size(); ++i)
    TORCH_CHECK(off[i] >= 0 && len[i] >= 0 && off[i] + len[i] <= W.numel(), "sgd_segs: range outside the buffer");
  // the kernel's vector body assumes the flat buffers start 16-B aligned (8-B for the bf16 mirror)
  TORCH_CHECK((((uintptr_t)W.data_ptr() | (uintptr_t)G.data_ptr() | (uintptr_t)mptr(V)) & 15) == 0 &&
                  (((uintptr_t)mptr(Wc)) & 7) == 0, "sgd_segs: 16-B aligned buffers");
  std::vector<long> o(off.begin(), off.end()), l(len.begin(), len.end());
  fm_sgd_update_segs(W.data_ptr<float>(), G.data_ptr<float>(), (float*)mptr(V), (unsigned short*)mptr(Wc),
                     lr.data_ptr<float>(), o.data(), l.data(), (int)o.size(), (float)wd, (float)mom, nesterov ? 1 : 0,
                     zero_g ? 1 : 0, cur());
}

// dW = dpre^T x with the SGD update fused into the epilogue (gemm.hip fm_gemm_dw_sgd): W [N_out, K_in]
// fp32 master, optional bf16 mirror Wc and momentum V of the same shape; db (optional) += column sums
// of dpre.  Returns the split-K factor, or -1 when the fused form does not apply (the caller then
// computes the gradient and runs the optimizer kernel itself).
int gemm_dw_sgd(torch::Tensor dpre, torch::Tensor x, torch::Tensor W, c10::optional<torch::Tensor> Wc,
                c10::optional<torch::Tensor> V, torch::Tensor lr, double wd, double mom, bool nesterov,
                c10::optional<torch::Tensor> db, torch::Tensor ws, int64_t cfg) {
  check_cuda(dpre, "dpre");
  check_cuda(x, "x");
  check_cuda(W, "W");
  const bool f32 = dpre.scalar_type() == torch::kFloat32;
  const int64_t B = dpre.size(0), Nout = dpre.size(1), Kin = x.size(1);
  TORCH_CHECK(x.scalar_type() == dpre.scalar_type() && (f32 || dpre.scalar_type() == torch::kBFloat16) && x.size(0) == B &&
                  dpre.stride(1) == 1 && x.stride(1) == 1,
              "gemm_dw_sgd: dpre [B, out], x [B, in] (both bf16 or both fp32), unit column stride");
  TORCH_CHECK(W.scalar_type() == torch::kFloat32 && W.is_contiguous() && W.numel() == Nout * Kin, "gemm_dw_sgd: W [out, in] fp32");
  if (Wc.has_value() && Wc->defined())
    TORCH_CHECK(Wc->scalar_type() == torch::kBFloat16 && Wc->is_contiguous() && Wc->numel() == W.numel(), "gemm_dw_sgd: Wc");
  if (V.has_value() && V->defined())
    TORCH_CHECK(V->scalar_type() == torch::kFloat32 && V->is_contiguous() && V->numel() == W.numel(), "gemm_dw_sgd: V");
  TORCH_CHECK(mom <= 0.0 || (V.has_value() && V->defined()), "gemm_dw_sgd: momentum needs V");
  TORCH_CHECK(lr.scalar_type() == torch::kFloat32 && lr.numel() >= 1 && lr.is_cuda(), "gemm_dw_sgd: lr device fp32 scalar");
  if (db.has_value() && db->defined())
    TORCH_CHECK(db->scalar_type() == torch::kFloat32 && db->numel() >= Nout, "gemm_dw_sgd: db fp32 [out]");
  TORCH_CHECK((B - 1) * dpre.stride(0) + Nout <= dpre.numel() && (B - 1) * x.stride(0) + Kin <= x.numel(), "gemm_dw_sgd: extents");
  if (f32)
    return fm_gemm_f32_dw_sgd(dpre.data_ptr<float>(), dpre.stride(0), x.data_ptr<float>(), x.stride(0),
                              W.data_ptr<float>(), Kin, (unsigned short*)mptr(Wc), (float*)mptr(V), lr.data_ptr<float>(),
                              (float)wd, (float)mom, nesterov ? 1 : 0, (int)Nout, (int)Kin, (int)B, ws.data_ptr<float>(),
                              ws.numel() * 4, (float*)mptr(db), (int)cfg, cur());
  return fm_gemm_dw_sgd(dpre.data_ptr(), dpre.stride(0), x.data_ptr(), x.stride(0), W.data_ptr<float>(), Kin,
                        (unsigned short*)mptr(Wc), (float*)mptr(V), lr.data_ptr<float>(), (float)wd, (float)mom,
                        nesterov ? 1 : 0, (int)Nout, (int)Kin, (int)B, ws.data_ptr<float>(), ws.numel() * 4,
                        (float*)mptr(db), (int)cfg, cur());
}

// thin-input Linear (gemm_small.hip): y = act(x W^T + b) for in_features K <= 32, K % 4 == 0; x, w,
// y all fp32 or all bf16 (fp32 accumulate).  Returns false (nothing launched) when the shape /
// alignment is outside the kernel's limits.
bool smallk_fwd(torch::Tensor x, torch::Tensor w, c10::optional<torch::Tensor> bias, torch::Tensor y, int64_t act) {
  check_cuda(x, "x");
  const bool bf = x.scalar_type() == torch::kBFloat16;
  const auto dt = bf ? torch::kBFloat16 : torch::kFloat32;
  TORCH_CHECK(x.scalar_type() == dt && w.scalar_type() == dt && y.scalar_type() == dt, "smallk_fwd: x, w, y all fp32 or all bf16");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && y.dim() == 2 && w.is_contiguous() && x.stride(1) == 1 && y.stride(1) == 1 &&
                  w.size(1) == x.size(1) && y.size(0) == x.size(0) && y.size(1) == w.size(0),
              "smallk_fwd: x [M, K], w [N, K], y [M, N]");
  if (bias.has_value() && bias->defined())
    TORCH_CHECK(bias->scalar_type() == torch::kFloat32 && bias->numel() == w.size(0), "smallk_fwd: bias [N] fp32");
  return fm_smallk_fwd_launch(x.data_ptr(), x.stride(0), w.data_ptr(), (const float*)mptr(bias), y.data_ptr(), y.stride(0),
                              x.size(0), (int)x.size(1), (int)w.size(0), (int)act, bf ? 1 : 0, cur()) == 0;
}

// dW [N, K] += dpre^T x and db [N] += colsum(dpre) (gemm_small.hip, deterministic two-pass); with lr
// the SGD step is applied to W = dw in the same pass instead (V / Wc optional, like gemm_dw_sgd).
bool smallk_dw(torch::Tensor dpre, torch::Tensor x, torch::Tensor dw, c10::optional<torch::Tensor> db, torch::Tensor ws,
               c10::optional<torch::Tensor> V, c10::optional<torch::Tensor> Wc, c10::optional<torch::Tensor> lr, double wd,
               double mom, bool nesterov) {
  check_cuda(dpre, "dpre");
  const bool bf = dpre.scalar_type() == torch::kBFloat16;
  TORCH_CHECK(dpre.scalar_type() == x.scalar_type() && (bf || dpre.scalar_type() == torch::kFloat32) &&
                  dw.scalar_type() == torch::kFloat32 && ws.scalar_type() == torch::kFloat32,
              "smallk_dw: dpre / x both fp32 or both bf16, fp32 dw");
  const int64_t M = dpre.size(0), N = dpre.size(1), K = x.size(1);
  TORCH_CHECK(x.size(0) == M && dpre.stride(1) == 1 && x.stride(1) == 1 && dw.is_contiguous() && dw.numel() == N * K,
              "smallk_dw: dpre [M, N], x [M, K], dw [N, K]");
  if (db.has_value() && db->defined()) TORCH_CHECK(db->scalar_type() == torch::kFloat32 && db->numel() >= N, "smallk_dw: db");
  const bool upd = lr.has_value() && lr->defined();
  if (upd) {
    TORCH_CHECK(lr->scalar_type() == torch::kFloat32 && lr->is_cuda(), "smallk_dw: lr device fp32 scalar");
    TORCH_CHECK(mom <= 0.0 || (V.has_value() && V->defined()), "smallk_dw: momentum needs V");
    if (V.has_value() && V->defined()) TORCH_CHECK(V->is_contiguous() && V->numel() == dw.numel(), "smallk_dw: V");
    if (Wc.has_value() && Wc->defined())
      TORCH_CHECK(Wc->scalar_type() == torch::kBFloat16 && Wc->is_contiguous() && Wc->numel() == dw.numel(), "smallk_dw: Wc");
  }
  return fm_smallk_dw_launch(dpre.data_ptr(), dpre.stride(0), x.data_ptr(), x.stride(0), dw.data_ptr<float>(),
                             (float*)mptr(db), M, (int)K, (int)N, ws.data_ptr<float>(), ws.numel() * 4,
                             upd ? (float*)mptr(V) : nullptr, upd ? (unsigned short*)mptr(Wc) : nullptr,
                             upd ? lr->data_ptr<float>() : nullptr, (float)wd, (float)mom, nesterov ? 1 : 0, bf ? 1 : 0,
                             cur()) == 0;
}

void skinny_fwd(torch::Tensor x, torch::Tensor w, c10::optional<torch::Tensor> bias, torch::Tensor y, int64_t act) {
  TORCH_CHECK(w.numel() == x.size(1) && y.size(1) == 1 && x.stride(1) == 1, "skinny_fwd: x[B,K] w[1,K] y[B,1]");
  TORCH_CHECK(x.scalar_type() == w.scalar_type() && x.scalar_type() == y.scalar_type(), "skinny_fwd: one dtype");
  if (x.scalar_type() == torch::kFloat32) {
    fm_skinny_fwd_f32_launch(x.data_ptr<float>(), x.stride(0), w.data_ptr<float>(),
                             bias.has_value() && bias->defined() ? bias->data_ptr<float>() : nullptr, y.data_ptr<float>(),
                             y.stride(0), x.size(0), (int)x.size(1), (int)act, cur());
    return;
  }
  fm_skinny_fwd(x.data_ptr(), x.stride(0), w.data_ptr(), bias.has_value() && bias->defined() ? bias->data_ptr<float>() : nullptr,
                y.data_ptr(), y.stride(0), x.size(0), (int)x.size(1), (int)act, cur());
}

void skinny_bwd(torch::Tensor x, torch::Tensor w, torch::Tensor y, torch::Tensor dy, c10::optional<torch::Tensor> dx, bool dx_acc,
                torch::Tensor dw, c10::optional<torch::Tensor> db, int64_t act, int64_t bact) {
  // bact: activation backward of the layer below (output x) fused into dX; 10 = none
  TORCH_CHECK(w.numel() == x.size(1) && dw.numel() == x.size(1), "skinny_bwd: shapes");
  long lddx = (dx.has_value() && dx->defined()) ? dx->stride(0) : 0;
  if (x.scalar_type() == torch::kFloat32) {
    TORCH_CHECK(w.scalar_type() == torch::kFloat32 && y.scalar_type() == torch::kFloat32 && dy.scalar_type() == torch::kFloat32,
                "skinny_bwd: fp32 operands");
    TORCH_CHECK(x.size(1) % 4 == 0 && x.stride(0) % 4 == 0 && lddx % 4 == 0,
                "skinny_bwd fp32: K % 4 == 0");
    fm_skinny_bwd_f32_launch(x.data_ptr<float>(), x.stride(0), w.data_ptr<float>(), y.data_ptr<float>(), y.stride(0),
                             dy.data_ptr<float>(), dy.stride(0), (float*)mptr(dx), lddx, dx_acc ? 1 : 0, dw.data_ptr<float>(),
                             (float*)mptr(db), x.size(0), (int)x.size(1), (int)act, (int)bact, cur());
    return;
  }
  TORCH_CHECK(x.size(1) % 8 == 0 && x.stride(0) % 8 == 0, "skinny_bwd: K % 8 == 0");
  fm_skinny_bwd(x.data_ptr(), x.stride(0), w.data_ptr(), y.data_ptr(), y.stride(0), dy.data_ptr(), dy.stride(0), mptr(dx), lddx,
                dx_acc ? 1 : 0, dw.data_ptr<float>(), (float*)mptr(db), x.size(0), (int)x.size(1), (int)act, (int)bact, cur());
}

void init_fill(torch::Tensor out, int64_t rows, int64_t cols, int64_t r0, int64_t c0, int64_t ldg, int64_t kind, int64_t seed,
               double a, double b) {
  check_cuda(out, "out");
  TORCH_CHECK(out.scalar_type() == torch::kFloat32 && out.is_contiguous(), "init_fill: fp32 contiguous");
  TORCH_CHECK(out.numel() == rows * cols, "init_fill: shape mismatch");
  fm_init_fill(out.data_ptr<float>(), rows, cols, r0, c0, ldg, (int)kind, (unsigned)seed, (float)a, (float)b, cur());
}

void embedding_fwd(torch::Tensor idx, torch::Tensor W, torch::Tensor out, int64_t ldo, double scale) {
  check_cuda(idx, "idx");
  check_cuda(W, "W");
  check_cuda(out, "out");
  TORCH_CHECK(W.scalar_type() == torch::kFloat32 && W.is_contiguous(), "table must be fp32 contiguous");
  TORCH_CHECK(idx.dim() == 2 && idx.is_contiguous(), "idx [B, bag] contiguous");
  long B = idx.size(0);
  int bag = idx.size(1);
  int D = W.size(1);
  TORCH_CHECK(out.numel() >= (B - 1) * ldo + D, "embedding out too small");
  fm_embedding_fwd(idx.data_ptr(), idx.scalar_type() == torch::kInt64, W.data_ptr<float>(), out.data_ptr(), is_bf16(out), B,
                   bag, (int)W.size(0), D, ldo, (float)scale, cur());
}

void embedding_bwd(torch::Tensor idx, torch::Tensor dy, int64_t ldg, torch::Tensor W, c10::optional<torch::Tensor> lr,
                   double scale) {
  check_cuda(idx, "idx");
  check_cuda(dy, "dy");
  check_cuda(W, "W");
  TORCH_CHECK(W.scalar_type() == torch::kFloat32 && W.is_contiguous(), "table must be fp32 contiguous");
  long B = idx.size(0);
  int bag = idx.size(1);
  fm_embedding_bwd(idx.data_ptr(), idx.scalar_type() == torch::kInt64, dy.data_ptr(), is_bf16(dy), W.data_ptr<float>(),
                   lr.has_value() && lr->defined() ? lr->data_ptr<float>() : nullptr, B, bag, (int)W.size(0),
                   (int)W.size(1), ldg, (float)scale, cur());
}

struct TabArgs {
  std::vector<const float*> Wc;
  std::vector<float*> Wm;
  std::vector<const void*> idx;
  std::vector<int> idx64, rows, D, bag;
  std::vector<void*> act;
  std::vector<const void*> cact;
  std::vector<long> ld;
  std::vector<float> scale;
  long B = 0;
};

TabArgs tab_args(const std::vector<torch::Tensor>& W, const std::vector<torch::Tensor>& idx, const std::vector<torch::Tensor>& act,
                 const std::vector<int64_t>& ld, const std::vector<double>& scale) {
  TabArgs a;
  size_t n = W.size();
  TORCH_CHECK(idx.size() == n && act.size() == n && ld.size() == n && scale.size() == n, "embedding multi: list sizes");
  for (size_t i = 0; i < n; ++i) {
    check_cuda(W[i], "W");
    check_cuda(idx[i], "idx");
    check_cuda(act[i], "act");
    TORCH_CHECK(W[i].scalar_type() == torch::kFloat32 && W[i].is_contiguous() && W[i].dim() == 2, "tables fp32 [rows, D]");
    TORCH_CHECK(idx[i].dim() == 2 && idx[i].is_contiguous(), "idx [B, bag]");
    long B = idx[i].size(0);
    if (i == 0) a.B = B;
    TORCH_CHECK(B == a.B, "embedding multi: same batch");
    TORCH_CHECK(act[i].numel() >= (B - 1) * ld[i] + W[i].size(1), "embedding act buffer too small");
    a.Wc.push_back(W[i].data_ptr<float>());
    a.Wm.push_back(W[i].data_ptr<float>());
    a.idx.push_back(idx[i].data_ptr());
    a.idx64.push_back(idx[i].scalar_type() == torch::kInt64);
    a.rows.push_back((int)W[i].size(0));
    a.D.push_back((int)W[i].size(1));
    a.bag.push_back((int)idx[i].size(1));
    a.act.push_back(act[i].data_ptr());
    a.cact.push_back(act[i].data_ptr());
    a.ld.push_back(ld[i]);
    a.scale.push_back((float)scale[i]);
  }
  return a;
}

// row_lo: first global row of each (row-sharded) table; empty = whole tables
std::vector<long> row_offsets(const std::vector<int64_t>& row_lo, size_t n) {
  TORCH_CHECK(row_lo.empty() || row_lo.size() == n, "embedding multi: one row offset per table");
  std::vector<long> lo(n, 0);
  for (size_t i = 0; i < row_lo.size(); ++i) lo[i] = (long)row_lo[i];
  return lo;
}

void embedding_fwd_multi(std::vector<torch::Tensor> W, std::vector<torch::Tensor> idx, std::vector<torch::Tensor> out,
                         std::vector<int64_t> ldo, std::vector<double> scale, std::vector<int64_t> row_lo) {
  if (W.empty()) return;
  TabArgs a = tab_args(W, idx, out, ldo, scale);
  std::vector<long> lo = row_offsets(row_lo, W.size());
  fm_embedding_fwd_multi((int)W.size(), a.Wc.data(), a.idx.data(), a.idx64.data(), a.act.data(), a.ld.data(), lo.data(),
                         a.rows.data(), a.D.data(), a.bag.data(), a.scale.data(), is_bf16(out[0]), a.B, cur());
}

// claim: optional per-table [owner (int32 [rows], -1 filled), dups (int32 [B*bag]), ndup (int32 [1])]
// triples (owner-computes sparse SGD for mostly-unique tables); None entries use the atomic path
void embedding_bwd_multi(std::vector<torch::Tensor> W, std::vector<torch::Tensor> idx, std::vector<torch::Tensor> dy,
                         std::vector<int64_t> ldg, std::vector<double> scale, c10::optional<torch::Tensor> lr,
                         c10::optional<std::vector<c10::optional<torch::Tensor>>> claim, std::vector<int64_t> row_lo) {
  if (W.empty()) return;
  TabArgs a = tab_args(W, idx, dy, ldg, scale);
  std::vector<long> lo = row_offsets(row_lo, W.size());
  std::vector<int*> own(W.size(), nullptr), dup(W.size(), nullptr), nd(W.size(), nullptr);
  bool any = false;
  if (claim.has_value()) {
    TORCH_CHECK(claim->size() == 3 * W.size(), "claim: 3 buffers per table");
    for (size_t k = 0; k < W.size(); ++k) {
      const auto& o = (*claim)[3 * k];
      if (!o.has_value() || !o->defined()) continue;
      const auto& d = (*claim)[3 * k + 1];
      const auto& c = (*claim)[3 * k + 2];
      TORCH_CHECK(o->scalar_type() == torch::kInt32 && o->numel() >= W[k].size(0), "claim owner: int32 [rows]");
      TORCH_CHECK(d.has_value() && d->scalar_type() == torch::kInt32 && d->numel() >= idx[k].numel(), "claim dups");
      TORCH_CHECK(c.has_value() && c->scalar_type() == torch::kInt32 && c->numel() >= 1, "claim ndup");
      own[k] = o->data_ptr<int>();
      dup[k] = d->data_ptr<int>();
      nd[k] = c->data_ptr<int>();
      any = true;
    }
  }
  fm_embedding_bwd_multi((int)W.size(), a.Wm.data(), a.idx.data(), a.idx64.data(), a.cact.data(), a.ld.data(), lo.data(),
                         a.rows.data(), a.D.data(), a.bag.data(), a.scale.data(), is_bf16(dy[0]),
                         lr.has_value() && lr->defined() ? lr->data_ptr<float>() : nullptr, a.B,
                         any ? own.data() : nullptr, any ? dup.data() : nullptr, any ? nd.data() : nullptr, cur());
}

// sparse data parallelism for replicated tables (embedding.hip): coalesce this rank's lookups
// into (count, unique local rows, summed gradients) payload views of the all-gather send buffer
void sdp_coalesce(std::vector<torch::Tensor> W, std::vector<torch::Tensor> idx, std::vector<torch::Tensor> dy,
                  std::vector<int64_t> ldg, std::vector<double> scale, std::vector<int64_t> row_lo,
                  std::vector<torch::Tensor> slot, std::vector<torch::Tensor> cid, std::vector<torch::Tensor> ids,
                  std::vector<torch::Tensor> g, std::vector<torch::Tensor> count) {
  if (W.empty()) return;
  TabArgs a = tab_args(W, idx, dy, ldg, scale);
  std::vector<long> lo = row_offsets(row_lo, W.size());
  const size_t n = W.size();
  TORCH_CHECK(slot.size() == n && cid.size() == n && ids.size() == n && g.size() == n && count.size() == n,
              "sdp_coalesce: one buffer of each kind per table");
  std::vector<int*> ps, pc, pi, pn;
  std::vector<float*> pg;
  for (size_t k = 0; k < n; ++k) {
    TORCH_CHECK(slot[k].scalar_type() == torch::kInt32 && slot[k].numel() >= W[k].size(0), "sdp slot: int32 [rows]");
    TORCH_CHECK(cid[k].scalar_type() == torch::kInt32 && cid[k].numel() >= idx[k].numel(), "sdp cid: int32 [B*bag]");
    TORCH_CHECK(ids[k].scalar_type() == torch::kInt32 && ids[k].numel() >= idx[k].numel(), "sdp ids: int32 [B*bag]");
    TORCH_CHECK(g[k].scalar_type() == torch::kFloat32 && g[k].numel() >= idx[k].numel() * W[k].size(1),
                "sdp g: fp32 [B*bag, D]");
    TORCH_CHECK(count[k].scalar_type() == torch::kInt32 && count[k].numel() >= 1, "sdp count: int32 [1]");
    ps.push_back(slot[k].data_ptr<int>());
    pc.push_back(cid[k].data_ptr<int>());
    pi.push_back(ids[k].data_ptr<int>());
    pg.push_back(g[k].data_ptr<float>());
    pn.push_back(count[k].data_ptr<int>());
  }
  fm_sdp_coalesce((int)n, a.idx.data(), a.idx64.data(), a.cact.data(), a.ld.data(), lo.data(), a.rows.data(), a.D.data(),
                  a.bag.data(), a.scale.data(), is_bf16(dy[0]), a.B, ps.data(), pc.data(), pi.data(), pg.data(), pn.data(),
                  cur());
}

// apply the gathered segments (segs x n payloads, segment-major) in order; own_seg frees the slots
void sdp_apply(std::vector<torch::Tensor> W, std::vector<torch::Tensor> seg_ids, std::vector<torch::Tensor> seg_g,
               std::vector<torch::Tensor> seg_count, std::vector<torch::Tensor> slot, std::vector<torch::Tensor> own_count,
               int64_t segs, int64_t own_seg, torch::Tensor lr) {
  const size_t n = W.size();
  if (n == 0) return;
  TORCH_CHECK(seg_ids.size() == n * segs && seg_g.size() == n * segs && seg_count.size() == n * segs,
              "sdp_apply: segs x tables payload views");
  TORCH_CHECK(slot.size() == n && own_count.size() == n, "sdp_apply: slot / own_count per table");
  check_cuda(lr, "lr");
  std::vector<float*> pw;
  std::vector<int> D, nmax;
  std::vector<const int*> pi, pn;
  std::vector<const float*> pg;
  std::vector<int*> ps, po;
  for (size_t k = 0; k < n; ++k) {
    check_cuda(W[k], "W");
    TORCH_CHECK(W[k].scalar_type() == torch::kFloat32 && W[k].is_contiguous() && W[k].dim() == 2, "tables fp32 [rows, D]");
    pw.push_back(W[k].data_ptr<float>());
    D.push_back((int)W[k].size(1));
    nmax.push_back((int)seg_ids[k].numel());
    ps.push_back(slot[k].data_ptr<int>());
    po.push_back(own_count[k].data_ptr<int>());
  }
  for (size_t j = 0; j < n * segs; ++j) {
    const size_t k = j % n;
    TORCH_CHECK(seg_ids[j].numel() == nmax[k] && seg_g[j].numel() >= (int64_t)nmax[k] * D[k], "sdp_apply: payload sizes");
    pi.push_back(seg_ids[j].data_ptr<int>());
    pg.push_back(seg_g[j].data_ptr<float>());
    pn.push_back(seg_count[j].data_ptr<int>());
  }
  fm_sdp_apply_segments((int)n, (int)segs, (int)own_seg, pw.data(), D.data(), pi.data(), pg.data(), pn.data(), ps.data(),
                        po.data(), nmax.data(), lr.data_ptr<float>(), cur());
}

// dst[to + sum i_k ts_k] (+)= src[so + sum i_k ss_k] over the box d[4] (element offsets / strides
// into the two buffers' storage; same dtype, bf16 or fp32)
void strided_copy4(torch::Tensor src, torch::Tensor dst, std::vector<int64_t> d, std::vector<int64_t> ss,
                   std::vector<int64_t> ts, int64_t so, int64_t to, bool acc) {
  check_cuda(src, "src");
  check_cuda(dst, "dst");
  TORCH_CHECK(src.scalar_type() == dst.scalar_type() && (is_bf16(src) || src.scalar_type() == torch::kFloat32),
              "strided_copy4: same dtype, bf16 or fp32");
  TORCH_CHECK(d.size() == 4 && ss.size() == 4 && ts.size() == 4, "strided_copy4: 4-D box");
  int64_t smax = so, tmax = to;
  for (int k = 0; k < 4; ++k) {
    TORCH_CHECK(d[k] >= 1 && ss[k] >= 0 && ts[k] >= 0, "strided_copy4: positive extents / strides");
    smax += (d[k] - 1) * ss[k];
    tmax += (d[k] - 1) * ts[k];
  }
  TORCH_CHECK(so >= 0 && to >= 0 && smax < src.numel() && tmax < dst.numel(), "strided_copy4: box outside the buffers");
  int di[4];
  long sl[4], tl[4];
  for (int k = 0; k < 4; ++k) {
    di[k] = (int)d[k];
    sl[k] = ss[k];
    tl[k] = ts[k];
  }
  fm_strided_copy4_run(src.data_ptr(), dst.data_ptr(), is_bf16(src), di, sl, tl, so, to, acc ? 1 : 0, cur());
}

void dot_fwd(std::vector<torch::Tensor> zs, int64_t ldz, torch::Tensor out, int64_t ldo, int64_t D, int64_t W, bool self) {
  TORCH_CHECK(zs.size() >= 1 && zs.size() <= 32, "dot interaction: 1..32 features");
  std::vector<const void*> p;
  long B = out.size(0);
  const auto dt = out.scalar_type();
  TORCH_CHECK(dt == torch::kBFloat16 || dt == torch::kFloat32, "dot interaction: bf16 or fp32");
  TORCH_CHECK(out.numel() >= (B - 1) * ldo + W, "dot output too small");
  for (auto& z : zs) {
    check_cuda(z, "z");
    TORCH_CHECK(z.scalar_type() == dt, "dot interaction inputs must match the output dtype");
    TORCH_CHECK(z.numel() >= (B - 1) * ldz + D, "dot input too small");
    p.push_back(z.data_ptr());
  }
  if (dt == torch::kFloat32) {
    TORCH_CHECK(D % 2 == 0, "dot interaction fp32: even D");
    fm_dot_interaction_fwd_f32((const float* const*)p.data(), (int)p.size(), ldz, out.data_ptr<float>(), ldo, B, (int)D,
                               (int)W, self ? 1 : 0, cur());
    return;
  }
  TORCH_CHECK(D % 16 == 0 && W % 8 == 0 && ldz % 8 == 0 && ldo % 8 == 0, "dot interaction: D%16, W%8, ld%8");
  fm_dot_interaction_fwd(p.data(), (int)p.size(), ldz, out.data_ptr(), ldo, B, (int)D, (int)W, self ? 1 : 0, cur());
}

// act0 (fp32 only): activation backward of feature 0's producer applied to dz[0] (10 = none)
void dot_bwd(std::vector<torch::Tensor> zs, int64_t ldz, torch::Tensor dout, int64_t ldo,
             std::vector<c10::optional<torch::Tensor>> dzs, int64_t lddz, int64_t acc_mask, int64_t D, bool self,
             int64_t act0) {
  std::vector<const void*> p;
  std::vector<void*> g;
  for (auto& z : zs) p.push_back(z.data_ptr());
  for (auto& d : dzs) g.push_back(mptr(d));
  TORCH_CHECK(zs.size() >= 1 && zs.size() <= 32 && dzs.size() == zs.size(), "dot interaction backward: 1..32 features");
  if (dout.scalar_type() == torch::kFloat32) {
    const long B = dout.size(0);
    const long F = (long)zs.size();
    const long np = self ? F * (F + 1) / 2 : F * (F - 1) / 2;
    TORCH_CHECK(D % 2 == 0 && D <= 256, "dot interaction backward fp32: even D <= 256");
    TORCH_CHECK(dout.numel() >= (B - 1) * ldo + ((D + np + 3) & ~3L) && ldo >= ((D + np + 3) & ~3L),
                "dot interaction backward: dOut row too small");
    for (size_t i = 0; i < zs.size(); ++i) {
      TORCH_CHECK(zs[i].scalar_type() == torch::kFloat32 && zs[i].numel() >= (B - 1) * ldz + D, "dot bwd: fp32 inputs");
      if (g[i]) TORCH_CHECK(dzs[i]->scalar_type() == torch::kFloat32 && dzs[i]->numel() >= (B - 1) * lddz + D, "dot bwd: fp32 grads");
    }
    fm_dot_interaction_bwd_f32((const float* const*)p.data(), (int)F, ldz, dout.data_ptr<float>(), ldo, (float* const*)g.data(),
                               lddz, (unsigned)acc_mask, B, (int)D, self ? 1 : 0, (int)act0, cur());
    return;
  }
  TORCH_CHECK(act0 == 10, "dot interaction backward: act0 is fp32-only");
  TORCH_CHECK(D % 8 == 0 && D <= 256, "dot interaction backward: D % 8 == 0, D <= 256");
  fm_dot_interaction_bwd(p.data(), (int)p.size(), ldz, dout.data_ptr(), ldo, g.data(), lddz, (unsigned)acc_mask,
                         dout.size(0), (int)D, self ? 1 : 0, cur());
}

void sgd(torch::Tensor W, torch::Tensor G, c10::optional<torch::Tensor> V, c10::optional<torch::Tensor> Wc, torch::Tensor lr,
         double wd, double mom, bool nesterov, bool zero_grad) {
  TORCH_CHECK(W.numel() == G.numel(), "sgd: size mismatch");
  fm_sgd_update(W.data_ptr<float>(), G.data_ptr<float>(), (float*)mptr(V), (unsigned short*)mptr(Wc), lr.data_ptr<float>(),
                W.numel(), (float)wd, (float)mom, nesterov ? 1 : 0, zero_grad ? 1 : 0, cur());
}

void adam(torch::Tensor W, torch::Tensor G, torch::Tensor M, torch::Tensor V, c10::optional<torch::Tensor> Wc,
          torch::Tensor alpha_t, double b1, double b2, double wd, double eps, bool zero_grad) {
  TORCH_CHECK(alpha_t.scalar_type() == torch::kFloat32 && alpha_t.is_cuda(), "alpha_t: fp32 device scalar");
  fm_adam_update(W.data_ptr<float>(), G.data_ptr<float>(), M.data_ptr<float>(), V.data_ptr<float>(), (unsigned short*)mptr(Wc),
                 W.numel(), alpha_t.data_ptr<float>(), (float)b1, (float)b2, (float)wd, (float)eps, zero_grad ? 1 : 0, cur());
}

void cast_bf16(torch::Tensor src, torch::Tensor dst) { fm_cast_bf16(src.data_ptr<float>(), (unsigned short*)dst.data_ptr(), src.numel(), cur()); }

void loss(int64_t loss_type, torch::Tensor logits, torch::Tensor labels, c10::optional<torch::Tensor> grad, double scale,
          torch::Tensor acc, int64_t mask, double clamp_t) {
  long B = logits.size(0);
  int C = (int)(logits.numel() / std::max<long>(1, B));
  int gb = (grad.has_value() && grad->defined()) ? is_bf16(*grad) : 0;
  fm_loss_fwd_bwd(logits.data_ptr(), is_bf16(logits), labels.data_ptr(), mptr(grad), gb, B, C, (int)loss_type, (float)scale,
                  acc.data_ptr<float>(), (int)mask, (float)clamp_t, cur());
}

void unary_fwd(int64_t code, torch::Tensor x, torch::Tensor y) { fm_unary_forward((int)code, x.data_ptr(), y.data_ptr(), x.numel(), is_bf16(x), cur()); }
void unary_bwd(int64_t code, torch::Tensor x, torch::Tensor y, torch::Tensor dy, torch::Tensor dx, bool acc) {
  fm_unary_backward((int)code, x.data_ptr(), y.data_ptr(), dy.data_ptr(), dx.data_ptr(), x.numel(), acc, is_bf16(x), cur());
}
// relu: y = relu(a op b); ymask (backward): the incoming gradient is zeroed where ymask <= 0
void binary_fwd(int64_t code, torch::Tensor a, torch::Tensor b, torch::Tensor y, bool relu) {
  TORCH_CHECK(a.numel() == b.numel() && a.numel() == y.numel() && a.scalar_type() == b.scalar_type() &&
                  a.scalar_type() == y.scalar_type(), "binary_fwd: same-size same-dtype operands");
  fm_binary_forward((int)code, a.data_ptr(), b.data_ptr(), y.data_ptr(), a.numel(), relu ? 1 : 0, is_bf16(a), cur());
}
void binary_bwd(int64_t code, torch::Tensor a, torch::Tensor b, torch::Tensor dy, c10::optional<torch::Tensor> ymask,
                c10::optional<torch::Tensor> da, c10::optional<torch::Tensor> db, bool acca, bool accb) {
  TORCH_CHECK(dy.numel() == a.numel() && dy.numel() == b.numel() && dy.scalar_type() == a.scalar_type(), "binary_bwd: operands");
  if (ymask.has_value() && ymask->defined())
    TORCH_CHECK(ymask->numel() == dy.numel() && ymask->scalar_type() == dy.scalar_type(), "binary_bwd: ymask");
  fm_binary_backward((int)code, a.data_ptr(), b.data_ptr(), dy.data_ptr(), cptr(ymask), mptr(da), mptr(db), a.numel(), acca,
                     accb, is_bf16(a), cur());
}
void act_bwd_bias(torch::Tensor y, torch::Tensor dy, c10::optional<torch::Tensor> dpre, c10::optional<torch::Tensor> db,
                  int64_t B, int64_t N, int64_t act) {
  TORCH_CHECK(y.scalar_type() == dy.scalar_type() && (y.scalar_type() == torch::kBFloat16 || y.scalar_type() == torch::kFloat32),
              "act_bwd_bias: bf16 or fp32");
  if (dpre.has_value() && dpre->defined()) TORCH_CHECK(dpre->scalar_type() == y.scalar_type(), "act_bwd_bias: dpre dtype");
  fm_act_bwd_bias(y.data_ptr(), dy.data_ptr(), mptr(dpre), (float*)mptr(db), B, (int)N, (int)act, is_bf16(y), cur());
}
// uint8 [N][H][W][3] decoded RGB -> normalized [N][3][H][W] fp32 / bf16 (image.hip)
void image_normalize(torch::Tensor src, torch::Tensor dst, std::vector<double> mean, std::vector<double> stdv) {
  check_cuda(src, "src");
  check_cuda(dst, "dst");
  TORCH_CHECK(src.scalar_type() == torch::kUInt8 && src.dim() == 4 && src.size(3) == 3 && src.is_contiguous(),
              "image_normalize: src must be contiguous uint8 [N][H][W][3]");
  TORCH_CHECK(dst.dim() == 4 && dst.size(0) == src.size(0) && dst.size(1) == 3 && dst.size(2) == src.size(1) &&
                  dst.size(3) == src.size(2) && dst.is_contiguous(),
              "image_normalize: dst must be contiguous [N][3][H][W] matching src");
  TORCH_CHECK(dst.scalar_type() == torch::kFloat32 || dst.scalar_type() == torch::kBFloat16, "image_normalize: fp32/bf16 dst");
  TORCH_CHECK(mean.size() == 3 && stdv.size() == 3, "image_normalize: 3 means and 3 stds");
  const float m[3] = {(float)mean[0], (float)mean[1], (float)mean[2]};
  const float sd[3] = {(float)stdv[0], (float)stdv[1], (float)stdv[2]};
  fm_image_normalize(src.data_ptr<uint8_t>(), dst.data_ptr(), src.size(0), (int)src.size(1), (int)src.size(2), m, sd,
                     dst.scalar_type() == torch::kBFloat16, cur());
}

void multi_copy(std::vector<torch::Tensor> src, std::vector<int64_t> src_off, std::vector<torch::Tensor> dst,
                std::vector<int64_t> dst_off, std::vector<int64_t> rows, std::vector<int64_t> cols, std::vector<int64_t> lds,
                std::vector<int64_t> ldd, int64_t add_mask) {
  int n = (int)src.size();
  std::vector<const void*> s(n);
  std::vector<void*> d(n);
  std::vector<long> r(n), c(n), a(n), b(n);
  int eb = src.empty() ? 4 : (int)src[0].element_size();
  for (int i = 0; i < n; ++i) {
    s[i] = (const char*)src[i].data_ptr() + src_off[i] * eb;
    d[i] = (char*)dst[i].data_ptr() + dst_off[i] * eb;
    r[i] = rows[i]; c[i] = cols[i]; a[i] = lds[i]; b[i] = ldd[i];
  }
  fm_multi_copy2d(n, s.data(), d.data(), r.data(), c.data(), a.data(), b.data(), (int)add_mask, eb, cur());
}
void permute(torch::Tensor x, torch::Tensor y, std::vector<int64_t> out_dims, std::vector<int64_t> in_strides, bool acc) {
  std::vector<long> od(out_dims.begin(), out_dims.end()), is(in_strides.begin(), in_strides.end());
  TORCH_CHECK(od.size() <= 6, "permute: <= 6 dims");
  fm_permute_nd(x.data_ptr(), y.data_ptr(), (int)od.size(), od.data(), is.data(), acc, is_bf16(x), cur());
}
void reverse(torch::Tensor x, torch::Tensor y, int64_t outer, int64_t len, int64_t inner, bool acc) {
  fm_reverse_axis(x.data_ptr(), y.data_ptr(), outer, len, inner, acc, is_bf16(x), cur());
}
void softmax(torch::Tensor x, torch::Tensor y, int64_t rows, int64_t C) { fm_softmax_fwd(x.data_ptr(), y.data_ptr(), rows, (int)C, is_bf16(x), cur()); }
void dropout(torch::Tensor x, torch::Tensor y, double rate, int64_t seed, int64_t step, bool acc) {
  fm_dropout_apply(x.data_ptr(), y.data_ptr(), x.numel(), (float)rate, (unsigned)seed, (unsigned)step, acc, is_bf16(x), cur());
}

}  // namespace

// ----------------------------------------------------------------------------- CNN
static void chk4(const torch::Tensor& t, const char* n) {
  check_cuda(t, n);
  TORCH_CHECK((t.scalar_type() == torch::kBFloat16 || t.scalar_type() == torch::kFloat32) && t.is_contiguous(), n,
              ": contiguous bf16 or fp32");
}
static void same_dt(const torch::Tensor& a, const torch::Tensor& b, const char* n) {
  TORCH_CHECK(a.scalar_type() == b.scalar_type(), n, ": operands must share one dtype");
}
void im2col(torch::Tensor x, torch::Tensor col, int64_t R, int64_t S, int64_t P, int64_t Q, int64_t sh, int64_t sw,
            int64_t pt, int64_t pl, int64_t ldcol) {
  chk4(x, "x");
  chk4(col, "col");
  TORCH_CHECK(x.dim() == 4, "im2col: NCHW");
  same_dt(x, col, "im2col");
  const long N = x.size(0), C = x.size(1);
  TORCH_CHECK(ldcol >= C * R * S && col.numel() >= N * P * Q * ldcol, "im2col: col too small");
  fm_im2col(x.data_ptr(), col.data_ptr(), N, C, x.size(2), x.size(3), R, S, P, Q, sh, sw, pt, pl, ldcol, is_bf16(x), cur());
}
void col2im(torch::Tensor dcol, torch::Tensor dx, int64_t R, int64_t S, int64_t P, int64_t Q, int64_t sh, int64_t sw,
            int64_t pt, int64_t pl, int64_t ldcol, bool acc) {
  chk4(dcol, "dcol");
  chk4(dx, "dx");
  same_dt(dcol, dx, "col2im");
  const long N = dx.size(0), C = dx.size(1);
  TORCH_CHECK(ldcol >= C * R * S && dcol.numel() >= N * P * Q * ldcol, "col2im: dcol too small");
  fm_col2im(dcol.data_ptr(), dx.data_ptr(), N, C, dx.size(2), dx.size(3), R, S, P, Q, sh, sw, pt, pl, ldcol, acc, is_bf16(dx),
            cur());
}
void transpose_batched(torch::Tensor in, c10::optional<torch::Tensor> yin, torch::Tensor out, int64_t N, int64_t A,
                       int64_t B, int64_t act, int64_t mode) {
  chk4(out, "out");
  TORCH_CHECK(in.scalar_type() == out.scalar_type() && in.numel() >= N * A * B && out.numel() >= N * A * B,
              "transpose_batched: one dtype, extents");
  if (mode == 1) TORCH_CHECK(yin.has_value() && yin->scalar_type() == in.scalar_type(), "transpose_batched: yin dtype");
  TORCH_CHECK(mode == 0 || (yin.has_value() && yin->numel() >= N * A * B), "transpose_batched: mode 1 needs yin");
  fm_transpose_batched(in.data_ptr(), cptr(yin), out.data_ptr(), N, A, B, act, mode, is_bf16(out), cur());
}
// implicit-GEMM convolution (csrc/kernels/conv_igemm.hip): x [N,C,H,W], w [K,C,R,S], y [N,K,P,Q]
static void conv_chk(const torch::Tensor& x, const torch::Tensor& w, const torch::Tensor& y, const char* n) {
  chk4(x, n);
  chk4(w, n);
  chk4(y, n);
  same_dt(x, w, n);
  same_dt(x, y, n);
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4 && y.dim() == 4 && w.size(1) == x.size(1) && y.size(1) == w.size(0) &&
                  y.size(0) == x.size(0), n, ": x [N,C,H,W], w [K,C,R,S], y [N,K,P,Q]");
  const long lim = (1L << 31) - 64;
  TORCH_CHECK(x.numel() * x.element_size() < lim && y.numel() * y.element_size() < lim &&
                  w.numel() * w.element_size() < lim, n, ": every operand must stay under 2 GiB (32-bit buffer offsets)");
  TORCH_CHECK(((uintptr_t)x.data_ptr() & 15) == 0 && ((uintptr_t)w.data_ptr() & 15) == 0 && ((uintptr_t)y.data_ptr() & 15) == 0,
              n, ": 16-B aligned operands");
}
#define CONV_GEOM_NO_K(x, w, y) (int)x.size(0), (int)x.size(1), (int)x.size(2), (int)x.size(3), (int)w.size(2), \
                                (int)w.size(3), (int)y.size(2), (int)y.size(3)
#define CONV_GEOM(x, w, y) (int)x.size(0), (int)x.size(1), (int)x.size(2), (int)x.size(3), (int)w.size(0), (int)w.size(2), \
                           (int)w.size(3), (int)y.size(2), (int)y.size(3)
int64_t conv_scratch(int64_t rows, int64_t cols) { return rows * fm_conv_lda((int)cols); }
void conv_fwd(torch::Tensor x, torch::Tensor w, torch::Tensor wpad, c10::optional<torch::Tensor> bias, torch::Tensor y,
              int64_t sh, int64_t sw, int64_t pt, int64_t pl, int64_t act) {
  conv_chk(x, w, y, "conv_fwd");
  chk4(wpad, "conv_fwd wpad");
  same_dt(w, wpad, "conv_fwd");
  TORCH_CHECK(wpad.numel() >= conv_scratch(w.size(0), w.size(1) * w.size(2) * w.size(3)) &&
                  ((uintptr_t)wpad.data_ptr() & 15) == 0, "conv_fwd: wpad scratch too small");
  const float* b = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == torch::kFloat32 && bias->numel() == w.size(0), "conv_fwd: fp32 bias[K]");
    b = bias->data_ptr<float>();
  }
  fm_conv_fwd(x.data_ptr(), w.data_ptr(), wpad.data_ptr(), b, y.data_ptr(), is_bf16(x), CONV_GEOM(x, w, y), sh, sw, pt, pl, act, cur());
}
void conv_dgrad(torch::Tensor g, torch::Tensor w, torch::Tensor wt, torch::Tensor dx, int64_t sh, int64_t sw, int64_t pt,
                int64_t pl, bool acc) {
  conv_chk(dx, w, g, "conv_dgrad");
  chk4(wt, "conv_dgrad wt");
  same_dt(w, wt, "conv_dgrad");
  TORCH_CHECK(wt.numel() >= conv_scratch(w.size(1), w.size(0) * w.size(2) * w.size(3)) && ((uintptr_t)wt.data_ptr() & 15) == 0,
              "conv_dgrad: wt scratch too small");
  fm_conv_dgrad(g.data_ptr(), w.data_ptr(), wt.data_ptr(), dx.data_ptr(), acc ? 1 : 0, is_bf16(g), CONV_GEOM(dx, w, g), sh, sw,
                pt, pl, cur());
}
void conv_wgrad(torch::Tensor g, torch::Tensor x, torch::Tensor dw, int64_t R, int64_t S, int64_t sh, int64_t sw, int64_t pt,
                int64_t pl) {
  check_cuda(dw, "dw");
  TORCH_CHECK(dw.scalar_type() == torch::kFloat32 && dw.is_contiguous() && dw.numel() == g.size(1) * x.size(1) * R * S,
              "conv_wgrad: contiguous fp32 dw[K*C*R*S]");
  chk4(g, "conv_wgrad g");
  chk4(x, "conv_wgrad x");
  same_dt(g, x, "conv_wgrad");
  TORCH_CHECK(g.dim() == 4 && x.dim() == 4 && g.size(0) == x.size(0), "conv_wgrad: g [N,K,P,Q], x [N,C,H,W]");
  TORCH_CHECK(x.numel() * x.element_size() < (1L << 31) - 64 && g.numel() * g.element_size() < (1L << 31) - 64,
              "conv_wgrad: operands under 2 GiB");
  fm_conv_wgrad(g.data_ptr(), x.data_ptr(), dw.data_ptr<float>(), is_bf16(x), (int)x.size(0), (int)x.size(1), (int)x.size(2),
                (int)x.size(3), (int)g.size(1), (int)R, (int)S, (int)g.size(2), (int)g.size(3), sh, sw, pt, pl, cur());
}
// stem convolutions (csrc/kernels/conv_stem.hip): bf16, 64 filters, few channels, stride 4 / 2
bool stem_supported(int64_t C, int64_t K, int64_t R, int64_t S, int64_t sh, int64_t sw) {
  return fm_stem_supported((int)C, (int)K, (int)R, (int)S, (int)sh, (int)sw) != 0;
}
int64_t stem_wgrad_ws(int64_t C, int64_t K, int64_t R, int64_t S, int64_t s) {
  return fm_stem_wgrad_ws((int)C, (int)K, (int)R, (int)S, (int)s);
}
int64_t stem_wf_elems(int64_t C, int64_t K, int64_t R, int64_t S, int64_t s) {
  return fm_stem_wf_elems((int)C, (int)K, (int)R, (int)S, (int)s);
}
void stem_fwd(torch::Tensor x, torch::Tensor w, torch::Tensor wf, c10::optional<torch::Tensor> bias, torch::Tensor y,
              int64_t s, int64_t pt, int64_t pl, int64_t act) {
  conv_chk(x, w, y, "stem_fwd");
  TORCH_CHECK(is_bf16(x), "stem_fwd: bf16 operands");
  TORCH_CHECK(stem_supported(x.size(1), w.size(0), w.size(2), w.size(3), s, s), "stem_fwd: unsupported geometry");
  const float* b = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == torch::kFloat32 && bias->numel() == w.size(0) && bias->is_contiguous(),
                "stem_fwd: fp32 bias[K]");
    b = bias->data_ptr<float>();
  }
  check_cuda(wf, "wf");
  TORCH_CHECK(wf.element_size() == 2 && wf.numel() >= stem_wf_elems(x.size(1), w.size(0), w.size(2), w.size(3), s) &&
                  ((uintptr_t)wf.data_ptr() & 15) == 0, "stem_fwd: 16-bit weight-fragment scratch of stem_wf_elems");
  TORCH_CHECK(fm_stem_fwd_run(x.data_ptr(), w.data_ptr(), wf.data_ptr(), b, y.data_ptr(), CONV_GEOM_NO_K(x, w, y), (int)s, (int)pt,
                              (int)pl, (int)act, cur()) == 0, "stem_fwd: launch");
}
void stem_wgrad(torch::Tensor x, torch::Tensor y, torch::Tensor dy, torch::Tensor dw, c10::optional<torch::Tensor> db,
                torch::Tensor ws, int64_t R, int64_t S, int64_t s, int64_t pt, int64_t pl, int64_t act) {
  chk4(x, "stem_wgrad x");
  chk4(y, "stem_wgrad y");
  chk4(dy, "stem_wgrad dy");
  TORCH_CHECK(is_bf16(x) && is_bf16(y) && is_bf16(dy), "stem_wgrad: bf16 x / y / dy");
  TORCH_CHECK(x.dim() == 4 && y.sizes() == dy.sizes() && y.size(0) == x.size(0), "stem_wgrad: x [N,C,H,W], y = dy [N,K,P,Q]");
  TORCH_CHECK(stem_supported(x.size(1), y.size(1), R, S, s, s), "stem_wgrad: unsupported geometry");
  TORCH_CHECK(x.numel() < (1L << 30) && y.numel() < (1L << 30), "stem_wgrad: operands under 2 GiB");
  TORCH_CHECK(((uintptr_t)dy.data_ptr() & 15) == 0 && ((uintptr_t)y.data_ptr() & 15) == 0, "stem_wgrad: 16-B aligned y / dy");
  check_cuda(dw, "dw");
  TORCH_CHECK(dw.scalar_type() == torch::kFloat32 && dw.is_contiguous() && dw.numel() == y.size(1) * x.size(1) * R * S,
              "stem_wgrad: contiguous fp32 dw[K*C*R*S]");
  float* dbp = nullptr;
  if (db.has_value() && db->defined()) {
    TORCH_CHECK(db->scalar_type() == torch::kFloat32 && db->is_contiguous() && db->numel() == y.size(1), "stem_wgrad: fp32 db[K]");
    dbp = db->data_ptr<float>();
  }
  check_cuda(ws, "ws");
  TORCH_CHECK(ws.scalar_type() == torch::kFloat32 && ws.numel() >= stem_wgrad_ws(x.size(1), y.size(1), R, S, s),
              "stem_wgrad: fp32 workspace of stem_wgrad_ws elements");
  TORCH_CHECK(fm_stem_wgrad_run(x.data_ptr(), y.data_ptr(), dy.data_ptr(), dw.data_ptr<float>(), dbp, ws.data_ptr<float>(),
                                (int)x.size(0), (int)x.size(1), (int)x.size(2), (int)x.size(3), (int)R, (int)S, (int)y.size(2),
                                (int)y.size(3), (int)s, (int)pt, (int)pl, (int)act, cur()) == 0,
              "stem_wgrad: launch");
}
// space-to-depth: x [N,C,H,W] <-> xs [N, C*s*s, Hs, Ws] (inv scatters xs back into x, acc adds)
void conv_s2d(torch::Tensor x, torch::Tensor xs, int64_t s, int64_t pt, int64_t pl, bool inv, bool acc) {
  chk4(x, "conv_s2d x");
  chk4(xs, "conv_s2d xs");
  same_dt(x, xs, "conv_s2d");
  TORCH_CHECK(x.dim() == 4 && xs.dim() == 4 && xs.size(0) == x.size(0) && xs.size(1) == x.size(1) * s * s,
              "conv_s2d: xs [N, C*s*s, Hs, Ws]");
  TORCH_CHECK(xs.numel() < (1L << 31) && x.numel() < (1L << 31), "conv_s2d: 32-bit indexing");
  fm_conv_s2d_run(x.data_ptr(), xs.data_ptr(), is_bf16(x), (int)x.size(0), (int)x.size(1), (int)x.size(2), (int)x.size(3),
                  (int)s, (int)pt, (int)pl, (int)xs.size(2), (int)xs.size(3), inv ? 1 : 0, acc ? 1 : 0, cur());
}
// kernel re-layout: ws = S2D(w) (inv = false), or dw += S2D^-1(dws) (inv = true, fp32 gradients)
void conv_w_s2d(torch::Tensor w, torch::Tensor ws, torch::Tensor dws, torch::Tensor dw, int64_t s, bool inv) {
  chk4(w, "conv_w_s2d w");
  chk4(ws, "conv_w_s2d ws");
  same_dt(w, ws, "conv_w_s2d");
  TORCH_CHECK(w.dim() == 4 && ws.dim() == 4 && ws.size(1) == w.size(1) * s * s, "conv_w_s2d: ws [K, C*s*s, Rs, Ss]");
  if (inv)
    TORCH_CHECK(dws.scalar_type() == torch::kFloat32 && dw.scalar_type() == torch::kFloat32 && dws.numel() == ws.numel() &&
                    dw.numel() == w.numel(), "conv_w_s2d: fp32 gradients");
  fm_conv_w_s2d_run(w.data_ptr(), ws.data_ptr(), inv ? dws.data_ptr<float>() : nullptr, inv ? dw.data_ptr<float>() : nullptr,
                    is_bf16(w), (int)w.size(0),
                    (int)w.size(1), (int)w.size(2), (int)w.size(3), (int)s, (int)ws.size(2), (int)ws.size(3), inv ? 1 : 0,
                    cur());
}
// NHWC-staged bf16 convolution (csrc/kernels/conv_nhwc.hip).  Every extent the kernels index is
// checked here: staged operands [N][Hp][Wp][Cp] (Cp % 8 == 0), 16-B aligned, under 2 GiB.
static void nhwc_chk(const torch::Tensor& t, long need, const char* n) {
  check_cuda(t, n);
  TORCH_CHECK(t.scalar_type() == torch::kBFloat16 && t.is_contiguous(), n, ": contiguous bf16");
  TORCH_CHECK(t.numel() >= need, n, ": too small (", t.numel(), " < ", need, ")");
  TORCH_CHECK(t.numel() * 2 < (1L << 31) - 64, n, ": under 2 GiB (32-bit buffer offsets)");
  TORCH_CHECK(((uintptr_t)t.data_ptr() & 15) == 0, n, ": 16-B aligned");
}
void nhwc_stage(torch::Tensor src, torch::Tensor dst, int64_t Cp, int64_t Hp, int64_t Wp, int64_t top, int64_t left, int64_t dh,
                int64_t dw) {
  TORCH_CHECK(dh >= 1 && dw >= 1, "nhwc_stage: dilation >= 1");
  TORCH_CHECK(src.dim() == 4, "nhwc_stage: src [N,C,H,W]");
  const long N = src.size(0), C = src.size(1);
  TORCH_CHECK(Cp % 8 == 0 && Cp >= C && Hp > 0 && Wp > 0, "nhwc_stage: Cp % 8 == 0, Cp >= C");
  nhwc_chk(src, src.numel(), "nhwc_stage src");
  nhwc_chk(dst, N * Hp * Wp * Cp, "nhwc_stage dst");
  TORCH_CHECK(N * Hp < (1L << 31), "nhwc_stage: grid");
  fm_nhwc_stage_run(src.data_ptr(), dst.data_ptr(), (int)N, (int)C, (int)src.size(2), (int)src.size(3), (int)Cp, (int)Hp,
                    (int)Wp, (int)top, (int)left, (int)dh, (int)dw, cur());
}
// gradient staging with the activation backward and bias gradient fused: dst = stage(act'(y)*dy)
void nhwc_stage_grad(torch::Tensor dy, torch::Tensor y, torch::Tensor dst, int64_t act, int64_t Cp, int64_t Hp, int64_t Wp,
                     int64_t top, int64_t left, int64_t dh, int64_t dw) {
  TORCH_CHECK(dy.dim() == 4 && y.sizes() == dy.sizes(), "nhwc_stage_grad: dy, y [N,K,P,Q]");
  TORCH_CHECK(dh >= 1 && dw >= 1, "nhwc_stage_grad: dilation >= 1");
  const long N = dy.size(0), C = dy.size(1);
  TORCH_CHECK(Cp % 8 == 0 && Cp >= C && Hp > 0 && Wp > 0, "nhwc_stage_grad: Cp % 8 == 0, Cp >= C");
  nhwc_chk(dy, dy.numel(), "nhwc_stage_grad dy");
  nhwc_chk(y, y.numel(), "nhwc_stage_grad y");
  nhwc_chk(dst, N * Hp * Wp * Cp, "nhwc_stage_grad dst");
  fm_nhwc_stage_grad_run(dy.data_ptr(), y.data_ptr(), dst.data_ptr(), (int)act, (int)N, (int)C, (int)dy.size(2),
                         (int)dy.size(3), (int)Cp, (int)Hp, (int)Wp, (int)top, (int)left, (int)dh, (int)dw, cur());
}
int64_t conv_nhwc_wgrad_ws(int64_t N, int64_t K, int64_t P, int64_t Q, int64_t R, int64_t S, int64_t Cp) {
  return fm_conv_nhwc_wgrad_ws((int)N, (int)K, (int)P, (int)Q, (int)R, (int)S, (int)Cp);
}
// mode 0: out = fwd weight matrix [K][R*S*Cp]; 1: dgrad matrix [C][R*S*Kp]; 3: both (out, out2);
// 2: dw (fp32 [K,C,R,S]) += fold(g2 slabs)
void cnhwc_wprep(torch::Tensor w, torch::Tensor out, torch::Tensor out2, torch::Tensor g2, torch::Tensor dw, int64_t Cp,
                 int64_t Kp, int64_t mode, int64_t nsplit) {
  TORCH_CHECK(nsplit >= 1 && mode >= 0 && mode <= 3, "cnhwc_wprep: mode 0..3, nsplit >= 1");
  TORCH_CHECK(w.dim() == 4, "cnhwc_wprep: w [K,C,R,S]");
  const long K = w.size(0), C = w.size(1), RS = w.size(2) * w.size(3);
  TORCH_CHECK(Cp % 8 == 0 && Cp >= C && Kp % 8 == 0 && Kp >= K, "cnhwc_wprep: padded channel counts");
  if (mode != 2) {
    TORCH_CHECK(K * RS * Cp + C * RS * Kp + 256L * 1024 < (1L << 31), "cnhwc_wprep: weight too large for 32-bit indexing");
    nhwc_chk(w, K * C * RS, "cnhwc_wprep w");
    if (mode == 0 || mode == 3) nhwc_chk(out, K * RS * Cp, "cnhwc_wprep out (fwd matrix)");
    if (mode == 1) nhwc_chk(out, C * RS * Kp, "cnhwc_wprep out (dgrad matrix)");
    if (mode == 3) nhwc_chk(out2, C * RS * Kp, "cnhwc_wprep out2 (dgrad matrix)");
  } else {
    check_cuda(g2, "g2");
    check_cuda(dw, "dw");
    TORCH_CHECK(g2.scalar_type() == torch::kFloat32 && g2.is_contiguous() && g2.numel() >= nsplit * K * RS * Cp,
                "cnhwc_wprep: fp32 g2 [nsplit][K][R*S*Cp]");
    TORCH_CHECK(dw.scalar_type() == torch::kFloat32 && dw.is_contiguous() && dw.numel() == K * C * RS,
                "cnhwc_wprep: fp32 dw [K*C*R*S]");
  }
  fm_cnhwc_wprep_run(w.data_ptr(), mode == 2 ? nullptr : out.data_ptr(), mode == 3 ? out2.data_ptr() : nullptr,
                     mode == 2 ? g2.data_ptr<float>() : nullptr, mode == 2 ? dw.data_ptr<float>() : nullptr, (int)K, (int)C,
                     (int)w.size(2), (int)w.size(3), (int)Cp, (int)Kp, (int)mode, (int)nsplit, cur());
}
// cnhwc_wprep mode 3 of several layers in one launch: w[i] [K,C,R,S] bf16 -> out[i] (fwd matrix
// [K][R*S*Cp[i]]) and out2[i] (dgrad matrix [C][R*S*Kp[i]])
void cnhwc_wprep_multi(std::vector<torch::Tensor> w, std::vector<torch::Tensor> out, std::vector<torch::Tensor> out2,
                       std::vector<int64_t> Cp, std::vector<int64_t> Kp) {
  const size_t n = w.size();
  TORCH_CHECK(out.size() == n && out2.size() == n && Cp.size() == n && Kp.size() == n, "cnhwc_wprep_multi: list sizes");
  std::vector<const void*> wp(n);
  std::vector<void*> op(n), o2(n);
  std::vector<int> K(n), C(n), R(n), S(n), cp(n), kp(n);
  for (size_t i = 0; i < n; ++i) {
    TORCH_CHECK(w[i].dim() == 4, "cnhwc_wprep_multi: w [K,C,R,S]");
    K[i] = (int)w[i].size(0);
    C[i] = (int)w[i].size(1);
    R[i] = (int)w[i].size(2);
    S[i] = (int)w[i].size(3);
    cp[i] = (int)Cp[i];
    kp[i] = (int)Kp[i];
    const long RS = (long)R[i] * S[i];
    TORCH_CHECK(cp[i] % 8 == 0 && cp[i] >= C[i] && kp[i] % 8 == 0 && kp[i] >= K[i], "cnhwc_wprep_multi: padded channel counts");
    TORCH_CHECK((long)K[i] * RS * cp[i] + (long)C[i] * RS * kp[i] + 256L * 1024 < (1L << 31),
                "cnhwc_wprep_multi: weight too large for 32-bit indexing");
    nhwc_chk(w[i], (long)K[i] * C[i] * RS, "cnhwc_wprep_multi w");
    nhwc_chk(out[i], (long)K[i] * RS * cp[i], "cnhwc_wprep_multi out (fwd matrix)");
    nhwc_chk(out2[i], (long)C[i] * RS * kp[i], "cnhwc_wprep_multi out2 (dgrad matrix)");
    wp[i] = w[i].data_ptr();
    op[i] = out[i].data_ptr();
    o2[i] = out2[i].data_ptr();
  }
  if (n) fm_cnhwc_wprep_multi_run((int)n, wp.data(), op.data(), o2.data(), K.data(), C.data(), R.data(), S.data(), cp.data(),
                                  kp.data(), cur());
}

// second output of a conv GEMM: a consumer's staged operand [N][H2][W2][C2] (o2 = {H2, W2, C2, t2, l2,
// d2h, d2w, write_nchw}); every position the epilogue can address lies inside it
static void* out2_chk(const c10::optional<torch::Tensor>& out2, const std::vector<int64_t>& o2, long N, long M, long OH,
                      long OW) {
  if (!out2.has_value() || !out2->defined()) return nullptr;
  TORCH_CHECK(o2.size() == 8, "out2 geometry: {H2, W2, C2, t2, l2, d2h, d2w, write_nchw}");
  TORCH_CHECK(o2[2] >= M && o2[5] >= 1 && o2[6] >= 1, "out2: C2 >= channels, dilation >= 1");
  nhwc_chk(*out2, N * o2[0] * o2[1] * o2[2], "out2");
  (void)OH; (void)OW;   // rows / columns outside [0,H2) x [0,W2) are dropped by the kernel
  return out2->data_ptr();
}
void conv_nhwc_fwd(torch::Tensor xs, torch::Tensor wf, c10::optional<torch::Tensor> bias, torch::Tensor y, int64_t R,
                   int64_t S, int64_t Cp, int64_t Hp, int64_t Wp, int64_t sh, int64_t sw, int64_t act,
                   c10::optional<torch::Tensor> out2, std::vector<int64_t> o2) {
  TORCH_CHECK(y.dim() == 4 && y.scalar_type() == torch::kBFloat16 && y.is_contiguous(), "conv_nhwc_fwd: bf16 y [N,K,P,Q]");
  const long N = y.size(0), K = y.size(1), P = y.size(2), Q = y.size(3);
  TORCH_CHECK(Cp % 8 == 0 && (P - 1) * sh + R <= Hp && (Q - 1) * sw + S <= Wp, "conv_nhwc_fwd: staged window extent");
  nhwc_chk(xs, N * Hp * Wp * Cp, "conv_nhwc_fwd xs");
  nhwc_chk(wf, K * R * S * Cp, "conv_nhwc_fwd wf");
  nhwc_chk(y, N * K * P * Q, "conv_nhwc_fwd y");
  const float* b = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == torch::kFloat32 && bias->numel() == K && bias->is_cuda(), "conv_nhwc_fwd: fp32 bias[K]");
    b = bias->data_ptr<float>();
  }
  void* o2p = out2_chk(out2, o2, N, K, P, Q);
  fm_conv_nhwc_fwd(xs.data_ptr(), xs.numel() * 2, wf.data_ptr(), b, y.data_ptr(), (int)N, (int)K, (int)P, (int)Q, (int)R,
                   (int)S, (int)Cp, (int)Hp, (int)Wp, (int)sh, (int)sw, (int)act, o2p, o2p ? (int)o2[0] : 0,
                   o2p ? (int)o2[1] : 0, o2p ? (int)o2[2] : 0, o2p ? (int)o2[3] : 0, o2p ? (int)o2[4] : 0,
                   o2p ? (int)o2[5] : 1, o2p ? (int)o2[6] : 1, o2p ? (int)o2[7] : 1, cur());
}
void conv_nhwc_dgrad(torch::Tensor gs, torch::Tensor wd, torch::Tensor dx, int64_t R, int64_t S, int64_t Kp, int64_t Hg,
                     int64_t Wg, bool acc, c10::optional<torch::Tensor> out2, std::vector<int64_t> o2) {
  TORCH_CHECK(dx.dim() == 4, "conv_nhwc_dgrad: dx [N,C,H,W]");
  const long N = dx.size(0), C = dx.size(1), H = dx.size(2), W = dx.size(3);
  TORCH_CHECK(Kp % 8 == 0 && H + R - 1 <= Hg && W + S - 1 <= Wg, "conv_nhwc_dgrad: staged G extent");
  nhwc_chk(gs, N * Hg * Wg * Kp, "conv_nhwc_dgrad gs");
  nhwc_chk(wd, C * R * S * Kp, "conv_nhwc_dgrad wd");
  nhwc_chk(dx, N * C * H * W, "conv_nhwc_dgrad dx");
  void* o2p = out2_chk(out2, o2, N, C, H, W);
  TORCH_CHECK(o2p == nullptr || !acc, "conv_nhwc_dgrad: a second output needs the non-accumulating data gradient");
  fm_conv_nhwc_dgrad(gs.data_ptr(), gs.numel() * 2, wd.data_ptr(), dx.data_ptr(), acc ? 1 : 0, (int)N, (int)C, (int)H, (int)W,
                     (int)R, (int)S, (int)Kp, (int)Hg, (int)Wg, o2p, o2p ? (int)o2[0] : 0, o2p ? (int)o2[1] : 0,
                     o2p ? (int)o2[2] : 0, o2p ? (int)o2[3] : 0, o2p ? (int)o2[4] : 0, o2p ? (int)o2[5] : 1,
                     o2p ? (int)o2[6] : 1, o2p ? (int)o2[7] : 1, cur());
}
// strided data gradient by stride phases over the stride-dilated staged G (w: the bf16 weights
// [K,C,R,S]; wsub: bf16 scratch of C*R*S*Kp for the phases' sub-kernels)
void conv_nhwc_dgrad_strided(torch::Tensor gs, torch::Tensor w, torch::Tensor wsub, torch::Tensor dx, int64_t Kp, int64_t Hg,
                             int64_t Wg, int64_t gt, int64_t gl, int64_t sh, int64_t sw, bool acc,
                             c10::optional<torch::Tensor> out2, std::vector<int64_t> o2) {
  TORCH_CHECK(dx.dim() == 4 && w.dim() == 4 && w.size(1) == dx.size(1), "conv_nhwc_dgrad_strided: dx [N,C,H,W], w [K,C,R,S]");
  const long N = dx.size(0), C = dx.size(1), H = dx.size(2), W = dx.size(3);
  const long K = w.size(0), R = w.size(2), S = w.size(3);
  TORCH_CHECK(sh >= 1 && sw >= 1 && Kp % 8 == 0 && Kp >= K && gt >= 0 && gl >= 0 && H + R - 1 <= Hg && W + S - 1 <= Wg,
              "conv_nhwc_dgrad_strided: staged G extent");
  nhwc_chk(gs, N * Hg * Wg * Kp, "conv_nhwc_dgrad_strided gs");
  nhwc_chk(w, K * C * R * S, "conv_nhwc_dgrad_strided w");
  nhwc_chk(wsub, C * R * S * Kp, "conv_nhwc_dgrad_strided wsub");
  nhwc_chk(dx, N * C * H * W, "conv_nhwc_dgrad_strided dx");
  void* o2p = out2_chk(out2, o2, N, C, H, W);
  TORCH_CHECK(o2p == nullptr || !acc, "conv_nhwc_dgrad_strided: a second output needs the non-accumulating data gradient");
  fm_conv_nhwc_dgrad_strided(gs.data_ptr(), gs.numel() * 2, w.data_ptr(), wsub.data_ptr(), dx.data_ptr(), acc ? 1 : 0, (int)N,
                             (int)C, (int)H, (int)W, (int)K, (int)R, (int)S, (int)Kp, (int)Hg, (int)Wg, (int)gt, (int)gl,
                             (int)sh, (int)sw, o2p, o2p ? (int)o2[0] : 0, o2p ? (int)o2[1] : 0, o2p ? (int)o2[2] : 0,
                             o2p ? (int)o2[3] : 0, o2p ? (int)o2[4] : 0, o2p ? (int)o2[5] : 1, o2p ? (int)o2[6] : 1,
                             o2p ? (int)o2[7] : 1, cur());
}
int64_t conv_nhwc_wgrad(torch::Tensor gs, torch::Tensor xs, torch::Tensor g2, c10::optional<torch::Tensor> db, int64_t N, int64_t K, int64_t Kp, int64_t P,
                     int64_t Q, int64_t Hg, int64_t Wg, int64_t gt, int64_t gl, int64_t gsh, int64_t gsw, int64_t R, int64_t S,
                     int64_t Cp, int64_t Hp, int64_t Wp, int64_t sh, int64_t sw, torch::Tensor ptab, bool build_tab) {
  TORCH_CHECK(Kp % 8 == 0 && Kp >= K && Cp % 8 == 0 && gt >= 0 && gl >= 0 && gsh >= 1 && gsw >= 1 &&
                  gt + (P - 1) * gsh < Hg && gl + (Q - 1) * gsw < Wg &&
                  (P - 1) * sh + R <= Hp && (Q - 1) * sw + S <= Wp,
              "conv_nhwc_wgrad: staged extents");
  nhwc_chk(gs, N * Hg * Wg * Kp, "conv_nhwc_wgrad gs");
  nhwc_chk(xs, N * Hp * Wp * Cp, "conv_nhwc_wgrad xs");
  check_cuda(g2, "g2");
  TORCH_CHECK(g2.scalar_type() == torch::kFloat32 && g2.is_contiguous() &&
                  g2.numel() >= fm_conv_nhwc_wgrad_ws((int)N, (int)K, (int)P, (int)Q, (int)R, (int)S, (int)Cp),
              "conv_nhwc_wgrad: fp32 g2 slabs (conv_nhwc_wgrad_ws floats)");
  float* dbp = nullptr;
  if (db.has_value() && db->defined()) {
    TORCH_CHECK(db->is_cuda() && db->scalar_type() == torch::kFloat32 && db->numel() == K && db->is_contiguous(),
                "conv_nhwc_wgrad: fp32 db[K]");
    dbp = db->data_ptr<float>();
  }
  TORCH_CHECK(N * P * Q < (1L << 28), "conv_nhwc_wgrad: pixel count");
  check_cuda(ptab, "ptab");
  TORCH_CHECK(ptab.scalar_type() == torch::kInt32 && ptab.is_contiguous() && ptab.numel() >= 2 * N * P * Q,
              "conv_nhwc_wgrad: int32 ptab[2*N*P*Q]");
  return fm_conv_nhwc_wgrad(gs.data_ptr(), gs.numel() * 2, xs.data_ptr(), xs.numel() * 2, g2.data_ptr<float>(), dbp, (int)N, (int)K,
                     (int)Kp, (int)P, (int)Q, (int)Hg, (int)Wg, (int)gt, (int)gl, (int)gsh, (int)gsw, (int)R, (int)S, (int)Cp,
                     (int)Hp, (int)Wp, (int)sh, (int)sw, ptab.data_ptr<int>(), build_tab ? 1 : 0, cur());
}
void conv_act_bwd(torch::Tensor dy, torch::Tensor y, torch::Tensor g, c10::optional<torch::Tensor> db, int64_t act) {
  chk4(dy, "dy");
  chk4(y, "y");
  chk4(g, "g");
  same_dt(dy, y, "conv_act_bwd");
  same_dt(dy, g, "conv_act_bwd");
  TORCH_CHECK(dy.dim() == 4 && y.sizes() == dy.sizes() && g.sizes() == dy.sizes(), "conv_act_bwd: [N,K,P,Q]");
  float* dbp = nullptr;
  if (db.has_value() && db->defined()) {
    TORCH_CHECK(db->scalar_type() == torch::kFloat32 && db->numel() == dy.size(1), "conv_act_bwd: fp32 db[K]");
    dbp = db->data_ptr<float>();
  }
  fm_conv_act_bwd(dy.data_ptr(), y.data_ptr(), g.data_ptr(), dbp, is_bf16(dy), (int)dy.size(0), (int)dy.size(1),
                  (int)(dy.size(2) * dy.size(3)), (int)act, cur());
}
static unsigned char* code_ptr(const c10::optional<torch::Tensor>& code, const torch::Tensor& y, const char* n) {
  if (!code.has_value() || !code->defined()) return nullptr;
  check_cuda(*code, n);
  TORCH_CHECK(code->scalar_type() == torch::kUInt8 && code->numel() >= y.numel(), n, ": uint8 code[y.numel()]");
  return code->data_ptr<uint8_t>();
}
// code (max pooling, optional): per-window argmax bytes for the backward pass
void pool_fwd(torch::Tensor x, torch::Tensor y, c10::optional<torch::Tensor> code, int64_t kh, int64_t kw, int64_t sh,
              int64_t sw, int64_t pt, int64_t pl, bool is_max, int64_t act) {
  chk4(x, "x");
  chk4(y, "y");
  same_dt(x, y, "pool_fwd");
  TORCH_CHECK(kh * kw < 255 && x.numel() < (1L << 31) && y.numel() < (1L << 31), "pool_fwd: window < 255, 32-bit indexing");
  fm_pool_fwd(x.data_ptr(), y.data_ptr(), code_ptr(code, y, "pool_fwd"), x.size(0), x.size(1), x.size(2), x.size(3),
              y.size(2), y.size(3), kh, kw, sh, sw, pt, pl, is_max, act, is_bf16(x), cur());
}
// code: uint8 scratch of y.numel() bytes (max pooling's per-window argmax); code_ready: the
// forward already filled it
void pool_bwd(torch::Tensor x, torch::Tensor y, torch::Tensor dy, torch::Tensor dx, torch::Tensor code, bool code_ready,
              int64_t kh, int64_t kw, int64_t sh, int64_t sw, int64_t pt, int64_t pl, bool is_max, int64_t act, bool acc) {
  TORCH_CHECK(kh * kw < 255 && x.numel() < (1L << 31), "pool_bwd: window < 255 elements, 32-bit indexing");
  chk4(x, "x");
  chk4(y, "y");
  chk4(dy, "dy");
  chk4(dx, "dx");
  same_dt(x, y, "pool_bwd");
  same_dt(x, dy, "pool_bwd");
  same_dt(x, dx, "pool_bwd");
  unsigned char* c = code_ptr(code, y, "pool_bwd");
  TORCH_CHECK(c != nullptr, "pool_bwd: code scratch required");
  fm_pool_bwd(x.data_ptr(), y.data_ptr(), dy.data_ptr(), dx.data_ptr(), c, code_ready ? 1 : 0, x.size(0), x.size(1),
              x.size(2), x.size(3), y.size(2), y.size(3), kh, kw, sh, sw, pt, pl, is_max, act, acc, is_bf16(x), cur());
}
void bn_fwd(torch::Tensor x, torch::Tensor y, torch::Tensor gamma, torch::Tensor beta, torch::Tensor stats,
            torch::Tensor meaninv, double eps, bool relu) {
  chk4(x, "x");
  chk4(y, "y");
  same_dt(x, y, "bn_fwd");
  const long C = x.size(1);
  TORCH_CHECK(gamma.scalar_type() == torch::kFloat32 && beta.scalar_type() == torch::kFloat32 && gamma.numel() >= C,
              "bn: fp32 gamma/beta [C]");
  TORCH_CHECK(stats.numel() >= 2 * C && meaninv.numel() >= 2 * C, "bn: stats [2C]");
  fm_bn_fwd(x.data_ptr(), y.data_ptr(), gamma.data_ptr<float>(), beta.data_ptr<float>(), stats.data_ptr<float>(),
            meaninv.data_ptr<float>(), x.size(0), C, x.size(2) * x.size(3), (float)eps, relu, is_bf16(x), cur());
}
void bn_bwd(torch::Tensor x, torch::Tensor y, torch::Tensor dy, torch::Tensor meaninv, torch::Tensor gamma,
            torch::Tensor gsum, torch::Tensor dgamma, torch::Tensor dbeta, c10::optional<torch::Tensor> dx, bool relu,
            bool acc) {
  chk4(x, "x");
  chk4(dy, "dy");
  same_dt(x, dy, "bn_bwd");
  same_dt(x, y, "bn_bwd");
  if (dx.has_value() && dx->defined()) same_dt(x, *dx, "bn_bwd");
  const long C = x.size(1);
  TORCH_CHECK(gsum.numel() >= 2 * C && dgamma.numel() >= C && dbeta.numel() >= C, "bn_bwd: sizes");
  fm_bn_bwd(x.data_ptr(), y.data_ptr(), dy.data_ptr(), meaninv.data_ptr<float>(), gamma.data_ptr<float>(),
            gsum.data_ptr<float>(), dgamma.data_ptr<float>(), dbeta.data_ptr<float>(), mptr(dx), x.size(0), C,
            x.size(2) * x.size(3), relu, acc, is_bf16(x), cur());
}
void compact_rows(torch::Tensor src, torch::Tensor dst, int64_t K, int64_t n, int64_t ldp, bool acc) {
  TORCH_CHECK(src.numel() >= K * ldp && dst.numel() >= K * n, "compact_rows: sizes");
  fm_compact_rows(src.data_ptr<float>(), dst.data_ptr<float>(), K, n, ldp, acc, cur());
}
void pad_rows(torch::Tensor src, torch::Tensor dst, int64_t K, int64_t n, int64_t ldp) {
  TORCH_CHECK(src.numel() >= K * n && dst.numel() >= K * ldp && src.scalar_type() == dst.scalar_type(), "pad_rows: sizes");
  fm_pad_rows(src.data_ptr(), dst.data_ptr(), K, n, ldp, is_bf16(src), cur());
}

// ----------------------------------------------------------------------------- LSTM
static float* fp(torch::Tensor& t, int64_t off) {
  TORCH_CHECK(t.scalar_type() == torch::kFloat32 && off >= 0 && off < t.numel(), "lstm: fp32 buffer/offset");
  return t.data_ptr<float>() + off;
}
// activation-dtype (bf16 or fp32) buffer at an element offset
static void* bp(torch::Tensor& t, int64_t off) {
  TORCH_CHECK((t.scalar_type() == torch::kBFloat16 || t.scalar_type() == torch::kFloat32) && off >= 0 && off < t.numel(),
              "lstm: bf16/fp32 buffer/offset");
  return (char*)t.data_ptr() + t.element_size() * off;
}
void lstm_init(c10::optional<torch::Tensor> h0, c10::optional<torch::Tensor> c0, torch::Tensor hprev, int64_t ldhp,
               torch::Tensor cinit, int64_t B, int64_t H) {
  TORCH_CHECK(hprev.numel() >= (B - 1) * ldhp + H && cinit.numel() >= B * H, "lstm_init: sizes");
  fm_lstm_init(cptr(h0), cptr(c0), bp(hprev, 0), ldhp, fp(cinit, 0), B, H, is_bf16(hprev), cur());
}
void lstm_cell_fwd(torch::Tensor G, int64_t g_off, int64_t ldg, torch::Tensor cprev, int64_t cp_off, int64_t ldcp,
                   torch::Tensor cout, int64_t c_off, int64_t ldc, torch::Tensor y, int64_t y_off, int64_t ldy,
                   torch::Tensor hprev, int64_t hp_off, int64_t ldhp, c10::optional<torch::Tensor> hT,
                   c10::optional<torch::Tensor> cT, int64_t B, int64_t H) {
  TORCH_CHECK(g_off + (B - 1) * ldg + 4 * H <= G.numel() && c_off + (B - 1) * ldc + H <= cout.numel() &&
                  y_off + (B - 1) * ldy + H <= y.numel(), "lstm_cell_fwd: extents");
  void* hn = hp_off >= 0 ? bp(hprev, hp_off) : nullptr;
  fm_lstm_cell_fwd(fp(G, g_off), ldg, fp(cprev, cp_off), ldcp, fp(cout, c_off), ldc, bp(y, y_off), ldy, hn, ldhp, mptr(hT),
                   mptr(cT), B, H, is_bf16(y), cur());
}
void lstm_cell_bwd(torch::Tensor A, int64_t a_off, int64_t lda, torch::Tensor ct, int64_t ct_off, int64_t ldc,
                   torch::Tensor cprev, int64_t cp_off, int64_t ldcp, c10::optional<torch::Tensor> dy, int64_t dy_off,
                   int64_t ldy, torch::Tensor dh, torch::Tensor dc, torch::Tensor dG, int64_t dg_off, int64_t lddg,
                   int64_t B, int64_t H) {
  TORCH_CHECK(a_off + (B - 1) * lda + 4 * H <= A.numel() && dg_off + (B - 1) * lddg + 4 * H <= dG.numel() &&
                  dh.numel() >= B * H && dc.numel() >= B * H, "lstm_cell_bwd: extents");
  const void* dyp = nullptr;
  if (dy.has_value() && dy->defined()) {
    TORCH_CHECK(dy_off + (B - 1) * ldy + H <= dy->numel() && dy->scalar_type() == dG.scalar_type(), "lstm_cell_bwd: dy extent");
    dyp = (const char*)dy->data_ptr() + dy->element_size() * dy_off;
  }
  fm_lstm_cell_bwd(fp(A, a_off), lda, fp(ct, ct_off), ldc, fp(cprev, cp_off), ldcp, dyp, ldy, fp(dh, 0), fp(dc, 0),
                   bp(dG, dg_off), lddg, B, H, is_bf16(dG), cur());
}

PYBIND11_MODULE(_C, m) {
  m.doc() = "flexmi HIP/CDNA4 kernels (gfx950)";
  m.def("gemm", &gemm, py::arg("A"), py::arg("lda"), py::arg("sA"), py::arg("a_kcontig"), py::arg("B"), py::arg("ldb"),
        py::arg("sB"), py::arg("b_kcontig"), py::arg("C"), py::arg("ldc"), py::arg("sC"), py::arg("bias"), py::arg("M"),
        py::arg("N"), py::arg("K"), py::arg("batch"), py::arg("alpha"), py::arg("beta"), py::arg("act"), py::arg("ws"),
        py::arg("ksplit"), py::arg("act_y"), py::arg("lday"), py::arg("bwd_act"), py::arg("colsum"), py::arg("rowsum_a"));
  m.def("gemm_dw_sgd", &gemm_dw_sgd, py::arg("dpre"), py::arg("x"), py::arg("W"), py::arg("Wc"), py::arg("V"),
        py::arg("lr"), py::arg("wd"), py::arg("mom"), py::arg("nesterov"), py::arg("db"), py::arg("ws"), py::arg("cfg") = 0);
  m.def("gemm_f32_last_form", []() { return fm_gemm_f32_last_form(); });
  m.def("sgd_segs", &sgd_segs);
  m.def("init_fill", &init_fill);
  m.def("smallk_fwd", &smallk_fwd);
  m.def("smallk_dw", &smallk_dw);
  m.def("skinny_fwd", &skinny_fwd);
  m.def("skinny_bwd", &skinny_bwd, py::arg("x"), py::arg("w"), py::arg("y"), py::arg("dy"), py::arg("dx"), py::arg("dx_acc"),
        py::arg("dw"), py::arg("db"), py::arg("act"), py::arg("bact") = 10);
  m.def("conv_scratch", &conv_scratch);
  m.def("conv_fwd", &conv_fwd);
  m.def("conv_dgrad", &conv_dgrad);
  m.def("conv_wgrad", &conv_wgrad);
  m.def("conv_act_bwd", &conv_act_bwd);
  m.def("nhwc_stage", &nhwc_stage);
  m.def("nhwc_stage_grad", &nhwc_stage_grad);
  m.def("conv_nhwc_wgrad_ws", &conv_nhwc_wgrad_ws);
  m.def("cnhwc_wprep_multi", &cnhwc_wprep_multi);
  m.def("conv_nhwc_set_shape", [](int64_t mode, int64_t shape) { fm_conv_nhwc_set_shape((int)mode, (int)shape); });
  m.def("cnhwc_wprep", &cnhwc_wprep);
  m.def("conv_nhwc_fwd", &conv_nhwc_fwd);
  m.def("conv_nhwc_dgrad", &conv_nhwc_dgrad);
  // 0 = native fp32 MFMA, 1 = split-bf16 kernel (gemm_f32.hip x3), 2 = its second form (gemm_x3.hip);
  // bools map to 0 / 1 for the older callers
  m.def("gemm_f32_set_split", [](int mode) { fm_gemm_f32_set_split(mode); });
  m.def("gemm_set_dma", [](int on) { fm_gemm_set_dma(on); });
  m.def("gemm_dma_enabled", []() { return fm_gemm_dma_enabled(); });
  m.def("gemm_f32_get_split", []() { return fm_gemm_f32_get_split(); });
  // sparse-SGD kernels of tables with slot buffers: 1 = count / update, 0 = claim / dup / owner
  m.def("embedding_set_bwd_mode", [](bool count) { fm_embedding_set_bwd_mode(count ? 1 : 0); });
  m.def("conv_nhwc_dgrad_strided", &conv_nhwc_dgrad_strided);
  m.def("conv_nhwc_wgrad", &conv_nhwc_wgrad);
  m.def("conv_s2d", &conv_s2d);
  m.def("stem_supported", &stem_supported);
  m.def("stem_wgrad_ws", &stem_wgrad_ws);
  m.def("stem_wf_elems", &stem_wf_elems);
  m.def("stem_fwd", &stem_fwd);
  m.def("stem_wgrad", &stem_wgrad);
  m.def("conv_w_s2d", &conv_w_s2d);
  m.def("embedding_fwd", &embedding_fwd);
  m.def("embedding_bwd", &embedding_bwd);
  m.def("embedding_fwd_multi", &embedding_fwd_multi, py::arg("W"), py::arg("idx"), py::arg("out"), py::arg("ldo"),
        py::arg("scale"), py::arg("row_lo") = std::vector<int64_t>{});
  m.def("embedding_bwd_multi", &embedding_bwd_multi, py::arg("W"), py::arg("idx"), py::arg("dy"), py::arg("ldg"),
        py::arg("scale"), py::arg("lr"), py::arg("claim"), py::arg("row_lo") = std::vector<int64_t>{});
  m.def("strided_copy4", &strided_copy4);
  m.def("sdp_coalesce", &sdp_coalesce);
  m.def("sdp_apply", &sdp_apply);
  m.def("dot_fwd", &dot_fwd);
  m.def("dot_bwd", &dot_bwd, py::arg("zs"), py::arg("ldz"), py::arg("dout"), py::arg("ldo"), py::arg("dzs"),
        py::arg("lddz"), py::arg("acc_mask"), py::arg("D"), py::arg("self"), py::arg("act0") = 10);
  m.def("sgd", &sgd);
  m.def("adam", &adam);
  m.def("cast_bf16", &cast_bf16);
  m.def("loss", &loss, py::arg("loss_type"), py::arg("logits"), py::arg("labels"), py::arg("grad"), py::arg("scale"),
        py::arg("acc"), py::arg("mask"), py::arg("clamp_t") = 0.0);
  m.def("unary_fwd", &unary_fwd);
  m.def("unary_bwd", &unary_bwd);
  m.def("binary_fwd", &binary_fwd);
  m.def("binary_bwd", &binary_bwd);
  m.def("act_bwd_bias", &act_bwd_bias);
  m.def("multi_copy", &multi_copy);
  m.def("image_normalize", &image_normalize);
  m.def("permute", &permute);
  m.def("reverse", &reverse);
  m.def("softmax", &softmax);
  m.def("dropout", &dropout);
  m.def("im2col", &im2col);
  m.def("col2im", &col2im);
  m.def("transpose_batched", &transpose_batched);
  m.def("pool_fwd", &pool_fwd);
  m.def("pool_bwd", &pool_bwd);
  m.def("bn_fwd", &bn_fwd);
  m.def("bn_bwd", &bn_bwd);
  m.def("compact_rows", &compact_rows);
  m.def("pad_rows", &pad_rows);
  m.def("lstm_init", &lstm_init);
  m.def("lstm_cell_fwd", &lstm_cell_fwd);
  m.def("lstm_cell_bwd", &lstm_cell_bwd);
  m.attr("arch") = "gfx950";
}
