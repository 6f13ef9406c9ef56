"""fp32 GEMM on the 16-bit matrix cores by operand splitting (csrc/kernels/gemm_x3.hip): the exact bf16
three-way split (gemm_f32_set_split(2) = every eligible GEMM, 3 = the big-GEMM policy) and the scaled
fp16 two-plane split (4 / 5: the same policies): every orientation, tails, epilogues, fused SGD, the fused
backward epilogue, row sums and split-K against a float64 oracle at the fp32 test tolerance, with
its error compared to the native v_mfma_f32_16x16x4_f32 kernel's on the same inputs."""
import pytest
import torch

from tests.test_gpu_fp32 import TOL, _fused_backward_epilogue, rel_err

pytestmark = pytest.mark.gpu


MODES = [2, 3, 4, 5]     # split mode (4 / 5: the fp16 two-plane scaled form)


@pytest.fixture(params=MODES)
def split(request):
    from flexmi.ops import _kernels as Kk
    prev = Kk.C().gemm_f32_get_split()
    Kk.C().gemm_f32_set_split(request.param)
    yield Kk
    Kk.C().gemm_f32_set_split(prev)


@pytest.fixture(autouse=True)
def _restore_split_mode():
    """Tests below switch the split mode explicitly; leave the process default (3) behind."""
    from flexmi.ops import _kernels as Kk
    prev = Kk.C().gemm_f32_get_split()
    yield
    Kk.C().gemm_f32_set_split(prev)


def _gemm(Kk, A, B, a_k, b_k, M, N, K):
    Ag = A if a_k else A.t().contiguous()
    Bg = B.t().contiguous() if b_k else B
    C = torch.empty(M, N, device=A.device)
    Kk.gemm(Ag, K if a_k else M, a_k, Bg, K if b_k else N, b_k, C, N, M, N, K)
    return C


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("a_k,b_k", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (300, 200, 130), (8192, 1024, 1024), (2048, 479, 512),
                                   (8192, 1024, 480), (1000, 1020, 8192), (256, 4096, 4096), (129, 67, 67),
                                   (330, 194, 96), (8192, 512, 1024), (1024, 480, 8192),
                                   # the default policy's boundaries (mode 3: min(M, N) >= 480, K >= 480)
                                   (480, 480, 480), (479, 1024, 1024), (1024, 479, 1024), (1024, 1024, 479),
                                   (480, 512, 512)])
def test_split_gemm_orientations_vs_native(gpu, mode, a_k, b_k, M, N, K):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(M + N + K)
    A, B = torch.randn(M, K, device=gpu), torch.randn(K, N, device=gpu)
    ref = A.double() @ B.double()
    Kk.C().gemm_f32_set_split(0)
    e_native = rel_err(_gemm(Kk, A, B, a_k, b_k, M, N, K), ref)
    Kk.C().gemm_f32_set_split(mode)
    try:
        e_split = rel_err(_gemm(Kk, A, B, a_k, b_k, M, N, K), ref)
    finally:
        Kk.C().gemm_f32_set_split(0)
    assert e_split < TOL, (e_split, e_native)
    assert e_split < 4 * e_native + 1e-6, (e_split, e_native)     # fp32-class accuracy, not bf16's ~1e-2


def test_split_epilogue_bias_act_beta(gpu, split):
    torch.manual_seed(1)
    M, N, K = 1000, 384, 192
    A, W, b = torch.randn(M, K, device=gpu), torch.randn(N, K, device=gpu), torch.randn(N, device=gpu)
    for act, fn in ((11, torch.relu), (12, torch.sigmoid), (13, torch.tanh)):
        C = torch.randn(M, N, device=gpu)
        C0 = C.double().clone()
        split.gemm(A, K, True, W, K, True, C, N, M, N, K, bias=b, act=act, beta=True)
        assert rel_err(C, fn(A.double() @ W.double().t() + b.double()) + C0) < TOL, act


@pytest.mark.parametrize("M,K,N", [(2048, 512, 256), (8192, 1024, 1024), (8192, 480, 1024)])
def test_split_fused_backward_epilogue(gpu, split, M, K, N):
    torch.manual_seed(3)
    _fused_backward_epilogue(split, gpu, M, K, N)


@pytest.mark.parametrize("ks", [2, 4, 8])
def test_split_splitk(gpu, split, ks):
    torch.manual_seed(2)
    M, N, K = 256, 128, 8192
    A, B = torch.randn(K, M, device=gpu), torch.randn(K, N, device=gpu)
    bias = torch.randn(N, device=gpu)
    C = torch.empty(M, N, device=gpu)
    assert split.gemm(A, M, False, B, N, False, C, N, M, N, K, bias=bias, ksplit=ks) == ks
    assert rel_err(C, A.double().t() @ B.double() + bias.double()) < TOL


@pytest.mark.parametrize("mode", MODES)
def test_split_wide_dynamic_range(gpu, mode):
    """Operands spanning many binades (the split terms are relative to each element's own exponent)."""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(5)
    M, N, K = 512, 256, 1024
    A = torch.randn(M, K, device=gpu) * torch.exp2(torch.randint(-20, 20, (M, K), device=gpu).float())
    B = torch.randn(K, N, device=gpu) * torch.exp2(torch.randint(-20, 20, (K, N), device=gpu).float())
    ref = A.double() @ B.double()
    Kk.C().gemm_f32_set_split(0)
    e_native = rel_err(_gemm(Kk, A, B, True, False, M, N, K), ref)
    Kk.C().gemm_f32_set_split(mode)
    try:
        e_split = rel_err(_gemm(Kk, A, B, True, False, M, N, K), ref)
    finally:
        Kk.C().gemm_f32_set_split(0)
    assert e_split < 4 * e_native + 1e-6, (e_split, e_native)


def test_split_dlrm_mlperf_widths_matches_cpu(gpu, split):
    from tests.test_gpu_fp32 import test_dlrm_mlperf_widths_fp32_gpu_matches_cpu as t
    t(gpu, True)


@pytest.mark.parametrize("Nout,Kin", [(1024, 480), (512, 1024), (256, 130)])
def test_split2_dw_rowsum(gpu, Nout, Kin):
    """dW += dpre^T x with the bias-gradient row sums (both operands MN-contiguous)."""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(6)
    B = 8192
    dpre, x = torch.randn(B, Nout, device=gpu), torch.randn(B, Kin, device=gpu)
    dw0, db0 = torch.randn(Nout, Kin, device=gpu), torch.randn(Nout, device=gpu)
    dw, db = dw0.clone(), db0.clone()
    Kk.C().gemm_f32_set_split(2)
    try:
        Kk.gemm(dpre, Nout, False, x, Kin, False, dw, Kin, Nout, Kin, B, beta=True, rowsum_a=db)
    finally:
        Kk.C().gemm_f32_set_split(0)
    assert rel_err(dw - dw0, dpre.double().t() @ x.double()) < TOL
    assert rel_err(db - db0, dpre.double().sum(0)) < TOL


@pytest.mark.parametrize("mom,nesterov", [(0.0, False), (0.9, True)])
@pytest.mark.parametrize("Nout,Kin", [(1024, 1024), (256, 512)])
def test_split2_dw_fused_sgd(gpu, mom, nesterov, Nout, Kin):
    """The SGD step fused into the split kernel's dW epilogue (unsplit) or its split-K reduce."""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(7)
    B, lr, wd = 8192, 0.05, 1e-4
    dpre, x = torch.randn(B, Nout, device=gpu), torch.randn(B, Kin, device=gpu)
    w = torch.randn(Nout, Kin, device=gpu)
    v = torch.randn(Nout, Kin, device=gpu) if mom > 0 else None
    db = torch.zeros(Nout, device=gpu)
    g = dpre.double().t() @ x.double() + wd * w.double()
    if mom > 0:
        v_ref = v.double() * mom + g
        g = g + mom * v_ref if nesterov else v_ref
    w_ref = w.double() - lr * g
    Kk.C().gemm_f32_set_split(2)
    try:
        ks = Kk.C().gemm_dw_sgd(dpre, x, w, None, v, torch.tensor([lr], device=gpu), wd, mom, nesterov, db,
                                Kk.workspace(gpu, Kk.GEMM_WS_BYTES))
    finally:
        Kk.C().gemm_f32_set_split(0)
    assert ks >= 1
    assert rel_err(w, w_ref) < TOL
    assert rel_err(db, dpre.double().sum(0)) < TOL


def test_split_nonfinite_operand(gpu):
    """Documented behaviour of the exact split (csrc/kernels/gemm_x3.hip split1): an inf operand turns
    the rows / columns it reaches into NaN (the native fp32 kernel gives inf); finite entries are
    unaffected."""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(21)
    M = N = K = 512
    A, B = torch.randn(M, K, device=gpu), torch.randn(K, N, device=gpu)
    A[3, 7] = float("inf")
    C = torch.empty(M, N, device=gpu)
    Kk.C().gemm_f32_set_split(2)
    try:
        Kk.gemm(A, K, True, B.t().contiguous(), K, True, C, N, M, N, K)
    finally:
        Kk.C().gemm_f32_set_split(3)
    assert torch.isnan(C[3]).all()
    mask = torch.ones(M, dtype=torch.bool, device=gpu)
    mask[3] = False
    ref = A[mask].double() @ B.double()
    assert rel_err(C[mask], ref) < TOL


@pytest.mark.parametrize("mode,a_k,b_k", [(4, True, True), (4, True, False), (5, True, True), (5, True, False),
                                          (5, False, False)])
def test_f16_split_row_scales(gpu, mode, a_k, b_k):
    """The fp16 form scales every A row and B column by its own power of two: rows and columns whose
    magnitudes span twelve decades, an all-zero row and column, subnormal-size and 1e30-size rows all
    come out at fp32 accuracy relative to EACH row's own magnitude (not only the global max).  (Mode 4
    runs the dW orientation on the bf16 three-plane split, whose bf16 MFMA inputs flush subnormals:
    only the F16 orientations are taken here.)"""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(7)
    M, N, K = 1024, 640, 1024
    A = torch.randn(M, K, device=gpu) * torch.pow(10.0, -12 * torch.rand(M, 1, device=gpu))
    B = torch.randn(K, N, device=gpu) * torch.pow(10.0, -6 * torch.rand(1, N, device=gpu))
    A[3] = 0.0
    B[:, 5] = 0.0
    A[7] *= 1e-30
    A[9] *= 1e30
    ref = A.double() @ B.double()
    Kk.C().gemm_f32_set_split(0)
    Cn = _gemm(Kk, A, B, a_k, b_k, M, N, K)
    Kk.C().gemm_f32_set_split(mode)
    Cs = _gemm(Kk, A, B, a_k, b_k, M, N, K)
    for C, name in ((Cs, "split"), (Cn, "native")):
        assert torch.isfinite(C).all(), name
    assert (Cs[3] == 0).all() and (Cs[:, 5] == 0).all()
    rowmax = ref.abs().amax(1, keepdim=True) + 1e-300
    e_split = ((Cs.double() - ref).abs() / rowmax).max().item()
    e_native = ((Cn.double() - ref).abs() / rowmax).max().item()
    assert e_split < 4 * e_native + 1e-6, (e_split, e_native)
