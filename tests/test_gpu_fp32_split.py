"""fp32 GEMM on the bf16 matrix cores by exact three-way operand splitting (csrc/kernels/gemm_f32.hip
fm_gemm_x3_kernel, FM_F32_SPLIT=1 / gemm_f32_set_split): every orientation, tails, epilogues, the
fused backward epilogue, row sums and split-K against a float64 oracle at the fp32 test tolerance,
with its error compared to the native v_mfma_f32_16x16x4_f32 kernel's on the same inputs."""
import pytest
import torch

from tests.test_gpu_fp32 import TOL, _fused_backward_epilogue, rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture
def split():
    from flexmi.ops import _kernels as Kk
    Kk.C().gemm_f32_set_split(True)
    yield Kk
    Kk.C().gemm_f32_set_split(False)


def _gemm(Kk, A, B, a_k, b_k, M, N, K):
    Ag = A if a_k else A.t().contiguous()
    Bg = B.t().contiguous() if b_k else B
    C = torch.empty(M, N, device=A.device)
    Kk.gemm(Ag, K if a_k else M, a_k, Bg, K if b_k else N, b_k, C, N, M, N, K)
    return C


@pytest.mark.parametrize("a_k,b_k", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (300, 200, 130), (8192, 1024, 1024), (2048, 479, 512),
                                   (8192, 1024, 480), (1000, 1020, 8192), (256, 4096, 4096), (129, 67, 67)])
def test_split_gemm_orientations_vs_native(gpu, a_k, b_k, M, N, K):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(M + N + K)
    A, B = torch.randn(M, K, device=gpu), torch.randn(K, N, device=gpu)
    ref = A.double() @ B.double()
    Kk.C().gemm_f32_set_split(False)
    e_native = rel_err(_gemm(Kk, A, B, a_k, b_k, M, N, K), ref)
    Kk.C().gemm_f32_set_split(True)
    try:
        e_split = rel_err(_gemm(Kk, A, B, a_k, b_k, M, N, K), ref)
    finally:
        Kk.C().gemm_f32_set_split(False)
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


def test_split_wide_dynamic_range(gpu):
    """Operands spanning many binades (the split terms are relative to each element's own exponent)."""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(5)
    M, N, K = 512, 256, 1024
    A = torch.randn(M, K, device=gpu) * torch.exp2(torch.randint(-20, 20, (M, K), device=gpu).float())
    B = torch.randn(K, N, device=gpu) * torch.exp2(torch.randint(-20, 20, (K, N), device=gpu).float())
    ref = A.double() @ B.double()
    Kk.C().gemm_f32_set_split(False)
    e_native = rel_err(_gemm(Kk, A, B, True, False, M, N, K), ref)
    Kk.C().gemm_f32_set_split(True)
    try:
        e_split = rel_err(_gemm(Kk, A, B, True, False, M, N, K), ref)
    finally:
        Kk.C().gemm_f32_set_split(False)
    assert e_split < 4 * e_native + 1e-6, (e_split, e_native)


def test_split_dlrm_mlperf_widths_matches_cpu(gpu, split):
    from tests.test_gpu_fp32 import test_dlrm_mlperf_widths_fp32_gpu_matches_cpu as t
    t(gpu, True)
