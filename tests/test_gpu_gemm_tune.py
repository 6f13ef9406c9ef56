"""Every GEMM configuration the tuner can select (flexmi/ops/gemm_tune.py: kernel form x split-K
depth, forced through the ksplit encoding) computes the same GEMM: fp32 forms against a float64
oracle at the fp32 tolerance (and run in the requested form where it applies), bf16 forms at the
bf16 tolerance, with the epilogues the step uses (bias + activation, beta accumulate, fused
backward epilogue, row sums, fused SGD)."""
import pytest
import torch

from tests.test_gpu_fp32 import TOL, rel_err

pytestmark = pytest.mark.gpu


def _mk(M, N, K, a_k, b_k, dev, dt):
    """Operands in the GEMM's storage orientation (dt) and their float64 [M, K] / [K, N] values."""
    A = torch.randn(M, K, device=dev).to(dt)
    B = (torch.randn(K, N, device=dev) * 0.05).to(dt)
    Ag = A if a_k else A.t().contiguous()
    Bg = B.t().contiguous() if b_k else B
    return Ag, Bg, A.double(), B.double()


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("M,N,K,a_k,b_k", [(8192, 1024, 480, True, True), (1024, 479, 8192, False, False),
                                           (8192, 512, 256, True, False), (256, 128, 8192, False, False),
                                           (300, 200, 4096, True, True)])
def test_every_candidate_matches_the_oracle(gpu, dtype, M, N, K, a_k, b_k):
    from flexmi.ops import _kernels as Kk
    from flexmi.ops import gemm_tune as T
    torch.manual_seed(M + N + K)
    dt = torch.float32 if dtype == "fp32" else torch.bfloat16
    Ag, Bg, A64, B64 = _mk(M, N, K, a_k, b_k, gpu, dt)
    bias = torch.randn(N, device=gpu)
    ref = torch.relu(A64 @ B64 + bias.double())
    C0 = torch.randn(M, N, device=gpu)
    tol = TOL if dtype == "fp32" else 1e-3
    prev = Kk.C().gemm_f32_get_split()
    Kk.C().gemm_f32_set_split(3)
    try:
        ran = set()
        for cfg in T.candidates(dtype, M, N, K):
            C = C0.clone()
            Kk.gemm(Ag, K if a_k else M, a_k, Bg, K if b_k else N, b_k, C, N, M, N, K, bias=bias, act=11, beta=True,
                    ksplit=cfg)
            form, ks = T.decode(cfg)
            err = rel_err(C, ref + C0.double())
            assert err < tol, (form, ks, err)
            if dtype == "fp32":
                ran.add(Kk.C().gemm_f32_last_form())
        if dtype == "fp32":
            assert {1, 2, 3} <= ran
    finally:
        Kk.C().gemm_f32_set_split(prev)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_candidates_with_fused_epilogues(gpu, dtype):
    from flexmi.ops import _kernels as Kk
    from flexmi.ops import gemm_tune as T
    torch.manual_seed(3)
    dt = torch.float32 if dtype == "fp32" else torch.bfloat16
    tol = TOL if dtype == "fp32" else 2e-2
    M, K, N = 2048, 512, 1024          # dX: dpre [M, N] . W [N, K] with act-bwd + column sums
    dpre = torch.randn(M, N, device=gpu).to(dt)
    W = (torch.randn(N, K, device=gpu) * 0.05).to(dt)
    yb = torch.randn(M, K, device=gpu).relu().to(dt)
    ref = (dpre.double() @ W.double()) * (yb.double() > 0)
    for cfg in T.candidates(dtype, M, K, N, fused=True):
        dx = torch.empty(M, K, device=gpu, dtype=dt)
        colsum = torch.zeros(K, device=gpu)
        Kk.gemm(dpre, N, True, W, K, False, dx, K, M, K, N, act_y=yb, bwd_act=11, colsum=colsum, ksplit=cfg)
        assert rel_err(dx, ref) < tol, T.decode(cfg)
        assert rel_err(colsum, ref.sum(0)) < (TOL if dtype == "fp32" else 1e-3), T.decode(cfg)
    # dW with the bias gradient as row sums, and with the SGD update fused
    B = 8192
    dp = torch.randn(B, 256, device=gpu).to(dt)
    x = torch.randn(B, 512, device=gpu).to(dt)
    gref = dp.double().t() @ x.double()
    for cfg in T.candidates(dtype, 256, 512, B):
        dw = torch.zeros(256, 512, device=gpu)
        db = torch.zeros(256, device=gpu)
        Kk.gemm(dp, 256, False, x, 512, False, dw, 512, 256, 512, B, beta=True, rowsum_a=db, ksplit=cfg)
        assert rel_err(dw, gref) < (TOL if dtype == "fp32" else 1e-3), T.decode(cfg)
        assert rel_err(db, dp.double().sum(0)) < (TOL if dtype == "fp32" else 1e-3), T.decode(cfg)
        w = torch.randn(256, 512, device=gpu)
        wref = w.double() - 0.01 * gref
        ks = Kk.C().gemm_dw_sgd(dp, x, w, None, None, torch.tensor([0.01], device=gpu), 0.0, 0.0, False, None,
                                Kk.workspace(gpu, Kk.GEMM_WS_BYTES), cfg)
        assert ks >= 1
        assert rel_err(w, wref) < (TOL if dtype == "fp32" else 1e-3), T.decode(cfg)
