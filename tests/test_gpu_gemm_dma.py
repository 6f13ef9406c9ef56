"""LDS-DMA operand staging of the bf16 GEMM (gemm.hip) and the native fp32 GEMM (gemm_f32.hip):
full-tile shapes take the DMA form (lanes load the chunks the swizzled LDS image puts at their
slots; the dW GEMMs' fused bias-gradient row sums read back from the image), others the
register-staged form.  Every orientation, split-K and the fused epilogues give
bit-identical results in both forms (same MFMA order) and match a float64 torch oracle."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(512, 256, 384), (1024, 128, 1024), (256, 512, 4096), (384, 192, 320)]   # last: off the tiles


def _mat(M, K, k_contig, dt, dev, scale=1.0):
    """A logical [M][K] operand stored K-contiguous ([M][K]) or MN-contiguous ([K][M])."""
    t = (torch.randn(M, K, device=dev) * scale).to(dt)
    return (t.contiguous(), K) if k_contig else (t.t().contiguous(), M)


def _run(Kk, dt, M, N, K, ak, bk, bias, act, dma):
    Kk.C().gemm_set_dma(dma)
    torch.manual_seed(M + N + K + 2 * ak + bk)
    dev = torch.device("cuda")
    A, lda = _mat(M, K, ak, dt, dev)
    B, ldb = _mat(N, K, bk, dt, dev, 0.05)
    C = torch.zeros(M, N, device=dev, dtype=torch.float32 if dt == torch.float32 else torch.bfloat16)
    b = torch.randn(N, device=dev) if bias else None
    rs = torch.zeros(M, device=dev) if not ak else None      # MN-contiguous A: fused row sums (bias grads)
    Kk.gemm(A, lda, ak, B, ldb, bk, C, N, M, N, K, bias=b, act=act, rowsum_a=rs)
    torch.cuda.synchronize()
    return A, B, b, C, rs


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32], ids=["bf16", "fp32"])
@pytest.mark.parametrize("ak,bk", [(1, 1), (1, 0), (0, 0)], ids=["kk", "km", "mm"])
@pytest.mark.parametrize("shape", SHAPES, ids=[f"{m}x{n}x{k}" for m, n, k in SHAPES])
def test_gemm_dma_matches_register_staging(dt, ak, bk, shape):
    from flexmi.ops import _kernels as Kk
    M, N, K = shape
    prev_dma = Kk.C().gemm_dma_enabled()
    prev_split = Kk.C().gemm_f32_get_split() if dt == torch.float32 else None
    if dt == torch.float32:
        Kk.C().gemm_f32_set_split(0)     # the native fp32 kernel (the split kernel has no DMA form)
    try:
        A, B, b, c1, rs1 = _run(Kk, dt, M, N, K, ak, bk, True, 11, 1)
        _, _, _, c0, rs0 = _run(Kk, dt, M, N, K, ak, bk, True, 11, 0)
    finally:
        Kk.C().gemm_set_dma(prev_dma)
        if prev_split is not None:
            Kk.C().gemm_f32_set_split(prev_split)
    assert torch.equal(c1, c0)
    a64 = (A.double() if ak else A.double().t())
    b64 = (B.double() if bk else B.double().t())
    ref = torch.relu(a64 @ b64.t() + b.double())
    err = ((c1.double() - ref).norm() / ref.norm()).item()
    assert err < (1e-5 if dt == torch.float32 else 1e-2), err
    if rs1 is not None:                     # row sums: same fp32 adds in both staging forms
        want = a64.sum(1)
        assert torch.allclose(rs1, rs0, rtol=1e-5, atol=1e-4)
        assert ((rs1.double() - want).norm() / want.norm()).item() < 1e-4
