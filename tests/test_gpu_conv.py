"""Implicit-GEMM convolution kernels (csrc/kernels/conv_igemm.hip) against a float64 PyTorch CPU
oracle: forward (+bias +ReLU), data gradient (overwrite and accumulate), weight gradient and
bias gradient, for bf16 and fp32, over the geometries the zoo uses -- AlexNet's 11x11/4 stem on
3 channels, 5x5 and 3x3 same-padding, ResNet 1x1 and strided 3x3, Inception's 1x7 / 7x1, tile tails
(odd pixel counts, channel counts off the tile) and asymmetric halo-shard pads.  Strided bf16 stems on
3 channels run through space-to-depth (one case with a saved forward buffer, one without)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _no_conv_tune(monkeypatch):
    """These tests target specific convolution paths: the heuristic form, no per-layer timing."""
    from flexmi.ops import _kernels as Kk
    monkeypatch.setattr(Kk, "CONV_TUNE", False)

CASES = [
    # N, C, H, W, K, R, S, sh, sw, pads(t,b,l,r)
    (2, 3, 67, 67, 64, 11, 11, 4, 4, (2, 2, 2, 2)),     # AlexNet stem (small image)
    (2, 64, 15, 15, 192, 5, 5, 1, 1, (2, 2, 2, 2)),
    (3, 96, 13, 13, 130, 3, 3, 1, 1, (1, 1, 1, 1)),     # K off the 128 tile
    (2, 64, 14, 14, 256, 1, 1, 1, 1, (0, 0, 0, 0)),     # 1x1
    (2, 32, 15, 15, 48, 3, 3, 2, 2, (1, 1, 1, 1)),      # strided 3x3 (dgrad parity gaps)
    (2, 24, 9, 9, 40, 1, 7, 1, 1, (0, 0, 3, 3)),        # Inception 1x7
    (2, 24, 9, 9, 40, 7, 1, 1, 1, (3, 3, 0, 0)),        # Inception 7x1
    (2, 8, 10, 7, 8, 3, 3, 2, 2, (0, 1, 1, 0)),         # asymmetric (halo-shard) pads
    (1, 5, 6, 5, 7, 2, 3, 1, 2, (1, 0, 0, 2)),          # everything odd
    (2, 3, 30, 30, 16, 7, 7, 2, 2, (3, 3, 3, 3)),       # ResNet stem 7x7/2 (bf16: space-to-depth path)
    (1, 3, 21, 19, 8, 11, 11, 4, 4, (2, 0, 1, 3)),      # strided stem with asymmetric halo pads
]


def _ref(x, w, b, st, pads, act):
    xd = F.pad(x.double().cpu(), (pads[2], pads[3], pads[0], pads[1])).requires_grad_(True)
    wd = w.double().cpu().requires_grad_(True)
    bd = b.double().cpu().requires_grad_(True) if b is not None else None
    y = F.conv2d(xd, wd, bd, st)
    return xd, wd, bd, (torch.relu(y) if act == 11 else y)


def _err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
@pytest.mark.parametrize("case", CASES, ids=[f"c{i}" for i in range(len(CASES))])
@pytest.mark.parametrize("act,bias", [(11, True), (10, False)])
def test_conv_igemm(gpu, dtype, case, act, bias):
    from flexmi.ops import _kernels as Kk
    N, C, H, W, K, R, S, sh, sw, pads = case
    dt = torch.bfloat16 if dtype == "bf16" else torch.float32
    tol = 1.5e-2 if dtype == "bf16" else 2e-5
    torch.manual_seed(hash(case) % 1000)
    x = torch.randn(N, C, H, W, device=gpu).to(dt)
    w = (torch.randn(K, C, R, S, device=gpu) / (C * R * S) ** 0.5).to(dt)
    b = torch.randn(K, device=gpu) if bias else None
    xd, wd, bd, yr = _ref(x, w, b, (sh, sw), pads, act)
    y = torch.empty(yr.shape, device=gpu, dtype=dt)
    saved = {} if CASES.index(case) % 2 else None       # saved-forward-buffer and recompute variants
    Kk.conv2d_forward(x, w, b, y, (sh, sw), pads, act, 1, saved)
    assert _err(y, yr.detach()) < tol
    dy = torch.randn(yr.shape, device=gpu).to(dt)
    # the backward consumes the ROUNDED forward output (the activation mask follows y as stored)
    g = dy.double().cpu() * ((y.double().cpu() > 0) if act == 11 else 1.0)
    yl = F.conv2d(xd, wd, None, (sh, sw))
    gx, gw = torch.autograd.grad(yl, [xd, wd], g)
    gx = gx[:, :, pads[0]: pads[0] + H, pads[2]: pads[2] + W]
    dx0 = torch.randn(N, C, H, W, device=gpu).to(dt)
    for acc in (False, True):
        dx = dx0.clone()
        dw = torch.full((K, C, R, S), 0.5, device=gpu)          # dW accumulates
        db = torch.full((K,), 0.25, device=gpu) if bias else None
        Kk.conv2d_backward(x, w, y, dy, dx, dw, db, (sh, sw), pads, act, 1, acc, saved)
        assert _err(dw - 0.5, gw) < tol
        if bias:
            assert _err(db - 0.25, g.sum((0, 2, 3))) < tol
        assert _err(dx, gx + (dx0.double().cpu() if acc else 0)) < tol


def test_conv_igemm_alexnet_width(gpu):
    """AlexNet conv2 at the bench batch slice: 64 -> 192, 5x5 on 27x27 (186 k output pixels per
    256 images; 24 images here), bf16, against the fp32 GPU GEMM reference (torch)."""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(3)
    x = torch.randn(24, 64, 27, 27, device=gpu).bfloat16()
    w = (torch.randn(192, 64, 5, 5, device=gpu) * 0.025).bfloat16()
    b = torch.randn(192, device=gpu)
    y = torch.empty(24, 192, 27, 27, device=gpu, dtype=torch.bfloat16)
    Kk.conv2d_forward(x, w, b, y, (1, 1), (2, 2, 2, 2), 11, 1)
    cols = F.unfold(x.float(), 5, padding=2)                                   # [N, CRS, PQ]
    ref = torch.relu(torch.einsum("kc,ncp->nkp", w.float().reshape(192, -1), cols) + b[None, :, None])
    assert _err(y.reshape(24, 192, -1), ref) < 1e-2
