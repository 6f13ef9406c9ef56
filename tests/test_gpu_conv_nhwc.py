"""NHWC-staged bf16 convolution (csrc/kernels/conv_nhwc.hip via flexmi/ops/_kernels.py
_nhwc_forward / _nhwc_backward) against a float64 torch oracle: forward (+bias +ReLU), data
gradient (overwrite / accumulate; strided layers through the stride-dilated staged G), weight
gradient (split-K float atomics + fold into [K,C,R,S]) and bias gradient, with the forward / data
gradient operands staged by LDS-DMA and by registers.  Geometries: ResNet /
Inception / AlexNet widths, channel counts off the 8-channel staging grain (C, K = 20, 36),
tile tails, 1x7 / 7x1, strides 2 and 3, negative (superset-box) pads, and the saved-forward vs
restaged backward."""
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
    # N, C, H, W, K, R, S, stride, pads (t, b, l, r)
    (2, 64, 14, 14, 64, 3, 3, 1, (1, 1, 1, 1)),       # ResNet 3x3
    (2, 64, 14, 14, 256, 1, 1, 1, (0, 0, 0, 0)),      # ResNet 1x1 expand
    (3, 256, 7, 7, 64, 1, 1, 1, (0, 0, 0, 0)),        # 1x1 reduce, 49-pixel images (odd epilogue)
    (2, 128, 15, 15, 128, 3, 3, 2, (1, 1, 1, 1)),     # strided 3x3 (dilated-G data gradient)
    (2, 64, 14, 14, 32, 1, 1, 2, (0, 0, 0, 0)),       # 1x1/2 shortcut
    (2, 20, 11, 9, 36, 3, 3, 1, (1, 1, 1, 1)),        # C, K off the 8-channel grain
    (2, 24, 9, 9, 40, 1, 7, 1, (0, 0, 3, 3)),         # Inception 1x7
    (2, 24, 9, 9, 40, 7, 1, 1, (3, 3, 0, 0)),         # Inception 7x1
    (2, 48, 17, 17, 64, 3, 3, 2, (0, 0, 0, 0)),       # Inception 3x3/2 valid
    (2, 16, 15, 15, 24, 5, 5, 3, (2, 2, 2, 2)),       # stride 3
    (2, 64, 15, 15, 192, 5, 5, 1, (2, 2, 2, 2)),      # AlexNet conv2 shape
    (2, 32, 14, 12, 48, 3, 3, 1, (-1, 1, -1, 1)),     # negative top/left pads (superset input box)
    (1, 16, 12, 13, 16, 3, 3, 1, (0, -1, 1, 0)),      # asymmetric halo-shard pads
    (1, 136, 6, 5, 136, 3, 3, 1, (1, 1, 1, 1)),       # M, N tails off the 128 / 64 tiles
]


@pytest.fixture(params=[1, 0], ids=["dma", "regstage"], autouse=True)
def staging(request):
    """Every case with the LDS-DMA operand staging (default for fwd / dgrad) and with register
    staging (fm_gemm_set_dma(0))."""
    from flexmi.ops import _kernels as Kk
    prev = Kk.C().gemm_dma_enabled()
    Kk.C().gemm_set_dma(request.param)
    yield request.param
    Kk.C().gemm_set_dma(prev)


def _oracle(x, w, b, st, pads):
    t, bt, l, r = pads
    xd = x.double().cpu().requires_grad_(True)
    xp = F.pad(xd, (max(l, 0), max(r, 0), max(t, 0), max(bt, 0)))
    xp = xp[:, :, max(-t, 0): xp.shape[2] - max(-bt, 0), max(-l, 0): xp.shape[3] - max(-r, 0)]
    wd = w.double().cpu().requires_grad_(True)
    y = F.conv2d(xp, wd, None if b is None else b.double().cpu(), st)
    return xd, wd, y


def _err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("case", CASES, ids=[f"n{i}" for i in range(len(CASES))])
@pytest.mark.parametrize("act,bias,save", [(11, True, True), (10, False, False)])
def test_conv_nhwc(gpu, case, act, bias, save):
    from flexmi.ops import _kernels as Kk
    assert Kk.NHWC_CONV
    N, C, H, W, K, R, S, s, pads = case
    torch.manual_seed(N * C + K * R + s)
    x = torch.randn(N, C, H, W, device=gpu).bfloat16()
    w = (torch.randn(K, C, R, S, device=gpu) / (C * R * S) ** 0.5).bfloat16()
    assert Kk._nhwc_ok(x, w, 1)
    b = torch.randn(K, device=gpu) if bias else None
    _, _, yr = _oracle(x, w, b, s, pads)
    if act == 11:
        yr = torch.relu(yr)
    y = torch.empty(yr.shape, device=gpu, dtype=torch.bfloat16)
    saved = {} if save else None
    Kk.conv2d_forward(x, w, b, y, (s, s), pads, act, 1, saved)
    assert _err(y, yr.detach()) < 1.5e-2, "forward"
    dy = torch.randn(yr.shape, device=gpu).bfloat16()
    g = dy.double().cpu() * ((y.double().cpu() > 0) if act == 11 else 1.0)
    gx, gw = _grads(x, w, s, pads, g)
    dx0 = torch.randn(N, C, H, W, device=gpu).bfloat16()
    for acc in (False, True):
        dx = dx0.clone()
        dw = torch.full((K, C, R, S), 0.5, device=gpu)
        db = torch.full((K,), 0.25, device=gpu) if bias else None
        Kk.conv2d_backward(x, w, y, dy, dx, dw, db, (s, s), pads, act, 1, acc, saved)
        assert _err(dw - 0.5, gw) < 1.5e-2, "wgrad"
        if bias:
            assert _err(db - 0.25, g.sum((0, 2, 3))) < 1.5e-2, "bias grad"
        assert _err(dx, gx + (dx0.double().cpu() if acc else 0)) < 1.5e-2, "dgrad"


def _grads(x, w, s, pads, g):
    xd, wd, y = _oracle(x, w, None, s, pads)
    return torch.autograd.grad(y, [xd, wd], g)


def test_conv_nhwc_weight_grad_only(gpu):
    """First layer of a network (no dX): G is staged unpadded and the weight gradient reads it with
    unit pixel strides, also for a strided layer."""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(7)
    N, C, H, W, K = 2, 32, 16, 16, 48
    x = torch.randn(N, C, H, W, device=gpu).bfloat16()
    w = (torch.randn(K, C, 3, 3, device=gpu) * 0.1).bfloat16()
    for s in (1, 2):
        _, _, yr = _oracle(x, w, None, s, (1, 1, 1, 1))
        y = torch.empty(yr.shape, device=gpu, dtype=torch.bfloat16)
        Kk.conv2d_forward(x, w, None, y, (s, s), (1, 1, 1, 1), 10, 1, {})
        dy = torch.randn(yr.shape, device=gpu).bfloat16()
        _, gw = _grads(x, w, s, (1, 1, 1, 1), dy.double().cpu())
        dw = torch.zeros(K, C, 3, 3, device=gpu)
        Kk.conv2d_backward(x, w, y, dy, None, dw, None, (s, s), (1, 1, 1, 1), 10, 1, False, None)
        assert _err(dw, gw) < 1.5e-2


def test_conv_nhwc_matches_nchw_path(gpu, monkeypatch):
    """The NHWC path and the NCHW kernels agree on a ResNet-width layer (both bf16 MFMA, fp32
    accumulate: only the summation order differs)."""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(11)
    x = torch.randn(4, 64, 28, 28, device=gpu).bfloat16()
    w = (torch.randn(128, 64, 3, 3, device=gpu) * 0.05).bfloat16()
    b = torch.randn(128, device=gpu)
    outs = []
    for on in (True, False):
        monkeypatch.setattr(Kk, "NHWC_CONV", on)
        y = torch.empty(4, 128, 28, 28, device=gpu, dtype=torch.bfloat16)
        Kk.conv2d_forward(x, w, b, y, (1, 1), (1, 1, 1, 1), 11, 1, {})
        outs.append(y.float())
    assert _err(outs[0], outs[1]) < 1e-2


@pytest.mark.parametrize("phase", [True, False])
def test_strided_dgrad_phase_and_dilated_agree(gpu, monkeypatch, phase):
    """Strided data gradient: the per-stride-phase GEMMs (default) and the single GEMM over the
    stride-dilated G both match the float64 oracle, incl. a phase without taps (1x1 / 2)."""
    from flexmi.ops import _kernels as Kk
    monkeypatch.setattr(Kk, "STRIDE_PHASE_DGRAD", phase)
    for (N, C, H, W, K, R, S, s, pads) in [(2, 32, 15, 14, 40, 3, 3, 2, (1, 1, 1, 1)), (2, 24, 13, 13, 16, 1, 1, 2, (0, 0, 0, 0)),
                                           (1, 16, 16, 17, 24, 5, 5, 3, (2, 2, 1, 1))]:
        torch.manual_seed(C + K)
        x = torch.randn(N, C, H, W, device=gpu).bfloat16()
        w = (torch.randn(K, C, R, S, device=gpu) / (C * R * S) ** 0.5).bfloat16()
        _, _, yr = _oracle(x, w, None, s, pads)
        y = torch.empty(yr.shape, device=gpu, dtype=torch.bfloat16)
        Kk.conv2d_forward(x, w, None, y, (s, s), pads, 10, 1, {})
        dy = torch.randn(yr.shape, device=gpu).bfloat16()
        gx, gw = _grads(x, w, s, pads, dy.double().cpu())
        for acc in (False, True):
            dx0 = torch.randn(N, C, H, W, device=gpu).bfloat16()
            dx = dx0.clone()
            dw = torch.zeros(K, C, R, S, device=gpu)
            Kk.conv2d_backward(x, w, y, dy, dx, dw, None, (s, s), pads, 10, 1, acc, None)
            assert _err(dx, gx + (dx0.double().cpu() if acc else 0)) < 1.5e-2, (phase, acc, R, s)
            assert _err(dw, gw) < 1.5e-2
