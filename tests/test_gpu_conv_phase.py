"""Strided convolution backward through the stride-phase decomposition (flexmi/ops/_kernels.py
_conv_backward_phases: s*s stride-1 pixel-vector dgrad / wgrad problems + strided copies)
against a float64 torch oracle, on the strided shapes of ResNet (3x3/2 pad 1, 1x1/2), Inception
(3x3/2 pad 0) and odd extents, with and without accumulation into dx."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _no_conv_tune(monkeypatch):
    """These tests target specific convolution paths: the heuristic form, no per-layer timing."""
    from flexmi.ops import _kernels as Kk
    monkeypatch.setattr(Kk, "CONV_TUNE", False)


@pytest.mark.parametrize("N,C,H,W,K,R,S,s,pt,pl", [
    (2, 16, 14, 14, 32, 3, 3, 2, 1, 1),     # ResNet downsampling 3x3/2
    (2, 32, 14, 14, 16, 1, 1, 2, 0, 0),     # ResNet 1x1/2 shortcut
    (2, 8, 17, 17, 16, 3, 3, 2, 0, 0),      # Inception 3x3/2 valid
    (1, 8, 13, 11, 8, 3, 3, 2, 1, 1),       # odd extents
    (2, 8, 15, 15, 16, 5, 5, 3, 2, 2),      # stride 3
])
@pytest.mark.parametrize("acc", [False, True])
def test_strided_conv_backward_phases(N, C, H, W, K, R, S, s, pt, pl, acc):
    from flexmi.ops import _kernels as Kk
    assert Kk.PHASE_CONV
    torch.manual_seed(N * H + K + R)
    dev = torch.device("cuda")
    x = torch.randn(N, C, H, W, device=dev).bfloat16()
    w = (torch.randn(K, C, R, S, device=dev) * 0.2).bfloat16()
    P = (H + 2 * pt - R) // s + 1
    Q = (W + 2 * pl - S) // s + 1
    xr = x.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    ref = F.conv2d(xr, wr, None, stride=s, padding=(pt, pl))
    assert ref.shape[2:] == (P, Q)
    dy = torch.randn(ref.shape, device=dev).bfloat16()
    gx, gw = torch.autograd.grad(ref, [xr, wr], dy.double())
    y = torch.empty(ref.shape, device=dev, dtype=torch.bfloat16)
    base = torch.randn_like(x) if acc else torch.full_like(x, float("nan"))
    dx = base.clone()
    dw = torch.zeros(w.shape, device=dev, dtype=torch.float32)
    Kk.conv2d_backward(x, w, y, dy, dx, dw, None, (s, s), (pt, pt, pl, pl), 10, 1, acc, {})
    exp = gx + (base.double() if acc else 0)
    scale = gx.abs().max().item()
    assert (dx.double() - exp).abs().max().item() < 2e-2 * scale + (0.02 if acc else 0), "dgrad"
    assert (dw.double() - gw).abs().max().item() < 1e-2 * gw.abs().max().item(), "wgrad"


@pytest.mark.parametrize("H,W,s,p", [(14, 14, 2, 0), (13, 15, 2, 0), (15, 15, 3, 1)])
def test_strided_1x1_forward_phase(H, W, s, p):
    """A strided 1x1 conv reads one input phase: gather + stride-1 pixel-vector forward."""
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(H + W)
    dev = torch.device("cuda")
    x = torch.randn(2, 16, H, W, device=dev).bfloat16()
    w = (torch.randn(24, 16, 1, 1, device=dev) * 0.2).bfloat16()
    b = torch.randn(24, device=dev)
    ref = torch.relu(F.conv2d(x.double(), w.double(), b.double(), stride=s, padding=p))
    y = torch.empty(ref.shape, device=dev, dtype=torch.bfloat16)
    Kk.conv2d_forward(x, w, b, y, (s, s), (p, p, p, p), 11, 1, {})
    assert (y.double() - ref).abs().max().item() < 2e-2 * ref.abs().max().item()
