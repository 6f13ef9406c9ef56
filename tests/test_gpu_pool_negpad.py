"""Pooling (row-segment backward) and convolution with NEGATIVE top/left pads against float64
torch oracles.  A spatially split conv / pool may read its producer's buffer in place when the
buffer box is a superset of the halo box (executor.superset_input_ok): the op then runs with
negative pads, i.e. its first window starts inside the buffer.  Also widths that the
backward's 8-column segments do not divide, accumulation into dx, max and avg."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref_pool(x, k, s, pt, pl, P, Q, is_max):
    """Pool of x with (possibly negative) top/left pads, P x Q outputs, bottom/right implied."""
    xd = x.double()
    H, W = x.shape[2], x.shape[3]
    hb = (P - 1) * s + k - pt - H       # bottom / right pads implied by the output extent
    wr = (Q - 1) * s + k - pl - W
    v = float("-inf") if is_max else 0.0
    xp = F.pad(xd, (max(pl, 0), max(wr, 0), max(pt, 0), max(hb, 0)), value=v)
    xp = xp[:, :, max(-pt, 0):, max(-pl, 0):]
    if is_max:
        return F.max_pool2d(xp, k, s)[:, :, :P, :Q]
    ones = F.pad(torch.ones_like(xd[:1, :1]), (max(pl, 0), max(wr, 0), max(pt, 0), max(hb, 0)))
    ones = ones[:, :, max(-pt, 0):, max(-pl, 0):]
    return (F.avg_pool2d(xp, k, s, divisor_override=1) / F.avg_pool2d(ones, k, s, divisor_override=1))[:, :, :P, :Q]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("is_max", [True, False])
@pytest.mark.parametrize("H,W,k,s,pt,pl", [(13, 27, 3, 2, 1, 1), (16, 16, 3, 2, -1, -1), (12, 55, 3, 2, 0, -1),
                                            (9, 33, 2, 2, -1, 0), (11, 8, 3, 1, 1, 1), (55, 55, 3, 2, 0, 0),
                                            (27, 27, 3, 2, 0, 0)])
def test_pool_rows_and_negative_pads(dt, is_max, H, W, k, s, pt, pl):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(H * W + k)
    dev = torch.device("cuda")
    x = torch.randn(2, 3, H, W, device=dev).to(dt)
    P = (H + pt - k) // s + 1 if pt < 0 else (H + 2 * pt - k) // s + 1
    Q = (W + pl - k) // s + 1 if pl < 0 else (W + 2 * pl - k) // s + 1
    xr = x.double().requires_grad_(True)
    ref = _ref_pool(xr, k, s, pt, pl, P, Q, is_max)
    y = torch.empty(ref.shape, device=dev, dtype=dt)
    saved = {}
    kind = 30 if is_max else 31
    Kk.pool2d_forward(x, y, (k, k), (s, s), (pt, pt, pl, pl), kind, 10, saved)
    tol = 1e-6 if dt == torch.float32 else 1e-2
    torch.testing.assert_close(y.double(), ref, rtol=tol, atol=tol)
    dy = torch.randn(ref.shape, device=dev).to(dt)
    gx, = torch.autograd.grad(ref, [xr], dy.double())
    for acc in (False, True):
        base = torch.randn_like(x) if acc else torch.empty_like(x)
        dx = base.clone()
        Kk.pool2d_backward(x, y, dy, dx, (k, k), (s, s), (pt, pt, pl, pl), kind, 10, acc, saved)
        exp = gx + (base.double() if acc else 0)
        torch.testing.assert_close(dx.double(), exp, rtol=tol * 2, atol=tol * 2)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("pt,pl", [(-1, -1), (0, -1), (-1, 1)])
def test_conv_negative_pads(dt, pt, pl):
    from flexmi.ops import _kernels as Kk
    torch.manual_seed(3)
    dev = torch.device("cuda")
    N, C, H, W, K, R = 2, 8, 14, 12, 16, 3
    x = torch.randn(N, C, H, W, device=dev).to(dt)
    w = (torch.randn(K, C, R, R, device=dev) * 0.2).to(dt)
    b = torch.randn(K, device=dev)
    P, Q = H + 2 * pt - R + 1 if pt >= 0 else H + pt - R + 1, W + 2 * pl - R + 1 if pl >= 0 else W + pl - R + 1
    xr = x.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    xp = F.pad(xr, (max(pl, 0), max(pl, 0), max(pt, 0), max(pt, 0)))[:, :, max(-pt, 0):, max(-pl, 0):]
    ref = F.conv2d(xp, wr, b.double())[:, :, :P, :Q]
    y = torch.empty(ref.shape, device=dev, dtype=dt)
    Kk.conv2d_forward(x, w, b, y, (1, 1), (pt, pt, pl, pl), 10, 1, {})
    tol = 1e-5 if dt == torch.float32 else 2e-2
    torch.testing.assert_close(y.double(), ref, rtol=tol, atol=tol * 4)
    dy = torch.randn(ref.shape, device=dev).to(dt)
    gx, gw = torch.autograd.grad(ref, [xr, wr], dy.double())
    dx = torch.empty_like(x)
    dw = torch.zeros(w.shape, device=dev, dtype=torch.float32)
    db = torch.zeros(K, device=dev)
    Kk.conv2d_backward(x, w, y, dy, dx, dw, db, (1, 1), (pt, pt, pl, pl), 10, 1, False, {})
    torch.testing.assert_close(dx.double(), gx, rtol=tol * 2, atol=tol * 8)
    torch.testing.assert_close(dw.double(), gw, rtol=tol * 2, atol=tol * 20)
    torch.testing.assert_close(db.double(), dy.double().sum((0, 2, 3)), rtol=tol, atol=tol * 20)
