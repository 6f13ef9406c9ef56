"""Dedicated stem convolution kernels (csrc/kernels/conv_stem.hip): the input tile is staged into LDS in
space-to-depth NHWC order by the convolution itself, forward on ds_read_b128 pixel runs, weight gradient
on ds_read_b64_tr_b16 transposed reads.  Checked against float64 torch oracles of the same convolution:
forward (+bias, +ReLU / no activation), weight and bias gradients ACCUMULATED onto existing values,
over AlexNet-class (11x11 / 4) and ResNet-class (7x7 / 2) geometries with partial row tiles, two column
tiles, odd output widths (scalar epilogue / gradient loads) and 1-3 input channels."""
import pytest
import torch

from tests.test_gpu_conv_nhwc import _err, _grads, _oracle

pytestmark = pytest.mark.gpu

CASES = [
    # N, C, H, W, R, S, stride, pad
    (2, 3, 229, 229, 11, 11, 4, 2),    # AlexNet stem: P = Q = 56
    (3, 3, 67, 75, 11, 11, 4, 2),      # 16 x 18 outputs: a partial row tile, Q % 4 != 0
    (2, 1, 40, 40, 11, 11, 4, 2),      # one channel
    (1, 3, 229, 229, 7, 7, 2, 3),      # ResNet stem: 115 x 115 (two column tiles, odd width)
    (2, 2, 33, 48, 7, 7, 2, 3),        # two channels, 17 x 24
]


def _case(gpu, case, seed=0):
    N, C, H, W, R, S, s, pad = case
    torch.manual_seed(seed + N * C + R * s + H)
    x = torch.randn(N, C, H, W, device=gpu).bfloat16()
    w = (torch.randn(64, C, R, S, device=gpu) / (C * R * S) ** 0.5).bfloat16()
    b = torch.randn(64, device=gpu)
    return x, w, b


@pytest.mark.parametrize("case", CASES, ids=[f"s{i}" for i in range(len(CASES))])
@pytest.mark.parametrize("act,bias", [(11, True), (10, False)])
def test_stem_forward_and_weight_grad_vs_float64(gpu, case, act, bias):
    from flexmi.ops import _kernels as Kk
    N, C, H, W, R, S, s, pad = case
    x, w, b = _case(gpu, case)
    b = b if bias else None
    pads = (pad, pad, pad, pad)
    _, _, yr = _oracle(x, w, b, s, pads)
    if act == 11:
        yr = torch.relu(yr)
    yr = yr.detach()
    y = torch.empty(yr.shape, device=gpu, dtype=torch.bfloat16)
    assert Kk.conv_forms(x, w, y, (s, s), 1)[0] == "stem"
    assert "stem" in Kk.conv_forms(x, w, y, (s, s), 1, "bwd", need_dx=False)
    assert "stem" not in Kk.conv_forms(x, w, y, (s, s), 1, "bwd", need_dx=True)
    Kk.conv2d_forward(x, w, b, y, (s, s), pads, act, 1, {}, form="stem")
    assert _err(y, yr) < 1.2e-2, "forward"
    dy = torch.randn(yr.shape, device=gpu).bfloat16()
    g = dy.double().cpu() * ((y.double().cpu() > 0) if act == 11 else 1.0)
    _, gw = _grads(x, w, s, pads, g)
    dw = torch.full((64, C, R, S), 0.5, device=gpu)
    db = torch.full((64,), 0.25, device=gpu)
    Kk.conv2d_backward(x, w, y, dy, None, dw, db, (s, s), pads, act, 1, False, {}, form="stem")
    assert _err(dw - 0.5, gw) < 1.2e-2, "wgrad"
    assert _err(db - 0.25, g.sum((0, 2, 3))) < 1e-4, "bias grad"


def test_stem_matches_the_generic_forms(gpu):
    """The stem form against the space-to-depth and implicit-GEMM forms on the AlexNet stem."""
    from flexmi.ops import _kernels as Kk
    case = CASES[0]
    N, C, H, W, R, S, s, pad = case
    x, w, b = _case(gpu, case, seed=5)
    pads = (pad, pad, pad, pad)
    P = (H + 2 * pad - R) // s + 1
    ys = {}
    for form in ("stem", "s2d", "igemm"):
        ys[form] = torch.empty(N, 64, P, P, device=gpu, dtype=torch.bfloat16)
        Kk.conv2d_forward(x, w, b, ys[form], (s, s), pads, 11, 1, {}, form=form)
    assert _err(ys["stem"], ys["igemm"]) < 1e-2 and _err(ys["s2d"], ys["igemm"]) < 1e-2
    dy = torch.randn(ys["stem"].shape, device=gpu).bfloat16()
    dws = {}
    for form in ("stem", "s2d"):
        dws[form] = torch.zeros(64, C, R, S, device=gpu)
        db = torch.zeros(64, device=gpu)
        Kk.conv2d_backward(x, w, ys["igemm"], dy, None, dws[form], db, (s, s), pads, 11, 1, False, {}, form=form)
    assert _err(dws["stem"], dws["s2d"]) < 1e-2


def test_stem_needs_input_gradient_falls_back(gpu):
    """A stem-shaped layer whose input needs a gradient is not given to the stem kernels: forced, the
    backward falls back to the implicit-GEMM form and still produces dX."""
    from flexmi.ops import _kernels as Kk
    case = (2, 3, 40, 40, 11, 11, 4, 2)
    N, C, H, W, R, S, s, pad = case
    x, w, b = _case(gpu, case)
    pads = (pad,) * 4
    _, _, yr = _oracle(x, w, b, s, pads)
    y = torch.relu(yr).detach().to(gpu).bfloat16()
    dy = torch.randn(y.shape, device=gpu).bfloat16()
    g = dy.double().cpu() * (y.double().cpu() > 0)
    gx, gw = _grads(x, w, s, pads, g)
    dx = torch.zeros(N, C, H, W, device=gpu, dtype=torch.bfloat16)
    dw = torch.zeros(64, C, R, S, device=gpu)
    Kk.conv2d_backward(x, w, y, dy, dx, dw, None, (s, s), pads, 11, 1, False, {}, form="stem")
    assert _err(dx, gx) < 1.5e-2 and _err(dw, gw) < 1.5e-2


def test_model_stem_runs_the_stem_kernels(gpu):
    """AlexNet's first layer picks (or is measured onto) a form; with tuning off the heuristic order
    starts with the stem kernels."""
    from flexmi.ops import _kernels as Kk
    x = torch.zeros(2, 3, 229, 229, device=gpu, dtype=torch.bfloat16)
    w = torch.zeros(64, 3, 11, 11, device=gpu, dtype=torch.bfloat16)
    y = torch.empty(2, 64, 56, 56, device=gpu, dtype=torch.bfloat16)
    assert Kk.conv_forms(x, w, y, (4, 4), 1) == ["stem", "s2d", "s2d_nhwc", "igemm"]
