"""Per-layer measured convolution forms (flexmi/ops/_kernels.py conv_forms / _conv_choose: the
cudnnFind*AlgorithmEx analogue of src/ops/conv_2d.cu:216-243, :872-930).  Every form applicable to a
layer -- NHWC-staged, NCHW implicit GEMM (with the stride-phase paths), space-to-depth stem on the NCHW
and on the NHWC kernels -- is forced on its own and checked against a float64 torch oracle (forward
+bias +ReLU, data gradient overwrite / accumulate, weight and bias gradients); then the tuner picks a
form per direction on first use, records it, and leaves dW / db / an accumulated dX touched exactly
once (its candidates run on scratch gradients)."""
import pytest
import torch

from tests.test_gpu_conv_nhwc import _err, _grads, _oracle

pytestmark = pytest.mark.gpu

CASES = [
    # N, C, H, W, K, R, S, stride, pads (t, b, l, r)
    (2, 3, 67, 67, 16, 11, 11, 4, (2, 2, 2, 2)),      # AlexNet stem (space-to-depth forms)
    (2, 3, 32, 32, 16, 7, 7, 2, (3, 3, 3, 3)),        # ResNet stem
    (2, 64, 15, 15, 96, 5, 5, 1, (2, 2, 2, 2)),       # AlexNet conv2-like
    (2, 32, 14, 14, 48, 3, 3, 1, (1, 1, 1, 1)),
    (2, 64, 14, 14, 32, 1, 1, 2, (0, 0, 0, 0)),       # strided 1x1 shortcut (phase forward)
    (2, 48, 17, 17, 64, 3, 3, 2, (1, 1, 1, 1)),       # strided 3x3 (phase backward)
    (2, 32, 15, 15, 48, 1, 1, 2, (0, 0, 0, 0)),       # strided 1x1, odd extent
]


def _case(gpu, case):
    N, C, H, W, K, R, S, s, pads = case
    torch.manual_seed(N * C + K * R + s)
    x = torch.randn(N, C, H, W, device=gpu).bfloat16()
    w = (torch.randn(K, C, R, S, device=gpu) / (C * R * S) ** 0.5).bfloat16()
    b = torch.randn(K, device=gpu)
    _, _, yr = _oracle(x, w, b, s, pads)
    return x, w, b, torch.relu(yr).detach()


@pytest.mark.parametrize("case", CASES, ids=[f"c{i}" for i in range(len(CASES))])
def test_every_conv_form_vs_float64(gpu, case):
    from flexmi.ops import _kernels as Kk
    N, C, H, W, K, R, S, s, pads = case
    x, w, b, yr = _case(gpu, case)
    y0 = torch.empty(yr.shape, device=gpu, dtype=torch.bfloat16)
    forms = Kk.conv_forms(x, w, y0, (s, s), 1)
    assert "igemm" in forms
    if C == 3:
        assert "s2d" in forms and (("s2d_nhwc" in forms) == (C * s * s >= 16))
    for form in forms:
        saved = {}
        y = torch.empty(yr.shape, device=gpu, dtype=torch.bfloat16)
        Kk.conv2d_forward(x, w, b, y, (s, s), pads, 11, 1, saved, form=form)
        assert _err(y, yr) < 1.5e-2, (form, "forward")
        dy = torch.randn(yr.shape, device=gpu).bfloat16()
        g = dy.double().cpu() * (y.double().cpu() > 0)
        gx, gw = _grads(x, w, s, pads, g)
        dx0 = torch.randn(N, C, H, W, device=gpu).bfloat16()
        for acc in (False, True):
            dx = dx0.clone()
            dw = torch.full((K, C, R, S), 0.5, device=gpu)
            db = torch.full((K,), 0.25, device=gpu)
            Kk.conv2d_backward(x, w, y, dy, dx, dw, db, (s, s), pads, 11, 1, acc, saved, form=form)
            assert _err(dw - 0.5, gw) < 1.5e-2, (form, "wgrad")
            assert _err(db - 0.25, g.sum((0, 2, 3))) < 1.5e-2, (form, "bias grad")
            assert _err(dx, gx + (dx0.double().cpu() if acc else 0)) < 1.5e-2, (form, "dgrad", acc)


@pytest.mark.parametrize("case", [CASES[0], CASES[2], CASES[5]], ids=["stem", "c5x5", "s2"])
def test_tuner_picks_and_records_a_form(gpu, case, monkeypatch):
    from flexmi.ops import _kernels as Kk
    monkeypatch.setattr(Kk, "CONV_TUNE", True)
    N, C, H, W, K, R, S, s, pads = case
    x, w, b, yr = _case(gpu, case)
    saved = {}
    y = torch.empty(yr.shape, device=gpu, dtype=torch.bfloat16)
    n0 = len(Kk.CONV_TUNE_LOG)
    Kk.conv2d_forward(x, w, b, y, (s, s), pads, 11, 1, saved)
    forms = Kk.conv_forms(x, w, y, (s, s), 1)
    assert saved["conv_form_fwd"] in forms
    assert _err(y, yr) < 1.5e-2
    dy = torch.randn(yr.shape, device=gpu).bfloat16()
    g = dy.double().cpu() * (y.double().cpu() > 0)
    gx, gw = _grads(x, w, s, pads, g)
    dx0 = torch.randn(N, C, H, W, device=gpu).bfloat16()
    dx = dx0.clone()
    dw = torch.full((K, C, R, S), 0.5, device=gpu)
    db = torch.full((K,), 0.25, device=gpu)
    Kk.conv2d_backward(x, w, y, dy, dx, dw, db, (s, s), pads, 11, 1, True, saved)
    assert saved["conv_form_bwd"] in forms
    # the candidates ran on scratch: the real gradients were accumulated exactly once
    assert _err(dw - 0.5, gw) < 1.5e-2 and _err(db - 0.25, g.sum((0, 2, 3))) < 1.5e-2
    assert _err(dx, gx + dx0.double().cpu()) < 1.5e-2
    log = Kk.CONV_TUNE_LOG[n0:]
    if len(forms) > 1:
        assert [e[0] for e in log] == ["fwd", "bwd"]
        for _, _, times, pick in log:
            assert set(times) == set(forms) and times[pick] == min(times.values())
    # later calls reuse the recorded forms without timing again
    Kk.conv2d_forward(x, w, b, y, (s, s), pads, 11, 1, saved)
    assert len(Kk.CONV_TUNE_LOG) == n0 + len(log)



def test_tuner_skips_a_form_that_does_not_apply(gpu, monkeypatch):
    """A backward candidate that falls through (returns False: the form does not apply to the layout)
    is not timed -- an early return once measured 1.5 us and was picked, and the step then ran the
    slow fallback."""
    from flexmi.ops import _kernels as Kk
    monkeypatch.setattr(Kk, "CONV_TUNE", True)
    x = torch.zeros(64, 64, device=gpu)

    def run(f):
        if f == "nope":
            return False
        x.add_(1.0)
        return True
    saved = {}
    assert Kk._conv_choose(saved, "bwd", ["nope", "works"], run, ("k",)) == "works"
    assert saved["conv_form_bwd"] == "works"
