"""GEMM configuration table (flexmi/ops/gemm_tune.py): key identity, the ksplit encoding the HIP
dispatch decodes (csrc/kernels/gemm_f32.hip gemm_f32_run: ks | form << 8), candidate enumeration
and table loading / FM_GEMM_TUNE=0.  The forced configurations themselves are checked against
float64 oracles on the GPU (tests/test_gpu_gemm_tune.py)."""
import json

from flexmi.ops import gemm_tune as T


def test_key_distinguishes_what_changes_the_configuration():
    base = T.key("fp32", 8192, 1024, 1024, True, True)
    assert base == "fp32|8192x1024x1024|kk|b1|-|c32"
    assert T.key("bf16", 8192, 1024, 1024, True, True) != base
    assert T.key("fp32", 8192, 1024, 1024, True, False) != base
    assert T.key("fp32", 8192, 1024, 1024, True, True, act_y=True, colsum=True) == "fp32|8192x1024x1024|kk|b1|yc|c32"
    assert T.key("fp32", 1024, 479, 8192, False, False, rowsum=True, sgd=True).endswith("|rs|c32")
    assert T.key("bf16", 64, 64, 64, True, True, c_fp32=False).endswith("c16")


def test_encoding_round_trips_and_fits_the_ksplit_argument():
    for form in range(7):
        for ks in T.KS_CHOICES:
            c = T.encode(form, ks)
            assert T.decode(c) == (form, ks)
            assert c & 255 == ks and c >> 8 == form


def test_candidates_respect_form_and_split_limits():
    c = T.candidates("fp32", 8192, 1024, 1024)
    forms = {T.decode(x)[0] for x in c}
    assert forms == {1, 2, 3, 4, 5, 6}
    for x in c:          # every split keeps >= 4 k-steps of 32
        assert T.decode(x)[1] * 4 <= 1024 // 32 or T.decode(x)[1] == 1
    # fused backward epilogue: the x3 split-K kernels (forms 4-6) carry it unsplit only
    fused = {T.decode(x) for x in T.candidates("fp32", 8192, 1024, 1024, fused=True)}
    assert {f for f, _ in fused} == {1, 2, 3, 4, 5, 6}
    assert all(ks == 1 for f, ks in fused if f >= 4)
    # tiny operands: no split kernel
    assert {T.decode(x)[0] for x in T.candidates("fp32", 8192, 32, 16)} == {1, 2, 3}
    assert {T.decode(x)[0] for x in T.candidates("bf16", 8192, 1024, 1024)} == {1, 2, 3}


def test_table_loading_and_switch(tmp_path, monkeypatch):
    k = T.key("fp32", 128, 256, 8192, False, False, rowsum=True)
    path = tmp_path / "t.json"
    T.save({k: {"cfg": T.encode(3, 32), "us": 9.0}, "other": {"cfg": 0}}, str(path))
    data = json.loads(path.read_text())
    assert data["entries"][k]["cfg"] == T.encode(3, 32)
    monkeypatch.setenv("FM_GEMM_TUNE", str(path))
    T.set_table(None)
    try:
        assert T.lookup(k) == T.encode(3, 32)
        assert T.lookup("other") == 0           # cfg 0 entries (heuristic kept) are not loaded
        assert T.lookup("absent") == 0
        monkeypatch.setenv("FM_GEMM_TUNE", "0")
        T.set_table(None)
        assert T.lookup(k) == 0
    finally:
        monkeypatch.delenv("FM_GEMM_TUNE", raising=False)
        T.set_table(None)


def test_shipped_table_is_well_formed():
    import os
    if not os.path.exists(T.DEFAULT_PATH):
        return
    with open(T.DEFAULT_PATH) as f:
        data = json.load(f)
    for k, v in data["entries"].items():
        dt, shape, orient, b, ep, c = k.split("|")
        assert dt in ("fp32", "bf16") and len(shape.split("x")) == 3 and len(orient) == 2
        form, ks = T.decode(int(v["cfg"]))
        assert form in (0, 1, 2, 3, 4, 5) and (ks in T.KS_CHOICES or v["cfg"] == 0)
        assert v["us"] <= v["heuristic_us"] + 1e-6
