"""Measured per-shape GEMM configurations (the MI355X analogue of the reference's per-layer
algorithm search: cudnnFind*AlgorithmEx over the conv forward / filter / data algorithms at init,
src/ops/conv_2d.cu:216-243, :332-347, :872-930; SURVEY V9 "autotune over tile configs").

Every GEMM the Linear / BatchMatmul kernels issue is identified by a key -- dtype, M, N, K, operand
orientations, batch and which fused epilogue it carries -- and the table maps a key to a
configuration measured on MI355X: the kernel form (native fp32 MFMA 128x128 / 128x64 / 64x64
tiles, the split-bf16 kernel with 256x128 / 128x128 tiles; bf16: the three tile shapes) and the
split-K depth.  The encoded value rides in the GEMM's ``ksplit`` argument (``ks | form << 8``, see
csrc/kernels/gemm_f32.hip gemm_f32_run); keys absent from the table keep the built-in heuristic.

``tools/tune_gemm.py`` records the keys a training step issues, times every candidate on the GPU
(isolated, CUDA events, operands of the recorded shapes and strides) and writes the table
``flexmi/ops/tuned/gemm_mi355x.json``, which is loaded here by default.  FM_GEMM_TUNE=0 disables
the table (heuristics only, for A/B); FM_GEMM_TUNE=<path> loads another table.
"""
import json
import os

_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned")
DEFAULT_PATH = os.path.join(_DIR, "gemm_mi355x.json")

FORMS_F32 = {1: "native128x128", 2: "native128x64", 3: "native64x64", 4: "x3_256x128", 5: "x3_128x128",
             6: "x3_128x64"}
FORMS_BF16 = {1: "128x128", 2: "128x64", 3: "64x64"}
KS_CHOICES = (1, 2, 4, 8, 16, 32, 64)

_table = None
RECORD = None        # a list while recording (tools/tune_gemm.py): one spec dict per GEMM call


def encode(form, ks):
    assert 0 <= form < 16 and 0 <= ks < 256
    return int(ks) | (int(form) << 8)


def decode(cfg):
    return cfg >> 8, cfg & 255


def key(dtype, M, N, K, a_k, b_k, batch=1, act_y=False, colsum=False, rowsum=False, sgd=False, c_fp32=True):
    """Identity of one GEMM for the table: operand dtype ('fp32' / 'bf16'), shape, orientations,
    batch and the fused epilogue kinds that constrain the split (act-bwd / column sums / row sums /
    fused SGD) -- everything that changes which configurations apply and how fast they run."""
    ep = ("y" if act_y else "") + ("c" if colsum else "") + ("r" if rowsum else "") + ("s" if sgd else "")
    return f"{dtype}|{int(M)}x{int(N)}x{int(K)}|{'k' if a_k else 'm'}{'k' if b_k else 'm'}|b{int(batch)}|{ep or '-'}|" \
           f"{'c32' if c_fp32 else 'c16'}"


def table():
    global _table
    if _table is None:
        _table = {}
        src = os.environ.get("FM_GEMM_TUNE", "1")
        if src != "0":
            path = DEFAULT_PATH if src in ("", "1") else src
            if os.path.exists(path):
                with open(path) as f:
                    data = json.load(f)
                _table = {k: int(v["cfg"]) for k, v in data.get("entries", {}).items() if int(v.get("cfg", 0)) > 0}
    return _table


def set_table(t):
    """Replace the active table (tests / the tuner); None reloads from FM_GEMM_TUNE on next use."""
    global _table
    _table = t


def lookup(k):
    return table().get(k, 0)


def candidates(dtype, M, N, K, fused=False, sgd=False):
    """Configurations worth timing for one key: every applicable form x the split depths that give
    each split at least 4 k-steps (and a single split for fused backward epilogues the split kernel
    cannot carry)."""
    out = []
    kstep = 32
    ktiles = max(1, (K + kstep - 1) // kstep)
    forms = list(FORMS_F32) if dtype == "fp32" else list(FORMS_BF16)
    for f in forms:
        x3 = dtype == "fp32" and f >= 4
        if x3 and (K % 32 or M < 64 or N < 64):
            continue
        for ks in KS_CHOICES:
            if x3 and fused and ks > 1:
                break               # the split kernel carries a fused epilogue unsplit only
            if ks > 1 and ks * 4 > ktiles:
                break
            out.append(encode(f, ks))
    return out


def save(entries, path=DEFAULT_PATH, meta=None):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        json.dump({"meta": meta or {}, "entries": entries}, f, indent=1, sort_keys=True)
