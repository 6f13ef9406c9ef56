#!/usr/bin/env python3
"""A/B of the fp32 GEMM forms on the DLRM shapes: native fp32 MFMA (split mode 0), the bf16 three-plane
split (mode 2, six products) and the fp16 two-plane scaled split (mode 5, three products): error vs a
float64 oracle (max-normalised, as tests/test_gpu_fp32.py) on N(0,1) operands and on operands whose rows
span six decades, and time per call (CUDA events, the amax pre-pass included)."""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from flexmi.ops import _kernels as K  # noqa: E402


def rel(a, b):
    return ((a.double() - b).abs().max() / (b.abs().max() + 1e-300)).item()


def run(M, N, Kd, a_k, b_k, spread, reps=20):
    g = torch.Generator(device="cuda").manual_seed(M + N + Kd)
    A = torch.randn(M, Kd, device="cuda", generator=g)
    B = torch.randn(Kd, N, device="cuda", generator=g)
    if spread:
        A *= torch.pow(10.0, -6 * torch.rand(M, 1, device="cuda", generator=g))
        B *= torch.pow(10.0, -6 * torch.rand(1, N, device="cuda", generator=g))
    ref = A.double() @ B.double()
    Ag = A if a_k else A.t().contiguous()
    Bg = B.t().contiguous() if b_k else B
    C = torch.empty(M, N, device="cuda")
    out = {"shape": f"{M}x{N}x{Kd}", "orient": ("k" if a_k else "m") + ("k" if b_k else "m"), "spread": spread}
    for mode in (0, 2, 5):
        K.C().gemm_f32_set_split(mode)
        f = lambda: K.gemm(Ag, Kd if a_k else M, a_k, Bg, Kd if b_k else N, b_k, C, N, M, N, Kd)
        f()
        torch.cuda.synchronize()
        err = rel(C, ref)
        # row-wise error relative to each row's own max (the per-row scaling's weak spot)
        rowerr = ((C.double() - ref).abs().amax(1) / (ref.abs().amax(1) + 1e-300)).max().item()
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        torch.cuda.synchronize()
        out[f"m{mode}"] = {"us": round(e0.elapsed_time(e1) * 1e3 / reps, 2), "err": float(f"{err:.3g}"),
                           "rowerr": float(f"{rowerr:.3g}")}
    K.C().gemm_f32_set_split(3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    for spread in (False, True):
        for (M, N, Kd, a_k, b_k) in [(8192, 1024, 1024, True, True), (8192, 1024, 1024, True, False),
                                     (1024, 1024, 8192, False, False), (8192, 1024, 480, True, True),
                                     (8192, 512, 1024, True, True), (512, 1024, 8192, False, False),
                                     (8192, 256, 512, True, True), (256, 512, 8192, False, False)]:
            run(M, N, Kd, a_k, b_k, spread)
