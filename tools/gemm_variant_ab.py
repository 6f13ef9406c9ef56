#!/usr/bin/env python3
"""A/B of flexmi GEMM variants (FM_GEMM[_F32]_VARIANT bits, set at run time) on the DLRM
MLPerf-like layer shapes at batch 8192, interleaved in one process (rule: compare arms in the same
process, several rounds, keep the minimum).
usage: gemm_variant_ab.py [--fp32] v0,v1,... ["M,K,N;..."]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexmi.ops import _kernels as K  # noqa: E402
from tools.bench_gemm import timeit  # noqa: E402

SHAPES = [(8192, 480, 1024), (8192, 1024, 1024), (8192, 1024, 512), (8192, 512, 256)]


def main():
    args = [a for a in sys.argv[1:] if a != "--fp32"]
    fp32 = "--fp32" in sys.argv
    variants = [int(v) for v in args[0].split(",")] if args else [0]
    shapes = SHAPES
    if len(args) > 1:
        shapes = [tuple(int(v) for v in t.split(",")) for t in args[1].split(";")]
    dt = torch.float32 if fp32 else torch.bfloat16
    setv = K.C().gemm_f32_set_variant if fp32 else K.C().gemm_set_variant
    dev = torch.device("cuda")
    tot = {v: 0.0 for v in variants}
    for B, k, n in shapes:
        x = torch.randn(B, k, device=dev).to(dt)
        w = torch.randn(n, k, device=dev).to(dt)
        dy = torch.randn(B, n, device=dev).to(dt)
        bias = torch.randn(n, device=dev)
        y = torch.empty(B, n, device=dev, dtype=dt)
        dx = torch.empty(B, k, device=dev, dtype=dt)
        dw = torch.empty(n, k, device=dev)
        cases = {
            "fwd": lambda: K.gemm(x, k, True, w, k, True, y, n, B, n, k, bias=bias, act=11),
            "dX": lambda: K.gemm(dy, n, True, w, k, False, dx, k, B, k, n),
            "dW": lambda: K.gemm(dy, n, False, x, k, False, dw, k, n, k, B),
        }
        for name, fn in cases.items():
            best = {v: 1e9 for v in variants}
            ref = None
            for _ in range(3):
                for v in variants:
                    setv(v)
                    best[v] = min(best[v], timeit(fn))
                    out = {"fwd": y, "dX": dx, "dW": dw}[name]
                    if ref is None:
                        ref = out.float().clone()
                    else:
                        err = ((out.float() - ref).abs().max() / ref.abs().max().clamp_min(1e-30)).item()
                        # bf16 outputs: kernels with different summation orders round differently
                        assert err < (1e-4 if out.dtype == torch.float32 else 1e-2), (name, v, err)
            setv(0)
            fl = 2.0 * B * k * n
            row = {"shape": f"{B}x{k}->{n}", "op": name}
            for v in variants:
                row[f"v{v}_us"] = round(best[v] * 1e6, 2)
                row[f"v{v}_TF"] = round(fl / best[v] / 1e12, 1)
                tot[v] += best[v] * 1e6
            print(json.dumps(row), flush=True)
    print(json.dumps({f"total_v{v}_us": round(t, 1) for v, t in tot.items()}))


if __name__ == "__main__":
    main()
