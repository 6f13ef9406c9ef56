#!/usr/bin/env python3
"""fp32 GEMM lab: every DLRM (MLPerf-like, batch 8192) layer shape in its three training
orientations, exactly as the executor issues them (fwd with bias+ReLU epilogue; dX; dW with
beta = 1 accumulation and the fused bias-gradient row sums), for a list of FM_GEMM_F32_VARIANT
values, against hipBLASLt (torch.matmul, fp32).  Checks every variant against a float64 oracle
and reports the best-of-rounds GPU time per call (hipGraph of 20 calls, interleaved rounds).
usage: gemm_f32_lab.py v0,v1,... ["M,K,N;..."]   (v: 0 = native fp32 MFMA kernel, -2 = split-bf16
kernel 16x16x32 form, -32 = split-bf16 kernel 32x32x16 form)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexmi.ops import _kernels as K  # noqa: E402
from tools.bench_gemm import timeit  # noqa: E402

SHAPES = [(8192, 16, 512), (8192, 512, 256), (8192, 256, 128), (8192, 480, 1024), (8192, 1024, 1024),
          (8192, 1024, 512), (8192, 512, 256)]


def main():
    args = sys.argv[1:]
    variants = [int(v) for v in args[0].split(",")] if args else [0]
    shapes = SHAPES
    if len(args) > 1:
        shapes = [tuple(int(v) for v in t.split(",")) for t in args[1].split(";")]
    torch.backends.cuda.matmul.allow_tf32 = False
    def setv(v):
        K.C().gemm_f32_set_split(2 if v < 0 else 0)

    dev = torch.device("cuda")
    torch.manual_seed(0)
    tot = {v: 0.0 for v in variants}
    tot["lib"] = 0.0
    for B, k, n in shapes:
        x = torch.randn(B, k, device=dev)
        w = torch.randn(n, k, device=dev) * 0.1
        dy = torch.randn(B, n, device=dev)
        bias = torch.randn(n, device=dev)
        y = torch.empty(B, n, device=dev)
        dx = torch.empty(B, k, device=dev)
        dw = torch.zeros(n, k, device=dev)
        db = torch.zeros(n, device=dev)
        ref = {
            "fwd": torch.relu(x.double() @ w.double().t() + bias.double()),
            "dX": dy.double() @ w.double(),
            "dW": dy.double().t() @ x.double(),
        }
        cases = {
            "fwd": (lambda: K.gemm(x, k, True, w, k, True, y, n, B, n, k, bias=bias, act=11), y,
                    lambda: torch.relu(x @ w.t() + bias)),
            "dX": (lambda: K.gemm(dy, n, True, w, k, False, dx, k, B, k, n), dx, lambda: dy @ w),
            "dW": (lambda: K.gemm(dy, n, False, x, k, False, dw, k, n, k, B, beta=True, rowsum_a=db), dw,
                   lambda: dy.t() @ x),
        }
        for name, (fn, out, lib) in cases.items():
            best = {v: 1e9 for v in variants}
            for v in variants:   # numerics first (fresh accumulators for beta = 1)
                setv(v)
                dw.zero_()
                db.zero_()
                fn()
                torch.cuda.synchronize()
                r = ref[name]
                err = ((out.double() - r).abs().max() / r.abs().max().clamp_min(1e-30)).item()
                assert err < 2e-5, (B, k, n, name, v, err)
                if name == "dW":
                    e2 = ((db.double() - dy.double().sum(0)).abs().max() / dy.double().sum(0).abs().max()).item()
                    assert e2 < 2e-5, ("db", v, e2)
            blib = 1e9
            for _ in range(3):
                for v in variants:
                    setv(v)
                    best[v] = min(best[v], timeit(fn))
                blib = min(blib, timeit(lib))
            setv(0)
            fl = 2.0 * B * k * n
            row = {"shape": f"{B}x{k}->{n}", "op": name, "lib_us": round(blib * 1e6, 2)}
            for v in variants:
                row[f"v{v}_us"] = round(best[v] * 1e6, 2)
                row[f"v{v}_TF"] = round(fl / best[v] / 1e12, 1)
                tot[v] += best[v] * 1e6
            tot["lib"] += blib * 1e6
            print(json.dumps(row), flush=True)
    print(json.dumps({f"total_{v}_us": round(t, 1) for v, t in tot.items()}), flush=True)


if __name__ == "__main__":
    main()
