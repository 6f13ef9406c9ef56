#!/usr/bin/env python3
"""Plane-GEMM lab (csrc/kernels/gemm_pl.hip): every DLRM (MLPerf-like, batch 8192) Linear shape in
its three training orientations as the executor issues them (fwd with bias + ReLU epilogue; dX; dW
with beta = 1 and the fused bias-gradient row sums), fp32 values from pre-split bf16 planes, against
the in-kernel split kernel (gemm_x3.hip, same call without planes) and hipBLASLt (torch.matmul fp32).
Checks both against a float64 oracle; reports best-of-rounds GPU time per call (hipGraph of 20 calls,
interleaved rounds) and the time of the split pass that produces one operand's planes.
usage: gemm_pl_lab.py ["M,K,N;..."] [--emit]   (--emit: the plane GEMM also writes C's planes)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexmi.ops import _kernels as K  # noqa: E402
from tools.bench_gemm import timeit  # noqa: E402

SHAPES = [(8192, 480, 1024), (8192, 1024, 1024), (8192, 1024, 512), (8192, 512, 256), (8192, 256, 128)]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    emit = "--emit" in sys.argv
    shapes = SHAPES
    if args:
        shapes = [tuple(int(v) for v in t.split(",")) for t in args[0].split(";")]
    torch.backends.cuda.matmul.allow_tf32 = False
    dev = torch.device("cuda")
    torch.manual_seed(0)
    tot = {"pl": 0.0, "x3": 0.0, "lib": 0.0, "split": 0.0}
    for B, k, n in shapes:
        x = torch.randn(B, k, device=dev)
        w = torch.randn(n, k, device=dev) * 0.1
        dy = torch.randn(B, n, device=dev)
        bias = torch.randn(n, device=dev)
        xp, wp, dyp = K.planes_like(x), K.planes_like(w), K.planes_like(dy)
        K.split_planes(x, xp)
        K.split_planes(w, wp)
        K.split_planes(dy, dyp)
        y = torch.empty(B, n, device=dev)
        yp = K.planes_like(y) if emit else None
        dx = torch.empty(B, k, device=dev)
        dw = torch.zeros(n, k, device=dev)
        db = torch.zeros(n, device=dev)
        ref = {
            "fwd": torch.relu(x.double() @ w.double().t() + bias.double()),
            "dX": dy.double() @ w.double(),
            "dW": dy.double().t() @ x.double(),
        }
        cases = {
            "fwd": (lambda pl: K.gemm(x, k, True, w, k, True, y, n, B, n, k, bias=bias, act=11,
                                      ap=xp if pl else None, bp=wp if pl else None, cp=yp if pl else None),
                    y, lambda: torch.relu(x @ w.t() + bias)),
            "dX": (lambda pl: K.gemm(dy, n, True, w, k, False, dx, k, B, k, n, ap=dyp if pl else None,
                                     bp=wp if pl else None), dx, lambda: dy @ w),
            "dW": (lambda pl: K.gemm(dy, n, False, x, k, False, dw, k, n, k, B, beta=True, rowsum_a=db,
                                     ap=dyp if pl else None, bp=xp if pl else None), dw, lambda: dy.t() @ x),
        }
        for name, (fn, out, lib) in cases.items():
            errs = {}
            for pl in (True, False):
                dw.zero_()
                db.zero_()
                fn(pl)
                torch.cuda.synchronize()
                r = ref[name]
                err = ((out.double() - r).abs().max() / r.abs().max().clamp_min(1e-30)).item()
                assert err < 2e-5, (B, k, n, name, pl, err)
                errs[pl] = err
                if name == "dW":
                    e2 = ((db.double() - dy.double().sum(0)).abs().max() / dy.double().sum(0).abs().max()).item()
                    assert e2 < 2e-5, ("db", pl, e2)
                if name == "fwd" and pl and emit:
                    back = yp[0].float() + yp[1].float() + yp[2].float()
                    assert torch.equal(back, y), "emitted planes do not sum back to C"
            bpl = bx3 = blib = 1e9
            for _ in range(3):
                bpl = min(bpl, timeit(lambda: fn(True)))
                bx3 = min(bx3, timeit(lambda: fn(False)))
                blib = min(blib, timeit(lib))
            fl = 2.0 * B * k * n
            row = {"shape": f"{B}x{k}->{n}", "op": name, "pl_us": round(bpl * 1e6, 2), "x3_us": round(bx3 * 1e6, 2),
                   "lib_us": round(blib * 1e6, 2), "pl_TF": round(fl / bpl / 1e12, 1),
                   "err_pl": f"{errs[True]:.2e}", "err_x3": f"{errs[False]:.2e}"}
            tot["pl"] += bpl * 1e6
            tot["x3"] += bx3 * 1e6
            tot["lib"] += blib * 1e6
            print(json.dumps(row), flush=True)
        bs = min(timeit(lambda: K.split_planes(x, xp)) for _ in range(3))
        tot["split"] += bs * 1e6
        print(json.dumps({"shape": f"{B}x{k}", "op": "split_x", "us": round(bs * 1e6, 2),
                          "GBps": round(B * k * 10 / bs / 1e9, 1)}), flush=True)
    print(json.dumps({f"total_{k_}_us": round(v, 1) for k_, v in tot.items()}), flush=True)


if __name__ == "__main__":
    main()
