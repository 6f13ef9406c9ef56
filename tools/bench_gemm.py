#!/usr/bin/env python3
"""GEMM microbenchmark on the DLRM (MLPerf-like, batch 8192) shapes: flexmi MFMA kernel vs
hipBLASLt (torch.matmul) on identical random operands (bf16, or fp32 with --fp32: the flexmi
f32-input MFMA kernel vs the library's fp32 GEMM).  Interleaved rounds in one process
(cdna_hip_programming.md rule 24); prints TFLOP/s per shape and orientation.
usage: bench_gemm.py [--fp32] ["M,K,N;M,K,N"]"""
import json
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from flexmi.ops import _kernels as K  # noqa: E402

B = 8192
LAYERS = [(16, 512), (512, 256), (256, 128), (480, 1024), (1024, 1024), (1024, 512), (512, 256), (256, 1)]


def timeit(fn, iters=20):
    """GPU time per call: `iters` calls captured in one hipGraph (host launch cost excluded)."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e-3 / iters


def main():
    dev = torch.device("cuda")
    rows = []
    global B
    layers = LAYERS
    args = [a for a in sys.argv[1:] if a != "--fp32"]
    dt = torch.float32 if "--fp32" in sys.argv else torch.bfloat16
    torch.backends.cuda.matmul.allow_tf32 = False
    if args:   # custom shapes "M,K,N;M,K,N"
        layers = []
        for t in args[0].split(";"):
            m_, k_, n_ = (int(v) for v in t.split(","))
            layers.append((m_, k_, n_))
    for spec in layers:
        if len(spec) == 3:
            B, k, n = spec
        else:
            k, n = spec
        x = torch.randn(B, k, device=dev).to(dt)
        w = torch.randn(n, k, device=dev).to(dt)
        dy = torch.randn(B, n, device=dev).to(dt)
        bias = torch.randn(n, device=dev)
        y = torch.empty(B, n, device=dev, dtype=dt)
        dx = torch.empty(B, k, device=dev, dtype=dt)
        dw = torch.empty(n, k, device=dev)
        cases = {
            "fwd": (2.0 * B * k * n,
                    lambda: K.gemm(x, k, True, w, k, True, y, n, B, n, k, bias=bias, act=11),
                    lambda: torch.relu(torch.addmm(bias.to(dt), x, w.t()))),
            "dX": (2.0 * B * k * n,
                   lambda: K.gemm(dy, n, True, w, k, False, dx, k, B, k, n),
                   lambda: torch.mm(dy, w)),
            "dW": (2.0 * B * k * n,
                   lambda: K.gemm(dy, n, False, x, k, False, dw, k, n, k, B),
                   lambda: torch.mm(dy.t(), x)),
        }
        for name, (fl, mine, ref) in cases.items():
            tm = min(timeit(mine) for _ in range(3))
            tr = min(timeit(ref) for _ in range(3))
            rows.append({"dtype": str(dt).replace("torch.", ""), "shape": f"{B}x{k}->{n}", "op": name, "flexmi_us": round(tm * 1e6, 2),
                         "hipblaslt_us": round(tr * 1e6, 2), "flexmi_TF": round(fl / tm / 1e12, 1),
                         "hipblaslt_TF": round(fl / tr / 1e12, 1)})
            print(json.dumps(rows[-1]), flush=True)
    tot_m = sum(r["flexmi_us"] for r in rows)
    tot_r = sum(r["hipblaslt_us"] for r in rows)
    print(json.dumps({"total_flexmi_us": round(tot_m, 1), "total_hipblaslt_us": round(tot_r, 1)}))


if __name__ == "__main__":
    main()
