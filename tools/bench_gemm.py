#!/usr/bin/env python3
"""GEMM microbenchmark on the DLRM (MLPerf-like, batch 8192) shapes: flexmi MFMA kernel vs
hipBLASLt (torch.matmul) on identical random bf16 operands.  Interleaved rounds in one process
(cdna_hip_programming.md rule 24); prints TFLOP/s per shape and orientation."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from flexmi.ops import _kernels as K  # noqa: E402

B = 8192
LAYERS = [(16, 512), (512, 256), (256, 128), (480, 1024), (1024, 1024), (1024, 512), (512, 256), (256, 1)]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    dev = torch.device("cuda")
    rows = []
    for (k, n) in LAYERS:
        x = torch.randn(B, k, device=dev).bfloat16()
        w = torch.randn(n, k, device=dev).bfloat16()
        dy = torch.randn(B, n, device=dev).bfloat16()
        bias = torch.randn(n, device=dev)
        y = torch.empty(B, n, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(B, k, device=dev, dtype=torch.bfloat16)
        dw = torch.empty(n, k, device=dev)
        cases = {
            "fwd": (2.0 * B * k * n,
                    lambda: K.gemm(x, k, True, w, k, True, y, n, B, n, k, bias=bias, act=11),
                    lambda: torch.relu(torch.addmm(bias.bfloat16(), x, w.t()))),
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
            rows.append({"shape": f"{B}x{k}->{n}", "op": name, "flexmi_us": round(tm * 1e6, 2),
                         "hipblaslt_us": round(tr * 1e6, 2), "flexmi_TF": round(fl / tm / 1e12, 1),
                         "hipblaslt_TF": round(fl / tr / 1e12, 1)})
            print(json.dumps(rows[-1]), flush=True)
    tot_m = sum(r["flexmi_us"] for r in rows)
    tot_r = sum(r["hipblaslt_us"] for r in rows)
    print(json.dumps({"total_flexmi_us": round(tot_m, 1), "total_hipblaslt_us": round(tot_r, 1)}))


if __name__ == "__main__":
    main()
