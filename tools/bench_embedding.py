#!/usr/bin/env python3
"""Embedding-bag kernel microbenchmark (fused sparse-SGD backward and forward) over table
sizes of the MLPerf DLRM set: per-table time, effective bytes/s.  hipGraph of reps launches."""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from flexmi.ops import _kernels as K  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(3):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
    return best


def main():
    dev = torch.device("cuda")
    D = 128
    for B in (8192, 65536):
        for rows in (3, 4, 10, 36, 108, 155, 976, 7120, 39884406):
            W = torch.randn(rows, D, device=dev)
            idx = torch.randint(0, rows, (B, 1), device=dev)
            dy = (torch.randn(B, D, device=dev) * 1e-3).bfloat16()
            out = torch.empty(B, D, device=dev, dtype=torch.bfloat16)
            lr = torch.tensor([0.01], device=dev)
            tf = timed(lambda: K.embedding_forward(idx, W, out, 20))
            tb = timed(lambda: K.embedding_backward_sgd(idx, dy, W, lr, 20, {}))
            print(json.dumps({"B": B, "rows": rows, "fwd_us": round(tf, 2), "bwd_us": round(tb, 2),
                              "bwd_GBps": round(B * D * 2 / tb / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
