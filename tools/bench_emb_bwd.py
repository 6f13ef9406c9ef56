#!/usr/bin/env python3
"""Embedding backward (fused sparse SGD) over a set of tables in ONE embedding_bwd_multi call,
timed with events over a hipGraph of reps launches.  Default set: the MLPerf tables that are not
owner-claimed at B = 8192 (<= 8192 rows).  Usage: bench_emb_bwd.py [rows,rows,...] [B] [reps]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexmi.ops import _kernels as K  # noqa: E402

MLPERF_SMALL = [7420, 7120, 1543, 63, 3, 10, 2208, 155, 4, 976, 14, 108, 36]


def main():
    rows = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 and sys.argv[1] else MLPERF_SMALL
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    D = 128
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(1)
    tabs = [torch.randn(r, D, device=dev) * 0.01 for r in rows]
    idx = [torch.randint(0, r, (B, 1), device=dev, generator=g) for r in rows]
    dy = [torch.randn(B, D, device=dev) for _ in rows]
    lr = torch.tensor([1e-6], device=dev)
    none = [None] * (3 * len(rows))

    def run():
        K.C().embedding_bwd_multi(tabs, idx, dy, [D] * len(rows), [1.0] * len(rows), lr, none)

    run()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(gr, stream=s):
            for _ in range(reps):
                run()
    torch.cuda.current_stream().wait_stream(s)
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(5):
        e0.record()
        gr.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1000 / reps)
    print(json.dumps({"rows": rows, "B": B, "us": round(best, 2),
                      "rowblock": os.environ.get("FM_EMB_ROWBLOCK", "0"),
                      "tiny_rows": os.environ.get("FM_EMB_TINY_ROWS", "64")}), flush=True)


if __name__ == "__main__":
    main()
