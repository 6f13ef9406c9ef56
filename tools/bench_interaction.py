#!/usr/bin/env python3
"""Dot-interaction microbenchmark at the DLRM MLPerf-like shape (B=8192, 1 dense + 26 sparse
features of D=128, pairs without self interaction): flexmi fwd/bwd kernels in fp32 and bf16,
GPU time per call from a captured hipGraph, plus the achieved HBM rate of the bytes each pass
must move (fwd: read Z, write out; bwd: read Z and dOut, write dZ).
usage: bench_interaction.py [B] [F] [D]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexmi.ops import _kernels as K  # noqa: E402
from tools.bench_gemm import timeit  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    F = int(sys.argv[2]) if len(sys.argv) > 2 else 27
    D = int(sys.argv[3]) if len(sys.argv) > 3 else 128
    dev = torch.device("cuda")
    npairs = F * (F - 1) // 2
    W = D + npairs
    for dt in (torch.float32, torch.bfloat16):
        es = torch.tensor([], dtype=dt).element_size()
        Wp = (W + 7) // 8 * 8
        zs = [torch.randn(B, D, device=dev).to(dt) for _ in range(F)]
        out = torch.zeros(B, Wp, device=dev, dtype=dt)
        dout = torch.randn(B, Wp, device=dev).to(dt)
        gs = [torch.zeros(B, D, device=dev, dtype=dt) for _ in range(F)]
        tf = min(timeit(lambda: K.dot_interaction_forward(zs, out, False)) for _ in range(3))
        tb = min(timeit(lambda: K.dot_interaction_backward(zs, dout, gs, [False] * F, False)) for _ in range(3))
        fb = (B * F * D + B * W) * es
        bb = (2 * B * F * D + B * W) * es
        print(json.dumps({"dtype": str(dt).replace("torch.", ""), "B": B, "F": F, "D": D,
                          "fwd_us": round(tf * 1e6, 2), "fwd_TBps": round(fb / tf / 1e12, 2),
                          "bwd_us": round(tb * 1e6, 2), "bwd_TBps": round(bb / tb / 1e12, 2)}), flush=True)


if __name__ == "__main__":
    main()
