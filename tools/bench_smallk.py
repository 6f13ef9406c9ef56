#!/usr/bin/env python3
"""Thin-input fp32 Linear (in_features <= 32): gemm_small.hip kernels vs the MFMA GEMM path and
hipBLASLt, standalone (hipGraph-timed, tools/bench_gemm.timeit), one JSON line per case.
usage: bench_smallk.py ["M,K,N;..."]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexmi.ops import _kernels as K  # noqa: E402
from tools.bench_gemm import timeit  # noqa: E402


def main():
    shapes = [(8192, 16, 512), (4096, 16, 512), (65536, 16, 512), (8192, 32, 256)]
    if len(sys.argv) > 1:
        shapes = [tuple(int(v) for v in t.split(",")) for t in sys.argv[1].split(";")]
    torch.backends.cuda.matmul.allow_tf32 = False
    dev = torch.device("cuda")
    torch.manual_seed(0)
    ws = K.workspace(dev, K.GEMM_WS_BYTES)
    for M, k, n in shapes:
        x = torch.randn(M, k, device=dev)
        w = torch.randn(n, k, device=dev)
        b = torch.randn(n, device=dev)
        y = torch.empty(M, n, device=dev)
        dpre = torch.randn(M, n, device=dev)
        dw = torch.zeros(n, k, device=dev)
        db = torch.zeros(n, device=dev)
        lr = torch.tensor([0.01], device=dev)
        t = {
            "fwd_smallk": timeit(lambda: K.C().smallk_fwd(x, w, b, y, 11)),
            "fwd_gemm": timeit(lambda: K.gemm(x, k, True, w, k, True, y, n, M, n, k, bias=b, act=11)),
            "fwd_lib": timeit(lambda: torch.relu(torch.addmm(b, x, w.t()))),
            "dw_smallk": timeit(lambda: K.C().smallk_dw(dpre, x, dw, db, ws, None, None, None, 0.0, 0.0, False)),
            "dw_smallk_sgd": timeit(lambda: K.C().smallk_dw(dpre, x, w, db, ws, None, None, lr, 0.0, 0.0, False)),
            "dw_gemm": timeit(lambda: K.gemm(dpre, n, False, x, k, False, dw, k, n, k, M, beta=True, rowsum_a=db)),
            "dw_lib": timeit(lambda: dw.addmm_(dpre.t(), x)),
        }
        row = {"shape": f"{M}x{k}->{n}"}
        row.update({kk: round(v * 1e6, 2) for kk, v in t.items()})
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
