#!/usr/bin/env python3
"""A/B the GEMM dispatch variants (fm_gemm_set_variant flags) on DLRM shapes in one process,
interleaved rounds (cdna_hip_programming.md §5.4 rule 24).  Flags: 1 = register kernel only,
2 = LDS-DMA kernel for every orientation, 4 = its 128x128 tile, 8 = s_setprio around MFMAs.
usage: gemm_probe.py [M,K,N ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flexmi.ops import _kernels as K  # noqa: E402
from tools.bench_gemm import timeit  # noqa: E402

VARIANTS = [int(v) for v in os.environ.get('VARIANTS', '0,16,32,2').split(',')]


def main():
    dev = torch.device("cuda")
    shapes = [tuple(int(v) for v in s.split(",")) for s in sys.argv[1:]] or [
        (8192, 1024, 1024), (8192, 1024, 512), (8192, 512, 256), (8192, 256, 128), (8192, 512, 1024)]
    C = K.C()
    for M, Kd, N in shapes:
        x = torch.randn(M, Kd, device=dev).bfloat16()
        w = torch.randn(N, Kd, device=dev).bfloat16()
        dy = torch.randn(M, N, device=dev).bfloat16()
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(M, Kd, device=dev, dtype=torch.bfloat16)
        dw = torch.empty(N, Kd, device=dev)
        ops = {"fwd": lambda: K.gemm(x, Kd, True, w, Kd, True, y, N, M, N, Kd, act=11),
               "dx": lambda: K.gemm(dy, N, True, w, Kd, False, dx, Kd, M, Kd, N),
               "dw": lambda: K.gemm(dy, N, False, x, Kd, False, dw, Kd, N, Kd, M)}
        fl = 2.0 * M * N * Kd
        # correctness of every variant against variant 0
        ref = {}
        for name, fn in ops.items():
            C.gemm_set_variant(0)
            fn()
            ref[name] = (y if name == "fwd" else dx if name == "dx" else dw).float().clone()
        res = {(n, v): [] for n in ops for v in VARIANTS}
        for _ in range(3):
            for v in VARIANTS:
                C.gemm_set_variant(v)
                for name, fn in ops.items():
                    res[(name, v)].append(timeit(fn))
        for v in VARIANTS:   # check outputs
            C.gemm_set_variant(v)
            for name, fn in ops.items():
                fn()
                out = (y if name == "fwd" else dx if name == "dx" else dw).float()
                err = (out - ref[name]).abs().max().item() / (ref[name].abs().max().item() + 1e-9)
                if err > 2e-2:
                    print(f"  MISMATCH variant {v} {name}: rel err {err:.3e}")
        C.gemm_set_variant(0)
        for name in ops:
            line = "  ".join(f"v{v}:{min(res[(name, v)]) * 1e6:6.1f}us/{fl / min(res[(name, v)]) / 1e12:4.0f}TF"
                             for v in VARIANTS)
            print(f"{M}x{Kd}->{N} {name:3s} {line}", flush=True)
        t = timeit(lambda: torch.matmul(x, w.t()))
        t2 = timeit(lambda: torch.matmul(dy, w))
        t3 = timeit(lambda: torch.matmul(dy.t(), x))
        print(f"   hipBLASLt fwd {t * 1e6:6.1f}us  dx {t2 * 1e6:6.1f}us  dw {t3 * 1e6:6.1f}us", flush=True)


if __name__ == "__main__":
    main()
