#!/usr/bin/env python3
"""Per-layer timing of the implicit-GEMM convolution kernels (csrc/kernels/conv_igemm.hip) on the
AlexNet / ResNet-50 / Inception shapes: fwd, dgrad, wgrad in µs and TFLOP/s.

    python tools/bench_conv.py [--dtype bf16|fp32] [--net alexnet|resnet|all] [--reps 20] [--only fwd|dgrad|wgrad]
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# name: N, C, H, W, K, R, S, stride, pad
NETS = {
    "alexnet": [("conv1", 256, 3, 229, 229, 64, 11, 11, 4, 2), ("conv2", 256, 64, 27, 27, 192, 5, 5, 1, 2),
                ("conv3", 256, 192, 13, 13, 384, 3, 3, 1, 1), ("conv4", 256, 384, 13, 13, 256, 3, 3, 1, 1),
                ("conv5", 256, 256, 13, 13, 256, 3, 3, 1, 1)],
    "resnet": [("r2_3x3", 64, 64, 56, 56, 64, 3, 3, 1, 1), ("r2_1x1", 64, 64, 56, 56, 256, 1, 1, 1, 0),
               ("r3_3x3", 64, 128, 28, 28, 128, 3, 3, 1, 1), ("r4_3x3", 64, 256, 14, 14, 256, 3, 3, 1, 1),
               ("r5_3x3", 64, 512, 7, 7, 512, 3, 3, 1, 1), ("r3_s2", 64, 128, 56, 56, 128, 3, 3, 2, 1)],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--net", default="alexnet", choices=["alexnet", "resnet", "all"])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="", help="fwd / dgrad / wgrad")
    ap.add_argument("--layer", default="", help="one layer name (e.g. conv2)")
    ap.add_argument("--shape", type=int, default=-1,
                    help="NHWC conv tile shape for every pass (0 128x128, 1 64x128, 2 64x64; -1 heuristic)")
    ap.add_argument("--path", default="raw", choices=["raw", "op"],
                    help="raw: the NCHW kernels (fwd / dgrad / wgrad); op: the framework's conv2d_forward / "
                         "conv2d_backward as dispatched (NHWC staging included; bwd = dgrad + wgrad + act/bias)")
    a = ap.parse_args()
    import torch
    from flexmi.ops import _kernels as K
    for mode in range(3):
        K.C().conv_nhwc_set_shape(mode, a.shape)
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    layers = sum((NETS[n] for n in (NETS if a.net == "all" else [a.net])), [])
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0, "bwd": 0.0}
    for name, N, C, H, W, Ko, R, S, st, pd in layers:
        if a.layer and name != a.layer:
            continue
        P = (H + 2 * pd - R) // st + 1
        Q = (W + 2 * pd - S) // st + 1
        x = torch.randn(N, C, H, W, device="cuda").to(dt)
        w = (torch.randn(Ko, C, R, S, device="cuda") * 0.05).to(dt)
        b = torch.zeros(Ko, device="cuda")
        y = torch.empty(N, Ko, P, Q, device="cuda", dtype=dt)
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        dw = torch.zeros(Ko, C, R, S, device="cuda")
        pads = (pd, pd, pd, pd)
        flop = 2.0 * N * Ko * P * Q * C * R * S
        C_ = K.C()
        wt = K.scratch(x.device, "bench_wt", C_.conv_scratch(C, Ko * R * S), dt)
        wp = K.scratch(x.device, "bench_wp", C_.conv_scratch(Ko, C * R * S), dt)
        if a.path == "raw":
            runs = {
                "fwd": lambda: C_.conv_fwd(x, w, wp, b, y, st, st, pd, pd, 11),
                "dgrad": lambda: C_.conv_dgrad(dy, w, wt, dx, st, st, pd, pd, False),
                "wgrad": lambda: C_.conv_wgrad(dy, x, dw.view(-1), R, S, st, st, pd, pd),
            }
        else:
            saved = {}
            db = torch.zeros(Ko, device="cuda")
            fm = "nhwc" if C >= 16 else None
            runs = {
                "fwd": lambda: K.conv2d_forward(x, w, b, y, (st, st), pads, 11, 1, saved, form=fm),
                "bwd": lambda: K.conv2d_backward(x, w, y, dy, dx, dw, db, (st, st), pads, 11, 1, False, saved,
                                                 form=fm),
            }
        line = f"{name:8s} N{N} C{C} {H}x{W} K{Ko} {R}x{S}/{st}:"
        for k, fn in runs.items():
            if a.only and k != a.only:
                continue
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.reps
            tot[k] += us
            fl = 2 * flop if k == "bwd" else flop
            line += f"  {k} {us:8.1f} us {fl / us / 1e6:6.1f} TF"
        print(line, flush=True)
    print("total us:", {k: round(v, 1) for k, v in tot.items()}, flush=True)


if __name__ == "__main__":
    main()
