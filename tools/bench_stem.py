#!/usr/bin/env python3
"""Time the stem convolution forms (flexmi/ops/_kernels.py conv forms) on the AlexNet / ResNet stems:
forward and weight-gradient (the first layer needs no dX), us per call.
usage: python tools/bench_stem.py [--reps 20]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from flexmi.ops import _kernels as Kk
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default=None, help="one form (e.g. stem)")
    ap.add_argument("--model", default=None, help="alexnet or resnet")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    for name, (N, H, R, s, pad) in {"alexnet b256": (256, 229, 11, 4, 2), "resnet b64": (64, 229, 7, 2, 3)}.items():
        if args.model and not name.startswith(args.model):
            continue
        x = torch.randn(N, 3, H, H, device=dev).bfloat16()
        w = (torch.randn(64, 3, R, R, device=dev) * 0.05).bfloat16()
        b = torch.randn(64, device=dev)
        P = (H + 2 * pad - R) // s + 1
        y = torch.empty(N, 64, P, P, device=dev, dtype=torch.bfloat16)
        dy = torch.randn_like(y)
        dw = torch.zeros(64, 3, R, R, device=dev)
        db = torch.zeros(64, device=dev)
        pads = (pad,) * 4
        for form in Kk.conv_forms(x, w, y, (s, s), 1):
            if args.only and form != args.only:
                continue
            f_us = Kk._time_us(lambda: Kk.conv2d_forward(x, w, b, y, (s, s), pads, 11, 1, {}, form=form), args.reps)
            b_us = Kk._time_us(lambda: Kk.conv2d_backward(x, w, y, dy, None, dw, db, (s, s), pads, 11, 1, False, {},
                                                          form=form), args.reps)
            print(f"{name:13s} {form:9s} fwd {f_us:8.1f} us  wgrad {b_us:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
