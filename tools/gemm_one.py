#!/usr/bin/env python3
"""Run one flexmi GEMM shape repeatedly (for rocprofv3 --pmc): gemm_one.py M K N orient [iters] [bf16|fp32]
orient: fwd (x[M,K] . W[N,K]^T), dx (dy[M,N] . W[N,K]), dw (dy^T . x)."""
import sys
import torch
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from flexmi.ops import _kernels as K  # noqa: E402

B, k, n = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
orient = sys.argv[4] if len(sys.argv) > 4 else "fwd"
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 50
mode = sys.argv[6] if len(sys.argv) > 6 else "bf16"
dt = torch.float32 if mode == "fp32" else torch.bfloat16
dev = torch.device("cuda")
x = torch.randn(B, k, device=dev).to(dt)
w = torch.randn(n, k, device=dev).to(dt)
dy = torch.randn(B, n, device=dev).to(dt)
y = torch.empty(B, n, device=dev, dtype=dt)
dx = torch.empty(B, k, device=dev, dtype=dt)
dw = torch.empty(n, k, device=dev)
for _ in range(iters):
    if orient == "fwd":
        K.gemm(x, k, True, w, k, True, y, n, B, n, k, act=11)
    elif orient == "dx":
        K.gemm(dy, n, True, w, k, False, dx, k, B, k, n)
    else:
        K.gemm(dy, n, False, x, k, False, dw, k, n, k, B)
torch.cuda.synchronize()
print("ok")
