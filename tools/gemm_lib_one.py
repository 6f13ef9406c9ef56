#!/usr/bin/env python3
"""hipBLASLt (torch.matmul) counterpart of gemm_one.py for rocprofv3 --pmc A/B:
gemm_lib_one.py M K N orient [iters] [bf16|fp32]  (fwd: x.W^T, dx: dy.W, dw: dy^T.x)"""
import sys
import torch

B, k, n = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
orient = sys.argv[4] if len(sys.argv) > 4 else "fwd"
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 50
dt = torch.float32 if (len(sys.argv) > 6 and sys.argv[6] == "fp32") else torch.bfloat16
torch.backends.cuda.matmul.allow_tf32 = False
dev = torch.device("cuda")
x = torch.randn(B, k, device=dev).to(dt)
w = torch.randn(n, k, device=dev).to(dt)
dy = torch.randn(B, n, device=dev).to(dt)
for _ in range(iters):
    if orient == "fwd":
        torch.matmul(x, w.t())
    elif orient == "dx":
        torch.matmul(dy, w)
    else:
        torch.matmul(dy.t(), x)
torch.cuda.synchronize()
print("ok")
