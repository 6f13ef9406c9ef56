#!/usr/bin/env python3
"""Run torch.matmul (hipBLASLt) on the DLRM GEMM shapes so rocprofv3 can report which library
kernels (macro-tile / MFMA / prefetch configuration encoded in the kernel name) it picks."""
import torch

dev = torch.device("cuda")
for M, K, N in [(8192, 1024, 1024), (8192, 1024, 512), (8192, 512, 256), (8192, 256, 128), (8192, 480, 1024)]:
    x = torch.randn(M, K, device=dev).bfloat16()
    w = torch.randn(N, K, device=dev).bfloat16()
    dy = torch.randn(M, N, device=dev).bfloat16()
    for _ in range(3):
        torch.matmul(x, w.t())
        torch.matmul(dy, w)
torch.cuda.synchronize()
print("ok")
