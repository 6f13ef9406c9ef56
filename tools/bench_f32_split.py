#!/usr/bin/env python3
"""fp32 GEMM timing on the DLRM MLPerf shapes (batch 8192): native fp32 MFMA kernel vs the exact
three-way bf16 split kernel (FM_F32_SPLIT) vs hipBLASLt (torch.matmul, fp32), every orientation the
framework uses (fwd: x W^T; dX: dy W; dW: dy^T x)."""
import json
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from flexmi.ops import _kernels as Kk
    shapes = [(8192, 512, 256), (8192, 256, 128), (8192, 480, 1024), (8192, 1024, 1024), (8192, 1024, 512),
              (8192, 512, 256), (256, 4096, 4096)]
    reps = 20

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps

    tot = {"native": 0.0, "split": 0.0, "hipblaslt": 0.0}
    for B, K, N in shapes:
        x = torch.randn(B, K, device="cuda")
        w = torch.randn(N, K, device="cuda")
        dy = torch.randn(B, N, device="cuda")
        out = torch.empty(B, N, device="cuda")
        dx = torch.empty(B, K, device="cuda")
        dw = torch.empty(N, K, device="cuda")
        ops = {
            "fwd": (lambda: Kk.gemm(x, K, True, w, K, True, out, N, B, N, K), lambda: torch.matmul(x, w.t(), out=out),
                    2.0 * B * K * N),
            "dX": (lambda: Kk.gemm(dy, N, True, w, K, False, dx, K, B, K, N), lambda: torch.matmul(dy, w, out=dx),
                   2.0 * B * K * N),
            "dW": (lambda: Kk.gemm(dy, N, False, x, K, False, dw, K, N, K, B), lambda: torch.matmul(dy.t(), x, out=dw),
                   2.0 * B * K * N),
        }
        for name, (fn, lib, flop) in ops.items():
            Kk.C().gemm_f32_set_split(False)
            t_n = timeit(fn)
            Kk.C().gemm_f32_set_split(True)
            t_s = timeit(fn)
            Kk.C().gemm_f32_set_split(False)
            t_l = timeit(lib)
            tot["native"] += t_n
            tot["split"] += t_s
            tot["hipblaslt"] += t_l
            print(json.dumps({"shape": f"{B}x{K}->{N}", "op": name, "native_us": round(t_n, 2), "split_us": round(t_s, 2),
                              "hipblaslt_us": round(t_l, 2), "native_TF": round(flop / t_n / 1e6, 1),
                              "split_TF": round(flop / t_s / 1e6, 1), "hipblaslt_TF": round(flop / t_l / 1e6, 1)}), flush=True)
    print(json.dumps({k + "_total_us": round(v, 1) for k, v in tot.items()}), flush=True)


if __name__ == "__main__":
    main()
