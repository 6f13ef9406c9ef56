#!/usr/bin/env python3
"""NMT placement on the MI355X simulator: data parallelism vs the reference's placement (source /
target embeddings on GPUs 0 / 1, LSTM chunks + projection data parallel, nmt/nmt.cc:269-309) vs
per-chunk pipeline placement (flexmi.models.nmt.nmt_strategy) vs the MCMC search seeded with the
best of them.  Every number is a simulator PROJECTION (cost DB of the compute precision, xGMI
machine model); the measured 1-GPU step is printed next to the 1-GPU projection when given.

    python tools/nmt_report.py [--dtype fp32] [--gpus 1,2,4,8] [--budget 500] [--measured-ms 18.7]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build(n, per_gpu, dtype):
    from flexmi.core import FFConfig, FFModel, SGDOptimizer
    from flexmi.models.nmt import NMTConfig, nmt
    cfg = FFConfig()
    cfg.batchSize = per_gpu * n
    cfg.device = "gpu"
    cfg.compute_dtype = dtype
    m = FFModel(cfg)
    nmt(m, NMTConfig())
    m.optimizer = SGDOptimizer(m, 0.01)
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--gpus", default="1,2,4,8")
    ap.add_argument("--batch-per-gpu", type=int, default=64)
    ap.add_argument("--budget", type=int, default=500)
    ap.add_argument("--measured-ms", type=float, default=0.0)
    a = ap.parse_args()
    from flexmi.models.nmt import nmt_strategy
    from flexmi.parallel.search import optimize
    print(f"# NMT (2 layers, seq 20, hidden 2048, vocab 20 K, batch {a.batch_per_gpu}/GPU) placement -- simulator "
          f"PROJECTIONS ({a.dtype} cost DB, xGMI model)")
    print(f"{'gpus':>4s} {'dp_ms':>9s} {'ref_ms':>9s} {'pipe_ms':>9s} {'search_ms':>9s}  note")
    for n in [int(x) for x in a.gpus.split(",")]:
        m = build(n, a.batch_per_gpu, a.dtype)
        ref = nmt_strategy(m, n, "reference") if n > 1 else {}
        pipe = nmt_strategy(m, n, "pipeline") if n > 1 else {}
        r0 = optimize(m, 0, 1.0, num_devices=n, init=None, seed=0, verbose=False)
        g = r0.graph
        ref_us = g.simulate(g.assign_from(ref))
        pipe_us = g.simulate(g.assign_from(pipe))
        seed = ref if ref_us <= pipe_us else pipe
        r = optimize(m, a.budget if n > 1 else 0, 1.0, num_devices=n, init=seed or None, seed=0, verbose=False)
        note = "projection"
        if n == 1 and a.measured_ms:
            note += f"; measured {a.measured_ms:.3f} ms ({100 * (r0.dp_us / 1e3 - a.measured_ms) / a.measured_ms:+.1f} %)"
        print(f"{n:4d} {r0.dp_us / 1e3:9.3f} {ref_us / 1e3:9.3f} {pipe_us / 1e3:9.3f} {r.best_us / 1e3:9.3f}  {note}")
        print("#", json.dumps({"gpus": n, "dtype": a.dtype, "dp_ms": r0.dp_us / 1e3, "reference_ms": ref_us / 1e3,
                               "pipeline_ms": pipe_us / 1e3, "search_ms": r.best_us / 1e3, "kind": "projection"}))


if __name__ == "__main__":
    main()
