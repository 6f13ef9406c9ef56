#!/usr/bin/env python3
"""SOAP strategy vs data parallelism on the MI355X simulator (the second half of the BASELINE
metric: "SOAP speedup vs pure DP").  Every number printed here is a PROJECTION of the simulator
(per-op costs from the measured MI355X cost DB for the compute precision, xGMI machine model for
the collectives); the measured 1-GPU step of bench.py is printed next to the 1-GPU projection as
the calibration check.

For each DLRM config and GPU count: predicted step time of
  dp      pure data parallelism (tables replicated; the sparse optimizer exchanges only the rows
          a step touches -- an all-gather of the global batch's row gradients, not the tables),
  hand    the HBM-balanced hand plan of bench.py (flexmi.models.dlrm.dlrm_strategy),
  search  the MCMC SOAP search seeded with the hand plan,
and the speedups search/dp and hand/dp.

    python tools/soap_report.py [--dtype fp32] [--budget 2000] [--measured-ms 1.65] > profiles/soap_vs_dp.txt
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = [("run_random", 256), ("criteo_kaggle", 256), ("mlperf", 8192)]


def build(name, n, per_gpu, dtype):
    from flexmi.core import FFConfig, FFModel, SGDOptimizer
    from flexmi.models.dlrm import DLRMConfig, build_dlrm
    cfg = FFConfig()
    cfg.batchSize = per_gpu * n
    cfg.device = "gpu"          # plan for the GPU (padded dense input); nothing is allocated
    cfg.compute_dtype = dtype
    m = FFModel(cfg)
    build_dlrm(m, DLRMConfig.preset(name))
    m.optimizer = SGDOptimizer(m, 0.01)
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--budget", type=int, default=2000)
    ap.add_argument("--gpus", default="1,2,4,8")
    ap.add_argument("--configs", default=",".join(c for c, _ in CONFIGS))
    ap.add_argument("--measured-ms", default="", help="config=ms,... measured bench.py N=1 steps (calibration)")
    a = ap.parse_args()
    from flexmi.models.dlrm import dlrm_strategy
    from flexmi.parallel.search import optimize
    measured = dict(kv.split("=") for kv in a.measured_ms.split(",") if "=" in kv)
    per = dict(CONFIGS)
    print(f"# SOAP vs DP on MI355X -- simulator PROJECTIONS ({a.dtype} cost DB, xGMI model); "
          f"search budget {a.budget}, seeded with the hand plan")
    print(f"{'config':14s} {'gpus':>4s} {'batch':>6s} {'dp_ms':>9s} {'hand_ms':>9s} {'search_ms':>9s} "
          f"{'hand/dp':>8s} {'search/dp':>9s}  note")
    for name in a.configs.split(","):
        for n in [int(x) for x in a.gpus.split(",")]:
            m = build(name, n, per[name], a.dtype)
            hand = dlrm_strategy(m, n) if n > 1 else {}
            r = optimize(m, a.budget if n > 1 else 0, 1.0, num_devices=n, init=hand or None, seed=0, verbose=False)
            g = r.graph
            hand_us = g.simulate(g.assign_from(hand))
            note = "projection"
            if n == 1 and name in measured:
                ms = float(measured[name])
                note = f"projection; measured {ms:.3f} ms ({100 * (r.dp_us / 1e3 - ms) / ms:+.1f} %)"
            print(f"{name:14s} {n:4d} {per[name] * n:6d} {r.dp_us / 1e3:9.3f} {hand_us / 1e3:9.3f} "
                  f"{r.best_us / 1e3:9.3f} {r.dp_us / hand_us:8.2f} {r.dp_us / r.best_us:9.2f}  {note}")
            rec = {"config": name, "gpus": n, "global_batch": per[name] * n, "dtype": a.dtype, "dp_ms": r.dp_us / 1e3,
                   "hand_ms": hand_us / 1e3, "search_ms": r.best_us / 1e3, "speedup_search_vs_dp": r.dp_us / r.best_us,
                   "speedup_hand_vs_dp": r.dp_us / hand_us, "kind": "projection",
                   "peak_hbm_GB": max(g.memory(r.assign)) / 1e9}
            print("#", json.dumps(rec))


if __name__ == "__main__":
    main()
