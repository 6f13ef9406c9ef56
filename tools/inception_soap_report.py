#!/usr/bin/env python3
"""InceptionV3 (BASELINE config 3: 8 x MI355X, MCMC-searched SOAP strategy with operator and
attribute splits) -- simulator PROJECTION of data parallelism vs the searched strategy at 1/2/4/8
GPUs (weak scaling, per-GPU batch fixed), with the per-op cost DB measured on MI355X for the
compute precision and the xGMI machine model.  Also reports what the searched strategy uses:
ops with a spatial (h/w) split, ops placed on a device subset, ops with a channel split.

    python tools/inception_soap_report.py [--dtype bf16] [--budget 3000] [--per-gpu 64] > profiles/inception_soap_vs_dp.txt
"""
from __future__ import annotations

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build(n, per_gpu, dtype, image):
    from flexmi.core import FFConfig, FFModel, SGDOptimizer
    from flexmi.models import cnn
    cfg = FFConfig()
    cfg.batchSize = per_gpu * n
    cfg.device = "gpu"          # plan for the GPU; nothing is allocated
    cfg.compute_dtype = dtype
    m = FFModel(cfg)
    cnn.inception_v3(m, image=image)
    m.optimizer = SGDOptimizer(m, 0.01)
    return m


def describe(model, strat, n):
    """(spatial-split ops, subset-placed ops, channel-split ops) of a strategy."""
    sp = sub = ch = 0
    for op in model.layers:
        pc = strat.get(op.name)
        if pc is None:
            continue
        d = list(pc.dims)
        if len(d) == 4 and (d[0] > 1 or d[1] > 1):
            sp += 1
        if len(d) == 4 and d[2] > 1 or len(d) == 2 and d[0] > 1:
            ch += 1
        if len(set(pc.device_ids)) < n:
            sub += 1
    return sp, sub, ch


def explain(model, r, n, top=12):
    """Why the searched strategy differs from DP: every op the search moved off data parallelism,
    its config and the simulated step-time cost of putting just that op back on DP (positive = the
    move pays), with the op's weight bytes (gradient all-reduce volume under DP)."""
    g = r.graph
    dp = g.dp_assign()
    rows = []
    for i, op in enumerate(g.ops):
        if r.assign[i] == dp[i]:
            continue
        a = list(r.assign)
        a[i] = dp[i]
        delta = g.simulate(a) - r.best_us
        wb = sum(_numel(w.dims) for w in op.weights) * 4
        pc = g.cands[i][r.assign[i]]
        rows.append((delta, op.name, op.op_type.name, list(pc.dims), len(set(pc.device_ids)), wb))
    rows.sort(reverse=True)
    out = [f"#   {n} GPUs: {len(rows)} ops off DP; the {min(top, len(rows))} that matter most "
           f"(delta = simulated ms/step added by reverting only that op to DP):"]
    for delta, name, t, dims, nd, wb in rows[:top]:
        out.append(f"#     {name:28s} {t:12s} dims={dims} on {nd} GPU(s), weights {wb / 2**20:7.2f} MiB, "
                   f"delta {delta / 1e3:+.3f} ms")
    return out


def _numel(d):
    n = 1
    for v in d:
        n *= v
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16", choices=["fp32", "bf16"])
    ap.add_argument("--budget", type=int, default=3000)
    ap.add_argument("--per-gpu", type=int, default=64)
    ap.add_argument("--image", type=int, default=299)
    ap.add_argument("--gpus", default="1,2,4,8")
    a = ap.parse_args()
    from flexmi.parallel.search import optimize
    print(f"# InceptionV3 {a.image}x{a.image}, {a.per_gpu} images per GPU (weak scaling), {a.dtype}: simulator "
          f"PROJECTIONS (measured MI355X cost DB, xGMI machine model); MCMC budget {a.budget} from data parallelism")
    print(f"{'gpus':>4s} {'batch':>6s} {'dp_ms':>9s} {'search_ms':>9s} {'search/dp':>9s} {'img/s(search)':>14s} "
          f"{'spatial':>7s} {'subset':>6s} {'channel':>7s} {'secs':>6s}")
    notes = []
    for n in [int(x) for x in a.gpus.split(",")]:
        m = build(n, a.per_gpu, a.dtype, a.image)
        t0 = time.time()
        r = optimize(m, a.budget if n > 1 else 1, 1.0, num_devices=n, seed=0, verbose=False)
        sp, sub, ch = describe(m, r.best, n)
        print(f"{n:4d} {m.config.batchSize:6d} {r.dp_us / 1e3:9.3f} {r.best_us / 1e3:9.3f} {r.speedup_vs_dp:9.3f} "
              f"{m.config.batchSize / (r.best_us * 1e-6):14.0f} {sp:7d} {sub:6d} {ch:7d} {time.time() - t0:6.1f}",
              flush=True)
        if n > 1:
            notes += explain(m, r, n)
    for line in notes:
        print(line)


if __name__ == "__main__":
    main()
