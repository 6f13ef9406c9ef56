#!/usr/bin/env python3
"""Sensitivity of the SOAP search's pick for the DLRM MLPerf config (BASELINE config 4, full-size
tables, 8192 samples per GPU) at 2 / 4 / 8 GPUs: the searched plan and the hand-written table plan it
is seeded with, re-simulated with every xGMI / all-reduce constant of the MI355X machine model at
0.5x and 2x (flexmi/parallel/search.py machine_corners).  The bench falls back to the table plan when
the pick loses more than --robust-threshold (10 %) in any corner.  Writes a text table.
usage: python tools/search_sensitivity.py [--budget 10000] [--out profiles/search_sensitivity_mlperf.txt]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build(world, dtype):
    from flexmi.core import FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
    from flexmi.models.dlrm import DLRMConfig, build_dlrm, dlrm_strategy
    dcfg = DLRMConfig.preset("mlperf")
    cfg = FFConfig()
    cfg.batchSize = 8192 * world
    cfg.compute_dtype = dtype
    m = FFModel(cfg)
    build_dlrm(m, dcfg)
    m.optimizer = SGDOptimizer(m, 0.01)
    return m, dlrm_strategy(m, world)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--budget", type=int, default=10000)
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from flexmi.parallel.search import optimize, sensitivity
    lines = [f"# SOAP search pick vs table plan under machine corners, DLRM mlperf {a.dtype}, 8192 samples/GPU, "
             f"search budget {a.budget} (tools/search_sensitivity.py)",
             "# ratio = simulated step of the pick / of the table plan; > 1.10 in any corner -> bench uses the table plan"]
    for w in [int(x) for x in a.worlds.split(",")]:
        m, table = build(w, a.dtype)
        res = optimize(m, a.budget, 1.0, num_devices=w, init=table, seed=0, verbose=False)
        rows, worst = sensitivity(m, dict(res.best), table, w)
        lines.append(f"world {w}: search {res.best_us / 1e3:.3f} ms, table {res.init_us / 1e3:.3f} ms, dp "
                     f"{res.dp_us / 1e3:.3f} ms (nominal constants); worst ratio {worst:.3f} -> "
                     f"{'TABLE PLAN (fallback)' if worst > 1.10 else 'search pick kept'}")
        for name, pu, bu, r in rows:
            lines.append(f"  {name:22s} pick {pu / 1e3:8.3f} ms  table {bu / 1e3:8.3f} ms  ratio {r:.3f}")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
