"""flexmi command line: strategy generators, the standalone SOAP simulator / search, .pb tools.

    python -m flexmi.cli gen-dlrm   --gpus 8 --emb 26 [--nodes 1] [-o FILE.pb]
    python -m flexmi.cli gen-dlrm-hetero --emb 8 [-o FILE.pb]
    python -m flexmi.cli show      FILE.pb
    python -m flexmi.cli simulate  --model dlrm-mlperf --gpus 8 [--strategy FILE.pb] [--trace T.json]
    python -m flexmi.cli search    --model inception_v3 --gpus 8 --budget 2000 [--export FILE.pb] [--trace T.json]

``gen-dlrm`` is the reference's DLRM strategy generator (``src/runtime/dlrm_strategy.cc:224-296``,
``gen_strategy.sh``): embedding i on GPU ``i mod (gpus*nodes)`` with dims [1, 1], the dense ops
(``linear``, ``concat``, ``mse_loss``) data parallel over every GPU, written with the reference's
op names so the files are interchangeable with the shipped ``dlrm_strategy_*.pb``;
``gen-dlrm-hetero`` is ``dlrm_strategy_hetero.cc`` (all embeddings on the CPU, the rest on one
GPU).  ``simulate`` / ``search`` are the standalone simulator (``scripts/simulator.cc``): build any
zoo model at the given batch, predict the per-iteration time of a strategy (default: data
parallel) on the calibrated MI355X machine model, or run the MCMC search and export the best.
"""
from __future__ import annotations

import argparse
import json
import sys

from flexmi.parallel.layout import ParallelConfig
from flexmi.parallel.strategy import load_strategies_from_file, save_strategies_to_file


def dlrm_reference_strategy(num_emb, gpus, nodes=1):
    total = gpus * nodes
    s = {f"embedding{i}": ParallelConfig([1, 1], [i % total]) for i in range(num_emb)}
    dp = ParallelConfig([1, total], list(range(total)))
    for name in ("linear", "concat", "mse_loss"):
        s[name] = ParallelConfig(list(dp.dims), list(dp.device_ids))
    return s


def dlrm_hetero_strategy(num_emb):
    s = {f"embedding{i}": ParallelConfig([1, 1], [0], ParallelConfig.CPU) for i in range(num_emb)}
    for name in ("linear", "concat", "mse_loss"):
        s[name] = ParallelConfig([1, 1], [0])
    return s


def _model(name, gpus, batch, small):
    from flexmi.core import FFConfig, FFModel, SGDOptimizer
    from flexmi.models import zoo
    cfg = FFConfig()
    cfg.device = "cpu"
    cfg.compute_dtype = "bf16"
    cfg.batchSize = batch
    m = FFModel(cfg)
    built = zoo.build(name, m, small=small)
    m.optimizer = SGDOptimizer(m, built.lr)
    return m


def main(argv=None):
    ap = argparse.ArgumentParser(prog="flexmi")
    sub = ap.add_subparsers(dest="cmd", required=True)
    g = sub.add_parser("gen-dlrm")
    g.add_argument("--gpus", type=int, required=True)
    g.add_argument("--emb", type=int, required=True)
    g.add_argument("--nodes", type=int, default=1)
    g.add_argument("-o", "--output")
    h = sub.add_parser("gen-dlrm-hetero")
    h.add_argument("--emb", type=int, required=True)
    h.add_argument("-o", "--output")
    s = sub.add_parser("show")
    s.add_argument("file")
    for name in ("simulate", "search"):
        p = sub.add_parser(name)
        p.add_argument("--model", required=True)
        p.add_argument("--gpus", type=int, default=8)
        p.add_argument("--batch", type=int, default=0, help="global batch (default 64 per GPU; DLRM 8192)")
        p.add_argument("--small", action="store_true")
        p.add_argument("--strategy", help="strategy .pb (simulate) / initial state (search)")
        p.add_argument("--trace", help="write the predicted timeline as Chrome trace JSON")
        p.add_argument("--machine", help="machine model JSON override")
        p.add_argument("--cost-db", help="measured cost DB JSON")
        if name == "search":
            p.add_argument("--budget", type=int, default=1000)
            p.add_argument("--alpha", type=float, default=1.0)
            p.add_argument("--seed", type=int, default=0)
            p.add_argument("--export", help="write the best strategy (.pb)")
    a = ap.parse_args(argv)

    if a.cmd in ("gen-dlrm", "gen-dlrm-hetero"):
        if a.cmd == "gen-dlrm":
            st = dlrm_reference_strategy(a.emb, a.gpus, a.nodes)
            out = a.output or f"dlrm_strategy_emb_{a.emb}_gpu_{a.gpus}_node_{a.nodes}.pb"
        else:
            st = dlrm_hetero_strategy(a.emb)
            out = a.output or f"dlrm_strategy_hetero_emb_{a.emb}.pb"
        save_strategies_to_file(out, st)
        print(f"wrote {len(st)} op configs to {out}")
        return 0
    if a.cmd == "show":
        st = load_strategies_from_file(a.file)
        for name in sorted(st):
            pc = st[name]
            dev = "CPU" if pc.device_type == ParallelConfig.CPU else "GPU"
            print(f"{name:24s} {dev} dims={list(pc.dims)} devices={list(pc.device_ids)}"
                  + (f" mem={list(pc.memory_types)}" if pc.memory_types else ""))
        return 0

    from flexmi.parallel.machine import MachineModel
    from flexmi.parallel.cost import CostModel
    from flexmi.parallel.search import SimGraph, optimize
    batch = a.batch or ((8192 if a.model.startswith("dlrm") else 64) * a.gpus)
    m = _model(a.model, a.gpus, batch, a.small)
    mach = MachineModel.load(a.machine, a.gpus) if a.machine else MachineModel.mi355x(a.gpus)
    init = None
    if a.strategy:
        from flexmi.parallel.strategy import resolve_reference_names
        init = resolve_reference_names(m, load_strategies_from_file(a.strategy))
    if a.cmd == "simulate":
        cost = CostModel(mach, a.cost_db) if a.cost_db else None
        graph = SimGraph(m, a.gpus, mach, cost, extra=init)
        asg = graph.assign_from(init or {})
        us = graph.simulate(asg)
        dp = graph.simulate(graph.dp_assign())
        mem = graph.memory(asg)
        print(json.dumps({"model": a.model, "gpus": a.gpus, "global_batch": batch, "predicted_ms": us / 1e3,
                          "data_parallel_ms": dp / 1e3, "speedup_vs_dp": dp / us if us > 0 else None,
                          "peak_mem_gb": [round(x / 1e9, 3) for x in mem] if isinstance(mem, (list, tuple)) else mem}))
        if a.trace:
            graph.chrome_trace(asg, a.trace)
        return 0
    res = optimize(m, a.budget, a.alpha, num_devices=a.gpus, machine=mach, cost_db=a.cost_db, seed=a.seed,
                   init=init, verbose=True)
    print(json.dumps({"model": a.model, "gpus": a.gpus, "global_batch": batch, **res.summary()}))
    if a.export:
        save_strategies_to_file(a.export, res.best)
        print(f"exported {len(res.best)} op configs to {a.export}")
    if a.trace:
        res.graph.chrome_trace(res.assign, a.trace)
    return 0


if __name__ == "__main__":
    sys.exit(main())
