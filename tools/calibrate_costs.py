#!/usr/bin/env python3
"""Calibrate the simulator's cost DB on a real MI355X (the analogue of the reference's
``measure_compute_time`` calls during search, done once, offline).

For every op of the model and every shard shape its candidate ParallelConfigs produce at
``--gpus`` device counts, measure forward/backward time with :func:`flexmi.runtime.measure.measure_op`
and write ``{"entries": {signature: [fwd_us, bwd_us]}, "scale": {op_type: measured/roofline}}``.

    python tools/calibrate_costs.py --model dlrm-mlperf --gpus 1,2,4,8 \
        --out flexmi/parallel/costdb/mi355x.json                       (bf16 fast mode)
    python tools/calibrate_costs.py --dtype fp32 --out flexmi/parallel/costdb/mi355x_fp32.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build_model(name, n, batch_per_gpu, device="gpu", dtype="bf16"):
    from flexmi.core import FFConfig, FFModel, SGDOptimizer
    cfg = FFConfig()
    cfg.batchSize = batch_per_gpu * n
    cfg.device = device
    cfg.compute_dtype = dtype if device == "gpu" else "fp32"
    m = FFModel(cfg)
    if name.startswith("dlrm"):
        from flexmi.models.dlrm import DLRMConfig, build_dlrm
        build_dlrm(m, DLRMConfig.preset(name.split("-", 1)[1] if "-" in name else "mlperf"))
    else:
        from flexmi.models import zoo
        zoo.build(name, m)
    m.optimizer = SGDOptimizer(m, 0.01)
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="dlrm-mlperf")
    ap.add_argument("--gpus", default="1,2,4,8")
    ap.add_argument("--batch-per-gpu", type=int, default=8192)
    ap.add_argument("--out", default=os.path.join(ROOT, "flexmi", "parallel", "costdb", "mi355x.json"))
    ap.add_argument("--limit", type=int, default=0)
    ap.add_argument("--device", default="gpu", choices=["gpu", "cpu"])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--time-budget", type=float, default=900.0, help="stop measuring after this many seconds")
    ap.add_argument("--refresh", default="", help="comma list of op types (e.g. OP_LINEAR) re-measured even when the "
                                                  "DB already holds them (after kernel changes)")
    a = ap.parse_args()

    from flexmi.parallel.cost import CostModel, op_signature
    from flexmi.parallel.machine import MachineModel
    from flexmi.parallel.search import candidate_configs
    from flexmi.runtime.measure import measure_op

    todo = {}
    for n in [int(x) for x in a.gpus.split(",")]:
        m = build_model(a.model, n, a.batch_per_gpu, a.device, a.dtype)
        for op in m.layers:
            for pc in candidate_configs(op, n):
                ins, outs = op.input_layouts(pc), op.output_layouts(pc)
                for p, dev in enumerate(pc.device_ids):
                    i_s = [tuple(hi - lo for lo, hi in l.part_box(l.parts_of(dev)[0])) for l in ins]
                    o_s = [tuple(hi - lo for lo, hi in l.part_box(p)) for l in outs]
                    key = op_signature(op, i_s, o_s)
                    if key not in todo:
                        todo[key] = (op, i_s, o_s)
    keys = sorted(todo)
    if a.limit:
        keys = keys[: a.limit]
    db = {"device": "MI355X", "dtype": a.dtype, "model": a.model, "entries": {}, "scale": {}}
    if os.path.exists(a.out):
        with open(a.out) as f:
            old = json.load(f)
        db["entries"].update(old.get("entries", {}))
        if "group_factor" in old:                      # measured on a DLRM run; keep it
            db["group_factor"] = old["group_factor"]
        # per-type scales of op types another model's run already fitted stay (a DB serves several
        # models: refitting OP_LINEAR on InceptionV3's one classifier would rescale every
        # unmeasured DLRM MLP shape); --refresh TYPE refits them
        db["scale_keep"] = {t: v for t, v in old.get("scale", {}).items() if t not in a.refresh.split(",")}
    cm = CostModel(MachineModel.mi355x(1), db_path="", dtype_bytes=4 if a.dtype == "fp32" else 2)
    t0 = time.time()
    done = 0
    refresh = tuple(t for t in a.refresh.split(",") if t)
    for k in keys:
        if k in db["entries"] and not (refresh and k.split("|")[0] in refresh):
            continue
        if time.time() - t0 > a.time_budget:
            print(f"[calibrate] time budget reached after {done} measurements", flush=True)
            break
        op, i_s, o_s = todo[k]
        r = measure_op(op, i_s, o_s, reps=a.reps, device=a.device, dtype=a.dtype)
        done += 1
        if r is None:
            continue
        db["entries"][k] = [round(r[0], 3), round(r[1], 3)]
        print(f"[calibrate] {done}/{len(keys)} {k}: fwd {r[0]:.2f} us bwd {r[1]:.2f} us", flush=True)
        if done % 20 == 0:
            _write(a.out, db, todo, cm)
    # fused embedding groups: the step runs every table of a placement in ONE forward and ONE
    # sparse-SGD launch, so the isolated per-table times overstate it; measure the whole group
    # at the 1-GPU batch and store measured(group) / sum(isolated tables) as group_factor
    from flexmi.core.types import OperatorType
    from flexmi.runtime.measure import measure_embedding_group
    m1 = build_model(a.model, 1, a.batch_per_gpu, a.device, a.dtype)
    embs = [op for op in m1.layers if op.op_type == OperatorType.OP_EMBEDDING]
    if len(embs) > 1 and a.model.startswith("dlrm"):   # the factor is the DLRM table group's
        iso = 0.0
        for op in embs:
            k = op_signature(op, [tuple(op.inputs[0].dims)], [tuple(op.outputs[0].dims)])
            if k in db["entries"]:
                iso += sum(db["entries"][k])
        gf, gb = measure_embedding_group(embs, a.batch_per_gpu, reps=a.reps, device=a.device, dtype=a.dtype)
        if iso > 0:
            db["group_factor"] = {"OP_EMBEDDING": round((gf + gb) / iso, 4)}
            print(f"[calibrate] embedding group of {len(embs)}: fwd {gf:.1f} us bwd {gb:.1f} us vs isolated "
                  f"{iso:.1f} us -> group_factor {db['group_factor']}", flush=True)
    _write(a.out, db, todo, cm)
    print(f"[calibrate] {len(db['entries'])} entries -> {a.out}; scales {db['scale']}", flush=True)


def _write(path, db, todo, cm):
    roof = {k: cm.roofline(*todo[k]) for k in db["entries"] if k in todo}
    fit = {t: round(v, 4) for t, v in cm.fit_scales({k: tuple(v) for k, v in db["entries"].items()}, roof).items()}
    keep = db.get("scale_keep", {})
    db["scale"] = {**fit, **keep}
    out = {k: v for k, v in db.items() if k != "scale_keep"}
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)


if __name__ == "__main__":
    main()
