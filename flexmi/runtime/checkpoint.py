"""Sharded checkpoint / resume with reshard-on-load.

The reference persisted nothing but the strategy ``.pb`` (``src/runtime/strategy.cc:137-172``);
training state was only reachable through ``Parameter::get_weights`` (``src/runtime/model.cu:260-334``).

flexmi writes, per rank, every parameter shard it is the FIRST holder of (replicas of
data-parallel weights are written once) together with its optimizer state (SGD velocity, Adam
m/v), plus a manifest with each shard's global box, the step counters (Adam β1ᵗ/β2ᵗ/α_t, the
device-side counters), the data position and the strategy.  Shards are one file per (rank,
parameter) so a 20 GB embedding table never has to pass through a single buffer, and they are
read back with ``torch.load(weights_only=True, mmap=True)``.  Loading intersects every local
shard box with the saved boxes, so a checkpoint written under one strategy / world size resumes
under any other (DP <-> table-wise <-> column-split, 2 ranks -> 1 or 4, ...).
"""
from __future__ import annotations

import json
import os
import re
from typing import Dict

import torch

FORMAT = "flexmi-ckpt-1"


def _fname(name):
    return re.sub(r"[^A-Za-z0-9_.-]", "_", name)


def _inter(a, b):
    out = []
    for (alo, ahi), (blo, bhi) in zip(a, b):
        lo, hi = max(alo, blo), min(ahi, bhi)
        if lo >= hi:
            return None
        out.append((lo, hi))
    return out


def _sl(box, origin):
    return tuple(slice(lo - o, hi - o) for (lo, hi), o in zip(box, origin))


def _keys(model):
    """Stable parameter keys: (layer position, weight index) -- auto-generated op names carry a
    process-local guid, so they are recorded for readability only."""
    out = {}
    for li, op in enumerate(model.layers):
        for wi, w in enumerate(op.weights):
            out[w.guid] = f"L{li}.{type(op).__name__}.w{wi}"
    return out


def save_checkpoint(model, path, extra: Dict = None):
    """Collective over all ranks of the model."""
    ex = model._ex()
    rank, world = ex.rank, ex.world
    os.makedirs(os.path.join(path, f"r{rank}"), exist_ok=True)
    if ex.backend == "hip":
        torch.cuda.synchronize()
    entries = []
    keys = _keys(model)
    ex.zero_materialize_state()          # ZeRO-1: gather the sharded optimizer state (collective)
    for e in ex.wentries.values():
        if e.box is None or (e.holders and e.holders[0] != rank):
            continue
        name = keys[e.param.guid]
        f = os.path.join(f"r{rank}", _fname(name) + ".pt")
        blob = {"master": e.master.detach().to("cpu").contiguous()}
        for sname, st in e.state.items():
            blob["state." + sname] = st.detach().to("cpu").contiguous()
        torch.save(blob, os.path.join(path, f))
        entries.append({"param": name, "name": e.param.name, "shape": list(e.param.dims),
                        "box": [list(b) for b in e.box], "file": f, "states": sorted(e.state)})
    with open(os.path.join(path, f"r{rank}", "shards.json"), "w") as fh:
        json.dump(entries, fh)
    ex.zero_release_state()
    ex.comm.barrier()
    if rank == 0:
        opt = model.optimizer
        man = {
            "format": FORMAT,
            "world": world,
            "step": ex.step_count,
            "optimizer": {"type": type(opt).__name__, "state": opt.state_dict() if opt else {}},
            "device_adam_state": [float(v) for v in ex.adam_state.detach().cpu()],
            "strategy": {op.name: {"dims": list(ex.pcs[op.guid].dims), "device_ids": list(ex.pcs[op.guid].device_ids)}
                         for op in model.layers},
            "ranks": list(range(world)),
            "extra": extra or {},
        }
        with open(os.path.join(path, "manifest.json"), "w") as fh:
            json.dump(man, fh, indent=1)
        from flexmi.parallel import strategy as S
        S.save_strategies_to_file(os.path.join(path, "strategy.pb"), dict(ex.pcs_by_name()))
    ex.comm.barrier()
    return path


def load_checkpoint(model, path, strict=True):
    """Collective.  Fills every local parameter shard (and optimizer state) of the running
    model from the saved shards, whatever strategy / world size wrote them."""
    ex = model._ex()
    with open(os.path.join(path, "manifest.json")) as fh:
        man = json.load(fh)
    if man.get("format") != FORMAT:
        raise ValueError(f"{path}: not a {FORMAT} checkpoint")
    shards: Dict[str, list] = {}
    for r in man["ranks"]:
        with open(os.path.join(path, f"r{r}", "shards.json")) as fh:
            for ent in json.load(fh):
                shards.setdefault(ent["param"], []).append(ent)
    cache = {}

    def blob(f):
        if f not in cache:
            cache[f] = torch.load(os.path.join(path, f), map_location="cpu", weights_only=True, mmap=True)
        return cache[f]

    keys = _keys(model)
    ex.zero_materialize_state()
    for e in ex.wentries.values():
        if e.box is None:
            continue
        name = keys[e.param.guid]
        got = shards.get(name)
        if not got:
            if strict:
                raise KeyError(f"checkpoint has no parameter {name!r}")
            continue
        mine = [tuple(b) for b in e.box]
        origin = [lo for lo, _ in mine]
        covered = 0
        for ent in got:
            if list(ent["shape"]) != list(e.param.dims):
                raise ValueError(f"{name}: checkpoint shape {ent['shape']} != model {list(e.param.dims)}")
            sbox = [tuple(b) for b in ent["box"]]
            it = _inter(mine, sbox)
            if it is None:
                continue
            b = blob(ent["file"])
            src = _sl(it, [lo for lo, _ in sbox])
            dst = _sl(it, origin)
            e.master[dst].copy_(b["master"][src])
            for sname, st in e.state.items():
                key = "state." + sname
                if key in b:
                    st[dst].copy_(b[key][src])
            vol = 1
            for lo, hi in it:
                vol *= hi - lo
            covered += vol
        if strict and covered != e.numel:
            raise ValueError(f"{name}: checkpoint covers {covered} of {e.numel} local elements")
    ex.zero_release_state(scatter=True)
    for g in ex.groups:
        if g.compute is not g.master:
            g.compute.copy_(g.master)
    ex.step_count = int(man["step"])
    opt = model.optimizer
    if opt is not None and man["optimizer"]["type"] == type(opt).__name__:
        opt.load_state_dict(man["optimizer"]["state"])
        if hasattr(opt, "lr"):
            ex.set_lr(opt.lr)
    ex.adam_state.copy_(torch.tensor(man["device_adam_state"], dtype=torch.float32))
    if ex.backend == "hip":
        torch.cuda.synchronize()
    return man
