"""SOAP strategy search: candidate configs -> native MI355X simulator -> Metropolis walk.

Reference: ``FFModel::optimize`` / ``rewrite`` (``src/runtime/model.cc:1082-1144``) start from
data parallelism, re-draw ONE op's ParallelConfig per step (``Op::get_random_parallel_config``,
``src/runtime/model.cc:295-324``), simulate (``src/runtime/simulator.cc:275-448``) and accept
with the Metropolis rule ``rand < exp(-alpha * (next - cur))``; the best strategy can be
exported to ``.pb`` but was never applied to the running model (caveat C6).

flexmi: every op gets an explicit, finite candidate list -- all degree vectors over the op's
SOAP-splittable dims (sample / attribute / parameter) whose product divides the device count,
each placed on every aligned contiguous device window (so table-wise embedding placement on
any single GPU is a candidate, as are column-parallel Linear groups and sub-node DP).  The
candidate tables (per-part costs from :mod:`flexmi.parallel.cost`, shard boxes, weight-sync
groups, per-device memory) are handed to the C++ simulator once (``csrc/sim/simulator.cc``);
the walk itself runs natively without the GIL.  The result IS applied: ``FFModel.compile``
installs the best strategy before ``init_layers``.
"""
from __future__ import annotations

import itertools
import json
import sys
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from flexmi.core.types import DataType, OperatorType
from flexmi.parallel.cost import CostModel
from flexmi.parallel.layout import Layout, ParallelConfig
from flexmi.parallel.machine import MachineModel

_FLOAT = (DataType.DT_FLOAT, DataType.DT_DOUBLE, DataType.DT_BF16, DataType.DT_HALF)


def _divisors(n):
    return [d for d in range(1, n + 1) if n % d == 0]


def candidate_configs(op, ndev: int, max_cands: int = 96) -> List[ParallelConfig]:
    """Enumerate valid ParallelConfigs of ``op`` on ``ndev`` devices (deterministic order;
    the data-parallel config first when valid)."""
    nd = op.out_ndims
    split = sorted(d for d in op.splittable_dims() if d < nd)
    out: List[ParallelConfig] = []
    seen = set()

    def add(pc):
        k = pc.key()
        if k not in seen and op.valid_pc(pc):
            seen.add(k)
            out.append(pc)

    add(ParallelConfig.data_parallel(nd, ndev))
    divs = _divisors(ndev)
    combos = []
    for degs in itertools.product(*[divs] * len(split)):
        p = 1
        for d in degs:
            p *= d
        if ndev % p == 0:
            combos.append(degs)
    combos.sort(key=lambda d: (-_prod(d), d))
    for degs in combos:
        user = [1] * nd
        for dim, d in zip(split, degs):
            user[dim] = d
        P = _prod(degs)
        for w in range(ndev // P):
            pc = ParallelConfig.from_user_degrees(user, list(range(w * P, (w + 1) * P)))
            add(pc)
            if len(out) >= max_cands:
                return out
    if not out:
        out.append(ParallelConfig([1] * nd, [0]))
    return out


def _prod(s):
    n = 1
    for d in s:
        n *= int(d)
    return n


def _box_shape(box):
    return tuple(hi - lo for lo, hi in box)


def _lay_parts(lay: Layout):
    return [(tuple(lo for lo, _ in lay.part_box(p)), tuple(hi for _, hi in lay.part_box(p)), tuple(lay.holders[p]))
            for p in range(lay.num_parts())]


@dataclass
class SearchResult:
    best: Dict[str, ParallelConfig]
    best_us: float
    init_us: float
    dp_us: float
    history: list = field(default_factory=list)
    accepted: int = 0
    iterations: int = 0
    seconds: float = 0.0

    @property
    def speedup_vs_dp(self):
        return self.dp_us / self.best_us if self.best_us > 0 else float("nan")

    def summary(self):
        return {"best_ms": self.best_us / 1e3, "dp_ms": self.dp_us / 1e3, "init_ms": self.init_us / 1e3,
                "speedup_vs_dp": self.speedup_vs_dp, "accepted": self.accepted, "iterations": self.iterations,
                "seconds": self.seconds}


def _rowwise(op):
    """Ops the executor runs as micro-batch chunks in a pipelined tail (Executor._plan_pipeline)."""
    return op.op_type in (OperatorType.OP_LINEAR, OperatorType.OP_DOT_INTERACTION) or (
        op.op_type == OperatorType.OP_CONCAT and op.axis != 0)


def auto_chunks(rows_per_gpu):
    """The executor's chunk count for a per-GPU batch (FLEXMI_XCHG_CHUNKS, default auto)."""
    from flexmi.runtime import executor as E
    if E.XCHG_CHUNKS != "auto":
        return max(1, int(E.XCHG_CHUNKS))
    return 2 if rows_per_gpu >= 1024 else 1


class SimGraph:
    """The model compiled into the native simulator's candidate tables."""

    def __init__(self, model, ndev: int, machine: Optional[MachineModel] = None, cost: Optional[CostModel] = None,
                 max_cands: int = 96, extra: Optional[Dict[str, ParallelConfig]] = None):
        from flexmi import _native
        self.model = model
        self.ndev = ndev
        self.machine = machine or MachineModel.mi355x(ndev)
        self.machine.ndev = ndev
        self.cost = cost or CostModel(self.machine, dtype_bytes=2 if model.config.compute_dtype == "bf16" else 4)
        opt = model.optimizer
        self.nstates = len(opt.state_names()) if opt is not None and hasattr(opt, "state_names") else 0
        self.sparse_ok = bool(getattr(opt, "sparse_capable", False))
        self.ops = list(model.layers)
        md = self.machine.native_dict()
        if not md["xchg_chunks"]:
            md["xchg_chunks"] = auto_chunks(model.config.batchSize // max(1, ndev))
        self.xchg_chunks = md["xchg_chunks"]
        self.sim = _native.Simulator(md)
        self.cands: List[List[ParallelConfig]] = []
        tid = {}
        for op in self.ops:
            for t in op.inputs:
                if t.guid not in tid:
                    prod = -1
                    if t.owner_op is not None:
                        raise RuntimeError(f"tensor {t.name} consumed before its producer {t.owner_op.name}")
                    tid[t.guid] = self.sim.add_tensor(self._eb(t), prod, 0, False)
            idx = len(self.cands)
            for j, o in enumerate(op.outputs):
                tid[o.guid] = self.sim.add_tensor(self._eb(o), idx, j, o.data_type in _FLOAT)
            cl = candidate_configs(op, ndev, max_cands)
            if extra and op.name in extra:
                pc = extra[op.name]
                if op.valid_pc(pc) and max(pc.device_ids) < ndev and pc not in cl:
                    cl.append(pc)
            self.cands.append(cl)
            self.sim.add_op(op.name, [tid[t.guid] for t in op.inputs], [tid[o.guid] for o in op.outputs],
                            [self._cand(op, pc) for pc in cl], ndev, _rowwise(op))

    def _eb(self, t):
        return self.cost.eb if t.data_type in _FLOAT else 8

    def _cand(self, op, pc: ParallelConfig):
        from flexmi.ops.embedding import Embedding
        outs = op.output_layouts(pc)
        ins = op.input_layouts(pc)
        wls = op.weight_layouts(pc)
        fwd, bwd = [], []
        mem, upd_bytes = {}, {}
        for p, dev in enumerate(pc.device_ids):
            in_shapes = []
            for lay in ins:
                ps = lay.parts_of(dev)
                in_shapes.append(_box_shape(lay.part_box(ps[0])) if ps else tuple(0 for _ in lay.shape))
            out_shapes = [_box_shape(lay.part_box(p)) for lay in outs]
            f, b = self.cost.op_cost(op, in_shapes, out_shapes)
            fwd.append(f)
            bwd.append(b)
            act = sum(_prod(s) for s in out_shapes)
            mem[dev] = mem.get(dev, 0.0) + act * self.cost.eb * 2
        wsync = []
        emb = op.op_type == OperatorType.OP_EMBEDDING
        for w, lay in zip(op.weights, wls):
            for p in range(lay.num_parts()):
                vol = _prod(_box_shape(lay.part_box(p)))
                h = lay.holders[p]
                sparse = emb and self.sparse_ok
                sdp_words = 0.0
                if sparse and len(h) > 1:
                    # the executor's per-table rule (Executor._sdp_pays): sparse DP only where the
                    # touched-row all-gather moves fewer bytes than the dense replica all-reduce
                    R = len(h)
                    B = op.inputs[0].dims[0]
                    bag = op.inputs[0].dims[1] if len(op.inputs[0].dims) > 1 else 1
                    box = lay.part_box(p)
                    rows = max(1, box[0][1] - box[0][0])
                    lookups = -(-B // R) * bag
                    sparse = Embedding.sdp_prefer_sparse(rows, vol // rows, lookups, R)
                    if sparse:
                        sdp_words = float(R * op.sdp_payload_words(lookups, vol // rows))
                if len(h) > 1:
                    if sparse:
                        # replicated table with the sparse optimizer = the executor's sparse data
                        # parallelism (Embedding.sdp_*): every replica all-gathers a fixed payload of
                        # its sample shard's lookups -- count + ids + fp32 row gradients, padded to
                        # one slot per lookup -- and applies all R segments.  A ring all-gather of
                        # R payloads moves what a ring all-reduce of R*payload/2 bytes moves.
                        R = len(h)
                        B = op.inputs[0].dims[0]
                        bag = op.inputs[0].dims[1] if len(op.inputs[0].dims) > 1 else 1
                        box = lay.part_box(p)
                        cols = vol // max(1, box[0][1] - box[0][0])
                        lookups = -(-B // R) * bag
                        payload = 4.0 * op.sdp_payload_words(lookups, cols)
                        wsync.append((R * payload / 2.0, list(h)))
                        for d in h:   # the apply: R segments of row read-modify-writes
                            upd_bytes[d] = upd_bytes.get(d, 0.0) + float(min(vol, B * bag * cols)) * 4.0
                    else:
                        wsync.append((float(vol * 4), list(h)))
                for d in h:
                    if sparse:
                        # the table + (sparse DP) the R-slot receive buffer of the all-gather
                        mem[d] = mem.get(d, 0.0) + vol * 4.0 + sdp_words * 4.0
                    else:
                        mem[d] = mem.get(d, 0.0) + vol * (4.0 + 4.0 + 2.0 + 4.0 * self.nstates)
                        upd_bytes[d] = upd_bytes.get(d, 0.0) + vol * 4.0
        W = self.ndev
        sample_only = (list(pc.device_ids) == list(range(W)) and all(
            l.degrees[0] == W and all(d == 1 for d in l.degrees[1:]) and l.replication() == 1 for l in outs + ins))
        return {"sample_only": sample_only, "part_dev": list(pc.device_ids), "fwd_us": fwd, "bwd_us": bwd,
                "out": [_lay_parts(l) for l in outs], "inp": [_lay_parts(l) for l in ins],
                "wsync": wsync, "mem": sorted(mem.items()),
                "upd": sorted((d, self.cost.update_us(b, self.nstates)) for d, b in upd_bytes.items()),
                "label": repr(pc)}

    # ------------------------------------------------------------------
    def dp_assign(self):
        out = []
        for op, cl in zip(self.ops, self.cands):
            dp = ParallelConfig.data_parallel(op.out_ndims, self.ndev)
            out.append(cl.index(dp) if dp in cl else 0)
        return out

    def assign_from(self, strategies: Dict[str, ParallelConfig]):
        a = self.dp_assign()
        for i, (op, cl) in enumerate(zip(self.ops, self.cands)):
            pc = strategies.get(op.name)
            if pc is not None and pc in cl:
                a[i] = cl.index(pc)
        return a

    def strategies(self, assign) -> Dict[str, ParallelConfig]:
        return {op.name: cl[a] for op, cl, a in zip(self.ops, self.cands, assign)}

    def simulate(self, assign):
        return self.sim.simulate(list(assign))

    def memory(self, assign):
        return self.sim.memory(list(assign))

    def chrome_trace(self, assign, path):
        """Predicted timeline (``chrome://tracing``): one row per GPU compute queue, collective
        channel and xGMI link (validate the cost model against rocprof)."""
        nd = self.ndev
        evs = []
        for name, kind, res, s, e in self.sim.trace(list(assign)):
            if res < nd:
                pid, tid = res, "compute"
            elif res < 2 * nd:
                pid, tid = res - nd, "collective"
            else:
                r = res - 2 * nd
                pid, tid = r // nd, f"xgmi->{r % nd}"
            evs.append({"name": f"{name}.{kind}", "ph": "X", "ts": s, "dur": max(e - s, 0.01), "pid": pid, "tid": tid,
                        "cat": kind})
        with open(path, "w") as f:
            json.dump({"traceEvents": evs, "displayTimeUnit": "ns"}, f)


def simulate(model, strategies=None, num_devices=None, machine=None, cost_db=None):
    n = num_devices or max(1, model.config.world_size)
    g = SimGraph(model, n, machine, CostModel(machine or MachineModel.mi355x(n), cost_db) if cost_db else None,
                 extra=strategies)
    return g.simulate(g.assign_from(strategies or {}))


def optimize(model, budget, alpha=1.0, num_devices=None, machine=None, cost_db=None, seed=0, init=None,
             verbose=None) -> SearchResult:
    """MCMC search (``FFModel::optimize``) over the native simulator; returns the best strategy."""
    n = num_devices or max(1, model.config.world_size)
    cfg = model.config
    if machine is None and getattr(cfg, "machine_file", None):
        machine = MachineModel.load(cfg.machine_file, n)
    machine = machine or MachineModel.mi355x(n)
    cost = CostModel(machine, cost_db if cost_db is not None else (getattr(cfg, "cost_db", "") or None),
                     dtype_bytes=2 if cfg.compute_dtype == "bf16" else 4)
    t0 = time.time()
    g = SimGraph(model, n, machine, cost, extra=init)
    dp = g.dp_assign()
    dp_us = g.simulate(dp)
    start = g.assign_from(init) if init else dp
    verbose = (cfg.rank == 0) if verbose is None else verbose
    best, best_us, init_us, hist, acc = g.sim.search(start, int(budget), float(alpha), int(seed), bool(verbose))
    res = SearchResult(g.strategies(best), best_us, init_us, dp_us, list(hist), acc, int(budget), time.time() - t0)
    res.graph = g
    res.assign = list(best)
    if verbose:
        print(f"[search] {n} devices, {budget} iters in {res.seconds:.1f}s: best {best_us / 1e3:.3f} ms/iter "
              f"(data parallel {dp_us / 1e3:.3f} ms, predicted speedup {res.speedup_vs_dp:.2f}x)", file=sys.stderr)
    return res


# machine corners of the sensitivity pass: every communication constant of the (spec-derived,
# uncalibrated above one GPU) MI355X model at half and at twice its value, one at a time, plus the
# all-pessimistic and all-optimistic combinations.  Reference: the simulator's fixed machine
# constants, src/runtime/simulator.cu:21-76.
SENS_KEYS = ("link_GBps", "link_lat_us", "ar_busbw_GBps", "ar_lat_us")


def machine_corners(base: MachineModel):
    corners = [("nominal", base)]
    for k in SENS_KEYS:
        for f in (0.5, 2.0):
            m = MachineModel(**{**base.__dict__})
            setattr(m, k, getattr(base, k) * f)
            corners.append((f"{k}x{f:g}", m))
    slow = MachineModel(**{**base.__dict__})
    fast = MachineModel(**{**base.__dict__})
    for k in SENS_KEYS:
        bw = k.endswith("GBps")
        setattr(slow, k, getattr(base, k) * (0.5 if bw else 2.0))
        setattr(fast, k, getattr(base, k) * (2.0 if bw else 0.5))
    corners += [("all_slow", slow), ("all_fast", fast)]
    return corners


def sensitivity(model, pick: Dict[str, ParallelConfig], base: Dict[str, ParallelConfig], num_devices, machine=None,
                cost_db=None):
    """Re-simulate the searched plan ``pick`` and a reference plan ``base`` (the hand-written table
    plan it was seeded with) on every machine corner.  Returns (rows, worst) with rows =
    [(corner, pick_us, base_us, pick_us / base_us)] and worst = the largest ratio: > 1.10 means
    the search's choice loses more than 10 % to the robust plan if a constant is off by 2x."""
    n = num_devices
    machine = machine or MachineModel.mi355x(n)
    rows = []
    for name, m in machine_corners(machine):
        m.ndev = n
        cost = CostModel(m, cost_db, dtype_bytes=2 if model.config.compute_dtype == "bf16" else 4)
        us = []
        for plan in (pick, base):
            g = SimGraph(model, n, m, cost, extra=plan)
            us.append(g.simulate(g.assign_from(plan)))
        rows.append((name, us[0], us[1], us[0] / us[1]))
    return rows, max(r[3] for r in rows)
