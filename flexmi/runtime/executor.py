"""Per-rank plan compiler + executor (SPMD: one process per GPU).

Replaces the reference's Legion machinery -- index launches per op (``src/runtime/model.cc``
``FFModel::forward/backward/update`` ``:948-993``), the FFMapper's point-task placement
(``src/mapper/mapper.cc:33-97``), region partitions and implicit DMA.  ``Executor.build``
compiles (graph, strategy, rank) into:

  * a layout for every tensor (producer's output partition) and every consumer view of it;
  * explicit reshard steps (one ``all_to_all`` each) wherever a consumer needs a different
    distribution than the producer made -- including partial-sum reductions in backward;
  * flat fp32 master/grad/optimizer-state buffers per gradient-sync group with bf16 compute
    mirrors, bucketed for async RCCL all-reduce overlapped with backward;
  * a fused sparse-SGD path for non-replicated embedding tables (no dense gradient).

All buffers are allocated once, so the whole step can be captured in a hipGraph
(``Executor.capture_step``) -- the analogue of Legion tracing (``dlrm.cc:178-185``).
"""
from __future__ import annotations

import math
import time
from collections import OrderedDict, defaultdict
from typing import Dict, List

import numpy as np
import torch

from flexmi.core.loss_metrics import NUM_SLOTS, PerfMetrics, loss_and_metrics_torch
from flexmi.core.optimizers import AdamOptimizer, SGDOptimizer
from flexmi.core.types import DataType, LossType, to_torch_dtype
from flexmi.ops.base import OpCtx
from flexmi.parallel.layout import Layout, ParallelConfig, ReshardPlan
from flexmi.utils.profiling import OpTimer


def _is_float(dt):
    return DataType(dt) in (DataType.DT_FLOAT, DataType.DT_DOUBLE, DataType.DT_BF16, DataType.DT_HALF)


def _slices(box, lo_box):
    return tuple(slice(b[0] - l[0], b[1] - l[0]) for b, l in zip(box, lo_box))


class ReshardStep:
    """One planned repartition of a tensor (forward copy or backward partial-sum reduce)."""

    def __init__(self, plan: ReshardPlan, rank, world, dtype=torch.float32, device=None):
        self.plan = plan
        self.dtype = dtype
        self.device = device
        self.rank = rank
        self.world = world
        self.local_only = all(t.src == t.dst for t in plan.transfers)
        self.sends = plan.sends_of(rank)
        self.recvs = plan.recvs_of(rank)
        self.recv_numel = [0] * world
        for t in self.recvs:
            n = 1
            for lo, hi in t.box:
                n *= hi - lo
            self.recv_numel[t.src] += n

    def run(self, comm, src_buf, dst_buf, accumulate=False):
        """src_buf: this rank's shard of the source layout (or None); dst_buf likewise."""
        plan, r = self.plan, self.rank
        reduce = plan.src.partial
        src_box = plan.src.local_box(r) if src_buf is not None else None
        dst_box = plan.dst.local_box(r) if dst_buf is not None else None
        if dst_buf is not None and (reduce or not self._covers()) and not accumulate:
            dst_buf.zero_()
            accumulate = True if reduce else accumulate
        if self.local_only or comm.world == 1:
            for t in self.recvs:
                piece = src_buf[_slices(t.box, src_box)]
                self._put(dst_buf, dst_box, t.box, piece, accumulate or reduce)
            return
        dtype, device = self.dtype, self.device
        send = [None] * comm.world
        per_peer = defaultdict(list)
        for t in self.sends:
            per_peer[t.dst].append(src_buf[_slices(t.box, src_box)].reshape(-1))
        for p, lst in per_peer.items():
            send[p] = torch.cat(lst) if len(lst) > 1 else lst[0]
        chunks = comm.all_to_all(send, self.recv_numel, dtype, device)
        offs = [0] * comm.world
        for t in self.recvs:
            shape = tuple(hi - lo for lo, hi in t.box)
            n = 1
            for s in shape:
                n *= s
            piece = chunks[t.src][offs[t.src]: offs[t.src] + n].view(shape)
            offs[t.src] += n
            self._put(dst_buf, dst_box, t.box, piece, accumulate or reduce)

    def _covers(self):
        return True

    @staticmethod
    def _put(dst_buf, dst_box, box, piece, add):
        v = dst_buf[_slices(box, dst_box)]
        if add:
            v.add_(piece.to(v.dtype))
        else:
            v.copy_(piece)


class WeightEntry:
    def __init__(self, param, op, widx, layout, rank):
        self.param = param
        self.op = op
        self.widx = widx
        self.layout = layout
        self.box = layout.local_box(rank)
        self.shape = tuple(hi - lo for lo, hi in self.box) if self.box is not None else None
        part = layout.parts_of(rank)
        self.holders = layout.holders[part[0]] if part else ()
        self.numel = int(np.prod(self.shape)) if self.shape else 0
        self.master = None
        self.grad = None
        self.compute = None
        self.state = {}
        self.sparse = False
        self.group = None
        self.offset = 0


class SyncGroup:
    """Weights sharing the same replica set: one flat master/grad/state/compute buffer."""

    def __init__(self, holders):
        self.holders = tuple(holders)
        self.entries: List[WeightEntry] = []
        self.numel = 0
        self.buckets = []  # list of (start, end, set(entry ids))

    @property
    def replicated(self):
        return len(self.holders) > 1


class Executor:
    def __init__(self, model, strategies: Dict[str, ParallelConfig], comm, optimizer, loss_type,
                 metrics, label_tensor):
        self.model = model
        self.cfg = model.config
        self.comm = comm
        self.rank = comm.rank
        self.world = comm.world
        self.backend = "hip" if self.cfg.device == "gpu" else "cpu"
        self.device = self.cfg.torch_device
        self.cdtype = torch.bfloat16 if (self.backend == "hip" and self.cfg.compute_dtype == "bf16") else torch.float32
        self.optimizer = optimizer
        self.loss_type = LossType(loss_type) if loss_type is not None else None
        self.metrics_obj = metrics
        self.label = label_tensor
        self.strategies = strategies
        self.timer = OpTimer(self.cfg.profiling, self.backend == "hip")
        self.training = True
        self.step_count = 0
        self._graph = None
        self.build()

    # ================================================================== build
    def pc_of(self, op):
        return self.pcs[op.guid]

    def _storage_dtype(self, t):
        if _is_float(t.data_type):
            return self.cdtype
        return to_torch_dtype(t.data_type)

    def _alloc(self, shape, dtype):
        return torch.empty(shape, dtype=dtype, device=self.device)

    def build(self):
        m = self.model
        ops = m.layers
        self.pcs = {}
        for op in ops:
            pc = self.strategies.get(op.name)
            if pc is None or not op.valid_pc(pc) or max(pc.device_ids) >= self.world:
                pc = ParallelConfig.data_parallel(op.out_ndims, self.world)
                if not op.valid_pc(pc):
                    pc = ParallelConfig([1] * op.out_ndims, [0])
            self.pcs[op.guid] = pc

        # ---- tensor layouts ---------------------------------------------------
        self.home: Dict[int, Layout] = {}
        self.consumers = defaultdict(list)     # guid -> [(op, idx)]
        self.need: Dict[tuple, Layout] = {}    # (op guid, input idx) -> layout
        for op in ops:
            pc = self.pcs[op.guid]
            for i, lay in enumerate(op.output_layouts(pc)):
                self.home[op.outputs[i].guid] = lay
            for i, lay in enumerate(op.input_layouts(pc)):
                t = op.inputs[i]
                self.need[(op.guid, i)] = lay
                self.consumers[t.guid].append((op, i))
                if t.owner_op is None and t.guid not in self.home:
                    self.home[t.guid] = lay.as_full()  # model input: first consumer's layout
        self.tensors = {}
        for op in ops:
            for t in op.inputs + op.outputs:
                self.tensors[t.guid] = t

        # ---- activation buffers ------------------------------------------------
        self.act: Dict[tuple, torch.Tensor] = {}
        self.grad: Dict[int, torch.Tensor] = {}
        for g, lay in self.home.items():
            t = self.tensors[g]
            shp = lay.local_shape(self.rank)
            if shp is not None:
                self.act[(g, lay.key())] = self._alloc(shp, self._storage_dtype(t))
        # view ops alias their input buffer (zero-copy Flat/Reshape)
        for op in ops:
            if getattr(op, "is_view", False):
                x = op.inputs[0]
                need = self.need[(op.guid, 0)]
                if need.same_as(self.home[x.guid]) and (x.guid, need.key()) in self.act:
                    out = op.outputs[0]
                    olay = self.home[out.guid]
                    src = self.act[(x.guid, need.key())]
                    self.act[(out.guid, olay.key())] = src.view(olay.local_shape(self.rank))

        # ---- forward/backward schedules ----------------------------------------
        self.fwd_steps = []
        self.bwd_steps = []
        for op in ops:
            pc = self.pcs[op.guid]
            for i, t in enumerate(op.inputs):
                need = self.need[(op.guid, i)]
                home = self.home[t.guid]
                if not need.same_as(home):
                    key = (t.guid, need.key())
                    if key not in self.act and need.local_shape(self.rank) is not None:
                        self.act[key] = self._alloc(need.local_shape(self.rank), self._storage_dtype(t))
                    self.fwd_steps.append(("reshard", t.guid, home, need, ReshardStep(ReshardPlan(home, need), self.rank, self.world, self._storage_dtype(t), self.device)))
            self.fwd_steps.append(("op", op))

        # grads: home-layout grad buffers for float tensors that need them
        self.grad_needed = set()
        for op in ops:
            for i, t in enumerate(op.inputs):
                if t.owner_op is not None and op.needs_input_grad(i) and _is_float(t.data_type):
                    self.grad_needed.add(t.guid)
        final = ops[-1].outputs[0]
        self.final = final
        self.grad_needed.add(final.guid)
        # outputs of ops whose inputs need grads must have grads too (transitively handled:
        # every op output that is consumed by a grad-needing op or is final)
        for g in list(self.grad_needed):
            pass
        for g in self.grad_needed:
            lay = self.home[g]
            shp = lay.local_shape(self.rank)
            if shp is not None:
                key = (g, lay.key())
                if getattr(self.tensors[g].owner_op, "is_view", False) and key in self.act:
                    pass
                self.grad[g] = self._alloc(shp, self.cdtype)
        # grads of view-op outputs alias the input grad buffer
        self.galias = {}
        for op in ops:
            if getattr(op, "is_view", False):
                x, out = op.inputs[0], op.outputs[0]
                if x.guid in self.grad and out.guid in self.grad and self.need[(op.guid, 0)].same_as(self.home[x.guid]):
                    self.grad[out.guid] = self.grad[x.guid].view(self.grad[out.guid].shape)
                    self.galias[out.guid] = self.gkey(x.guid)
        self.tmp_grad: Dict[tuple, torch.Tensor] = {}
        for op in reversed(ops):
            self.bwd_steps.append(("op", op))
            for i, t in enumerate(op.inputs):
                if t.guid not in self.grad_needed or not op.needs_input_grad(i):
                    continue
                need = self.need[(op.guid, i)]
                home = self.home[t.guid]
                if not need.same_as(home):
                    shp = need.local_shape(self.rank)
                    if shp is not None:
                        self.tmp_grad[(op.guid, i)] = self._alloc(shp, self.cdtype)
                    self.bwd_steps.append(("reduce", op, i, t.guid,
                                           ReshardStep(ReshardPlan(need.as_partial(), home), self.rank, self.world, self.cdtype, self.device)))

        # ---- weights ------------------------------------------------------------
        self._build_weights(ops)

        # ---- loss / label -------------------------------------------------------
        self._build_loss()

        # ---- op contexts --------------------------------------------------------
        self.ctx: Dict[int, OpCtx] = {}
        for op in ops:
            pc = self.pcs[op.guid]
            if self.rank not in pc.device_ids:
                continue
            c = OpCtx(op, self.rank, self.backend, self.cdtype)
            for i, t in enumerate(op.inputs):
                need = self.need[(op.guid, i)]
                c.inputs.append(self.act.get((t.guid, need.key())))
                c.in_boxes.append(need.local_box(self.rank))
                if t.guid in self.grad_needed and op.needs_input_grad(i):
                    if need.same_as(self.home[t.guid]):
                        c.in_grads.append(self.grad.get(t.guid))
                    else:
                        c.in_grads.append(self.tmp_grad.get((op.guid, i)))
                else:
                    c.in_grads.append(None)
                c.in_grad_accumulate.append(False)
            for o in op.outputs:
                lay = self.home[o.guid]
                c.outputs.append(self.act.get((o.guid, lay.key())))
                c.out_boxes.append(lay.local_box(self.rank))
                c.out_grads.append(self.grad.get(o.guid))
            for wi, w in enumerate(op.weights):
                e = self.wentries.get(w.guid)
                c.weights.append(e.master if e else None)
                c.wcompute.append(e.compute if e else None)
                c.weight_grads.append(e.grad if e else None)
                c.w_boxes.append(e.box if e else None)
            c.lr = self.lr_tensor
            op.prepare(c)
            self.ctx[op.guid] = c
        self.grad_written = set()
        self._build_groups(ops)

    def _build_groups(self, ops):
        """Fuse independent ops of the same kind and placement into one launch (embedding
        tables of a DLRM graph: 26 ops -> 1 forward + 2 backward launches).  Members run at the
        first member's position in forward and at the last position (in backward order, i.e.
        the first member) in backward, when every member's output gradient is final."""
        from flexmi.core.types import OperatorType
        self.group_of = {}
        groups = []
        for op in ops:
            c = self.ctx.get(op.guid)
            if c is None or op.op_type != OperatorType.OP_EMBEDDING:
                continue
            pc = self.pcs[op.guid]
            for g in groups:
                lead = g[0]
                if (self.pcs[lead.guid] == pc and type(lead).can_group(lead, op, self.ctx[lead.guid], c)):
                    g.append(op)
                    break
            else:
                groups.append([op])
        for g in groups:
            if len(g) > 1:
                for op in g:
                    self.group_of[op.guid] = g

    # ------------------------------------------------------------------
    def _build_weights(self, ops):
        self.wentries: Dict[int, WeightEntry] = {}
        groups: "OrderedDict[tuple, SyncGroup]" = OrderedDict()
        sparse_ok = isinstance(self.optimizer, SGDOptimizer) and self.optimizer.sparse_capable
        for op in reversed(ops):  # backward order => buckets fill contiguously
            pc = self.pcs[op.guid]
            lays = op.weight_layouts(pc)
            for wi, w in enumerate(op.weights):
                e = WeightEntry(w, op, wi, lays[wi], self.rank)
                self.wentries[w.guid] = e
                if e.box is None:
                    continue
                from flexmi.core.types import OperatorType
                if (op.op_type == OperatorType.OP_EMBEDDING and sparse_ok and lays[wi].replication() == 1):
                    e.sparse = True
                    op.sparse_sgd = True
                    e.master = self._alloc(e.shape, torch.float32)
                    e.compute = e.master
                    continue
                key = e.holders
                if key not in groups:
                    groups[key] = SyncGroup(key)
                g = groups[key]
                e.group = g
                e.offset = g.numel
                g.numel += (e.numel + 63) // 64 * 64  # 256-B aligned views: 16-B vector loads in every kernel
                g.entries.append(e)
        self.groups = list(groups.values())
        mixed = self.cdtype != torch.float32
        for g in self.groups:
            g.master = self._alloc((g.numel,), torch.float32)
            g.gradbuf = self._alloc((g.numel,), torch.float32)
            g.gradbuf.zero_()
            g.compute = self._alloc((g.numel,), self.cdtype) if mixed else g.master
            g.state = {n: torch.zeros(g.numel, dtype=torch.float32, device=self.device)
                       for n in (self.optimizer.state_names() if self.optimizer else [])}
            for e in g.entries:
                sl = slice(e.offset, e.offset + e.numel)
                e.master = g.master[sl].view(e.shape)
                e.grad = g.gradbuf[sl].view(e.shape)
                e.compute = g.compute[sl].view(e.shape)
                e.state = {n: s[sl].view(e.shape) for n, s in g.state.items()}
            # buckets (only meaningful for replicated groups)
            cap = max(1, int(self.cfg.grad_bucket_mb * (1 << 20) / 4))
            start, ids = 0, set()
            for e in g.entries:
                end = e.offset + (e.numel + 63) // 64 * 64
                if ids and end - start > cap:
                    g.buckets.append([start, e.offset, ids])
                    start, ids = e.offset, set()
                ids.add(e.param.guid)
            if ids:
                g.buckets.append([start, g.numel, ids])
        # communicators for every replicated subset, created in the same order everywhere
        all_sets = []
        for op in ops:
            for lay in op.weight_layouts(self.pcs[op.guid]):
                for h in lay.holders:
                    if len(h) > 1 and tuple(sorted(h)) not in all_sets:
                        all_sets.append(tuple(sorted(h)))
        for s in all_sets:
            self.comm.group_for(s)
        # initialise every shard directly from the counter-based initializers
        for e in self.wentries.values():
            if e.box is None:
                continue
            init = e.param.initializer
            from flexmi.core.initializers import ZeroInitializer
            (init or ZeroInitializer()).fill(e.param.dims, e.box, e.master)
        for g in self.groups:
            if g.compute is not g.master:
                g.compute.copy_(g.master)
        lr = getattr(self.optimizer, "lr", 0.01) if self.optimizer else 0.0
        self.lr_tensor = torch.tensor([lr], dtype=torch.float32, device=self.device)
        self.pending = {}

    def set_lr(self, lr):
        self.lr_tensor.fill_(float(lr))

    def _build_loss(self):
        final = self.final
        # BCE on a sigmoid output: the loss kernel emits dL/dz = p - y (numerically exact), so the
        # producing op must not apply the sigmoid derivative again (fused sigmoid + BCE).
        if self.loss_type == LossType.LOSS_BINARY_CROSSENTROPY:
            from flexmi.core.types import ActiMode, OperatorType
            fop = final.owner_op
            if getattr(fop, "activation", None) == ActiMode.AC_MODE_SIGMOID:
                fop.skip_act_grad = True
            elif fop.op_type == OperatorType.OP_SIGMOID:
                fop.skip_act_grad = True
            else:
                raise ValueError("LOSS_BINARY_CROSSENTROPY expects the model to end in a sigmoid "
                                 "(dense(..., AC_MODE_SIGMOID) or sigmoid())")
        home = self.home[final.guid]
        deg = [1] * len(final.dims)
        deg[0] = home.degrees[0]
        # loss layout: same sample split, other dims whole (one holder per sample part)
        holders = []
        for i in range(deg[0]):
            hs = [home.holders[p] for p in range(home.num_parts()) if home.part_coords(p)[0] == i]
            holders.append((hs[0][0],))
        self.loss_layout = Layout(final.dims, tuple(deg), holders)
        self.loss_reshard = None
        if not self.loss_layout.same_as(home):
            self.loss_reshard = ReshardStep(ReshardPlan(home, self.loss_layout), self.rank, self.world, self.cdtype, self.device)
            self.loss_back = ReshardStep(ReshardPlan(self.loss_layout.as_partial(), home), self.rank, self.world, self.cdtype, self.device)
        shp = self.loss_layout.local_shape(self.rank)
        self.logits_buf = None
        self.logit_grad = None
        if shp is not None:
            if self.loss_reshard is None:
                self.logits_buf = self.act[(final.guid, home.key())]
                self.logit_grad = self.grad[final.guid]
            else:
                self.logits_buf = self._alloc(shp, self.cdtype)
                self.logit_grad = self._alloc(shp, self.cdtype)
        # label
        lab = self.label
        if lab is not None:
            ldeg = [1] * len(lab.dims)
            ldeg[0] = deg[0]
            self.label_layout = Layout(lab.dims, tuple(ldeg), holders)
            self.home[lab.guid] = self.label_layout
            self.tensors[lab.guid] = lab
            lshp = self.label_layout.local_shape(self.rank)
            ldt = torch.float32 if _is_float(lab.data_type) else to_torch_dtype(lab.data_type)
            self.label_buf = self._alloc(lshp, ldt) if lshp is not None else None
            if self.label_buf is not None:
                self.label_buf.zero_()
            self.act[(lab.guid, self.label_layout.key())] = self.label_buf
        self.metric_acc = torch.zeros(NUM_SLOTS, dtype=torch.float32, device=self.device)

    def gkey(self, g):
        while g in self.galias:
            g = self.galias[g]
        return g

    # ================================================================== run
    def local_buffer(self, t):
        lay = self.home[t.guid]
        return self.act.get((t.guid, lay.key()))

    def forward(self):
        tm = self.timer
        for st in self.fwd_steps:
            if st[0] == "reshard":
                _, g, home, need, rs = st
                src = self.act.get((g, home.key()))
                dst = self.act.get((g, need.key()))
                rs.run(self.comm, src, dst)
            else:
                op = st[1]
                c = self.ctx.get(op.guid)
                if c is not None:
                    c.training = self.training
                    grp = self.group_of.get(op.guid)
                    if grp is not None:
                        if grp[0] is op:
                            with tm.scope(op.name + ".group_fwd"):
                                type(op).forward_group(grp, [self.ctx[o.guid] for o in grp])
                        continue
                    with tm.scope(op.name + ".fwd"):
                        op.forward(c)

    def zero_gradients(self):
        """Reference semantics (``model.cc:1146-1169``): gradients start at zero.  flexmi
        kernels overwrite on first write, so this only resets the bookkeeping."""
        self.grad_written = set()

    def backward(self):
        tm = self.timer
        self.grad_written = set()
        # 1. loss gradient (+ metrics) ----------------------------------------
        with tm.scope("loss"):
            self._loss_step(compute_grad=True)
        self.grad_written.add(self.gkey(self.final.guid))
        # 2. reverse ops ------------------------------------------------------
        self.pending = {}
        for g in self.groups:
            if g.replicated:
                g.bucket_left = [len(b[2]) for b in g.buckets]
                g.works = [None] * len(g.buckets)
        for st in self.bwd_steps:
            if st[0] == "op":
                op = st[1]
                c = self.ctx.get(op.guid)
                if c is not None:
                    for i, t in enumerate(op.inputs):
                        if c.in_grads[i] is not None and self.need[(op.guid, i)].same_as(self.home[t.guid]):
                            c.in_grad_accumulate[i] = self.gkey(t.guid) in self.grad_written
                        else:
                            c.in_grad_accumulate[i] = False
                    if all(g is None for g in c.out_grads) and not op.weights:
                        pass
                    for o in op.outputs:
                        if o.guid in self.grad and self.gkey(o.guid) not in self.grad_written:
                            self.grad[o.guid].zero_()   # unused output
                            self.grad_written.add(self.gkey(o.guid))
                    grp = self.group_of.get(op.guid)
                    if grp is not None:
                        if grp[0] is op:
                            with tm.scope(op.name + ".group_bwd"):
                                type(op).backward_group(grp, [self.ctx[o.guid] for o in grp])
                    else:
                        with tm.scope(op.name + ".bwd"):
                            op.backward(c)
                    for i, t in enumerate(op.inputs):
                        if c.in_grads[i] is not None and self.need[(op.guid, i)].same_as(self.home[t.guid]):
                            self.grad_written.add(self.gkey(t.guid))
                self._weights_done(op)
            else:
                _, op, i, g, rs = st
                src = self.tmp_grad.get((op.guid, i))
                dst = self.grad.get(g)
                acc = self.gkey(g) in self.grad_written
                rs.run(self.comm, src, dst, accumulate=acc)
                self.grad_written.add(self.gkey(g))

    def _weights_done(self, op):
        for w in op.weights:
            e = self.wentries.get(w.guid)
            if e is None or e.group is None or not e.group.replicated:
                continue
            g = e.group
            for bi, b in enumerate(g.buckets):
                if w.guid in b[2]:
                    g.bucket_left[bi] -= 1
                    if g.bucket_left[bi] == 0 and self.cfg.overlap_grad_sync:
                        g.works[bi] = self.comm.all_reduce_async(g.gradbuf[b[0]:b[1]], g.holders)

    def _sync_grads(self):
        for g in self.groups:
            if not g.replicated:
                continue
            for bi, b in enumerate(g.buckets):
                w = g.works[bi] if hasattr(g, "works") else None
                if w is None:
                    w = self.comm.all_reduce_async(g.gradbuf[b[0]:b[1]], g.holders)
                if w is not None:
                    w.wait()
                g.works[bi] = None

    def update(self):
        from flexmi.ops import _kernels as K
        self._sync_grads()
        opt = self.optimizer
        if opt is None:
            return
        opt.next()
        with self.timer.scope("update"):
            for g in self.groups:
                if g.numel == 0:
                    continue
                if self.backend == "hip":
                    if isinstance(opt, SGDOptimizer):
                        K.sgd_update(g.master, g.gradbuf, g.state.get("v"), g.compute if g.compute is not g.master else None,
                                     self.lr_tensor, opt.weight_decay, opt.momentum, opt.nesterov)
                    else:
                        K.adam_update(g.master, g.gradbuf, g.state["m"], g.state["v"],
                                      g.compute if g.compute is not g.master else None,
                                      opt.alpha_t, opt.beta1, opt.beta2, opt.weight_decay, opt.epsilon)
                else:
                    if isinstance(opt, SGDOptimizer):
                        st = {"v": g.state["v"]} if "v" in g.state else {}
                        gt = g.gradbuf + opt.weight_decay * g.master
                        if opt.momentum > 0:
                            st["v"].mul_(opt.momentum).add_(gt)
                            gt = gt + opt.momentum * st["v"] if opt.nesterov else st["v"]
                        g.master.sub_(self.lr_tensor * gt)
                    else:
                        opt.update_torch(g.master, g.gradbuf, g.state)
                    if g.compute is not g.master:
                        g.compute.copy_(g.master)
        self.step_count += 1

    # ------------------------------------------------------------------ loss
    def _loss_step(self, compute_grad):
        from flexmi.ops import _kernels as K
        if self.loss_type is None:
            return
        if self.loss_reshard is not None:
            self.loss_reshard.run(self.comm, self.local_buffer(self.final), self.logits_buf)
        if self.logits_buf is not None:
            scale = 1.0 / self.final.dims[0]
            mask = self.metrics_obj.mask if self.metrics_obj else 0
            if self.backend == "hip":
                K.loss_forward_backward(int(self.loss_type), self.logits_buf, self.label_buf,
                                        self.logit_grad if compute_grad else None, scale,
                                        self.metric_acc, mask)
            else:
                loss_and_metrics_torch(self.loss_type, self.logits_buf, self.label_buf, self.logit_grad,
                                       scale, self.metric_acc, mask, compute_grad)
        if compute_grad and self.loss_reshard is not None:
            self.loss_back.run(self.comm, self.logit_grad, self.grad.get(self.final.guid))

    def compute_metrics(self):
        self._loss_step(compute_grad=False)

    def reset_metrics(self):
        self.metric_acc.zero_()

    def perf_metrics(self):
        acc = self.metric_acc.clone()
        if self.world > 1:
            self.comm.all_reduce(acc)
        return PerfMetrics(acc.cpu().double().numpy(), self.metrics_obj.metrics if self.metrics_obj else [])

    # ------------------------------------------------------------------ host views
    def _gather_full(self, lay: Layout, local, dtype):
        full_shape = lay.shape
        out = torch.zeros(full_shape, dtype=dtype)
        if self.world == 1:
            box = lay.local_box(0)
            out[_slices(box, tuple((0, 0) for _ in box))] = local.detach().to("cpu", dtype)
            return out
        # replicate to everyone through a reshard to a fully replicated layout
        rep = Layout.replicated(lay.shape, list(range(self.world)))
        sdt = local.dtype if local is not None else (self.cdtype if dtype == torch.float32 else dtype)
        rs = ReshardStep(ReshardPlan(lay.as_full(), rep), self.rank, self.world, sdt, self.device)
        dst = torch.empty(full_shape, dtype=sdt, device=self.device)
        rs.run(self.comm, local, dst)
        return dst.to("cpu", dtype)

    def gather_to_host(self, t):
        lay = self.home.get(t.guid)
        buf = self.local_buffer(t)
        dt = torch.float32 if _is_float(t.data_type) else to_torch_dtype(t.data_type)
        return self._gather_full(lay, buf, dt).numpy()

    def scatter_from_host(self, t, arr):
        lay = self.home.get(t.guid)
        buf = self.local_buffer(t)
        if buf is None:
            return
        box = lay.local_box(self.rank)
        full = torch.as_tensor(np.asarray(arr)).reshape(lay.shape)
        buf.copy_(full[_slices(box, tuple((0, 0) for _ in box))].to(buf.dtype))

    def get_param_full(self, p):
        e = self.wentries[p.guid]
        return self._gather_full(e.layout, e.master, torch.float32)

    def set_param_full(self, p, full):
        e = self.wentries[p.guid]
        if e.box is None:
            return
        e.master.copy_(full[_slices(e.box, tuple((0, 0) for _ in e.box))].to(e.master.dtype))
        if e.compute is not e.master and e.compute is not None:
            e.compute.copy_(e.master)

    def load_batch(self, t, full_batch: torch.Tensor, start=0):
        """Copy this rank's shard of rows [start, start+B) of a host/device array into the
        tensor's home buffer (per-rank loader: SURVEY §2.4 X7)."""
        buf = self.local_buffer(t)
        if buf is None:
            return
        lay = self.home[t.guid]
        box = lay.local_box(self.rank)
        src = full_batch[start + box[0][0]: start + box[0][1]]
        rest = tuple(slice(lo, hi) for lo, hi in box[1:])
        if rest:
            src = src[(slice(None),) + rest]
        buf.copy_(src.to(buf.dtype), non_blocking=True)

    def load_local_many(self, pairs):
        """Copy several (tensor, source-shard) pairs into their home buffers; on MI355X in one
        multi-copy launch per 16 tensors (bytes moved as 16-bit words)."""
        if self.backend != "hip":
            for t, src in pairs:
                self.local_buffer(t).copy_(src)
            return
        from flexmi.ops import _kernels as K
        src, dst, n = [], [], []
        for t, s_ in pairs:
            d = self.local_buffer(t)
            if d is None:
                continue
            sv = s_.contiguous().view(-1).view(torch.int16)
            dv = d.view(-1).view(torch.int16)
            src.append(sv)
            dst.append(dv)
            n.append(dv.numel())
        if src:
            K.C().multi_copy(src, [0] * len(src), dst, [0] * len(dst), [1] * len(n), n, n, n, 0)

    # ------------------------------------------------------------------ hipGraph
    def train_step(self):
        self.forward()
        self.zero_gradients()
        self.backward()
        self.update()

    def capture_step(self, warmup=2):
        """Capture forward+backward+update into one hipGraph (static buffers)."""
        assert self.backend == "hip"
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.train_step()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.train_step()
        self._graph = g
        return g

    def replay(self):
        self._graph.replay()
        self.step_count += 1

    # ------------------------------------------------------------------ introspection
    def memory_report(self):
        n = 0
        for v in self.act.values():
            if v is not None:
                n += v.numel() * v.element_size()
        w = sum(g.numel * 4 * (2 + len(g.state)) for g in self.groups)
        sp = sum(e.numel * 4 for e in self.wentries.values() if e.sparse)
        return {"activations": n, "dense_params": w, "sparse_tables": sp}
