"""Embedding bag (``OP_EMBEDDING``).

Reference: ``src/ops/embedding.cu`` -- lookup ``out[b,:] = Σ_j W[idx[b,j],:]`` (``:173-197``),
backward = atomicAdd of the output grad into a dense ``W_grad`` (``:199-224``), partitions
allow only the sample dim or whole-table placement (``:108-135``).  AVG divided inside the bag
loop (bug, ``:187-195``); here AVG divides once.

MI355X: ``csrc/kernels/embedding.hip`` -- lanes gather whole rows with 16-B loads and write bf16
activations; the executor fuses all embedding ops of one placement into ONE launch (descriptor
table).  The backward never materialises a dense gradient for SGD: rows are updated in place
(W[idx] -= lr*dy).  Mostly-unique (large) tables use owner-computes: each row is claimed by one
lookup (CAS), duplicates add with atomics, the owner applies a plain 16-B read-modify-write;
other tables use 256-B-contiguous fp32 atomics; tiny tables accumulate in LDS first.
SOAP: sample split, **column (parameter) split** of the table, whole-table placement
(``dims=[1,1]``, device k) -- a 100 M-row table fits one MI355X's 288 GB of HBM -- and **row
split** (flexmi extension of the strategy format: a third internal degree, ``dims=[c, n, r]``):
each of r shards holds a contiguous block of rows, looks up only the indices it holds and emits
a PARTIAL output; the consumer's reshard sums the r partials (one all_to_all with add), and in
backward every shard receives the full output gradient and updates only its own rows.  Row
shards split tables too big for one GPU and spread a hot table's lookups over several GPUs.
"""
from __future__ import annotations

import math
import os

import torch

from flexmi.core.initializers import UniformInitializer
from flexmi.core.types import AggrMode, DataType, OperatorType
from flexmi.parallel.layout import Layout

from .base import Op, OpCtx, store
from . import _kernels as K



NATIVE_CPU = os.environ.get("FM_CPU_NATIVE", "1") != "0"
_CPU_MOD = []


def _cpu_ext():
    """The native CPU kernel module, or None when it was not built."""
    if not _CPU_MOD:
        try:
            from flexmi import _cpu as m
        except ImportError:
            m = None
        _CPU_MOD.append(m)
    return _CPU_MOD[0]

class SparseDPState:
    """Payload buffers of one replicated embedding group (see :meth:`Embedding.sdp_pack`).

    One int32 send buffer per rank: [count per table (padded to 64)] [ids per table: B*bag]
    [gradients per table: B*bag*D fp32 bits]; the all-gather fills ``recv`` = R segments of that
    layout in replica-rank order (the order of the sorted replica set = the group's rank order)."""

    def __init__(self, ops, ctxs, holders, rank):
        self.holders = tuple(sorted(holders))
        self.R = len(self.holders)
        self.seg = self.holders.index(rank)
        dev = ctxs[0].weights[0].device
        n = len(ctxs)
        nmax = [c.inputs[0].numel() for c in ctxs]
        D = [c.weights[0].shape[1] for c in ctxs]
        hdr = (n + 63) // 64 * 64
        offs_i, offs_g, o = [], [], hdr
        for k in range(n):
            offs_i.append(o)
            o += (nmax[k] + 63) // 64 * 64
        for k in range(n):
            offs_g.append(o)
            o += (nmax[k] * D[k] + 63) // 64 * 64
        self.P = o
        self.send = torch.zeros(self.P, dtype=torch.int32, device=dev)
        self.recv = torch.zeros(self.R * self.P, dtype=torch.int32, device=dev)

        def views(buf):
            cnt = [buf[k:k + 1] for k in range(n)]
            ids = [buf[offs_i[k]:offs_i[k] + nmax[k]] for k in range(n)]
            g = [buf[offs_g[k]:offs_g[k] + nmax[k] * D[k]].view(torch.float32) for k in range(n)]
            return cnt, ids, g
        # own payload lives in the send buffer; every segment (own included) is read from recv
        self.count, self.ids, self.g = {}, {}, {}
        self.count[self.seg], self.ids[self.seg], self.g[self.seg] = views(self.send)
        self.rcount, self.rids, self.rg = [], [], []
        for s in range(self.R):
            c, i, g = views(self.recv[s * self.P:(s + 1) * self.P])
            self.rcount.append(c)
            self.rids.append(i)
            self.rg.append(g)
        hip = ctxs[0].hip
        self.slot = [torch.full((c.weights[0].shape[0],), -1, dtype=torch.int32, device=dev) for c in ctxs] if hip else []
        self.cid = [torch.empty(nmax[k], dtype=torch.int32, device=dev) for k in range(n)] if hip else []

    def exchange(self, comm):
        comm.all_gather(self.recv, self.send, self.holders)


class Embedding(Op):
    op_type = OperatorType.OP_EMBEDDING
    name_prefix = "Embed"

    def __init__(self, model, input, num_entries, out_dim, aggr=AggrMode.AGGR_MODE_SUM,
                 kernel_initializer=None, name=None):
        super().__init__(model, [input], name)
        self.num_entries = int(num_entries)
        self.out_dim = int(out_dim)
        self.aggr = AggrMode(aggr)
        if self.name is None:
            self.name = self.auto_name(f"{num_entries}x{out_dim}")
        if kernel_initializer is None:
            r = math.sqrt(1.0 / self.num_entries)
            kernel_initializer = UniformInitializer(model._next_seed() if model else 0, -r, r)
        self._add_weight((self.num_entries, self.out_dim), kernel_initializer, "weight")
        self._finish([(input.dims[0], self.out_dim)])
        # set by the executor when a fused sparse optimizer applies to this table; sparse_dp =
        # the replica set of a replicated table trained by touched-row exchange
        self.sparse_sgd = False
        self.sparse_dp = None

    def splittable_dims(self):
        return {0, 1}

    @staticmethod
    def _grid(pc):
        """(n, c, r, dev): sample / column / row degrees and the device of part (i, j, k); the
        internal dims are [c, n] or [c, n, r] (internal dim 0 fastest in the device list)."""
        d = list(pc.dims) + [1] * (3 - len(pc.dims))
        c, n, r = int(d[0]), int(d[1]), int(d[2])
        ids = pc.device_ids

        def dev(i, j, k):
            return ids[j + c * (i + n * k)]
        return n, c, r, dev

    def valid_pc(self, pc):
        if len(pc.dims) <= 2:
            return super().valid_pc(pc)
        if len(pc.dims) != 3 or len(pc.device_ids) != pc.num_parts() or min(pc.device_ids) < 0:
            return False
        n, c, r, _ = self._grid(pc)
        B, D = self.outputs[0].dims
        # a rank holds at most one part of each layout: row shards on distinct devices
        return (n <= B and c <= D and r <= self.num_entries and len(set(pc.device_ids)) == len(pc.device_ids))

    def output_layouts(self, pc):
        n, c, r, dev = self._grid(pc)
        if r == 1:
            return super().output_layouts(pc)
        holders = [tuple(dev(i, j, k) for k in range(r)) for i in range(n) for j in range(c)]
        return [Layout(self.outputs[0].dims, (n, c), holders, partial=True)]

    def input_layouts(self, pc):
        n, c, r, dev = self._grid(pc)
        holders = [tuple(dev(i, j, k) for k in range(r) for j in range(c)) for i in range(n)]
        return [Layout(self.inputs[0].dims, (n, 1), holders)]

    def weight_layouts(self, pc):
        n, c, r, dev = self._grid(pc)
        holders = [tuple(dev(i, j, k) for i in range(n)) for k in range(r) for j in range(c)]
        return [Layout(self.weights[0].dims, (r, c), holders)]

    @staticmethod
    def _row_lo(ctx):
        b = ctx.w_boxes[0] if ctx.w_boxes else None
        return int(b[0][0]) if b is not None else 0

    @staticmethod
    def _local_rows(idx, lo, rows):
        """(local row per lookup clamped into the shard, mask of the lookups this shard holds)."""
        li = idx.long() - lo
        ok = (li >= 0) & (li < rows)
        return li.clamp(0, rows - 1), ok

    def needs_input_grad(self, i):
        return False

    # ---------------------------------------------------------- compute
    @staticmethod
    def _native_cpu(*ts):
        """flexmi._cpu (csrc/cpu/cpu_ops.cc) when built and the operands fit it: fp32 tables and
        rows, integer indices; FM_CPU_NATIVE=0 selects the torch reference path instead."""
        if not NATIVE_CPU:
            return None
        m = _cpu_ext()
        if m is None:
            return None
        w, idx, rows = ts
        if (w.dtype != torch.float32 or rows.dtype != torch.float32 or not w.is_contiguous()
                or idx.dtype not in (torch.int32, torch.int64) or rows.stride(-1) != 1 or w.device.type != "cpu"):
            return None
        return m

    def forward(self, ctx: OpCtx):
        idx = ctx.inputs[0]
        w = ctx.weights[0]
        out = ctx.outputs[0]
        if ctx.hip:
            Embedding.forward_group([self], [ctx])
        elif self._native_cpu(w, idx, out) is not None:
            scale = 1.0 / idx.shape[1] if self.aggr == AggrMode.AGGR_MODE_AVG else 1.0
            _cpu_ext().embedding_fwd(w, idx.contiguous(), out, self._row_lo(ctx), scale)
        else:
            bag = idx.shape[1]
            li, ok = self._local_rows(idx, self._row_lo(ctx), w.shape[0])
            rows = w.index_select(0, li.reshape(-1)).view(idx.shape[0], bag, -1) * ok.unsqueeze(-1).to(w.dtype)
            r = rows.sum(1)
            if self.aggr == AggrMode.AGGR_MODE_AVG:
                r = r / bag
            out.copy_(r)

    def backward(self, ctx: OpCtx):
        idx = ctx.inputs[0]
        dy = ctx.out_grads[0]
        if self.sparse_sgd:
            # fused sparse SGD (no dense grad): W[idx] -= lr * dy  (duplicates summed first)
            scale = 1.0 / idx.shape[1] if self.aggr == AggrMode.AGGR_MODE_AVG else 1.0
            if ctx.hip:
                Embedding.backward_group([self], [ctx])
            elif self._native_cpu(ctx.weights[0], idx, dy) is not None:
                _cpu_ext().embedding_bwd(ctx.weights[0], idx.contiguous(), dy, self._row_lo(ctx),
                                         -float(ctx.lr) * scale)
            else:
                g = dy.float()
                if self.aggr == AggrMode.AGGR_MODE_AVG:
                    g = g / idx.shape[1]
                bag = idx.shape[1]
                li, ok = self._local_rows(idx, self._row_lo(ctx), ctx.weights[0].shape[0])
                gg = g.repeat_interleave(bag, dim=0) * ok.reshape(-1, 1).to(g.dtype)
                upd = torch.zeros_like(ctx.weights[0])
                upd.index_add_(0, li.reshape(-1), gg)
                ctx.weights[0].sub_(ctx.lr.to(upd.dtype) * upd)
            return
        dw = ctx.weight_grads[0]
        if ctx.hip:
            Embedding.backward_group([self], [ctx])
        elif self._native_cpu(dw, idx, dy) is not None:
            scale = 1.0 / idx.shape[1] if self.aggr == AggrMode.AGGR_MODE_AVG else 1.0
            _cpu_ext().embedding_bwd(dw, idx.contiguous(), dy, self._row_lo(ctx), scale)
        else:
            g = dy.float()
            if self.aggr == AggrMode.AGGR_MODE_AVG:
                g = g / idx.shape[1]
            bag = idx.shape[1]
            li, ok = self._local_rows(idx, self._row_lo(ctx), dw.shape[0])
            dw.index_add_(0, li.reshape(-1), g.repeat_interleave(bag, dim=0) * ok.reshape(-1, 1).to(g.dtype))

    # ---------------------------------------------------------- fused groups
    @staticmethod
    def can_group(a, b, ca, cb):
        """Executor fusion: independent embeddings with the same placement run as ONE launch."""
        return (ca.outputs[0].dtype == cb.outputs[0].dtype and a.sparse_sgd == b.sparse_sgd
                and getattr(a, "sparse_dp", None) == getattr(b, "sparse_dp", None)
                and ca.inputs[0].shape[0] == cb.inputs[0].shape[0])

    @staticmethod
    def forward_group(ops, ctxs):
        if not ctxs[0].hip:
            for op, c in zip(ops, ctxs):
                op.forward(c)
            return
        K.C().embedding_fwd_multi([c.weights[0] for c in ctxs], [c.inputs[0] for c in ctxs],
                                  [c.outputs[0] for c in ctxs], [c.outputs[0].stride(0) for c in ctxs],
                                  [1.0 / c.inputs[0].shape[1] if op.aggr == AggrMode.AGGR_MODE_AVG else 1.0
                                   for op, c in zip(ops, ctxs)],
                                  [Embedding._row_lo(c) for c in ctxs])

    @staticmethod
    def backward_group(ops, ctxs):
        if not ctxs[0].hip:
            for op, c in zip(ops, ctxs):
                op.backward(c)
            return
        scales = [1.0 / c.inputs[0].shape[1] if op.aggr == AggrMode.AGGR_MODE_AVG else 1.0 for op, c in zip(ops, ctxs)]
        if ops[0].sparse_sgd:
            tables = [c.weights[0] for c in ctxs]
            lr = ctxs[0].lr
        else:
            tables = [c.weight_grads[0] for c in ctxs]   # accumulate (zeroed once per step)
            lr = None
        claim = None
        if ops[0].sparse_sgd:
            bufs = [op._claim_buffers(c) for op, c in zip(ops, ctxs)]
            if any(b is not None for b in bufs):
                claim = []
                for b in bufs:
                    claim.extend(b if b is not None else (None, None, None))
        K.C().embedding_bwd_multi(tables, [c.inputs[0] for c in ctxs], [c.out_grads[0] for c in ctxs],
                                  [c.out_grads[0].stride(0) for c in ctxs], scales, lr, claim,
                                  [Embedding._row_lo(c) for c in ctxs])

    # ---------------------------------------------------------- sparse data parallelism
    # A table REPLICATED over a set of ranks (sample-split lookups, e.g. pure DP) is trained with
    # touched-row exchange instead of the reference's dense per-replica gradient + replica sum
    # (src/ops/embedding.cu:108-135 partitions, src/runtime/model.cc:697-724 grad replicas,
    # src/runtime/optimizer_kernel.cu:96-101 replica reduction -- a table-sized gradient, 96 GB
    # at MLPerf scale).  Per step: (1) pack -- each replica coalesces its lookups into (unique
    # local rows, summed gradients) payloads; (2) one all-gather of the payloads over the replica
    # set; (3) apply -- every replica applies the R segments in rank order (plain row updates,
    # rows unique per segment), so all replicas perform the same fp32 operations and stay
    # bit-identical.  Nothing table-sized is allocated besides the table itself and an int32
    # claim slot per row (GPU).
    @staticmethod
    def sdp_state(ops, ctxs, holders, rank):
        c0 = ctxs[0]
        st = c0.saved.get("sdp")
        if st is None:
            st = SparseDPState(ops, ctxs, holders, rank)
            c0.saved["sdp"] = st
        return st

    @staticmethod
    def sdp_pack(ops, ctxs):
        st = ctxs[0].saved["sdp"]
        scales = [1.0 / c.inputs[0].shape[1] if op.aggr == AggrMode.AGGR_MODE_AVG else 1.0 for op, c in zip(ops, ctxs)]
        if ctxs[0].hip:
            K.C().sdp_coalesce([c.weights[0] for c in ctxs], [c.inputs[0] for c in ctxs], [c.out_grads[0] for c in ctxs],
                               [c.out_grads[0].stride(0) for c in ctxs], scales, [Embedding._row_lo(c) for c in ctxs],
                               st.slot, st.cid, st.ids[st.seg], st.g[st.seg], st.count[st.seg])
            return
        for k, (op, c) in enumerate(zip(ops, ctxs)):
            idx, w = c.inputs[0], c.weights[0]
            bag = idx.shape[1]
            li, ok = Embedding._local_rows(idx, Embedding._row_lo(c), w.shape[0])
            sel = ok.reshape(-1)
            rows = li.reshape(-1)[sel]
            g = (c.out_grads[0].float() * scales[k]).repeat_interleave(bag, dim=0)[sel]
            uniq, inv = torch.unique(rows, return_inverse=True)
            summed = torch.zeros((uniq.numel(), w.shape[1]), dtype=torch.float32).index_add_(0, inv, g)
            n = uniq.numel()
            st.count[st.seg][k].fill_(n)
            st.ids[st.seg][k][:n].copy_(uniq.to(torch.int32))
            st.g[st.seg][k][:n * w.shape[1]].copy_(summed.reshape(-1))

    @staticmethod
    def sdp_apply(ops, ctxs):
        st = ctxs[0].saved["sdp"]
        lr = ctxs[0].lr
        if ctxs[0].hip:
            K.C().sdp_apply([c.weights[0] for c in ctxs], [t for s in range(st.R) for t in st.rids[s]],
                            [t for s in range(st.R) for t in st.rg[s]], [t for s in range(st.R) for t in st.rcount[s]],
                            st.slot, st.count[st.seg], st.R, st.seg, lr)
            return
        mlr = -lr.to(torch.float32)
        for s in range(st.R):
            for k, c in enumerate(ctxs):
                w = c.weights[0]
                n = int(st.rcount[s][k].item())
                if n:
                    D = w.shape[1]
                    w.index_add_(0, st.rids[s][k][:n].long(), mlr * st.rg[s][k][:n * D].view(n, D))

    CLAIM = True                 # owner-computes path for mostly-unique tables (tests may switch it)
    # owner-computes when rows exceed CLAIM_RATIO x lookups per step (few enough duplicates for the
    # claim / dup / owner kernels to beat per-lookup atomics): 0.2 takes the 2208..7420-row MLPerf
    # tables off the atomic kernel, 1.162-1.163 vs 1.171 ms/step at ratio 1
    # (profiles/bench_ab_claim_ratio_r5cr.txt)
    CLAIM_RATIO = 0.2
    # the count / update kernel pair (csrc/kernels/embedding.hip, fm_embedding_set_bwd_mode(1)) for
    # every table above the tiny-table LDS kernel's rows, on the same slot / flag buffers: an
    # alternative form kept tested (tests/test_gpu_kernels.py), off by default
    COUNT = False
    # the wave-private LDS kernel's table-size limit: the same constant as the C++ dispatcher
    # (embedding.hip kind_of TINY_ROWS)
    TINY_ROWS = 64

    def _claim_buffers(self, ctx):
        """Owner-computes sparse SGD buffers for a mostly-unique table (rows > lookups per step):
        a per-row claim slot (int32, -1 = free; restored after every step), the duplicate list
        and its counter.  Smaller tables keep the atomic / LDS-privatised kernels."""
        if not Embedding.CLAIM:
            return None
        s = ctx.saved
        if "claim" not in s:
            w, idx = ctx.weights[0], ctx.inputs[0]
            big = w.shape[0] > (Embedding.TINY_ROWS if Embedding.COUNT else Embedding.CLAIM_RATIO * idx.numel())
            if big and self.out_dim % 4 == 0:
                dev = w.device
                s["claim"] = (torch.full((w.shape[0],), -1, dtype=torch.int32, device=dev),
                              torch.empty(idx.numel(), dtype=torch.int32, device=dev),
                              torch.zeros(1, dtype=torch.int32, device=dev))
            else:
                s["claim"] = None
        return s["claim"]

    def flops(self, in_shapes, out_shapes):
        return float(in_shapes[0][0] * in_shapes[0][1] * out_shapes[0][1])

    @staticmethod
    def sdp_payload_words(lookups, D):
        """int32 words one replica contributes per table to the sparse-DP all-gather (the worst
        case: every lookup a distinct row) -- used by the cost model (flexmi/parallel/search.py)."""
        return 1 + lookups * (1 + D)

    @staticmethod
    def sdp_prefer_sparse(rows, D, lookups, R):
        """Replicated table over R holders: train it by sparse data parallelism (touched-row
        all-gather of R fixed payloads) only when that moves fewer bytes than the dense replica
        all-reduce of the table's rows x D gradient.  A ring all-gather of R payloads moves what a
        ring all-reduce of R * payload / 2 words moves, so sparse wins iff R * payload / 2 < rows * D.
        The tiny Criteo tables (3..10 rows) stay dense; 1e5+-row tables go sparse.  One rule for
        the executor (Executor._build_weights) and the search's cost model (SimGraph._cand)."""
        if R <= 1:
            return True
        return R * Embedding.sdp_payload_words(lookups, D) / 2.0 < float(rows) * D

    def bytes_moved(self, in_shapes, out_shapes, elem=2):
        b, bag = in_shapes[0]
        d = out_shapes[0][1]
        return float(b * bag * d * 4 + b * d * elem + b * bag * 8)
