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
import os
import time
from collections import OrderedDict, defaultdict
from typing import Dict, List

import numpy as np
import torch

from flexmi.core.loss_metrics import NUM_SLOTS, PerfMetrics, loss_and_metrics_torch
from flexmi.core.initializers import _native_cpu
from flexmi.core.optimizers import AdamOptimizer, SGDOptimizer
from flexmi.core.types import DataType, LossType, to_torch_dtype
from flexmi.ops.base import OpCtx
from flexmi.parallel.layout import Layout, ParallelConfig, ReshardPlan, box_intersect, box_volume
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
        run_reshards(comm, [(self, src_buf, dst_buf, accumulate)])

    # --- phases used by run_reshards (several reshards share ONE all_to_all) ---------------
    def prepare_dst(self, dst_buf, accumulate):
        """Zero the destination when contributions are summed into it; returns add-mode."""
        reduce = self.plan.src.partial
        if dst_buf is not None and reduce and not accumulate:
            dst_buf.zero_()
        return accumulate or reduce

    def local_copies(self, src_buf, dst_buf, add):
        r = self.rank
        if not self.recvs:
            return
        src_box = self.plan.src.local_box(r)
        dst_box = self.plan.dst.local_box(r)
        for t in self.recvs:
            if t.src == r:
                self._put(dst_buf, dst_box, t.box, src_buf[_slices(t.box, src_box)], add)

    def remote_sends(self, src_buf):
        """{peer: [flat pieces]} in plan order (same order the peer unpacks)."""
        out = defaultdict(list)
        if not self.sends:
            return out
        src_box = self.plan.src.local_box(self.rank)
        for t in self.sends:
            if t.dst != self.rank:
                out[t.dst].append(src_buf[_slices(t.box, src_box)].reshape(-1))
        return out

    def remote_recv_numel(self):
        n = defaultdict(int)
        for t in self.recvs:
            if t.src != self.rank:
                n[t.src] += box_volume(t.box)
        return n

    def unpack(self, chunks, offs, dst_buf, add):
        if not self.recvs:
            return
        dst_box = self.plan.dst.local_box(self.rank)
        for t in self.recvs:
            if t.src == self.rank:
                continue
            shape = tuple(hi - lo for lo, hi in t.box)
            n = box_volume(t.box)
            piece = chunks[t.src][offs[t.src]: offs[t.src] + n].view(shape)
            offs[t.src] += n
            self._put(dst_buf, dst_box, t.box, piece, add)

    @staticmethod
    def _put(dst_buf, dst_box, box, piece, add):
        v = dst_buf[_slices(box, dst_box)]
        if add:
            v.add_(piece.to(v.dtype))
        else:
            v.copy_(piece)


def run_reshards(comm, items):
    """Execute several reshard steps with ONE all_to_all (collective fusion: e.g. the 26
    embedding outputs of a DLRM interaction move in a single RCCL call per direction).
    items: [(ReshardStep, src_buf, dst_buf, accumulate)], all of the same dtype."""
    adds = []
    for st, src, dst, acc in items:
        adds.append(st.prepare_dst(dst, acc))
    for (st, src, dst, acc), add in zip(items, adds):
        st.local_copies(src, dst, add)
    if comm.world == 1 or all(st.local_only for st, *_ in items):
        return
    W = comm.world
    per_peer = defaultdict(list)
    recv = [0] * W
    for st, src, dst, acc in items:
        for p, lst in st.remote_sends(src).items():
            per_peer[p].extend(lst)
        for p, n in st.remote_recv_numel().items():
            recv[p] += n
    send = [None] * W
    for p, lst in per_peer.items():
        send[p] = torch.cat(lst) if len(lst) > 1 else lst[0]
    st0 = items[0][0]
    chunks = comm.all_to_all(send, recv, st0.dtype, st0.device)
    offs = [0] * W
    for (st, src, dst, acc), add in zip(items, adds):
        st.unpack(chunks, offs, dst, add)


# FM_OVERLAP_EMB=1/0/auto (default auto: on when an embedding table is >= 128 wide).  Inside a
# captured segment, fused embedding-group kernels run on a
# second HIP stream so they overlap the bottom-MLP GEMMs (forward: hoisted to the fork point and
# joined before their first consumer; backward: forked after the interaction gradient and joined
# before the dense update or the segment end).  Embedding kernels use no shared GEMM workspace.
# Measured N=1 (100 steps, samples/s): mlperf d=128 11.45 M -> 12.37 M; run_random and criteo_kaggle
# (narrow tables) lose 3-6 %, hence the width rule.
OVERLAP_EMB = os.environ.get("FM_OVERLAP_EMB", "auto")

# FM_P2P=1/0/auto (default auto): a fused exchange whose transfer graph is sparse -- some pair of
# participants never exchanges (spatial halos, pipeline hand-offs between neighbouring chunks) --
# posts grouped point-to-point send/recv with only its real peers (one coalesced RCCL launch, each
# transfer on its own xGMI link) instead of an all-to-all over every participant.
P2P_MODE = os.environ.get("FM_P2P", "auto")


# FLEXMI_XCHG_CHUNKS=K / auto (default auto: 2 when every rank holds >= 1024 samples): micro-batch
# pipelining of the last cross-device exchange of the forward when everything after it is a
# sample-split row-wise tail (DLRM: embedding all-to-all -> interaction -> top MLP).  The exchange
# is split into K all-to-alls over row chunks of the destination's samples; chunk c's tail
# forward runs as soon as chunk c has landed, overlapping the all-to-all of chunk c+1.  Backward
# mirrors it: the tail's input-gradient passes run per chunk and each chunk's gradient
# all-to-all starts right after, overlapping the next chunk; the tail's weight gradients run on
# the whole batch afterwards (overlapping the last chunk).  Reference: the DLRM strategy moves
# every embedding output in one exchange (src/runtime/dlrm_strategy.cc:252-263).
XCHG_CHUNKS = os.environ.get("FLEXMI_XCHG_CHUNKS", "auto")
# test hook: chunk the row-wise tail at world 1 too (no exchange; exercises the chunked kernels)
XCHG_LOCAL = False
PIPE_ROW_ALIGN = 8          # chunk boundaries on 8-row multiples: 16-B aligned rows for the kernels
# the NHWC convolutions' weight re-layouts as one launch per step (conv_wprep_all): ResNet-50 b64
# 6.62 -> 6.69 k img/s, AlexNet b256 within noise (profiles/conv_wprep_all_ab_r7.txt); tests flip it
CONV_WPREP_ALL = True
# smallest weight (elements) whose SGD is fused into its dW GEMM (FM_FUSED_SGD); tests lower it
FUSED_SGD_MIN = 1 << 21


def chunk_bounds(n, k):
    """Row boundaries of k micro-batch chunks of n local rows (boundaries on 8-row multiples)."""
    return [0] + [(n * c // k) // PIPE_ROW_ALIGN * PIPE_ROW_ALIGN for c in range(1, k)] + [n]


def overlap_embeddings_enabled(ex):
    """Whether captured steps of executor ``ex`` run the fused embedding groups on a second HIP
    stream (``OVERLAP_EMB``: "1" / "0" / "auto" = on when an embedding table is >= 128 wide)."""
    if OVERLAP_EMB == "1":
        return True
    if OVERLAP_EMB != "auto":
        return False
    return any(st[0] == "op" and type(st[1]).__name__ == "Embedding" and st[1].out_dim >= 128 for st in ex.fwd_steps)


def _run_overlapped(items, s, side):
    """Issue one graph segment's items with the embedding groups on ``side`` (fork/join by events,
    which stream capture records as graph edges).  A group forward is hoisted only across plain
    op forwards that declare what they write (``Item.writes``) and write none of the group's
    inputs (``Item.reads``): never across reshards, exchange unpacks or another group.
    (Measured and dropped: forking the group forward later than its earliest point, letting the
    optimizer skip the join of a pending group backward, and weight-gradient GEMMs on a third
    stream -- profiles/bench_ab_emb_fwd_delay_r5za.txt, bench_ab_late_join_r5w.txt,
    dw_stream_ab_r5p4.txt, dw_stream_chain_tail_ab_r6.txt.)"""
    # without the side stream the embedding-group items run in place on the main stream
    fwd = [k for k, it in enumerate(items) if it.name.endswith(".group_fwd")] if side is not None else []
    hoist, fork_at = set(), {}
    for k in fwd:
        j = k
        reads = items[k].reads
        while j > 0 and reads is not None:
            prev = items[j - 1]
            if prev.writes is None or prev.name.endswith(".group_fwd") or (prev.writes & reads):
                break
            j -= 1
        if j < k:
            hoist.add(k)
            fork_at.setdefault(j, []).append(k)
    joined_fwd = set()
    bwd_pending = False
    for k, it in enumerate(items):
        if k in fork_at:
            side.wait_stream(s)
            with torch.cuda.stream(side):
                for h in fork_at[k]:
                    items[h].fn()
        if k in hoist:
            s.wait_stream(side)      # join at the item's original position (before its consumer)
            joined_fwd.add(k)
            continue
        if side is not None and it.name.endswith(".group_bwd"):
            side.wait_stream(s)
            with torch.cuda.stream(side):
                it.fn()
            bwd_pending = True
            continue
        if bwd_pending and not it.name.endswith((".bwd", ".bwd_dw", ".bwd_dx")):
            s.wait_stream(side)
            bwd_pending = False
        it.fn()
    if side is not None:
        s.wait_stream(side)


class Item:
    __slots__ = ("kind", "fn", "name", "check", "native", "zero_group", "reads", "writes")

    def __init__(self, kind, fn, name, check=None, native=None):
        self.kind, self.fn, self.name = kind, fn, name
        self.zero_group = None  # the per-step gradient memset of this weight group
        # tensor guids this item reads / writes (op forwards and embedding-group forwards);
        # None = unknown -- the second-stream scheduler never reorders across it
        self.reads = None
        self.writes = None
        self.check = check      # debug mode: callable(item) run after fn (NaN/Inf guard)
        self.native = native    # comm items: structured form for the native runner (flexmi._rt)

    def __repr__(self):
        return f"{self.kind}:{self.name}"


def _rt_module():
    try:
        from flexmi import _rt
        return _rt
    except ImportError:
        return None


_LIVE_RUNNERS = None
# replicated embedding tables (DP) trained by touched-row exchange instead of a dense gradient
# all-reduce (FLEXMI_SPARSE_DP=0: the reference's dense replica gradients, for A/B)
SPARSE_DP = os.environ.get("FLEXMI_SPARSE_DP", "1") != "0"


def release_native_runners():
    """Drop the native runners' references to c10d process groups, tensors and callables.  Runs
    before ``torch.distributed.destroy_process_group`` (hooked) and at exit: a group must be
    destroyed while every rank is still alive -- one whose last reference goes away during
    interpreter shutdown, after the peer ranks (and the TCP store host) have exited, aborts."""
    for r in list(_LIVE_RUNNERS or ()):
        r.rt.release()


def _hook_destroy_process_group():
    from flexmi.parallel.comm import install_teardown_hook
    install_teardown_hook()


class NativeRunner:
    """Compiles item lists into programs of the native step runner (``csrc/runtime/step_runner.cc``):
    compute items stay callables (or, once captured, hipGraph launches), comm items become c10d
    collectives issued from C++ with their Work handles kept in runner slots -- the step loop and
    every RCCL call run without the Python interpreter in between."""

    def __init__(self, ex):
        import torch.distributed as dist
        self.ex = ex
        self.rt = _rt_module().StepRunner()
        self.world_pg = dist.group.WORLD if ex.world > 1 else None
        self.slots = {}
        self.pids = {}
        self.step_items = {}
        self.keep = []          # Python objects referenced by native steps (graphs, callables)
        global _LIVE_RUNNERS
        if _LIVE_RUNNERS is None:
            import atexit
            import weakref
            _LIVE_RUNNERS = weakref.WeakSet()
            atexit.register(release_native_runners)
            _hook_destroy_process_group()
        _LIVE_RUNNERS.add(self)

    def slot(self, key):
        s = self.slots.get(key)
        if s is None:
            s = self.slots[key] = self.rt.new_slot()
        return s

    def _pg(self, ranks):
        g = self.ex.comm.group_for(ranks) if ranks is not None else None
        return self.world_pg if g is None else g

    def add_item(self, pid, it):
        rt, ex = self.rt, self.ex
        nat = it.native
        if nat is None:
            rt.add_call(pid, it.fn, it.name)
            return
        kind = nat[0]
        if kind in ("a2a", "a2a_sync"):
            x = nat[1]
            s = self.slot(("a2a", id(x)))
            self.keep.append(x)
            if not x.active:        # this rank has no piece in the exchange
                return
            rs_, ss_ = x.group_splits()
            add = rt.add_p2p if x.p2p else rt.add_all_to_all
            add(pid, s, x.pg if x.pg is not None else self.world_pg, x.recv_buf, x.send_buf, rs_, ss_, it.name)
            if kind == "a2a_sync":
                rt.add_wait(pid, s, it.name + ".wait")
        elif kind == "wait":
            rt.add_wait(pid, self.slot(("a2a", id(nat[1]))), it.name)
        elif kind == "ar":
            g, bi = nat[1], nat[2]
            b = g.buckets[bi]
            rt.add_all_reduce(pid, self.slot(("ar", id(g), bi)), self._pg(g.holders), g.gradbuf[b[0]:b[1]], False,
                              it.name)
        elif kind == "rs":
            g, bi = nat[1], nat[2]
            b = g.buckets[bi]
            sh = ex._zero_pieces(g)[bi][1]
            rt.add_reduce_scatter(pid, self.slot(("ar", id(g), bi)), self._pg(g.holders), g.gshard[sh],
                                  g.gradbuf[b[0]:b[1]], False, it.name)
        elif kind == "ar_sync":
            for g in ex.groups:
                if not g.replicated:
                    continue
                for bi, b in enumerate(g.buckets):
                    if g.zero:
                        sh = ex._zero_pieces(g)[bi][1]
                        rt.add_reduce_scatter(pid, self.slot(("ar", id(g), bi)), self._pg(g.holders), g.gshard[sh],
                                              g.gradbuf[b[0]:b[1]], True, f"{it.name}.bucket{bi}")
                        continue
                    rt.add_all_reduce(pid, self.slot(("ar", id(g), bi)), self._pg(g.holders), g.gradbuf[b[0]:b[1]],
                                      True, f"{it.name}.bucket{bi}")
        elif kind == "ag_buf":      # all-gather of explicit buffers over a replica set (sparse DP)
            out, inp, ranks = nat[1], nat[2], nat[3]
            rt.add_all_gather(pid, self.slot(("agb", id(out))), self._pg(ranks), out, inp, it.name)
        elif kind == "ag_sync":
            for g in ex.groups:
                if not g.zero:
                    continue
                for bi, (fsl, sh) in enumerate(ex._zero_pieces(g)):
                    b = g.buckets[bi]
                    rt.add_all_gather(pid, self.slot(("ag", id(g), bi)), self._pg(g.holders), g.master[b[0]:b[1]],
                                      g.mshard[sh], f"{it.name}.bucket{bi}")
        else:
            raise ValueError(f"unknown native item {kind}")

    def program(self, items):
        """Program id for an item list (compiled once per list).  ``step_items[pid][i]`` is the
        (item, last step of that item) behind native step i (hooks map steps back to items)."""
        pid = self.pids.get(id(items))
        if pid is None:
            pid = self.rt.new_program()
            owner = []
            for it in items:
                n0 = self.rt.program_size(pid)
                self.add_item(pid, it)
                n1 = self.rt.program_size(pid)
                owner.extend((it, k == n1 - 1) for k in range(n0, n1))
            self.pids[id(items)] = pid
            self.step_items[pid] = owner
            self.keep.append(items)
        return pid

    def run(self, pid, pre=None, post=None):
        rt, comm = self.rt, self.ex.comm
        c0, b0 = rt.collectives, rt.bytes_sent
        rt.run(pid, pre, post)
        comm.calls += rt.collectives - c0
        comm.bytes_sent += rt.bytes_sent - b0


def _box2d(buf, buf_lo, box):
    """A box of a contiguous shard buffer as one strided 2-D copy: (elem offset, rows, cols,
    leading dim) -- or None when the box is not row x contiguous-span shaped."""
    shape = tuple(buf.shape)
    nd = len(shape)
    ext = [hi - lo for lo, hi in box]
    strides = buf.stride()
    off = sum((lo - l) * st for (lo, _), l, st in zip(box, buf_lo, strides))
    if nd == 1:
        return off, 1, ext[0], ext[0]
    part = [d for d in range(1, nd) if ext[d] != shape[d]]
    if not part:
        return off, ext[0], int(np.prod(shape[1:])), strides[0]
    j = part[0]
    if any(ext[k] != shape[k] for k in range(j + 1, nd)) or any(shape[k] != 1 for k in range(1, j)):
        return None
    return off, ext[0], ext[j] * int(np.prod(shape[j + 1:], dtype=np.int64)), strides[0]


class FusedExchange:
    """Several reshards moved by ONE all_to_all through persistent send/recv buffers, split in
    pack (compute) / exchange (RCCL, asynchronous) / wait / unpack (compute) so the compute halves
    live inside hipGraph segments and independent work overlaps the collective.  On MI355X the
    pack and unpack phases are each ONE multi-descriptor copy launch (per 16 pieces) instead of
    a copy per (tensor, peer) piece."""

    def __init__(self, items, world, rank, comm=None):
        self.items = items
        self.world = world
        self.rank = rank
        # ranks that send or receive anything in this exchange: a strict subset exchanges on its
        # own communicator (created here, on every rank in plan order -- new_group is collective)
        # and the other ranks skip the collective entirely
        parts = set()
        for st, *_ in items:
            for t in st.plan.transfers:
                if t.src != t.dst:
                    parts.update((t.src, t.dst))
        self.participants = sorted(parts)
        self.active = rank in parts
        peers = defaultdict(set)
        for st, *_ in items:
            for t in st.plan.transfers:
                if t.src != t.dst:
                    peers[t.src].add(t.dst)
                    peers[t.dst].add(t.src)
        n = len(self.participants)
        # point-to-point when some participants never exchange, or when only two ranks of a
        # larger world do (a pipeline hand-off: send/recv on the world communicator instead of a
        # new two-rank communicator).  Decided from the global transfer plan, so every rank picks
        # the same collective.
        sparse = (n >= 3 and max(len(v) for v in peers.values()) < n - 1) or (n == 2 and world > 2)
        self.p2p = n >= 2 and (P2P_MODE == "1" or (P2P_MODE == "auto" and sparse))
        self.pg = None
        if comm is not None and 0 < n < world and not self.p2p:
            self.pg = comm.group_for(self.participants)
        st0 = items[0][0]
        self.dtype, self.device = st0.dtype, st0.device
        self.adds = [acc or st.plan.src.partial for st, src, dst, acc in items]
        send = [0] * world
        recv = [0] * world
        for st, src, dst, acc in items:
            for t in st.sends:
                if t.dst != rank:
                    send[t.dst] += box_volume(t.box)
            for t in st.recvs:
                if t.src != rank:
                    recv[t.src] += box_volume(t.box)
        self.send_sizes, self.recv_sizes = send, recv
        self.send_buf = torch.empty(sum(send), dtype=self.dtype, device=self.device)
        self.recv_buf = torch.empty(sum(recv), dtype=self.dtype, device=self.device)
        self.send_off = [sum(send[:p]) for p in range(world)]
        self.recv_off = [sum(recv[:p]) for p in range(world)]
        self.work = None
        self.tag = None            # program item name prefix (micro-batch chunk exchanges)
        self._plan_descriptors()

    def _plan_descriptors(self):
        """Pre-plan every piece as a strided 2-D copy (HIP backend); falls back to per-piece
        tensor copies when a box is not 2-D expressible or dtypes differ."""
        self.fast = self.device is not None and torch.device(self.device).type == "cuda"
        if not self.fast:
            return
        r = self.rank
        pack, unpack, zero = [], [], []
        soff = list(self.send_off)
        roff = list(self.recv_off)
        per_send = defaultdict(list)
        for (st, src, dst, acc), add in zip(self.items, self.adds):
            if dst is not None and st.plan.src.partial and not acc:
                zero.append(dst)
            for b in (src, dst):
                if b is not None and (b.dtype != self.dtype or not b.is_contiguous()):
                    self.fast = False
                    return
            src_lo = [lo for lo, _ in st.plan.src.local_box(r)] if src is not None else None
            dst_lo = [lo for lo, _ in st.plan.dst.local_box(r)] if dst is not None else None
            for t in st.recvs:
                if t.src == r:          # local piece: src box -> dst box
                    a, b = _box2d(src, src_lo, t.box), _box2d(dst, dst_lo, t.box)
                    if a is None or b is None or a[1:3] != b[1:3]:
                        self.fast = False
                        return
                    pack.append((src, a[0], dst, b[0], a[1], a[2], a[3], b[3], add, t.box))
            for t in st.sends:
                if t.dst != r:
                    a = _box2d(src, src_lo, t.box)
                    if a is None:
                        self.fast = False
                        return
                    per_send[t.dst].append((src, a))
            for t in st.recvs:
                if t.src != r:
                    b = _box2d(dst, dst_lo, t.box)
                    if b is None:
                        self.fast = False
                        return
                    n = box_volume(t.box)
                    unpack.append((self.recv_buf, roff[t.src], dst, b[0], b[1], b[2], b[2], b[3], add, t.box))
                    roff[t.src] += n
        for p in range(self.world):     # sends grouped by peer, in plan order (= peer's unpack order)
            for src, a in per_send.get(p, []):
                off, rows, cols, ld = a
                pack.append((src, off, self.send_buf, soff[p], rows, cols, ld, cols, False, None))
                soff[p] += rows * cols
        self.zero_list = zero
        self.pack_desc, self.unpack_desc = self._launches(pack), self._launches(unpack)

    @staticmethod
    def _launches(desc):
        """Split descriptors into launches in which no two pieces write intersecting boxes of
        the same buffer (pieces of one launch run concurrently; partial-sum pieces add)."""
        from flexmi.parallel.layout import _native
        ids = {}
        dst = [ids.setdefault(id(d[2]), len(ids)) for d in desc]
        sizes = _native().split_launches(dst, [None if d[9] is None else [list(r) for r in d[9]] for d in desc], 32)
        out, k = [], 0
        for n in sizes:
            out.append(desc[k:k + n])
            k += n
        return out

    @staticmethod
    def _run_desc(launches):
        from flexmi.ops import _kernels as K
        for ch in launches:
            mask = 0
            for k, d in enumerate(ch):
                if d[8]:
                    mask |= 1 << k
            K.C().multi_copy([d[0] for d in ch], [d[1] for d in ch], [d[2] for d in ch], [d[3] for d in ch],
                             [d[4] for d in ch], [d[5] for d in ch], [d[6] for d in ch], [d[7] for d in ch], mask)

    def pack(self):
        if self.fast:
            for z in self.zero_list:
                z.zero_()
            self._run_desc(self.pack_desc)
            return
        for (st, src, dst, acc), add in zip(self.items, self.adds):
            st.prepare_dst(dst, acc)
            st.local_copies(src, dst, add)
        off = list(self.send_off)
        per = defaultdict(list)
        for st, src, dst, acc in self.items:
            for p, lst in st.remote_sends(src).items():
                per[p].extend(lst)
        for p in range(self.world):
            for piece in per.get(p, []):
                n = piece.numel()
                self.send_buf[off[p]: off[p] + n].copy_(piece)
                off[p] += n

    def exchange(self, comm):
        self.start(comm)
        self.wait()

    def start(self, comm):
        """Launch the all_to_all asynchronously (RCCL runs on its own stream; the current
        stream keeps executing independent work until :meth:`wait`)."""
        import torch.distributed as dist
        if not self.active:
            return
        rs, ss = self.group_splits()
        if self.p2p:
            ops = []
            so = ro = 0
            for q, peer in enumerate(self._group_ranks()):
                if ss[q] > 0:
                    ops.append(dist.P2POp(dist.isend, self.send_buf[so:so + ss[q]], peer, group=self.pg))
                if rs[q] > 0:
                    ops.append(dist.P2POp(dist.irecv, self.recv_buf[ro:ro + rs[q]], peer, group=self.pg))
                so += ss[q]
                ro += rs[q]
            self.work = dist.batch_isend_irecv(ops) if ops else None
        else:
            self.work = dist.all_to_all_single(self.recv_buf, self.send_buf, rs, ss, group=self.pg, async_op=True)
        comm.calls += 1
        comm.bytes_sent += self.send_buf.numel() * self.send_buf.element_size()

    def _group_ranks(self):
        """Global ranks in the order of the exchange's communicator."""
        return list(self.participants) if self.pg is not None else list(range(self.world))

    def group_splits(self):
        """(recv, send) split sizes in the order of the exchange's communicator."""
        if self.pg is None:
            return list(self.recv_sizes), list(self.send_sizes)
        return [self.recv_sizes[p] for p in self.participants], [self.send_sizes[p] for p in self.participants]

    def wait(self):
        if self.work is not None:
            for w in (self.work if isinstance(self.work, list) else [self.work]):
                w.wait()
            self.work = None

    def unpack(self):
        if self.fast:
            self._run_desc(self.unpack_desc)
            return
        chunks = list(torch.split(self.recv_buf, self.recv_sizes))
        offs = [0] * self.world
        for (st, src, dst, acc), add in zip(self.items, self.adds):
            st.unpack(chunks, offs, dst, add)


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
        self.zero = False   # ZeRO-1 sharded optimizer state (Executor._zero_layout)
        self.shard_numel = 0

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
        self.debug = bool(getattr(self.cfg, "debug", False))
        self.watchdog = None
        if getattr(self.cfg, "watchdog_s", 0) > 0:
            from flexmi.runtime.health import Watchdog
            self.watchdog = Watchdog(self.cfg.watchdog_s, getattr(self.cfg, "watchdog_mode", "exit"))
        self.training = True
        self.step_count = 0
        self._grads_dirty = False       # gradients not yet consumed by an update (see capture_step)
        self._graph = None
        self._native = None
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
            owner = getattr(op, "shared_from", None)
            if owner is not None and owner.guid in self.pcs and op.valid_pc(self.pcs[owner.guid]):
                self.pcs[op.guid] = self.pcs[owner.guid]   # tied weights: the owner's shards
                continue
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
        # halo consumers (conv / pool) read the producer's buffer in place when every rank's need
        # box lies inside the box that rank already holds (no cross-rank halo; e.g. a 3x3/2 pool
        # that never reads the last row): no copy in forward, no zero + accumulate of the input
        # gradient in backward -- the op derives its pads from the bigger box
        for op in ops:
            if not getattr(op, "superset_input_ok", False):
                continue
            for i, t in enumerate(op.inputs):
                need, home = self.need[(op.guid, i)], self.home.get(t.guid)
                if home is None or need.same_as(home) or need.partial or home.partial or need.shape != home.shape:
                    continue
                if need.ranks() != home.ranks():
                    continue
                inside = True
                for r in need.ranks():
                    if len(need.parts_of(r)) != 1 or len(home.parts_of(r)) != 1:
                        inside = False
                        break
                    nb, hb = need.local_box(r), home.local_box(r)
                    if any(a0 < b0 or a1 > b1 for (a0, a1), (b0, b1) in zip(nb, hb)):
                        inside = False
                        break
                if inside:
                    self.need[(op.guid, i)] = home
        self.tensors = {}
        for op in ops:
            for t in op.inputs + op.outputs:
                self.tensors[t.guid] = t
        self.final_op = ops[-1]
        plan = self._native_plan(ops)
        by_guid = {op.guid: op for op in ops}
        ops = [by_guid[g] for g in plan[0]]
        self.ops = ops

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

        # ---- forward/backward schedules (graph planner: csrc/runtime/planner.cc) ---
        self.fwd_steps = []
        self.bwd_steps = []
        for kind, g, idxs in plan[1]:
            op = by_guid[g]
            if kind == 0:
                self.fwd_steps.append(("op", op))
                continue
            lst = []
            for i in idxs:
                t = op.inputs[i]
                need, home = self.need[(op.guid, i)], self.home[t.guid]
                key = (t.guid, need.key())
                if key not in self.act and need.local_shape(self.rank) is not None:
                    self.act[key] = self._alloc(need.local_shape(self.rank), self._storage_dtype(t))
                dt = self._storage_dtype(t)
                lst.append((t.guid, home, need, ReshardStep(ReshardPlan(home, need), self.rank, self.world, dt, self.device)))
            self.fwd_steps.append(("reshard", lst))

        # grads: home-layout grad buffers for float tensors that need them.  Backward liveness
        # (planner): an op runs backward only when one of its outputs reaches the loss; its float
        # inputs then need gradients (graph inputs only when asked, e.g. for the cost measurement of
        # a single op).  Dead branches (an encoder's unused top output) are skipped.
        final = self.final_op.outputs[0]
        self.final = final
        self.bwd_live = set(plan[2])
        self.grad_needed = set(plan[3])
        for g in self.grad_needed:
            lay = self.home[g]
            shp = lay.local_shape(self.rank)
            if shp is not None:
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
        for kind, g, idxs in plan[4]:
            op = by_guid[g]
            if kind == 0:
                self.bwd_steps.append(("op", op))
                continue
            red = []
            for i in idxs:
                t = op.inputs[i]
                need, home = self.need[(op.guid, i)], self.home[t.guid]
                shp = need.local_shape(self.rank)
                if shp is not None:
                    self.tmp_grad[(op.guid, i)] = self._alloc(shp, self.cdtype)
                # the gradient of a partial-sum output (row-sharded embedding) is the FULL
                # gradient on every holder: reduce into home.as_full()
                red.append((op, i, t.guid,
                            ReshardStep(ReshardPlan(need.as_partial(), home.as_full()), self.rank, self.world,
                                        self.cdtype, self.device)))
            self.bwd_steps.append(("reduce", red))

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
            # a split whose extent does not divide the degree can leave this rank an empty output
            # box (e.g. 6 rows over 4 ranks -> 2/2/2/0): nothing to compute, zero input gradients
            c.empty = bool(c.outputs) and all(o is None or o.numel() == 0 for o in c.outputs)
            op.prepare(c)
            self.ctx[op.guid] = c
        self._build_groups(ops)
        self._build_epilogue_fusion(ops)
        self._build_binary_relu_fusion(ops)
        self._build_conv_chain_fusion(ops)
        self._build_interaction_act_fusion(ops)
        self.adam_state = torch.tensor([1.0, 1.0, 0.0], dtype=torch.float32, device=self.device)
        self._compile_program()

    def _native_plan(self, ops):
        """Graph-level plan from the native planner (csrc/runtime/planner.cc, flexmi._native):
        the communication-first topological order (producers of cross-device reshards and their
        ancestors first, so the asynchronous exchanges started after them overlap the remaining
        independent ops: DLRM embeddings first, their all-to-all hides behind the bottom MLP),
        the forward schedule (input reshards per dtype, each (tensor, layout) once, then the op),
        backward liveness and the backward schedule (live ops in reverse, each followed by the
        gradient reduce of its resharded inputs).  Depends only on the graph and layouts, so every
        rank derives the same plan (collectives are issued in the same order everywhere).
        Reference: the op walk of FFModel::compile / the task launches of forward/backward,
        src/runtime/model.cc:374-1180."""
        from flexmi import _native
        producer = {t.guid: op.guid for op in ops for t in op.outputs}
        need_ids, dt_ids = {}, {}
        spec = []
        for op in ops:
            ins = []
            for i, t in enumerate(op.inputs):
                need, home = self.need[(op.guid, i)], self.home[t.guid]
                reshard = not need.same_as(home)
                prod = producer.get(t.guid, -1)
                remote = (reshard and prod >= 0 and self.world > 1
                          and any(tr.src != tr.dst for tr in ReshardPlan(home, need).transfers))
                nid = need_ids.setdefault(need.key(), len(need_ids))
                did = dt_ids.setdefault(self._storage_dtype(t), len(dt_ids))
                ins.append((t.guid, prod, did, nid, _is_float(t.data_type), bool(op.needs_input_grad(i)),
                            reshard, remote))
            spec.append((op.guid, ins, [o.guid for o in op.outputs]))
        return _native.plan_graph(spec, self.world, bool(getattr(self.cfg, "input_grads", False)))

    def _build_epilogue_fusion(self, ops):
        """Linear L1 -> Linear L2 (L1's output consumed only by L2, same layout): L2's dX GEMM
        epilogue applies L1's activation backward and accumulates L1's bias gradient, so L1 skips
        its separate act-bwd/bias-grad pass (one full read+write of the activation gradient)."""
        from flexmi.core.types import ActiMode, OperatorType
        if self.backend != "hip":
            return
        for op in ops:
            if op.op_type != OperatorType.OP_LINEAR or getattr(op, "skip_act_grad", False):
                continue
            c1 = self.ctx.get(op.guid)
            t = op.outputs[0]
            cons = self.consumers.get(t.guid, [])
            if c1 is None or len(cons) != 1 or t is self.final:
                continue
            l2, idx = cons[0]
            c2 = self.ctx.get(l2.guid)
            # (a 1-wide L2 runs the skinny kernel, which applies L1's activation backward to its dX too)
            if (l2.op_type != OperatorType.OP_LINEAR or c2 is None or op.out_dim == 1
                    or not self.need[(l2.guid, idx)].same_as(self.home[t.guid]) or c2.in_grads[0] is None):
                continue
            c2.saved["fuse_below"] = (c1.outputs[0], op.activation)
            c1.saved["grad_is_dpre"] = True

    def _build_interaction_act_fusion(self, ops):
        """Linear L -> DotInteraction input 0 (the DLRM bottom MLP's last layer; L's output consumed
        only there, same layout, fp32): the interaction backward applies L's activation backward to
        the gradient it writes (interaction.hip act0), so L skips its separate act-bwd / bias-grad
        pass and sums its bias gradient in its dW GEMM."""
        from flexmi.core.types import OperatorType
        if self.backend != "hip" or self.cfg.compute_dtype != "fp32":
            return
        for op in ops:
            if op.op_type != OperatorType.OP_LINEAR or getattr(op, "skip_act_grad", False):
                continue
            c1 = self.ctx.get(op.guid)
            t = op.outputs[0]
            cons = self.consumers.get(t.guid, [])
            if c1 is None or len(cons) != 1 or t is self.final or c1.saved.get("grad_is_dpre"):
                continue
            dop, idx = cons[0]
            cd = self.ctx.get(dop.guid)
            if (type(dop).__name__ != "DotInteraction" or idx != 0 or cd is None or cd.in_grads[0] is None
                    or not self.need[(dop.guid, idx)].same_as(self.home[t.guid])):
                continue
            cd.saved["act0"] = int(op.activation)
            c1.saved["grad_is_dpre"] = True

    def _build_binary_relu_fusion(self, ops):
        """ElementBinary A -> ReLU B (A's output consumed only by B, same layout, B's input gradient
        A's output gradient): A writes relu(a op b) straight into B's output and, in backward, masks
        B's output gradient by (B's output > 0) itself; B runs nothing.  The ResNet residual add +
        ReLU then costs one pass per direction instead of two (reference: element_binary.cu and
        element_unary.cu as separate cuDNN calls).  Off under --debug (A's own output stays unwritten)."""
        from flexmi.core.types import OperatorType
        if self.backend != "hip" or self.debug:
            return
        bin_types = (OperatorType.OP_EW_ADD, OperatorType.OP_EW_SUB, OperatorType.OP_EW_MUL, OperatorType.OP_EW_DIV)
        for op in ops:
            if op.op_type not in bin_types:
                continue
            ca = self.ctx.get(op.guid)
            t = op.outputs[0]
            cons = self.consumers.get(t.guid, [])
            if ca is None or ca.empty or len(cons) != 1 or t is self.final:
                continue
            b, idx = cons[0]
            cb = self.ctx.get(b.guid)
            if (b.op_type != OperatorType.OP_RELU or cb is None or cb.empty
                    or op.guid in self.group_of or b.guid in self.group_of
                    or not self.need[(b.guid, idx)].same_as(self.home[t.guid])
                    or not self.home[b.outputs[0].guid].same_as(self.home[t.guid])
                    or cb.outputs[0] is None or cb.out_grads[0] is None
                    or cb.outputs[0].shape != ca.outputs[0].shape):
                continue
            ca.saved["fused_relu"] = (cb.outputs[0], cb.out_grads[0])
            cb.saved["fused_into_binary"] = True

    def _build_conv_chain_fusion(self, ops):
        """Conv A -> Conv B (A's output consumed only by B, same layout, both on the NHWC-staged bf16
        path): A's forward epilogue also writes its output straight into B's staged NHWC input, so B
        skips its staging pass, and when A is linear (no activation) A's NCHW output is not written
        at all.  Backward mirror (A linear, B the sole consumer): B's data-gradient epilogue writes
        A's staged output gradient (padded / stride-dilated for A's own data gradient), so A skips
        its gradient staging and B's NCHW dX is not written.  The staged buffers are per-op and
        zero-initialised once: their halos / dilation gaps are never written.  FM_CONV_CHAIN=0 turns
        it off (A/B); off under --debug (skipped NCHW buffers stay unwritten)."""
        from flexmi.core.types import ActiMode, OperatorType
        from flexmi.ops import _kernels as K
        if self.backend != "hip" or self.debug or os.environ.get("FM_CONV_CHAIN", "1") == "0":
            return
        for op in ops:
            if op.op_type != OperatorType.OP_CONV2D:
                continue
            ca = self.ctx.get(op.guid)
            t = op.outputs[0]
            cons = self.consumers.get(t.guid, [])
            if ca is None or ca.empty or len(cons) != 1 or t is self.final or op.guid in self.group_of:
                continue
            b, idx = cons[0]
            cb = self.ctx.get(b.guid)
            if (b.op_type != OperatorType.OP_CONV2D or cb is None or cb.empty or b.guid in self.group_of
                    or not self.need[(b.guid, idx)].same_as(self.home[t.guid])):
                continue
            xa, wa, ya = ca.inputs[0], ca.wcompute[0], ca.outputs[0]
            xb, wb, yb = cb.inputs[0], cb.wcompute[0], cb.outputs[0]
            if any(v is None for v in (xa, wa, ya, xb, wb, yb)) or xb.shape != ya.shape:
                continue
            if not (K._nhwc_ok(xa, wa, op.groups) and K._nhwc_ok(xb, wb, b.groups)):
                continue
            dev = ya.device
            # forward: A's epilogue -> B's staged input
            N, Hp, Wp, Cp, top, left = K.nhwc_x_geometry(xb.shape, wb.shape, yb.shape, (b.sh, b.sw), b._pads(cb))
            xs_b = torch.zeros((N, Hp, Wp, Cp), dtype=ya.dtype, device=dev)
            cb.saved["nhwc_x"], cb.saved["nhwc_x_prestaged"] = xs_b, True
            linear = op.activation == ActiMode.AC_MODE_NONE
            ca.saved["nhwc_out2"] = (xs_b, (Hp, Wp, Cp, top, left, 1, 1, 0 if linear else 1))
            # backward: B's data gradient -> A's staged output gradient (G_A = dY_A for a linear A)
            if not linear or not cb.in_grads or cb.in_grads[0] is None or cb.in_grad_accumulate[0]:
                continue
            need_dx = bool(ca.in_grads) and ca.in_grads[0] is not None
            geo = K.nhwc_g_geometry(xa.shape, wa.shape, ya.shape, (op.sh, op.sw), op._pads(ca), need_dx)
            if geo is None:
                continue
            N, Hg, Wg, Kp, gt, gl, dh, dw = geo
            gs_a = torch.zeros((N, Hg, Wg, Kp), dtype=ya.dtype, device=dev)
            ca.saved["nhwc_gs"], ca.saved["nhwc_g_prestaged"] = gs_a, True
            cb.saved["nhwc_dgrad_out2"] = (gs_a, (Hg, Wg, Kp, gt, gl, dh, dw, 0))

    def _build_groups(self, ops):
        """Fuse independent ops of the same kind and placement into one launch (embedding
        tables of a DLRM graph: 26 ops -> 1 forward + 2 backward launches).  Members run at the
        first member's position in forward and at the last position (in backward order, i.e.
        the first member) in backward, when every member's output gradient is final."""
        from flexmi.core.types import OperatorType
        self.group_of = {}
        groups = []
        pos = {st[1].guid: k for k, st in enumerate(self.fwd_steps) if st[0] == "op"}

        def ready_at(op, lead):
            # a member runs at the leader's forward position: every input must already hold its
            # values there -- needed in its home layout (no reshard emitted later) and either a
            # model input or produced by an op scheduled before the leader
            for i, t in enumerate(op.inputs):
                if not self.need[(op.guid, i)].same_as(self.home[t.guid]):
                    return False
                if t.owner_op is not None and pos.get(t.owner_op.guid, 1 << 30) >= pos[lead.guid]:
                    return False
            return True

        for op in ops:
            c = self.ctx.get(op.guid)
            if c is None or op.op_type != OperatorType.OP_EMBEDDING or getattr(op, "host_exec", False):
                continue
            pc = self.pcs[op.guid]
            for g in groups:
                lead = g[0]
                if (self.pcs[lead.guid] == pc and ready_at(op, lead)
                        and type(lead).can_group(lead, op, self.ctx[lead.guid], c)):
                    g.append(op)
                    break
            else:
                groups.append([op])
        for g in groups:
            if len(g) > 1:
                for op in g:
                    self.group_of[op.guid] = g

    # ------------------------------------------------------------------
    @staticmethod
    def _sdp_pays(op, lay):
        """Replicated table: sparse DP (touched-row all-gather) only where it moves fewer bytes
        than the dense replica all-reduce (Embedding.sdp_prefer_sparse; the search prices the same
        rule).  Every rank decides from global shapes only, so all replicas agree."""
        from flexmi.ops.embedding import Embedding
        R = lay.replication()
        box = lay.part_box(0)
        rows = box[0][1] - box[0][0]
        cols = 1
        for lo, hi in box[1:]:
            cols *= hi - lo
        B = op.inputs[0].dims[0]
        bag = op.inputs[0].dims[1] if len(op.inputs[0].dims) > 1 else 1
        return Embedding.sdp_prefer_sparse(rows, cols, -(-B // R) * bag, R)

    def _build_weights(self, ops):
        self.wentries: Dict[int, WeightEntry] = {}
        groups: "OrderedDict[tuple, SyncGroup]" = OrderedDict()
        sparse_ok = isinstance(self.optimizer, SGDOptimizer) and self.optimizer.sparse_capable
        for op in reversed(ops):  # backward order => buckets fill contiguously
            pc = self.pcs[op.guid]
            lays = op.weight_layouts(pc)
            for wi, w in enumerate(op.weights):
                if w.guid in self.wentries:   # tied weight (shared_op): one entry, grads summed
                    assert self.wentries[w.guid].layout.same_as(lays[wi]), f"{op.name}: tied weight sharded differently"
                    continue
                e = WeightEntry(w, op, wi, lays[wi], self.rank)
                self.wentries[w.guid] = e
                if e.box is None:
                    continue
                from flexmi.core.types import OperatorType
                if pc.device_type == ParallelConfig.CPU:
                    # heterogeneous placement (dlrm_strategy_hetero.cc): the table
                    # lives in (pinned) host memory and its lookups / sparse SGD run on the host
                    if op.op_type != OperatorType.OP_EMBEDDING or not sparse_ok:
                        raise NotImplementedError(f"{op.name}: CPU placement is supported for embedding "
                                                  "tables trained with SGD (the reference's hetero strategy)")
                    e.sparse = True
                    op.sparse_sgd = True
                    op.host_exec = True
                    e.master = torch.empty(e.shape, dtype=torch.float32, pin_memory=self.backend == "hip")
                    e.compute = e.master
                    continue
                if op.op_type == OperatorType.OP_EMBEDDING:
                    op.sparse_dp = None
                if (op.op_type == OperatorType.OP_EMBEDDING and sparse_ok
                        and (lays[wi].replication() == 1 or (SPARSE_DP and self._sdp_pays(op, lays[wi])))):
                    # non-replicated: fused sparse SGD; replicated: sparse data parallelism
                    # (touched-row all-gather over the replica set, Embedding.sdp_*)
                    e.sparse = True
                    op.sparse_sgd = True
                    if lays[wi].replication() > 1:
                        op.sparse_dp = tuple(sorted(e.holders))
                    e.master = self._alloc(e.shape, torch.float32)
                    e.compute = e.master
                    continue
                key = e.holders
                if key not in groups:
                    groups[key] = SyncGroup(key)
                g = groups[key]
                e.group = g
                g.entries.append(e)
        self.groups = list(groups.values())
        mixed = self.cdtype != torch.float32
        cap = max(1, int(self.cfg.grad_bucket_mb * (1 << 20) / 4))
        zero = int(getattr(self.cfg, "zero_stage", 0)) >= 1
        from flexmi import _native
        for g in self.groups:
            g.zero = zero and g.replicated
            if g.zero:
                self._zero_layout(g, cap)
            else:
                # flat buffer layout + all-reduce buckets from the native plan compiler (the same
                # planner as the C++ model, csrc/runtime/native_model.cc plan_weights): 256-B aligned
                # views (16-B vector loads in every kernel), buckets in backward order
                offs, g.numel, bks = _native.plan_weights([e.numel for e in g.entries], cap)
                for e, o in zip(g.entries, offs):
                    e.offset = int(o)
                g.buckets = [[int(b[0]), int(b[1]), {g.entries[int(i)].param.guid for i in b[2:]}] for b in bks]
            # zeroed: the 256-B alignment gaps between entries are never written by an initializer,
            # and the replica checksums / finiteness checks (--debug) read the whole flat buffer --
            # uninitialised gaps made identical replicas look divergent (or non-finite)
            g.master = torch.zeros((g.numel,), dtype=torch.float32, device=self.device)
            g.gradbuf = self._alloc((g.numel,), torch.float32)
            g.gradbuf.zero_()
            g.compute = torch.zeros((g.numel,), dtype=self.cdtype, device=self.device) if mixed else g.master
            snames = self.optimizer.state_names() if self.optimizer else []
            # ZeRO-1: optimizer state exists only for this rank's shard of every bucket
            g.state = {n: torch.zeros(g.shard_numel if g.zero else g.numel, dtype=torch.float32, device=self.device)
                       for n in snames}
            if g.zero:
                g.gshard = self._alloc((g.shard_numel,), torch.float32)
                g.mshard = self._alloc((g.shard_numel,), torch.float32)
            for e in g.entries:
                sl = slice(e.offset, e.offset + e.numel)
                e.master = g.master[sl].view(e.shape)
                e.grad = g.gradbuf[sl].view(e.shape)
                e.compute = g.compute[sl].view(e.shape)
                e.state = {} if g.zero else {n: s[sl].view(e.shape) for n, s in g.state.items()}

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
            if g.zero:
                for full, sh in self._zero_pieces(g):
                    g.mshard[sh].copy_(g.master[full])
        lr = getattr(self.optimizer, "lr", 0.01) if self.optimizer else 0.0
        self.lr_tensor = torch.tensor([lr], dtype=torch.float32, device=self.device)
        self.pending = {}

    # ------------------------------------------------------------------ ZeRO-1
    # Optimizer-state sharding for replicated weight groups.  Every gradient bucket is padded to a
    # multiple of (replicas x 64) elements; backward reduce-scatters each bucket as soon as it is
    # final (RCCL ring reduce-scatter: half the bytes of the all-reduce it replaces), each replica
    # updates only its 1/R slice of every bucket -- fp32 master shard + optimizer state exist for
    # that slice only -- and the update all-gathers the fresh master slices back into the full
    # replicated buffer (the other half of the ring all-reduce).  Same bytes on xGMI as plain DP,
    # 1/R of the optimizer state and optimizer-kernel work per GPU.
    def _zero_layout(self, g, cap):
        R = len(g.holders)
        quant = R * 64
        off = start = 0
        ids = set()
        g.buckets = []
        for e in g.entries:
            sz = (e.numel + 63) // 64 * 64
            if ids and off + sz - start > cap:
                end = start + -(-(off - start) // quant) * quant
                g.buckets.append([start, end, ids])
                start = off = end
                ids = set()
            e.offset = off
            off += sz
            ids.add(e.param.guid)
        end = start + -(-(off - start) // quant) * quant
        g.buckets.append([start, end, ids])
        g.numel = end
        g.zero_rank = sorted(g.holders).index(self.rank)
        g.zero_R = R
        g.shard_numel = sum((b[1] - b[0]) // R for b in g.buckets)

    def _zero_pieces(self, g):
        """[(slice of the full flat buffer owned by this rank, slice of the shard buffers)] per bucket."""
        out, so = [], 0
        for b0, b1, _ in g.buckets:
            n = (b1 - b0) // g.zero_R
            lo = b0 + g.zero_rank * n
            out.append((slice(lo, lo + n), slice(so, so + n)))
            so += n
        return out

    def _zero_rs(self, g, bi, sync=True):
        b0, b1, _ = g.buckets[bi]
        sh = self._zero_pieces(g)[bi][1]
        return self.comm.reduce_scatter_async(g.gshard[sh], g.gradbuf[b0:b1], g.holders) if not sync else \
            self.comm.reduce_scatter(g.gshard[sh], g.gradbuf[b0:b1], g.holders)

    def _zero_gather(self):
        for g in self.groups:
            if not g.zero:
                continue
            for bi, (full, sh) in enumerate(self._zero_pieces(g)):
                b0, b1, _ = g.buckets[bi]
                self.comm.all_gather(g.master[b0:b1], g.mshard[sh], g.holders)

    def _zero_cast(self):
        for g in self.groups:
            if g.zero and g.compute is not g.master:
                g.compute.copy_(g.master)

    def zero_materialize_state(self):
        """Collective: full-size optimizer state for every ZeRO group (entries' ``state`` views
        point into it) -- for checkpointing, which stores per-parameter state."""
        for g in self.groups:
            if not g.zero:
                continue
            g.state_full = {}
            for n, st in g.state.items():
                full = torch.zeros(g.numel, dtype=torch.float32, device=self.device)
                for bi, (fsl, sh) in enumerate(self._zero_pieces(g)):
                    b0, b1, _ = g.buckets[bi]
                    self.comm.all_gather(full[b0:b1], st[sh].contiguous(), g.holders)
                g.state_full[n] = full
            for e in g.entries:
                sl = slice(e.offset, e.offset + e.numel)
                e.state = {n: f[sl].view(e.shape) for n, f in g.state_full.items()}

    def zero_release_state(self, scatter=False):
        """Drop the full-size state views; with ``scatter`` (after a load) keep this rank's slice."""
        for g in self.groups:
            if not g.zero or getattr(g, "state_full", None) is None:
                continue
            if scatter:
                for n, st in g.state.items():
                    for fsl, sh in self._zero_pieces(g):
                        st[sh].copy_(g.state_full[n][fsl])
                for fsl, sh in self._zero_pieces(g):
                    g.mshard[sh].copy_(g.master[fsl])
            g.state_full = None
            for e in g.entries:
                e.state = {}

    def set_lr(self, lr):
        self.lr_tensor.fill_(float(lr))

    def pcs_by_name(self):
        return {op.name: self.pcs[op.guid] for op in self.model.layers}

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

    # The step is compiled ONCE into a flat program of items; "compute" items only enqueue
    # HIP work on the current stream (capturable), "comm" items call RCCL.  Eager execution runs
    # the items in order; graph mode captures every maximal run of compute items into one
    # hipGraph and runs the collectives eagerly between replays (segmented capture).
    # ------------------------------------------------------------ micro-batch pipeline
    def _plan_pipeline(self):
        """The chunked tail of XCHG_CHUNKS, or None.  Decided from global layouts only (every rank
        takes the same decision: the chunk all-to-alls are collectives).  Conditions: the last
        cross-device forward exchange is followed by ops only; each is a row-wise kind (Linear,
        DotInteraction, Concat off the sample dim) whose outputs and needed inputs are one-holder sample splits over the
        whole world with identical per-rank rows; every rank holds >= 8 rows per chunk."""
        from flexmi.core.types import OperatorType
        if self.world == 1 and not XCHG_LOCAL:
            return None
        steps = self.fwd_steps
        W = self.world

        def rowwise(op):
            return op.op_type in (OperatorType.OP_LINEAR, OperatorType.OP_DOT_INTERACTION) or (
                op.op_type == OperatorType.OP_CONCAT and op.axis != 0)

        xk = [k for k, st in enumerate(steps)
              if st[0] == "reshard" and not all(rs.local_only for *_, rs in st[1])]
        if xk:
            k0 = xk[-1]
        elif XCHG_LOCAL:
            k0 = len(steps) - 1       # the longest row-wise suffix, after an op step
            while k0 >= 0 and steps[k0][0] == "op" and rowwise(steps[k0][1]):
                k0 -= 1
            if k0 < 0 or steps[k0][0] != "op":
                return None
        else:
            return None
        if k0 == len(steps) - 1 or any(st[0] != "op" for st in steps[k0 + 1:]):
            return None
        region = [st[1] for st in steps[k0 + 1:]]

        def sample_split(lay):
            return (not lay.partial and lay.boxes is None and all(d == 1 for d in lay.degrees[1:])
                    and lay.degrees[0] == W and all(len(h) == 1 for h in lay.holders)
                    and sorted(h[0] for h in lay.holders) == list(range(W)))

        rows = None
        for op in region:
            if not rowwise(op) or getattr(op, "host_exec", False) or op.guid in self.group_of:
                return None
            lays = [self.home[o.guid] for o in op.outputs] + [self.need[(op.guid, i)] for i in range(len(op.inputs))]
            for lay in lays:
                if not sample_split(lay):
                    return None
                ext = tuple(tuple(lay.local_box(r)[0]) for r in range(W))
                if rows is None:
                    rows = ext
                elif ext != rows:
                    return None
        nmin = min(hi - lo for lo, hi in rows)
        K = (2 if nmin >= 1024 else 1) if XCHG_CHUNKS == "auto" else int(XCHG_CHUNKS)
        if K <= 1 or nmin < PIPE_ROW_ALIGN * K:
            return None
        # backward: the tail's ops contiguous in backward order, then the gradient return of
        # exactly their inputs -- otherwise the backward runs whole-batch (forward still chunked)
        rset = {op.guid for op in region}
        bs = self.bwd_steps
        pos = [k for k, st in enumerate(bs) if st[0] == "op" and st[1].guid in rset]
        kb = None
        if pos and pos == list(range(pos[0], pos[0] + len(region))) and [bs[k][1] for k in pos] == list(reversed(region)):
            nxt = bs[pos[-1] + 1] if pos[-1] + 1 < len(bs) else None
            if nxt is None or nxt[0] != "reduce":
                kb = pos[0] if not xk else None          # world-1 test hook: no gradient return
            elif all(op.guid in rset for op, *_ in nxt[1]):
                kb = pos[0]
        lo_r, hi_r = rows[self.rank]
        b = chunk_bounds(hi_r - lo_r, K)
        ctx = [{op.guid: self._chunk_ctx(op, b[c], b[c + 1]) for op in region} for c in range(K)]
        return {"k": k0, "region": region, "K": K, "rows": rows, "kb": kb, "ctx": ctx}

    def _chunk_ctx(self, op, a, b):
        """Op context of local rows [a, b): row views of the whole-batch buffers (so the chunks'
        forward fills the same activations the backward reads), shared weights / gradients; a
        Linear's act-backward scratch is one whole-batch buffer whose row slices the chunks'
        input-gradient passes fill and the whole-batch weight-gradient pass reads."""
        import copy
        from flexmi.core.types import ActiMode, OperatorType
        c = self.ctx[op.guid]
        cc = copy.copy(c)

        def rows(t):
            if t is None:
                return None
            return t[a:b]

        cc.inputs = [rows(t) for t in c.inputs]
        cc.outputs = [rows(t) for t in c.outputs]
        cc.in_grads = [rows(t) for t in c.in_grads]
        cc.out_grads = [rows(t) for t in c.out_grads]
        cc.in_grad_accumulate = list(c.in_grad_accumulate)
        cc.in_boxes = [None if bx is None else ((bx[0][0] + a, bx[0][0] + b),) + tuple(bx[1:]) for bx in c.in_boxes]
        cc.out_boxes = [None if bx is None else ((bx[0][0] + a, bx[0][0] + b),) + tuple(bx[1:]) for bx in c.out_boxes]
        cc.saved = dict(c.saved)
        fb = c.saved.get("fuse_below")
        if fb is not None:
            cc.saved["fuse_below"] = (fb[0][a:b], fb[1])
        cc.workspace = {}
        if (op.op_type == OperatorType.OP_LINEAR and c.hip and op.activation != ActiMode.AC_MODE_NONE
                and not getattr(op, "skip_act_grad", False) and not c.saved.get("grad_is_dpre", False)
                and c.out_grads and c.out_grads[0] is not None):
            y = c.outputs[0]
            inner = y.numel() // max(1, y.shape[0] * y.shape[-1])
            full = c.workspace.get("dpre")
            shp = (y.numel() // y.shape[-1], y.shape[-1])
            if full is None or tuple(full.shape) != shp:
                full = torch.empty(shp, dtype=c.out_grads[0].dtype, device=y.device)
                c.workspace["dpre"] = full
            cc.workspace["dpre"] = full[a * inner: b * inner]
        return cc

    def _chunk_items(self, items, side, c, pipe):
        """Reshard items of chunk c: each plan clipped to chunk c of the sample-split side's rows;
        a partial-sum destination is zeroed by chunk 0 only (later chunks add into it)."""
        K = pipe["K"]

        def rows(lo, hi):
            b = chunk_bounds(hi - lo, K)
            return lo + b[c], lo + b[c + 1]

        out = []
        for rs, src, dst, acc in items:
            st = ReshardStep(rs.plan.clip_rows(side, rows), self.rank, self.world, rs.dtype, rs.device)
            out.append((st, src, dst, acc if c == 0 else (acc or rs.plan.src.partial)))
        return out

    def _emit_pipelined_fwd(self, fwd, exs, pipe):
        for c in range(pipe["K"]):
            if exs:
                self._emit_exchange_finish(fwd, exs[c], "reshard.fwd")
            for op in pipe["region"]:
                cc = pipe["ctx"][c][op.guid]
                fwd.append(Item("compute", (lambda op=op, cc=cc: self._fwd_op(op, cc)), f"{op.name}.c{c}.fwd"))
                fwd[-1].reads = {t.guid for t in op.inputs}
                fwd[-1].writes = {t.guid for t in op.outputs}
                fwd[-1].check = (lambda op=op, cc=cc: self._check_op(op.name + ".fwd", cc.outputs, "output"))

    def _compile_program(self):
        tm = self.timer
        fwd, bwd, upd = [], [], []

        def C(lst, name, fn):
            lst.append(Item("compute", fn, name))

        # the NHWC convolutions' weight re-layouts of the step in one launch before the forward
        # (flexmi/ops/_kernels.py conv_wprep_all; layers join after their first NHWC forward)
        from flexmi.core.types import OperatorType as _OT
        convs = [st[1] for st in self.fwd_steps if st[0] == "op" and st[1].op_type == _OT.OP_CONV2D]
        if self.backend == "hip" and convs and CONV_WPREP_ALL:
            def wprep_all(convs=convs):
                from flexmi.ops import _kernels as K
                layers = []
                for op in convs:
                    c = self.ctx.get(op.guid)
                    if c is not None and not c.empty and c.wcompute and c.wcompute[0] is not None:
                        layers.append((c.wcompute[0], c.saved))
                K.conv_wprep_all(layers)
            C(fwd, "conv.wprep_all", wprep_all)

        # ---------------- forward
        # cross-device reshards are split: pack + asynchronous all_to_all right after the last
        # producer of their sources, wait + unpack right before the consumer -- so the ops in
        # between (e.g. the DLRM bottom MLP) overlap the embedding exchange
        pipe = self.pipe = self._plan_pipeline()
        op_pos = {st[1].guid: k for k, st in enumerate(self.fwd_steps) if st[0] == "op"}
        launch_after = defaultdict(list)     # fwd step index -> exchanges to start after it
        deferred = {}                        # fwd step index of a reshard -> its exchange
        for k, st in enumerate(self.fwd_steps):
            if st[0] != "reshard":
                continue
            items = [(rs, self.act.get((g, home.key())), self.act.get((g, need.key())), False)
                     for g, home, need, rs in st[1]]
            if self.world == 1 or all(rs.local_only for rs, *_ in items):
                continue
            prods = [op_pos[self.tensors[g].owner_op.guid] for g, *_ in st[1]
                     if self.tensors[g].owner_op is not None and self.tensors[g].owner_op.guid in op_pos]
            if pipe is not None and k == pipe["k"]:
                exs = [FusedExchange(self._chunk_items(items, "dst", c, pipe), self.world, self.rank, self.comm)
                       for c in range(pipe["K"])]
                for c, ex in enumerate(exs):
                    ex.tag = f"reshard.fwd.c{c}"
            else:
                exs = [FusedExchange(items, self.world, self.rank, self.comm)]
            deferred[k] = exs
            launch_after[max(prods) if prods else -1].extend(exs)
        for ex in launch_after.get(-1, []):
            self._emit_exchange_start(fwd, ex, "reshard.fwd")
        for k, st in enumerate(self.fwd_steps):
            if pipe is not None and k > pipe["k"]:
                break                          # the tail was emitted chunk by chunk
            if st[0] == "reshard":
                if k in deferred:
                    if pipe is not None and k == pipe["k"]:
                        self._emit_pipelined_fwd(fwd, deferred[k], pipe)
                    else:
                        self._emit_exchange_finish(fwd, deferred[k][0], "reshard.fwd")
                else:
                    items = [(rs, self.act.get((g, home.key())), self.act.get((g, need.key())), False)
                             for g, home, need, rs in st[1]]
                    self._emit_reshards(fwd, items, "reshard.fwd")
                continue
            self._emit_fwd_op(fwd, st[1])
            for ex in launch_after.get(k, []):
                self._emit_exchange_start(fwd, ex, "reshard.fwd")
            if pipe is not None and k == pipe["k"]:
                self._emit_pipelined_fwd(fwd, [], pipe)     # world-1 test hook: no exchange

        # ---------------- backward (accumulate flags resolved at compile time)
        self._compile_backward(bwd, C)

        # ---------------- update
        if any(g.replicated for g in self.groups):
            upd.append(Item("comm", self._sync_grads, "allreduce.wait", native=("ar_sync",)))
        if self.optimizer is not None:
            C(upd, "update", self._optimizer_step)
            if any(g.zero for g in self.groups):
                upd.append(Item("comm", self._zero_gather, "zero.allgather", native=("ag_sync",)))
                C(upd, "zero.cast", self._zero_cast)
        self.prog_fwd, self.prog_bwd, self.prog_upd = fwd, bwd, upd
        self._plan_fused_sgd()

    def _plan_fused_sgd(self):
        """SGD fused into the weight-gradient GEMMs of the training step (FM_FUSED_SGD, default on).

        A Linear weight qualifies when its gradient has no consumer besides the optimizer: SGD,
        HIP backend, the weight's group is not replicated (no all-reduce) nor ZeRO-sharded, the
        weight belongs to one op (not tied), and no debug guards.  For those, the step program
        (``step_program`` / ``train_step``) runs the backward with ``ctx.fused_sgd`` armed: the op's
        dW GEMM updates master, momentum and bf16 mirror in its epilogue after the op's dX GEMM
        (csrc/kernels/gemm.hip fm_gemm_dw_sgd), and the update program runs the optimizer over the
        remaining ranges only (one segmented launch).  ``backward()`` / ``update()`` called
        separately keep the unfused semantics (gradients materialised, then updated).
        Reference: the separate dW (linear.cu:592-635) and sgd_update (optimizer_kernel.cu:23-41)
        tasks, which this removes the gradient's HBM round trip (write, read, re-zero) between."""
        from flexmi.core.types import OperatorType
        from flexmi.ops import _kernels as K
        self.fused_sgd_state = {"on": False}
        self.fused_sgd_entries = []
        self.prog_bwd_fused = self.prog_upd_fused = None
        opt = self.optimizer
        if (self.backend != "hip" or not isinstance(opt, SGDOptimizer) or self.debug
                or os.environ.get("FM_FUSED_SGD", "1") == "0"):
            return
        # only weights big enough for the saved gradient round trip to matter: on the MLPerf DLRM
        # (<= 1 M-element candidates) fusing measured 0.3-0.9 % slower, on summit_large
        # (16-42 M-element layers) 1.61 -> 1.17 ms bf16 (profiles/fused_sgd_ab_r4i.txt)
        min_numel = FUSED_SGD_MIN
        uses = defaultdict(int)
        for st in self.bwd_steps:
            if st[0] == "op":
                for w in st[1].weights:
                    uses[w.guid] += 1
        for e in self.wentries.values():
            g = e.group
            if (g is None or g.replicated or g.zero or e.numel < max(1, min_numel) or e.widx != 0 or uses[e.param.guid] != 1
                    or e.op.op_type != OperatorType.OP_LINEAR):
                continue
            c = self.ctx.get(e.op.guid)
            if c is None or not c.weight_grads or c.weight_grads[0] is not e.grad or not c.inputs:
                continue
            # weights whose dW runs in the library GEMM (fp32 big layers) or the skinny kernel keep
            # their gradient and stay in the one segmented optimizer launch
            n_out, n_in = e.master.shape[0], e.master.numel() // max(1, e.master.shape[0])
            rows = c.inputs[0].numel() // max(1, c.inputs[0].shape[-1])
            if n_out == 1 or K._dw_lib(rows, n_out, n_in, self.cdtype):
                continue
            c.fused_sgd = K.FusedSGD(e.master, e.compute if g.compute is not g.master else None,
                                     e.state.get("v") if opt.momentum > 0 else None, self.lr_tensor,
                                     opt.weight_decay, opt.momentum, opt.nesterov)
            c.fused_sgd_state = self.fused_sgd_state
            self.fused_sgd_entries.append(e)
        if not self.fused_sgd_entries:
            return
        # per group: the ranges the update program still covers (gaps between fused weights)
        fused = defaultdict(list)
        for e in self.fused_sgd_entries:
            fused[id(e.group)].append((e.offset, e.offset + e.numel))
        for g in self.groups:
            spans = sorted(fused.get(id(g), []))
            rest, at = [], 0
            for lo, hi in spans:
                if lo > at:
                    rest.append((at, lo - at))
                at = max(at, hi)
            if at < g.numel:
                rest.append((at, g.numel - at))
            g.sgd_rest = rest if spans else None

        def arm(on):
            self.fused_sgd_state["on"] = on
        self.prog_bwd_fused = ([Item("compute", (lambda: arm(True)), "fused_sgd.arm")] + self.prog_bwd +
                               [Item("compute", (lambda: arm(False)), "fused_sgd.disarm")])
        self.prog_upd_fused = [Item("compute", (lambda: self._optimizer_step(fused=True)), "update")
                               if it.name == "update" else it for it in self.prog_upd]

    def _emit_exchange_start(self, lst, ex, name):
        name = getattr(ex, "tag", None) or name
        lst.append(Item("compute", ex.pack, name + ".pack"))
        lst.append(Item("comm", (lambda ex=ex: ex.start(self.comm)), name + ".a2a", native=("a2a", ex)))

    def _emit_exchange_finish(self, lst, ex, name):
        name = getattr(ex, "tag", None) or name
        lst.append(Item("comm", ex.wait, name + ".wait", native=("wait", ex)))
        lst.append(Item("compute", ex.unpack, name + ".unpack"))

    def _emit_fwd_op(self, fwd, op):
        c = self.ctx.get(op.guid)
        if c is None:
            return
        grp = self.group_of.get(op.guid)
        if grp is not None:
            if grp[0] is op:
                fwd.append(Item("compute", (lambda grp=grp: type(grp[0]).forward_group(grp, [self.ctx[o.guid] for o in grp])),
                                op.name + ".group_fwd"))
                fwd[-1].reads = {t.guid for o in grp for t in o.inputs}
                fwd[-1].writes = {t.guid for o in grp for t in o.outputs}
            return
        kind = "comm" if getattr(op, "host_exec", False) else "compute"   # host ops are never captured
        fwd.append(Item(kind, (lambda op=op, c=c: self._fwd_op(op, c)), op.name + ".fwd"))
        fwd[-1].reads = {t.guid for t in op.inputs}
        fwd[-1].writes = {t.guid for t in op.outputs}
        fwd[-1].check = (lambda op=op, c=c: self._check_op(op.name + ".fwd", c.outputs, "output"))

    def _compile_backward(self, bwd, C):
        written = set()
        # gradient reductions into a tensor's home grad buffer are started where the consumer's
        # backward produced them and finished right before the first later step that touches
        # that buffer (normally the producer op's backward), overlapping the steps in between
        finish_before = defaultdict(list)
        for g in self.groups:   # weight/bias grads accumulate (atomics in fused epilogues): one memset
            if g.numel:
                C(bwd, "zero_grads", (lambda g=g: g.gradbuf.zero_()))
                bwd[-1].zero_group = g   # dropped from captured steps: the update kernel re-zeroes
        self._emit_loss(bwd, compute_grad=True)
        written.add(self.gkey(self.final.guid))
        bucket_left = {}
        for g in self.groups:
            if g.replicated:
                bucket_left[id(g)] = [len(b[2]) for b in g.buckets]
                g.works = [None] * len(g.buckets)
        steps = self.bwd_steps
        # a tied weight's gradient is final after the LAST op (in backward order) that uses it
        uses_left = defaultdict(int)
        for st in steps:
            if st[0] == "op":
                for w in st[1].weights:
                    uses_left[w.guid] += 1

        def touches(st, keys):
            if st[0] == "op":
                return any(self.gkey(t.guid) in keys for t in st[1].inputs + st[1].outputs)
            return any(self.gkey(g) in keys for _, _, g, _ in st[1])

        # dW of the Linear ops that precede the FIRST cross-device gradient exchange in backward order
        # (DLRM: the top MLP ahead of the embedding-gradient all-to-all) is deferred until that
        # exchange has been started, so the weight-gradient GEMMs overlap the all-to-all instead of
        # delaying it; their bucket all-reduces follow them.
        from flexmi.core.types import OperatorType
        has_xchg = self.world > 1 and any(
            st[0] != "op" and not all(rs.local_only for _, _, _, rs in st[1]) for st in steps)
        mode = os.environ.get("FLEXMI_DEFER_DW", "1")     # 0: off, force: also without an exchange (tests)
        defer_ok = (has_xchg or mode == "force") and mode != "0"
        deferred = []          # [(op, ctx)] whose dW items wait for the first exchange start

        def bucket_done(done_ops):
            for w in [w for o in done_ops for w in o.weights]:
                uses_left[w.guid] -= 1
                e = self.wentries.get(w.guid)
                if e is None or e.group is None or not e.group.replicated or uses_left[w.guid] > 0:
                    continue
                g = e.group
                for bi, b in enumerate(g.buckets):
                    if w.guid in b[2]:
                        bucket_left[id(g)][bi] -= 1
                        if bucket_left[id(g)][bi] == 0 and self.cfg.overlap_grad_sync:
                            if g.zero:
                                bwd.append(Item("comm", (lambda g=g, bi=bi: self._launch_bucket(g, bi)),
                                                f"reducescatter.bucket{bi}", native=("rs", g, bi)))
                            else:
                                bwd.append(Item("comm", (lambda g=g, bi=bi: self._launch_bucket(g, bi)),
                                                f"allreduce.bucket{bi}", native=("ar", g, bi)))

        def flush_deferred():
            for dop, dc in deferred:
                C(bwd, dop.name + ".bwd_dw", (lambda op=dop, c=dc: op.backward(c, "dw")))
                bucket_done([dop])
            deferred.clear()

        pipe = getattr(self, "pipe", None)
        kb = pipe["kb"] if pipe is not None else None
        skip_to = -1
        for k, st in enumerate(steps):
            for ex in finish_before.pop(k, []):
                self._emit_exchange_finish(bwd, ex, "reshard.bwd")
            if k < skip_to:
                continue
            if k == kb:
                skip_to = self._emit_pipelined_bwd(bwd, C, pipe, k, written, bucket_done, finish_before, touches)
                if defer_ok:
                    flush_deferred()
                    defer_ok = False
                continue
            if st[0] == "op":
                op = st[1]
                c = self.ctx.get(op.guid)
                if c is not None:
                    flags = []
                    for i, t in enumerate(op.inputs):
                        same = c.in_grads[i] is not None and self.need[(op.guid, i)].same_as(self.home[t.guid])
                        flags.append(bool(same and self.gkey(t.guid) in written))
                    for o in op.outputs:
                        if o.guid in self.grad and self.gkey(o.guid) not in written:
                            C(bwd, o.name + ".zero_unused_grad", (lambda t=self.grad[o.guid]: t.zero_()))
                            written.add(self.gkey(o.guid))
                    grp = self.group_of.get(op.guid)
                    if getattr(op, "sparse_dp", None) and (grp is None or grp[0] is op):
                        self._emit_sparse_dp(bwd, grp or [op])
                    elif grp is not None:
                        if grp[0] is op:
                            C(bwd, op.name + ".group_bwd",
                              (lambda grp=grp: type(grp[0]).backward_group(grp, [self.ctx[o.guid] for o in grp])))
                    elif defer_ok and op.op_type == OperatorType.OP_LINEAR and op.weights:
                        C(bwd, op.name + ".bwd_dx", (lambda op=op, c=c, flags=flags: self._bwd_op(op, c, flags, "dx")))
                        bwd[-1].check = (lambda op=op, c=c: self._check_op(op.name + ".bwd", c.in_grads, "input grad"))
                        deferred.append((op, c))
                    else:
                        bwd.append(Item("comm" if getattr(op, "host_exec", False) else "compute",
                                        (lambda op=op, c=c, flags=flags: self._bwd_op(op, c, flags)), op.name + ".bwd"))
                        bwd[-1].check = (lambda op=op, c=c: self._check_op(op.name + ".bwd", c.in_grads, "input grad"))
                    for i, t in enumerate(op.inputs):
                        if c.in_grads[i] is not None and self.need[(op.guid, i)].same_as(self.home[t.guid]):
                            written.add(self.gkey(t.guid))
                # gradient buckets completed by this op -> async all-reduce (overlaps the rest of bwd).
                # A fused group's members all run backward at the group's step (grp[0]): their
                # weight gradients are final only there, not at the members' own positions.
                grp = self.group_of.get(op.guid)
                done_ops = [op] if grp is None else (list(grp) if grp[0] is op else [])
                if deferred and deferred[-1][0] is op:
                    done_ops = []            # its dW (and bucket) come with the deferred items
                bucket_done(done_ops)
            else:
                items, seen = [], set()
                for op, i, g, rs in st[1]:
                    key = self.gkey(g)
                    items.append((rs, self.tmp_grad.get((op.guid, i)), self.grad.get(g), key in written or key in seen))
                    seen.add(key)
                if self.world == 1 or all(rs.local_only for rs, *_ in items):
                    self._emit_reshards(bwd, items, "reshard.bwd")
                else:
                    ex = FusedExchange(items, self.world, self.rank, self.comm)
                    self._emit_exchange_start(bwd, ex, "reshard.bwd")
                    if defer_ok:
                        flush_deferred()          # dW GEMMs overlap this exchange
                        defer_ok = False
                    keys = {self.gkey(g) for _, _, g, _ in st[1]}
                    nxt = next((j for j in range(k + 1, len(steps)) if touches(steps[j], keys)), len(steps))
                    finish_before[nxt].append(ex)
                for op, i, g, rs in st[1]:
                    written.add(self.gkey(g))
        flush_deferred()
        for ex in finish_before.pop(len(steps), []):
            self._emit_exchange_finish(bwd, ex, "reshard.bwd")
        assert not finish_before

    def _emit_pipelined_bwd(self, bwd, C, pipe, kb, written, bucket_done, finish_before, touches):
        """The tail's backward chunk by chunk (see XCHG_CHUNKS); returns the first step after the
        tail's gradient return."""
        from flexmi.core.types import OperatorType
        steps = self.bwd_steps
        region_b = list(reversed(pipe["region"]))
        kr = kb + len(region_b)
        flags = {}
        for op in region_b:
            c = self.ctx[op.guid]
            fl = []
            for i, t in enumerate(op.inputs):
                same = c.in_grads[i] is not None and self.need[(op.guid, i)].same_as(self.home[t.guid])
                fl.append(bool(same and self.gkey(t.guid) in written))
            for o in op.outputs:
                if o.guid in self.grad and self.gkey(o.guid) not in written:
                    C(bwd, o.name + ".zero_unused_grad", (lambda t=self.grad[o.guid]: t.zero_()))
                    written.add(self.gkey(o.guid))
            flags[op.guid] = fl
            for i, t in enumerate(op.inputs):
                if c.in_grads[i] is not None and self.need[(op.guid, i)].same_as(self.home[t.guid]):
                    written.add(self.gkey(t.guid))
        red = steps[kr][1] if kr < len(steps) and steps[kr][0] == "reduce" else []
        items, seen = [], set()
        for op, i, g, rs in red:
            key = self.gkey(g)
            items.append((rs, self.tmp_grad.get((op.guid, i)), self.grad.get(g), key in written or key in seen))
            seen.add(key)
        exs = []
        if items:
            exs = [FusedExchange(self._chunk_items(items, "src", c, pipe), self.world, self.rank, self.comm)
                   for c in range(pipe["K"])]
        for c, ex in enumerate(exs):
            ex.tag = f"reshard.bwd.c{c}"
        split = {op.guid for op in region_b if op.op_type == OperatorType.OP_LINEAR and op.weights}
        for c in range(pipe["K"]):
            for op in region_b:
                cc = pipe["ctx"][c][op.guid]
                fl = flags[op.guid]
                if op.guid in split:
                    C(bwd, f"{op.name}.c{c}.bwd_dx", (lambda op=op, cc=cc, fl=fl: self._bwd_op(op, cc, fl, "dx")))
                else:
                    bwd.append(Item("compute", (lambda op=op, cc=cc, fl=fl: self._bwd_op(op, cc, fl)), f"{op.name}.c{c}.bwd"))
                bwd[-1].check = (lambda op=op, cc=cc: self._check_op(op.name + ".bwd", cc.in_grads, "input grad"))
            if exs:
                self._emit_exchange_start(bwd, exs[c], "reshard.bwd")
        # whole-batch weight gradients (overlapping the last chunk's all-to-all), then their buckets
        for op in region_b:
            if op.guid in split:
                C(bwd, op.name + ".bwd_dw", (lambda op=op: op.backward(self.ctx[op.guid], "dw")))
            bucket_done([op])
        if not red:
            return kr
        keys = {self.gkey(g) for _, _, g, _ in red}
        nxt = next((j for j in range(kr + 1, len(steps)) if touches(steps[j], keys)), len(steps))
        finish_before[nxt].extend(exs)
        for op, i, g, rs in red:
            written.add(self.gkey(g))
        return kr + 1

    def _emit_sparse_dp(self, bwd, grp):
        """Replicated embedding tables: pack (coalesce this rank's lookups) -> all-gather of the
        payloads over the replica set (RCCL) -> apply every replica's segment in rank order."""
        ctxs = [self.ctx[o.guid] for o in grp]
        op = grp[0]
        cls = type(op)
        st = cls.sdp_state(grp, ctxs, op.sparse_dp, self.rank)
        name = op.name + (".group" if len(grp) > 1 else "")
        bwd.append(Item("compute", (lambda grp=grp, ctxs=ctxs: cls.sdp_pack(grp, ctxs)), name + ".sdp_pack"))
        bwd.append(Item("comm", (lambda st=st: st.exchange(self.comm)), name + ".sdp_allgather",
                        native=("ag_buf", st.recv, st.send, st.holders)))
        bwd.append(Item("compute", (lambda grp=grp, ctxs=ctxs: cls.sdp_apply(grp, ctxs)), name + ".sdp_apply"))

    def _fwd_op(self, op, c):
        c.training = self.training
        if getattr(c, "empty", False):
            return
        if getattr(op, "host_exec", False):
            return self._host_op(op, c, "forward")
        op.forward(c)

    def _bwd_op(self, op, c, flags, phase=None):
        for i, f in enumerate(flags):
            c.in_grad_accumulate[i] = f
        if getattr(c, "empty", False):
            if phase in (None, "dx"):
                for g, acc in zip(c.in_grads, c.in_grad_accumulate):
                    if g is not None and not acc:
                        g.zero_()
            return
        if getattr(op, "host_exec", False):
            return self._host_op(op, c, "backward")
        if phase is None:
            op.backward(c)
        else:
            op.backward(c, phase)

    def _host_op(self, op, c, phase):
        """A CPU-placed op (P6) runs its CPU (fp32 torch) path on the host: host copies of the
        device inputs / output grads in, forward outputs back to the device buffers (H2D).  Its
        weights -- a host-resident table -- are updated in place by the host sparse SGD."""
        h = c.saved.get("host_ctx")
        if h is None:
            h = OpCtx(op, self.rank, "cpu", torch.float32)
            h.w_boxes, h.weights, h.wcompute = c.w_boxes, c.weights, c.wcompute
            h.weight_grads = [None] * len(c.weights)
            h.in_boxes, h.out_boxes = c.in_boxes, c.out_boxes
            h.outputs = [torch.empty(tuple(o.shape), dtype=torch.float32) for o in c.outputs]
            h.in_grads = [None] * len(c.inputs)
            h.in_grad_accumulate = [False] * len(c.inputs)
            c.saved["host_ctx"] = h
        h.training = c.training
        h.inputs = [x.cpu() if x is not None else None for x in c.inputs]
        if phase == "forward":
            op.forward(h)
            for dev, host in zip(c.outputs, h.outputs):
                dev.copy_(host)
        else:
            h.out_grads = [g.float().cpu() if g is not None else None for g in c.out_grads]
            h.lr = self.lr_tensor.cpu()
            op.backward(h)

    def _emit_reshards(self, lst, items, name):
        if not items:
            return
        if self.world == 1 or all(rs.local_only for rs, *_ in items):
            lst.append(Item("compute", (lambda items=items: run_reshards(self.comm, items)), name))
            return
        ex = FusedExchange(items, self.world, self.rank, self.comm)
        lst.append(Item("compute", ex.pack, name + ".pack"))
        lst.append(Item("comm", (lambda ex=ex: ex.exchange(self.comm)), name + ".a2a", native=("a2a_sync", ex)))
        lst.append(Item("compute", ex.unpack, name + ".unpack"))

    def _emit_loss(self, lst, compute_grad):
        if self.loss_type is None:
            return
        if self.loss_reshard is not None:
            self._emit_reshards(lst, [(self.loss_reshard, self.local_buffer(self.final), self.logits_buf, False)],
                                "loss.gather")
        if self.logits_buf is not None:
            lst.append(Item("compute", (lambda: self._loss_kernel(compute_grad)), "loss"))
        if compute_grad and self.loss_reshard is not None:
            self._emit_reshards(lst, [(self.loss_back, self.logit_grad, self.grad.get(self.final.guid), False)],
                                "loss.scatter")

    def release(self):
        """Drop this executor's native-runner references (callables, tensors, process groups held
        from C++ -- invisible to Python's cycle collector) and its captured graphs, so the model's
        device memory is freed once the Python objects go away (bench.py builds a second model)."""
        nr = self._native if self._native not in (None, False) else None
        if nr is not None:
            nr.rt.release()
            nr.keep.clear()
        self._native = None
        self._graph = None
        self._graphs = []
        self._graph_segments = []

    def native_runner(self):
        """The native step runner when it can execute this executor's programs: ``flexmi._rt``
        built, plain Comm (fault-injecting wrappers stay on the Python path), no per-item
        debug / watchdog / timer hooks; FLEXMI_NATIVE_RUNNER=0 disables it."""
        if self._native is None:
            from flexmi.parallel.comm import Comm
            from flexmi.runtime.health import FaultyComm
            comm = self.comm
            faults = None
            if isinstance(comm, FaultyComm) and type(comm.inner) is Comm:
                faults, comm = comm.faults, comm.inner
            ok = (os.environ.get("FLEXMI_NATIVE_RUNNER", "1") != "0" and _rt_module() is not None
                  and type(comm) is Comm and not self.timer.enabled)
            self._native = NativeRunner(self) if ok else False
            if ok and faults:
                # FaultyComm's injections on the native path: the runner counts its collectives
                self._native.rt.set_faults({int(k): (str(v[0]), float(v[1]) if len(v) > 1 else 0.0)
                                            for k, v in faults.items()})
        return self._native or None

    def _run(self, prog):
        nr = self.native_runner()
        if self.debug or self.watchdog is not None:
            return self._run_guarded(prog, nr)
        if nr is not None:
            nr.run(nr.program(prog))
            return
        tm = self.timer
        if tm.enabled:
            for it in prog:
                with tm.scope(it.name):
                    it.fn()
        else:
            for it in prog:
                it.fn()

    def _run_guarded(self, prog, nr=None):
        """Debug / watchdog execution: heartbeat per item; in debug mode every item is followed
        by a device synchronisation and its NaN/Inf guard.  With the native
        step runner the heartbeat and the guards are its per-step hooks, so fault / debug /
        watchdog runs execute the production program (native collectives included)."""
        from flexmi.runtime.health import WatchdogTimeout
        wd = self.watchdog
        if wd is not None:
            wd.arm()
        try:
            if nr is not None:
                pid = nr.program(prog)
                owner = nr.step_items[pid]

                def pre(i, name):
                    if wd is not None:
                        wd.beat(name)

                def post(i, name):
                    if not self.debug or not owner[i][1]:      # guard after an item's last step
                        return
                    if self.backend == "hip":
                        torch.cuda.synchronize()
                    it = owner[i][0]
                    if it.check is not None:
                        it.check()
                nr.run(pid, pre, post)
                return
            for it in prog:
                if wd is not None:
                    wd.beat(it.name)
                with self.timer.scope(it.name):
                    it.fn()
                if self.debug:
                    if self.backend == "hip":
                        torch.cuda.synchronize()
                    if it.check is not None:
                        it.check()
        except KeyboardInterrupt:
            if wd is not None and wd.fired:
                raise WatchdogTimeout(f"rank {self.rank}: no progress in '{wd.fired_tag}' for "
                                      f"{wd.timeout_s:.1f}s") from None
            raise
        finally:
            if wd is not None:
                wd.disarm()

    def _check_op(self, where, tensors, kind):
        from flexmi.runtime.health import check_finite
        check_finite(where, tensors, kind)

    def forward(self):
        self._run(self.prog_fwd)

    def zero_gradients(self):
        """Reference semantics (``model.cc:1146-1169``): gradients start at zero.  flexmi
        kernels overwrite on first write (decided when the program is compiled), so there is
        nothing to clear."""
        return None

    def backward(self):
        self._run(self.prog_bwd)
        self._grads_dirty = True

    def update(self):
        self._run(self.prog_upd)
        self._after_update()

    def _after_update(self):
        if self.backend == "hip" and self.optimizer is not None:
            self._grads_dirty = any(g.zero for g in self.groups)   # update kernels re-zeroed the rest
        if self.optimizer is not None:
            self.optimizer.next()   # host mirror of the device-side step counters
        self.step_count += 1
        if self.debug:
            from flexmi.runtime.health import check_finite, check_replicas
            for g in self.groups:
                if g.numel:
                    check_finite(f"update step {self.step_count}", [g.master], "weights")
            check_replicas(self)

    def _launch_bucket(self, g, bi):
        b = g.buckets[bi]
        if g.zero:
            g.works[bi] = self._zero_rs(g, bi, sync=False)
            return
        g.works[bi] = self.comm.all_reduce_async(g.gradbuf[b[0]:b[1]], g.holders)

    def _sync_grads(self):
        for g in self.groups:
            if not g.replicated:
                continue
            for bi, b in enumerate(g.buckets):
                w = g.works[bi]
                if w is None:
                    w = self._zero_rs(g, bi, sync=False) if g.zero else \
                        self.comm.all_reduce_async(g.gradbuf[b[0]:b[1]], g.holders)
                if w is not None:
                    w.wait()
                g.works[bi] = None

    def _optimizer_step(self, fused=False):
        """fused: the weights in ``fused_sgd_entries`` were already updated inside their dW GEMMs
        (_plan_fused_sgd); only the remaining ranges of each group are updated here."""
        from flexmi.ops import _kernels as K
        opt = self.optimizer
        if isinstance(opt, AdamOptimizer):
            # device-side bias-correction counters (capturable): [beta1^t, beta2^t, alpha_t]
            st = self.adam_state
            st[0:1].mul_(opt.beta1)
            st[1:2].mul_(opt.beta2)
            st[2:3].copy_(opt.alpha * torch.sqrt(1 - st[1:2]) / (1 - st[0:1]))
        for g in self.groups:
            if g.numel == 0:
                continue
            if g.zero:
                self._zero_opt_step(g, opt)
                continue
            comp = g.compute if g.compute is not g.master else None
            rest = getattr(g, "sgd_rest", None) if fused else None
            if rest is not None:
                if rest:
                    K.C().sgd_segs(g.master, g.gradbuf, g.state.get("v") if opt.momentum > 0 else None, comp,
                                   self.lr_tensor, [r[0] for r in rest], [r[1] for r in rest], opt.weight_decay,
                                   opt.momentum, opt.nesterov, True)
                continue
            if self.backend == "hip":
                # the kernels consume the gradient and leave it zeroed for the next backward
                if isinstance(opt, SGDOptimizer):
                    K.sgd_update(g.master, g.gradbuf, g.state.get("v"), comp, self.lr_tensor, opt.weight_decay,
                                 opt.momentum, opt.nesterov, zero_grad=True)
                else:
                    K.adam_update(g.master, g.gradbuf, g.state["m"], g.state["v"], comp, self.adam_state[2:3],
                                  opt.beta1, opt.beta2, opt.weight_decay, opt.epsilon, zero_grad=True)
            else:
                if isinstance(opt, SGDOptimizer):
                    gt = g.gradbuf + opt.weight_decay * g.master
                    if opt.momentum > 0:
                        v = g.state["v"]
                        v.mul_(opt.momentum).add_(gt)
                        gt = gt + opt.momentum * v if opt.nesterov else v
                    g.master.sub_(self.lr_tensor * gt)
                else:
                    gt = g.gradbuf + opt.weight_decay * g.master
                    m_, v_ = g.state["m"], g.state["v"]
                    m_.mul_(opt.beta1).add_((1 - opt.beta1) * gt)
                    v_.mul_(opt.beta2).add_((1 - opt.beta2) * gt * gt)
                    g.master.sub_(self.adam_state[2] * m_ / (v_.sqrt() + opt.epsilon))
                if comp is not None:
                    comp.copy_(g.master)

    def _zero_opt_step(self, g, opt):
        """The optimizer on this rank's shard: fp32 master shard, reduce-scattered gradient shard
        and the sharded state, one fused kernel launch over the whole shard buffer (the slices of
        all buckets are packed back to back)."""
        from flexmi.ops import _kernels as K
        m, gr, st = g.mshard, g.gshard, g.state
        if self.backend == "hip":
            if isinstance(opt, SGDOptimizer):
                K.sgd_update(m, gr, st.get("v"), None, self.lr_tensor, opt.weight_decay, opt.momentum, opt.nesterov)
            else:
                K.adam_update(m, gr, st["m"], st["v"], None, self.adam_state[2:3], opt.beta1, opt.beta2,
                              opt.weight_decay, opt.epsilon)
        elif isinstance(opt, SGDOptimizer):
            gt = gr + opt.weight_decay * m
            if opt.momentum > 0:
                v = st["v"]
                v.mul_(opt.momentum).add_(gt)
                gt = gt + opt.momentum * v if opt.nesterov else v
            m.sub_(self.lr_tensor * gt)
        else:
            gt = gr + opt.weight_decay * m
            m_, v_ = st["m"], st["v"]
            m_.mul_(opt.beta1).add_((1 - opt.beta1) * gt)
            v_.mul_(opt.beta2).add_((1 - opt.beta2) * gt * gt)
            m.sub_(self.adam_state[2] * m_ / (v_.sqrt() + opt.epsilon))

    # ------------------------------------------------------------------ loss
    def _loss_kernel(self, compute_grad):
        from flexmi.ops import _kernels as K
        scale = 1.0 / self.final.dims[0]
        mask = self.metrics_obj.mask if self.metrics_obj else 0
        clamp = float(getattr(self.model, "loss_threshold", 0.0) or 0.0)
        if self.backend == "hip":
            K.loss_forward_backward(int(self.loss_type), self.logits_buf, self.label_buf,
                                    self.logit_grad if compute_grad else None, scale, self.metric_acc, mask, clamp)
        elif (_native_cpu() is not None and self.logits_buf.dtype == torch.float32 and self.logits_buf.is_contiguous()
              and self.metric_acc.device.type == "cpu"):
            # csrc/cpu/init_metrics.cc loss_metrics: one pass, gradient + metrics
            _native_cpu().loss_metrics(int(self.loss_type), self.logits_buf, self.label_buf,
                                       self.logit_grad if compute_grad else None, scale, self.metric_acc, mask, clamp)
        else:
            loss_and_metrics_torch(self.loss_type, self.logits_buf, self.label_buf, self.logit_grad,
                                   scale, self.metric_acc, mask, compute_grad, clamp=clamp)

    def compute_metrics(self):
        if not hasattr(self, "prog_metrics"):
            self.prog_metrics = []
            self._emit_loss(self.prog_metrics, compute_grad=False)
        self._run(self.prog_metrics)

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
        if e.group is not None and e.group.zero:
            for fsl, sh in self._zero_pieces(e.group):
                e.group.mshard[sh].copy_(e.group.master[fsl])

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
        if self.prog_bwd_fused is None:
            self.backward()
            self.update()
            return
        self._run(self.prog_bwd_fused)     # dW GEMMs of fused weights update them in place
        self._grads_dirty = True
        self._run(self.prog_upd_fused)
        self._after_update()

    def step_program(self):
        if self.prog_bwd_fused is not None:
            return self.prog_fwd + self.prog_bwd_fused + self.prog_upd_fused
        return self.prog_fwd + self.prog_bwd + self.prog_upd

    def capture_step(self, pre=None):
        """The training step as a replayable hipGraph program (see ``_capture_step``).  The
        per-step gradient memset is left out of the graph: the update kernels consume the
        gradients and write them back as zeros, and a replay that follows an eager backward
        (gradients still dirty) clears them first."""
        assert self.backend == "hip"
        memset = [it for it in self.step_program() if getattr(it, "zero_group", None) is not None
                  and not it.zero_group.zero]
        skip = {id(it) for it in memset} if self.optimizer is not None else set()
        replay = self._capture_step(pre, skip)
        groups = [it.zero_group for it in memset]

        def run():
            if self._grads_dirty:
                for g in groups:
                    g.gradbuf.zero_()
            replay()
            self._grads_dirty = bool(skip) and any(g.zero for g in self.groups)
        return run

    def _capture_step(self, pre=None, skip=()):
        """Capture the training step as hipGraph segments split at the collectives.
        ``pre``: optional compute callable (e.g. input staging) captured at the head.
        Returns a callable that replays one step.  The caller must have run >= 1 eager step
        (allocator warm-up, lazily created workspaces)."""
        prog = ([Item("compute", pre, "pre")] if pre is not None else []) + \
            [it for it in self.step_program() if id(it) not in skip]
        segments = []
        cur = []
        for it in prog:
            if it.kind == "compute":
                cur.append(it)
            else:
                if cur:
                    segments.append(("graph", cur))
                    cur = []
                segments.append(("comm", it))
        if cur:
            segments.append(("graph", cur))
        # (a high-priority main stream measured much slower: 2.08-2.19 vs 1.15 ms/step,
        # profiles/bench_ab_stream_prio_r5p.txt -- the graph started the MLP chain ~30 us late)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        ov = overlap_embeddings_enabled(self)
        side = torch.cuda.Stream() if ov else None
        runs = []
        graphs = []
        # thread_local capture: the RCCL process group's watchdog thread queries events while
        # a segment is being captured; only this thread's calls belong to the graph
        for kind, x in segments:
            if kind == "graph":
                g = torch.cuda.CUDAGraph()
                with torch.cuda.stream(s):
                    with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                        if ov:
                            _run_overlapped(x, s, side)
                        else:
                            for it in x:
                                it.fn()
                graphs.append(g)
                runs.append(g.replay)
            else:
                runs.append(x.fn)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self._graph_segments = segments
        self._graphs = graphs
        opt = self.optimizer
        nr = self.native_runner()
        if nr is not None:
            # the whole step as ONE native program: hipGraphLaunch per segment, collectives
            # issued by the C++ runner in between
            pid = nr.rt.new_program()
            gi = iter(graphs)
            for k, (kind, x) in enumerate(segments):
                if kind == "graph":
                    g = next(gi)
                    nr.rt.add_graph(pid, int(g.raw_cuda_graph_exec()), f"segment{k}")
                else:
                    nr.add_item(pid, x)
            nr.keep.append(graphs)

            def replay():
                nr.run(pid)
                if opt is not None:
                    opt.next()
                self.step_count += 1
            return replay

        def replay():
            for r in runs:
                r()
            if opt is not None:
                opt.next()
            self.step_count += 1
        return replay

    # ------------------------------------------------------------------ introspection
    def memory_report(self):
        n = 0
        for v in self.act.values():
            if v is not None:
                n += v.numel() * v.element_size()
        w = sum(g.numel * 4 * 2 + sum(t.numel() for t in g.state.values()) * 4 for g in self.groups)
        sp = sum(e.numel * 4 for e in self.wentries.values() if e.sparse)
        # sparse data parallelism: the all-gather payload buffers (send + R segments) and the
        # claim slots -- per-step lookups, not table-sized gradients
        sdp = 0
        for c in self.ctx.values():
            st = c.saved.get("sdp")
            if st is not None:
                sdp += (st.send.numel() + st.recv.numel()) * 4 + sum(t.numel() * 4 for t in st.slot + st.cid)
        return {"activations": n, "dense_params": w, "sparse_tables": sp, "sparse_dp_payload": sdp}
