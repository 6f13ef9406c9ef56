"""Sharding algebra: ParallelConfig, Layout (shard boxes + holders) and reshard plans.

This replaces what Legion did implicitly in the reference -- logical regions, restriction
partitions (``src/runtime/model.cc:457-875``) and the dependence analysis that inserted DMA
copies between producer and consumer partitions (``src/runtime/simulator.cc:295-326`` models
exactly those intersection copies).  Here every cross-device byte is planned explicitly:
a :class:`ReshardPlan` lists (src rank, dst rank, box) transfers that the executor runs as
one RCCL ``all_to_all`` (``flexmi/parallel/comm.py``).  The transfer planning itself (box
intersections over all part pairs, holder choice, ordering) is C++: ``csrc/runtime/shard.cc``.

Conventions:
  * ParallelConfig ``dims`` are kept in the reference's *internal* order (innermost first,
    last entry = sample dim) so ``.pb`` strategy files round-trip unchanged;
  * Layout ``degrees`` are in *user* order (outer -> inner, batch first); part index is the
    row-major linearisation of the part coordinates, which equals the reference's
    linearisation with internal dim 0 fastest (``src/mapper/mapper.cc:62-95``).
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass, field
from typing import List, Sequence, Tuple

Box = Tuple[Tuple[int, int], ...]  # per dim [lo, hi)

_NATIVE = None


def _native():
    """flexmi._native (C++ sharding algebra, strategy codec, simulator): always built by
    tools/build_ext.py -- no Python fallback for the plan compiler's transfer planning."""
    global _NATIVE
    if _NATIVE is None:
        try:
            from flexmi import _native as mod
        except ImportError as e:
            raise RuntimeError("flexmi._native is not built: run `python tools/build_ext.py --only native`") from e
        _NATIVE = mod
    return _NATIVE


@dataclass
class ParallelConfig:
    """Per-op partitioning: degrees per dim (internal order) + explicit device list.
    ``include/config.h:41-50``."""
    GPU = 0
    CPU = 1
    dims: List[int] = field(default_factory=lambda: [1])
    device_ids: List[int] = field(default_factory=lambda: [0])
    device_type: int = 0
    memory_types: List[int] = field(default_factory=list)

    @property
    def nDims(self):
        return len(self.dims)

    def num_parts(self):
        n = 1
        for d in self.dims:
            n *= d
        return n

    def user_degrees(self):
        return tuple(reversed(self.dims))

    @staticmethod
    def from_user_degrees(degrees, device_ids, device_type=0):
        return ParallelConfig(list(reversed(list(degrees))), list(device_ids), device_type)

    @staticmethod
    def data_parallel(ndims, num_devices, devices=None):
        """Default DP config (``src/runtime/model.cc:282-293``): split the sample dim."""
        dims = [1] * ndims
        dims[-1] = num_devices
        ids = list(devices) if devices is not None else list(range(num_devices))
        return ParallelConfig(dims, ids)

    def key(self):
        return (tuple(self.dims), tuple(self.device_ids), self.device_type)

    def __hash__(self):
        return hash(self.key())

    def __eq__(self, o):
        return isinstance(o, ParallelConfig) and self.key() == o.key()

    def __repr__(self):
        return f"PC(dims={self.dims}, devs={self.device_ids})"


def split_extent(n: int, d: int, k: int) -> Tuple[int, int]:
    """Equal-block partition of extent n into d parts (ceil blocks, last part short)."""
    b = -(-n // d)
    lo = min(n, k * b)
    hi = min(n, (k + 1) * b)
    return lo, hi


def box_intersect(a: Box, b: Box):
    out = []
    for (alo, ahi), (blo, bhi) in zip(a, b):
        lo, hi = max(alo, blo), min(ahi, bhi)
        if lo >= hi:
            return None
        out.append((lo, hi))
    return tuple(out)


def box_volume(b: Box) -> int:
    v = 1
    for lo, hi in b:
        v *= hi - lo
    return v


@dataclass
class Layout:
    """How one logical tensor is distributed over ranks.

    ``holders[p]`` lists the ranks that hold part ``p`` (more than one = replication).
    ``partial`` marks gradient layouts in which holders of a part own partial sums that must
    be added (the reference's ``replica`` tensors + ``backward2`` saxpy,
    ``src/ops/linear.cu:766-794``)."""
    shape: Tuple[int, ...]
    degrees: Tuple[int, ...]
    holders: List[Tuple[int, ...]]
    partial: bool = False
    boxes: object = None  # optional explicit per-part boxes (overlapping halos for spatial splits)

    def __post_init__(self):
        self.shape = tuple(int(s) for s in self.shape)
        self.degrees = tuple(int(d) for d in self.degrees)
        assert len(self.shape) == len(self.degrees), (self.shape, self.degrees)
        assert len(self.holders) == self.num_parts(), (len(self.holders), self.degrees)
        self.holders = [tuple(h) for h in self.holders]

    def num_parts(self):
        n = 1
        for d in self.degrees:
            n *= d
        return n

    def part_coords(self, p):
        coords = []
        for d in reversed(self.degrees):
            coords.append(p % d)
            p //= d
        return tuple(reversed(coords))

    def part_box(self, p) -> Box:
        if self.boxes is not None:
            return self.boxes[p]
        c = self.part_coords(p)
        return tuple(split_extent(n, d, k) for n, d, k in zip(self.shape, self.degrees, c))

    def parts_of(self, rank):
        return [p for p, h in enumerate(self.holders) if rank in h]

    def local_box(self, rank):
        """The (single) box a rank holds.  A rank holds at most one part per layout in every
        strategy flexmi generates (same restriction as the reference mapper)."""
        ps = self.parts_of(rank)
        if not ps:
            return None
        assert len(ps) == 1, f"rank {rank} holds several parts {ps} of {self}"
        return self.part_box(ps[0])

    def local_shape(self, rank):
        b = self.local_box(rank)
        return None if b is None else tuple(hi - lo for lo, hi in b)

    def ranks(self):
        s = set()
        for h in self.holders:
            s.update(h)
        return sorted(s)

    def replication(self):
        return max(len(h) for h in self.holders)

    def same_as(self, o: "Layout"):
        return self.key() == o.key()

    def as_partial(self):
        return Layout(self.shape, self.degrees, list(self.holders), True, self.boxes)

    def as_full(self):
        return Layout(self.shape, self.degrees, list(self.holders), False, self.boxes)

    def key(self):
        bx = None if self.boxes is None else tuple(self.boxes)
        return (self.shape, self.degrees, tuple(self.holders), self.partial, bx)

    def native(self):
        """The (shape, degrees, holders, boxes|None, partial) tuple of flexmi._native."""
        bx = None if self.boxes is None else [list(b) for b in self.boxes]
        return (list(self.shape), list(self.degrees), [list(h) for h in self.holders], bx, bool(self.partial))

    # --- constructors -------------------------------------------------
    @staticmethod
    def from_pc(shape, pc: ParallelConfig, replicate_over=None):
        """Layout of an op output under ParallelConfig ``pc`` (degrees in internal order,
        trailing/leading dims padded with 1 when the tensor rank differs)."""
        nd = len(shape)
        deg = list(pc.user_degrees())
        if len(deg) < nd:
            deg = deg + [1] * (nd - len(deg))  # pad inner dims (sample stays first)
        elif len(deg) > nd:
            # collapse extra degrees into the sample dim
            extra = 1
            for d in deg[nd:]:
                extra *= d
            deg = deg[:nd]
            deg[-1] *= extra
        holders = [(pc.device_ids[p],) for p in range(pc.num_parts())]
        return Layout(tuple(shape), tuple(deg), holders)

    @staticmethod
    def replicated(shape, ranks):
        return Layout(tuple(shape), (1,) * len(shape), [tuple(ranks)])


@dataclass
class Transfer:
    src: int
    dst: int
    box: Box           # global coordinates
    src_part: int
    dst_part: int


class ReshardPlan:
    """Explicit transfers turning ``src`` into ``dst`` (SURVEY §7.5 hard part #1)."""

    def __init__(self, src: Layout, dst: Layout):
        assert src.shape == dst.shape, (src.shape, dst.shape)
        self.src, self.dst = src, dst
        self.reduce = src.partial and not dst.partial
        # box intersections + holder choice in C++ (csrc/runtime/shard.cc: reshard_transfers)
        self.transfers: List[Transfer] = [
            Transfer(s, d, tuple(tuple(r) for r in box), sp, dp)
            for s, d, box, sp, dp in _native().reshard_transfers(src.native(), dst.native())]

    def is_identity(self):
        return all(t.src == t.dst for t in self.transfers) and not self.reduce_needed_local()

    def reduce_needed_local(self):
        # local partial sums from several holders that live on one rank never happen (one part per rank)
        return False

    def bytes_between(self, elem_size=4):
        """{(src,dst): bytes} -- used by the simulator's comm tasks."""
        out = {}
        for t in self.transfers:
            if t.src != t.dst:
                out[(t.src, t.dst)] = out.get((t.src, t.dst), 0) + box_volume(t.box) * elem_size
        return out

    def clip_rows(self, side, rows):
        """The part of this plan that moves one micro-batch chunk: every transfer's dim-0 extent
        clipped to ``rows(lo, hi) -> (a, b)``, the chunk's global rows inside the [lo, hi) rows
        held by the transfer's destination (``side="dst"``: a forward exchange into a sample
        split) or source (``side="src"``: the gradient return out of one).  Transfers outside the
        chunk are dropped; the chunks of 0..K-1 partition the plan."""
        lay = self.dst if side == "dst" else self.src
        out = ReshardPlan.__new__(ReshardPlan)
        out.src, out.dst, out.reduce = self.src, self.dst, self.reduce
        out.transfers = []
        for t in self.transfers:
            lo, hi = lay.local_box(t.dst if side == "dst" else t.src)[0]
            a, b = rows(lo, hi)
            x0, x1 = max(a, t.box[0][0]), min(b, t.box[0][1])
            if x0 < x1:
                out.transfers.append(Transfer(t.src, t.dst, ((x0, x1),) + tuple(t.box[1:]), t.src_part, t.dst_part))
        return out

    def sends_of(self, rank):
        return [t for t in self.transfers if t.src == rank]

    def recvs_of(self, rank):
        return [t for t in self.transfers if t.dst == rank]


def enumerate_degree_splits(n_devices: int, ndims: int, max_parts=None):
    """All degree vectors (user order) whose product divides ``n_devices`` -- used by the
    search's proposal generator."""
    out = []
    for degs in itertools.product(*[range(1, n_devices + 1)] * ndims):
        p = 1
        for d in degs:
            p *= d
        if n_devices % p == 0 and (max_parts is None or p <= max_parts):
            out.append(degs)
    return out
