"""Native sharding algebra (csrc/runtime/shard.cc via flexmi._native) against a plain-Python
oracle of the same semantics: transfer lists for random layout pairs (splits, replication,
partial sums, explicit halo boxes) and launch splitting of copy pieces."""
import random

import pytest

from flexmi.parallel.layout import Layout, ReshardPlan, box_intersect, box_volume, split_extent


def _oracle_transfers(src, dst):
    reduce = src.partial and not dst.partial
    out = []
    for dp in range(dst.num_parts()):
        dbox = dst.part_box(dp)
        for sp in range(src.num_parts()):
            inter = box_intersect(dbox, src.part_box(sp))
            if inter is None:
                continue
            sh = src.holders[sp]
            for d in dst.holders[dp]:
                if reduce:
                    out.extend((s, d, inter, sp, dp) for s in sh)
                else:
                    s = d if d in sh else sh[(dp + sp) % len(sh)]
                    out.append((s, d, inter, sp, dp))
    out.sort(key=lambda t: (t[0], t[1], t[4], t[3], t[2]))
    return out


def _rand_layout(rng, shape, world, partial=False, halo=False):
    degrees = []
    left = world
    for n in shape:
        d = rng.choice([k for k in (1, 2, 3, 4) if k <= max(1, min(n, left))])
        degrees.append(d)
        left = max(1, left // d)
    lay_parts = 1
    for d in degrees:
        lay_parts *= d
    holders = []
    for _ in range(lay_parts):
        k = min(world, rng.choice([1, 1, 2]))
        holders.append(tuple(sorted(rng.sample(range(world), k))))
    lay = Layout(tuple(shape), tuple(degrees), holders, partial)
    if halo:
        boxes = []
        for p in range(lay_parts):
            b = lay.part_box(p)
            boxes.append(tuple((max(0, lo - 1), min(n, hi + 1)) for (lo, hi), n in zip(b, shape)))
        lay = Layout(tuple(shape), tuple(degrees), holders, partial, boxes)
    return lay


@pytest.mark.parametrize("seed", range(40))
def test_reshard_transfers_match_oracle(seed):
    rng = random.Random(seed)
    world = rng.choice([1, 2, 3, 4, 8])
    shape = tuple(rng.randint(1, 13) for _ in range(rng.randint(1, 4)))
    src = _rand_layout(rng, shape, world, partial=rng.random() < 0.3, halo=rng.random() < 0.2)
    dst = _rand_layout(rng, shape, world, halo=rng.random() < 0.2)
    got = [(t.src, t.dst, t.box, t.src_part, t.dst_part) for t in ReshardPlan(src, dst).transfers]
    assert got == _oracle_transfers(src, dst)
    if not src.partial and src.boxes is None and dst.boxes is None:
        # every destination element is delivered exactly once per holder
        vol = sum(box_volume(t[2]) for t in got)
        per_part = sum(box_volume(dst.part_box(p)) * len(dst.holders[p]) for p in range(dst.num_parts()))
        assert vol == per_part


def test_split_extent_matches():
    from flexmi import _native
    for n in range(0, 20):
        for d in range(1, 6):
            for k in range(d):
                assert tuple(_native.split_extent(n, d, k)) == split_extent(n, d, k)


def test_split_launches():
    from flexmi import _native
    b = lambda *r: [list(x) for x in r]  # noqa: E731
    # pieces 0,1 write disjoint boxes of buffer 0; piece 2 overlaps piece 0 -> new launch
    sizes = _native.split_launches([0, 0, 0, 1], [b((0, 2)), b((2, 4)), b((1, 3)), b((0, 4))], 32)
    assert sizes == [2, 2]
    # no boxes never clash; the per-launch cap applies
    assert _native.split_launches([0] * 5, [None] * 5, 2) == [2, 2, 1]
    # different buffers never clash
    assert _native.split_launches([0, 1, 2], [b((0, 4))] * 3, 32) == [3]
