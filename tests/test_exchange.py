"""Fused reshard exchange (FusedExchange): the MI355X pack/unpack plan (one multi-descriptor
copy launch per phase, vectorised 16-B pieces) must move exactly what the per-piece tensor
path moves.  All ranks of a world-W exchange are simulated in ONE process: every rank packs,
the all_to_all is emulated by slicing the send buffers, every rank unpacks."""
import numpy as np
import pytest
import torch

from flexmi.parallel.layout import Layout, ParallelConfig, ReshardPlan
from flexmi.runtime.executor import FusedExchange, ReshardStep

W = 4


def _pc(dims, devs):
    return ParallelConfig(list(dims), list(devs))


CASES = {
    # DLRM forward: table output on its owner (full batch) -> data-parallel rows
    "emb_fwd": ((64, 128), _pc([1, 1], [2]), _pc([1, W], range(W)), False),
    # DLRM backward: row-split gradient contributions (partial) -> owner, summed
    "emb_bwd": ((64, 128), _pc([1, W], range(W)), _pc([1, 1], [1]), True),
    # channel-parallel Linear input gradients: replicated partials reduced to DP rows
    "chan_reduce": ((32, 48), _pc([1, 1], [0]), _pc([1, W], range(W)), True),
    # column split -> row split (transposing repartition)
    "col_to_row": ((32, 64), _pc([W, 1], range(W)), _pc([1, W], range(W)), False),
    # 4-D spatial split -> sample split (boxes not 2-D expressible: per-piece fallback)
    "spatial": ((4, 3, 8, 8), _pc([1, W, 1, 1], range(W)), _pc([W, 1, 1, 1], range(W)), False),
}


def _layouts(name):
    shape, a, b, partial = CASES[name]
    src = Layout.from_pc(shape, a)
    dst = Layout.from_pc(shape, b)
    if partial:
        if name == "chan_reduce":   # every rank holds a full partial sum
            src = Layout.replicated(shape, list(range(W))).as_partial()
        else:
            src = src.as_partial()
    return shape, src, dst


def _run(name, device, dtype, fast):
    shape, src_l, dst_l = _layouts(name)
    g = torch.Generator().manual_seed(3)
    srcs, dsts, exs = [], [], []
    for r in range(W):
        ss = src_l.local_shape(r)
        ds = dst_l.local_shape(r)
        s = torch.randn(ss, generator=g).to(device, dtype) if ss is not None else None
        d = torch.full(ds, 7.0).to(device, dtype) if ds is not None else None
        st = ReshardStep(ReshardPlan(src_l, dst_l), r, W, dtype, device)
        ex = FusedExchange([(st, s, d, False)], W, r)
        if not fast:
            ex.fast = False
        srcs.append(s)
        dsts.append(d)
        exs.append(ex)
    for ex in exs:
        ex.pack()
    for r, ex in enumerate(exs):      # emulated all_to_all_single
        for p in range(W):
            n = ex.recv_sizes[p]
            if n:
                o = exs[p]
                so = o.send_off[r]
                ex.recv_buf[ex.recv_off[p]: ex.recv_off[p] + n].copy_(o.send_buf[so: so + n])
    for ex in exs:
        ex.unpack()
    return [d.float().cpu() if d is not None else None for d in dsts], exs


def _reference(name):
    """Ground truth from the full logical tensor."""
    shape, src_l, dst_l = _layouts(name)
    g = torch.Generator().manual_seed(3)
    full = torch.zeros(shape)
    for r in range(W):
        ss = src_l.local_shape(r)
        if ss is None:
            continue
        s = torch.randn(ss, generator=g)
        box = src_l.local_box(r)
        sl = tuple(slice(lo, hi) for lo, hi in box)
        if src_l.partial:
            full[sl] += s
        else:
            full[sl] = s
    out = []
    for r in range(W):
        box = dst_l.local_box(r)
        out.append(None if box is None else full[tuple(slice(lo, hi) for lo, hi in box)].clone())
    return out


@pytest.mark.parametrize("name", list(CASES))
def test_exchange_cpu_matches_logical_reshard(name):
    got, _ = _run(name, "cpu", torch.float32, fast=False)
    for a, b in zip(got, _reference(name)):
        if b is not None:
            torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("name", list(CASES))
def test_exchange_hip_plan_matches_tensor_path(name, dtype):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    fast, exs = _run(name, "cuda", dtype, fast=True)
    slow, _ = _run(name, "cuda", dtype, fast=False)
    if name != "spatial":
        assert all(ex.fast for ex in exs), "2-D expressible boxes must take the multi-copy plan"
    for a, b in zip(fast, slow):
        if b is not None:
            torch.testing.assert_close(a, b, rtol=0, atol=0)
    ref = _reference(name)
    tol = 1e-5 if dtype == torch.float32 else 3e-2
    for a, b in zip(fast, ref):
        if b is not None:
            torch.testing.assert_close(a, b, rtol=tol, atol=tol)
