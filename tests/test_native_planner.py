"""Native graph planner (csrc/runtime/planner.cc via flexmi._native.plan_graph): order, forward
reshard schedule, backward liveness and gradient-reduce schedule on hand-built graphs, plus the
executor's use of it on a two-rank DLRM plan (CPU only)."""
import pytest

from flexmi import _native


def inp(t, prod=-1, dtype=0, need=0, is_float=True, needs_grad=True, reshard=False, remote=False):
    return (t, prod, dtype, need, is_float, needs_grad, reshard, remote)


def test_single_rank_keeps_model_order_and_schedules():
    # op1: x(100) -> t11 ; op2: t11 (resharded) -> t12 ; op3: t12, idx(101, int) -> t13 (loss)
    ops = [(1, [inp(100, needs_grad=False)], [11]),
           (2, [inp(11, 1, reshard=True)], [12]),
           (3, [inp(12, 2), inp(101, is_float=False, dtype=1, reshard=True, need=5)], [13])]
    order, fwd, live, gn, bwd = _native.plan_graph(ops, 1)
    assert order == [1, 2, 3]
    assert fwd == [(0, 1, []), (1, 2, [0]), (0, 2, []), (1, 3, [1]), (0, 3, [])]
    assert live == [3, 2, 1]
    assert gn == [11, 12, 13]
    # op2's resharded input gets its gradient reduced home; the int input of op3 does not
    assert bwd == [(0, 3, []), (0, 2, []), (1, 2, [0]), (0, 1, [])]


def test_comm_first_order_hoists_remote_producers_and_ancestors():
    # a: dense chain d1 -> d2 ; b: e0 -> e1 whose output crosses ranks into the join j
    ops = [(1, [inp(100)], [11]),            # d1
           (2, [inp(11, 1)], [12]),          # d2
           (3, [inp(101)], [13]),            # e0 (ancestor of the remote producer)
           (4, [inp(13, 3)], [14]),          # e1 (remote producer)
           (5, [inp(12, 2), inp(14, 4, reshard=True, remote=True)], [15])]
    order = _native.plan_graph(ops, 2)[0]
    assert order == [3, 4, 1, 2, 5]
    # a local-only reshard does not reorder
    ops[4] = (5, [inp(12, 2), inp(14, 4, reshard=True, remote=False)], [15])
    assert _native.plan_graph(ops, 2)[0] == [1, 2, 3, 4, 5]


def test_dead_branch_and_dedup_and_dtype_groups():
    # op1 has two outputs; only the first reaches the loss through op2.  op3 consumes the unused
    # output (dead).  The loss is the LAST op in model order (op2), not the last in topo order.
    ops = [(1, [inp(100)], [11, 12]),
           (3, [inp(12, 1)], [13]),
           (2, [inp(11, 1, reshard=True, need=7), inp(11, 1, reshard=True, need=7),
                inp(200, dtype=1, reshard=True, need=8, is_float=False, needs_grad=False),
                inp(201, dtype=0, reshard=True, need=9)], [14])]
    order, fwd, live, gn, bwd = _native.plan_graph(ops, 1)
    assert 3 not in live and set(live) == {1, 2}
    # same (tensor, layout) resharded once; one exchange per dtype in first-seen order
    assert (1, 2, [0, 3]) in fwd and (1, 2, [2]) in fwd
    assert fwd.index((1, 2, [0, 3])) < fwd.index((1, 2, [2]))
    assert 201 not in gn          # graph input: no gradient unless input_grads
    assert 201 in _native.plan_graph(ops, 1, True)[3]


def test_cycle_is_rejected():
    ops = [(1, [inp(12, 2)], [11]), (2, [inp(11, 1)], [12])]
    with pytest.raises(RuntimeError, match="cycle"):
        _native.plan_graph(ops, 2)
