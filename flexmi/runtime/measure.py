"""Measure one op's forward/backward time at a shard shape on the local MI355X.

Reference: ``Op::measure_compute_time`` (e.g. ``src/ops/linear.cu:973-1049``) allocated the
shard's tensors in a simulator arena on GPU 0 and timed 5 warm-up + 10 runs of the op's CUDA
kernels with cudaEvents.

flexmi builds a one-op model with the shard shapes (same op type and attributes, same HIP
kernels and fused epilogues the executor runs), captures ``reps`` back-to-back forward (resp.
backward) calls into one hipGraph -- the way the training step runs them -- and reports the
mean per call.  Used by ``tools/calibrate_costs.py`` to fill the simulator's cost DB.
"""
from __future__ import annotations

import torch

from flexmi.core.types import DataType, OperatorType


def _make_clone(op, m, in_shapes, out_shapes):
    """Build the op again inside model ``m`` on fresh inputs with shard shapes; None if the op
    type has no measurable kernel (views) or is unsupported."""
    from flexmi.ops.elementwise import ElementBinary, ElementUnary
    t = op.op_type
    ins = [m.create_tensor(list(s), op.inputs[i].data_type) for i, s in enumerate(in_shapes)]
    if t == OperatorType.OP_LINEAR:
        m.dense(ins[0], out_shapes[0][-1], op.activation, op.use_bias)
    elif t == OperatorType.OP_EMBEDDING:
        m.embedding(ins[0], op.num_entries, out_shapes[0][-1], op.aggr)
    elif t == OperatorType.OP_DOT_INTERACTION:
        m.dot_interaction(ins[0], ins[1:], op.self_interaction)
    elif t == OperatorType.OP_CONCAT:
        m.concat(ins, op.axis)
    elif t == OperatorType.OP_BATCHMATMUL:
        m.batch_matmul(ins[0], ins[1])
    elif t == OperatorType.OP_SOFTMAX:
        m.softmax(ins[0])
    elif t == OperatorType.OP_CONV2D:
        m.conv2d(ins[0], out_shapes[0][1], op.kh, op.kw, op.sh, op.sw, op.ph, op.pw, op.activation, op.use_bias)
    elif t == OperatorType.OP_POOL2D:
        m.pool2d(ins[0], op.kh, op.kw, op.sh, op.sw, op.ph, op.pw, op.pool_type, op.activation)
    elif t == OperatorType.OP_LSTM:
        st = op.has_state
        m.lstm(ins[0], op.H, ins[1] if st else None, ins[2] if st else None)
    elif isinstance(op, ElementUnary):
        m._add(ElementUnary(m, op.op_type, ins[0]))
    elif isinstance(op, ElementBinary):
        m._add(ElementBinary(m, op.op_type, ins[0], ins[1]))
    else:
        return None
    return ins


def measure_op(op, in_shapes, out_shapes, reps=20, index_range=None, device="gpu", dtype="bf16"):
    """(fwd_us, bwd_us) of ``op`` at the given shard shapes on ``cuda`` in compute precision
    ``dtype`` (bf16 fast mode or the fp32 reference-precision kernels; ``device="cpu"``: host
    timing of the fp32 reference path, used by the CPU tests)."""
    from flexmi.core import FFConfig, FFModel, SGDOptimizer, LossType
    cfg = FFConfig()
    cfg.batchSize = int(in_shapes[0][0]) if in_shapes and in_shapes[0] else 1
    cfg.device = device
    cfg.compute_dtype = dtype if device == "gpu" else "fp32"
    # the op's input gradient is part of its backward unless the input is a graph input
    cfg.input_grads = not (op.op_type == OperatorType.OP_LINEAR and op.inputs[0].owner_op is None)
    m = FFModel(cfg)
    ins = _make_clone(op, m, in_shapes, out_shapes)
    if ins is None:
        return None
    m.compile(SGDOptimizer(m, 0.001), LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE, [])
    ex = m.init_layers()
    g = torch.Generator(device=ex.device)
    g.manual_seed(0)
    for t in ins:
        buf = ex.local_buffer(t)
        if buf is None:
            continue
        if t.data_type in (DataType.DT_INT32, DataType.DT_INT64):
            hi = index_range or getattr(m.layers[0], "num_entries", 2)
            buf.copy_(torch.randint(0, hi, buf.shape, generator=g, device=ex.device))
        else:
            buf.copy_(torch.randn(buf.shape, generator=g, device=ex.device))
    new = m.layers[0]
    mine = lambda it: (it.kind == "compute" and it.name.startswith(new.name + ".")
                       and "zero_unused" not in it.name)
    fwd = [it for it in ex.prog_fwd if mine(it)]
    bwd = [it for it in ex.prog_bwd if mine(it)]
    out_grad = ex.grad.get(new.outputs[0].guid)
    if out_grad is not None:
        out_grad.copy_(torch.randn(out_grad.shape, generator=g, device=ex.device) * 1e-3)

    def timed(items):
        if not items:
            return 0.0
        if device != "gpu":
            import time
            t0 = time.perf_counter()
            for _ in range(reps):
                for it in items:
                    it.fn()
            return (time.perf_counter() - t0) * 1e6 / reps
        for it in items:           # warm-up (lazy workspaces)
            it.fn()
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(gr, stream=s):
                for _ in range(reps):
                    for it in items:
                        it.fn()
        torch.cuda.current_stream().wait_stream(s)
        gr.replay()
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        best = float("inf")
        for _ in range(3):
            e0.record()
            gr.replay()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
        del gr
        return best

    f = timed(fwd)
    b = timed(bwd)
    m.executor = None
    del ex
    if device == "gpu":
        torch.cuda.empty_cache()
    return f, b


def measure_embedding_group(ops, batch, reps=20, device="gpu", dtype="bf16"):
    """(fwd_us, bwd_us) of ALL embedding ``ops`` looked up together at ``batch`` rows -- the fused
    group launch the executor actually runs (one forward, one sparse-SGD backward for every table
    of a placement).  tools/calibrate_costs.py divides it by the sum of the per-table isolated
    measurements to get the DB's ``group_factor``."""
    from flexmi.core import FFConfig, FFModel, SGDOptimizer, LossType
    cfg = FFConfig()
    cfg.batchSize = int(batch)
    cfg.device = device
    cfg.compute_dtype = dtype if device == "gpu" else "fp32"
    m = FFModel(cfg)
    ins = []
    for op in ops:
        t = m.create_tensor([batch, op.inputs[0].dims[1]], op.inputs[0].data_type)
        m.embedding(t, op.num_entries, op.out_dim, op.aggr)
        ins.append((t, op.num_entries))
    last = [m.concat([l.outputs[0] for l in m.layers], 1)] if len(m.layers) > 1 else [m.layers[0].outputs[0]]
    m.compile(SGDOptimizer(m, 0.001), LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE, [])
    ex = m.init_layers()
    g = torch.Generator(device=ex.device)
    g.manual_seed(0)
    for t, rows in ins:
        buf = ex.local_buffer(t)
        buf.copy_(torch.randint(0, rows, buf.shape, generator=g, device=ex.device))
    names = tuple(l.name + "." for l in m.layers if l.op_type == OperatorType.OP_EMBEDDING)
    fwd = [it for it in ex.prog_fwd if it.kind == "compute" and it.name.startswith(names)]
    bwd = [it for it in ex.prog_bwd if it.kind == "compute" and it.name.startswith(names)]
    for gr in ex.grad.values():
        gr.normal_(0, 1e-3)

    def timed(items):
        if not items:
            return 0.0
        import time
        for it in items:
            it.fn()
        if device != "gpu":
            t0 = time.perf_counter()
            for _ in range(reps):
                for it in items:
                    it.fn()
            return (time.perf_counter() - t0) * 1e6 / reps
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            for it in items:
                it.fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / reps

    f, b = timed(fwd), timed(bwd)
    m.executor = None
    del ex
    if device == "gpu":
        torch.cuda.empty_cache()
    return f, b
