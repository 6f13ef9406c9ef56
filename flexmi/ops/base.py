"""Operator base class.

Reference: ``class Op`` (``include/model.h:240-281``) with init/forward/backward tasks,
``create_output_and_partition``/``create_weights`` and ``measure_compute_time``.  In flexmi an
op is split into

  * graph semantics: shape inference, parameters, initializers (constructor);
  * parallel semantics: for a ParallelConfig, the *layouts* (shard boxes + holders) of its
    outputs, required inputs and weights -- what the reference expressed as Legion
    partitions in ``create_output_and_partition`` (e.g. ``src/ops/linear.cu:188-293``);
  * local compute: ``forward(ctx)`` / ``backward(ctx)`` on this rank's shards, dispatched to
    the HIP kernels (``flexmi/ops/_kernels.py``) on MI355X or to fp32 PyTorch on CPU;
  * cost hints for the simulator (``flops``/``bytes`` of a shard).

All backward kernels honour ``ctx.in_grad_accumulate`` (β=1 accumulate vs β=0 overwrite);
the reference always accumulated after ``zero_gradients`` (``src/ops/linear.cu:614-634``).
"""
from __future__ import annotations

import itertools
from typing import List

import torch

from flexmi.core.tensor import Parameter, Tensor
from flexmi.core.types import DataType, OperatorType
from flexmi.parallel.layout import Layout, ParallelConfig

_op_guid = itertools.count(100)  # reference guids start at 100 (src/runtime/model.cc:142)


class OpCtx:
    """Per-rank execution context of one op (buffers fixed at plan time)."""

    def __init__(self, op, rank, backend, compute_dtype):
        self.op = op
        self.rank = rank
        self.backend = backend            # "cpu" | "hip"
        self.compute_dtype = compute_dtype  # torch dtype of float activations
        self.inputs: List[torch.Tensor] = []
        self.outputs: List[torch.Tensor] = []
        self.weights: List[torch.Tensor] = []   # fp32 master shards
        self.wcompute: List[torch.Tensor] = []  # compute copies (bf16) or the masters
        self.wcompute_t: List[torch.Tensor] = []  # transposed compute copies (GEMM dX), optional
        self.in_boxes = []
        self.out_boxes = []
        self.w_boxes = []
        self.out_grads: List[torch.Tensor] = []
        self.in_grads: List[torch.Tensor] = []
        self.in_grad_accumulate: List[bool] = []
        self.weight_grads: List[torch.Tensor] = []
        self.saved = {}
        self.training = True
        self.sparse_update = None   # callable(lr) for fused sparse optimizers (embeddings)
        self.lr = None              # device scalar tensor (SGD lr) for fused updates
        self.workspace = {}

    @property
    def hip(self):
        return self.backend == "hip"


def store(dst: torch.Tensor, val: torch.Tensor, accumulate: bool):
    if accumulate:
        dst.add_(val.to(dst.dtype))
    else:
        dst.copy_(val)


class Op:
    op_type = OperatorType.OP_ANY
    name_prefix = "Op"

    def __init__(self, model, inputs: List[Tensor], name=None):
        self.model = model
        self.guid = next(_op_guid)
        self.inputs = list(inputs)
        self.outputs: List[Tensor] = []
        self.weights: List[Parameter] = []
        self.name = name
        self.profiling = getattr(model.config, "profiling", False) if model is not None else False
        self.layer_id = None

    # ------------------------------------------------------------------ graph
    def _finish(self, out_dims_list, out_dtypes=None):
        for i, d in enumerate(out_dims_list):
            dt = out_dtypes[i] if out_dtypes else DataType.DT_FLOAT
            self.outputs.append(Tensor(d, dt, owner_op=self, owner_idx=i, model=self.model,
                                       name=f"{self.name}:out{i}"))
        return self

    def _add_weight(self, dims, init, suffix, dtype=DataType.DT_FLOAT):
        p = Parameter(dims, dtype, owner_op=self, owner_idx=len(self.weights), model=self.model,
                      name=f"{self.name}.{suffix}", initializer=init)
        self.weights.append(p)
        return p

    def auto_name(self, params: str):
        """``"<Type>_<params>_<guid>"`` (e.g. ``"Dense_512"``; ``src/ops/linear.cu:67``)."""
        return f"{self.name_prefix}_{params}_{self.guid}" if params else f"{self.name_prefix}_{self.guid}"

    # reference Python wrapper API (flexflow_cbinding.py:52-344)
    def get_weight_tensor(self):
        return self.weights[0] if self.weights else None

    def get_bias_tensor(self):
        return self.weights[1] if len(self.weights) > 1 else None

    def get_input_tensor(self, idx=0):
        return self.inputs[idx]

    def get_output_tensor(self, idx=0):
        return self.outputs[idx]

    def get_parameter_by_id(self, idx):
        return self.weights[idx]

    def get_input_by_id(self, idx):
        return self.inputs[idx]

    def get_output_by_id(self, idx):
        return self.outputs[idx]

    def init(self, model=None):
        """Per-op init is folded into the executor build (``Op::init`` index launch)."""
        return None

    # ------------------------------------------------------------------ parallel
    @property
    def out_ndims(self):
        return len(self.outputs[0].dims)

    def splittable_dims(self):
        """User-order dims of output 0 that may be partitioned (SOAP sample/attribute/parameter)."""
        return {0}

    def valid_pc(self, pc: ParallelConfig):
        deg = Layout.from_pc(self.outputs[0].dims, pc).degrees
        ok = all(d == 1 or (i in self.splittable_dims() and d <= self.outputs[0].dims[i]) for i, d in enumerate(deg))
        return ok and all(0 <= x for x in pc.device_ids) and len(pc.device_ids) == pc.num_parts()

    def output_layouts(self, pc: ParallelConfig):
        return [Layout.from_pc(o.dims, pc) for o in self.outputs]

    def input_layouts(self, pc: ParallelConfig):
        """Default: inputs partitioned exactly like output 0 (elementwise semantics)."""
        lo = Layout.from_pc(self.outputs[0].dims, pc)
        return [Layout(t.dims, lo.degrees, lo.holders) for t in self.inputs]

    def weight_layouts(self, pc: ParallelConfig):
        """Default: weights replicated on every device of the op."""
        devs = tuple(sorted(set(pc.device_ids)))
        return [Layout.replicated(w.dims, devs) for w in self.weights]

    def sample_replica_groups(self, pc):
        return None

    # ------------------------------------------------------------------ compute
    def forward(self, ctx: OpCtx):
        raise NotImplementedError(type(self).__name__)

    def backward(self, ctx: OpCtx):
        raise NotImplementedError(type(self).__name__)

    def needs_input_grad(self, i):
        t = self.inputs[i]
        return t.data_type in (DataType.DT_FLOAT, DataType.DT_DOUBLE, DataType.DT_BF16, DataType.DT_HALF)

    def prepare(self, ctx: OpCtx):
        """Called once after buffers are bound (kernel-side workspaces, descriptors)."""
        return None

    # ------------------------------------------------------------------ cost hints
    def flops(self, in_shapes, out_shapes):
        """Forward FLOPs of a shard; backward assumed 2x (GEMM-like ops)."""
        v = 0
        for s in out_shapes:
            n = 1
            for d in s:
                n *= d
            v += n
        return float(v)

    def bytes_moved(self, in_shapes, out_shapes, elem=2):
        n = 0
        for s in list(in_shapes) + list(out_shapes):
            m = 1
            for d in s:
                m *= d
            n += m
        return float(n * elem)

    def __repr__(self):
        return f"{type(self).__name__}({self.name})"
