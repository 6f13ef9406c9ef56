"""Replay a ``.ff`` file onto an FFModel (``python/flexflow/torch/model.py:18-149``), plus
:func:`from_torch` which also copies the module's trained weights into the flexmi parameters."""
from __future__ import annotations

from flexmi.core.types import ActiMode, OpType, PoolType


class PyTorchModel:
    def __init__(self, filename):
        self.filename = filename
        self.tensor_dict = {}
        self.op_of_node = {}

    def apply(self, ffmodel, input_tensors):
        outputs = []
        idx = 0
        with open(self.filename) as f:
            lines = [ln.strip() for ln in f if ln.strip()]
        for line in lines:
            items = [i.strip() for i in line.split(",")]
            name = items[0]
            prev = [p.strip() for p in items[1].split(":") if p.strip()]
            op = OpType(int(items[2]))
            ins = [self.tensor_dict[p] for p in prev]
            t = None
            if op == OpType.INPUT:
                t = input_tensors[idx]
                idx += 1
            elif op == OpType.OUTPUT:
                outputs = ins
                continue
            elif op == OpType.LINEAR:
                t = ffmodel.dense(ins[0], int(items[3]), ActiMode(int(items[4])), bool(int(items[5])), name=name)
            elif op == OpType.CONV2D:
                t = ffmodel.conv2d(ins[0], int(items[3]), int(items[4]), int(items[5]), int(items[6]), int(items[7]),
                                   int(items[8]), int(items[9]), ActiMode(int(items[10])), bool(int(items[11])), name=name)
            elif op == OpType.POOL2D:
                k, s, p = int(items[3]), int(items[4]), int(items[5])
                t = ffmodel.pool2d(ins[0], k, k, s, s, p, p, PoolType(int(items[6])), ActiMode(int(items[7])), name=name)
            elif op == OpType.BATCH_NORM:
                t = ffmodel.batch_norm(ins[0], False, name=name)
            elif op == OpType.DROPOUT:
                t = ffmodel.dropout(ins[0], float(items[3]), 0, name=name)
            elif op == OpType.FLAT:
                t = ins[0] if len(ins[0].dims) == 2 else ffmodel.flat(ins[0], name=name)
            elif op in (OpType.RELU, OpType.SIGMOID, OpType.TANH, OpType.ELU, OpType.SOFTMAX, OpType.EXP):
                fn = {OpType.RELU: "relu", OpType.SIGMOID: "sigmoid", OpType.TANH: "tanh", OpType.ELU: "elu",
                      OpType.SOFTMAX: "softmax", OpType.EXP: "exp"}[op]
                t = getattr(ffmodel, fn)(ins[0], name=name)
            elif op == OpType.CONCAT:
                t = ffmodel.concat(ins, int(items[3]), name=name)
            elif op == OpType.ADD:
                t = ffmodel.add(ins[0], ins[1], name=name)
            elif op == OpType.SUBTRACT:
                t = ffmodel.subtract(ins[0], ins[1], name=name)
            elif op == OpType.MULTIPLY:
                t = ffmodel.multiply(ins[0], ins[1], name=name)
            else:
                raise ValueError(f"unsupported op {op!r} in {self.filename}")
            self.tensor_dict[name] = t
            if t is not None and t.owner_op is not None and all(t is not x for x in ins):
                self.op_of_node[name] = t.owner_op
        return outputs


def from_torch(module, ffmodel, input_tensors, filename=None):
    """Trace ``module`` (torch.fx), build it on ``ffmodel`` and return (outputs, PyTorchModel).
    After ``ffmodel.compile(...)`` + ``init_layers()`` call :func:`copy_weights`."""
    import os
    import tempfile
    from .fx import torch_to_flexflow
    import torch.fx
    path = filename or os.path.join(tempfile.mkdtemp(), "model.ff")
    torch_to_flexflow(module, path)
    pm = PyTorchModel(path)
    pm.targets = {n.name: n.target for n in torch.fx.symbolic_trace(module).graph.nodes if n.op == "call_module"}
    return pm.apply(ffmodel, input_tensors), pm


def copy_weights(module, ffmodel, pm):
    """Copy Linear / Conv2d / BatchNorm2d parameters of ``module`` into the flexmi model."""
    import torch
    mods = dict(module.named_modules())
    for node_name, op in pm.op_of_node.items():
        tgt = getattr(pm, "targets", {}).get(node_name, node_name)
        m = mods.get(tgt)
        if m is None:
            continue
        if isinstance(m, (torch.nn.Linear, torch.nn.Conv2d)):
            op.weights[0].set_weights(ffmodel, m.weight.detach().cpu().numpy())
            if m.bias is not None and len(op.weights) > 1:
                op.weights[1].set_weights(ffmodel, m.bias.detach().cpu().numpy())
        elif isinstance(m, torch.nn.BatchNorm2d) and m.affine:
            op.weights[0].set_weights(ffmodel, m.weight.detach().cpu().numpy())
            op.weights[1].set_weights(ffmodel, m.bias.detach().cpu().numpy())
