"""PyTorch -> flexmi via torch.fx (``python/flexflow/torch/fx.py``).

``torch_to_flexflow(module, filename)`` symbolically traces the module and writes the reference's
line format ``name, in1:in2:, <OpType int>, params...`` (one op per line; OpType values of
``flexflow_type.py:39-65``) so files round-trip with the reference tools.  Beyond the reference
it understands tuple kernel/stride/padding for pooling (written as the first component, like
the reference), functional ``relu/sigmoid/tanh/mul/sub/flatten``, ``operator.add`` and
``torch.cat(dim=...)``.
"""
from __future__ import annotations

import operator

import torch
import torch.fx

from flexmi.core.types import ActiMode, OpType, PoolType


def _first(v):
    return v[0] if isinstance(v, (tuple, list)) else v


def _args_names(args):
    a = args[0] if len(args) == 1 and isinstance(args[0], (list, tuple)) else args
    return [x.name for x in a if isinstance(x, torch.fx.Node)]


def _module_line(m):
    T = torch.nn
    if isinstance(m, T.Linear):
        return [int(OpType.LINEAR), m.out_features, int(ActiMode.AC_MODE_NONE), 1 if m.bias is not None else 0]
    if isinstance(m, T.Conv2d):
        return [int(OpType.CONV2D), m.out_channels, m.kernel_size[0], m.kernel_size[1], m.stride[0], m.stride[1],
                m.padding[0], m.padding[1], int(ActiMode.AC_MODE_NONE), 1 if m.bias is not None else 0]
    if isinstance(m, (T.MaxPool2d, T.AvgPool2d)):
        pt = PoolType.POOL_MAX if isinstance(m, T.MaxPool2d) else PoolType.POOL_AVG
        return [int(OpType.POOL2D), _first(m.kernel_size), _first(m.stride), _first(m.padding), int(pt),
                int(ActiMode.AC_MODE_NONE)]
    if isinstance(m, T.BatchNorm2d):
        return [int(OpType.BATCH_NORM)]
    if isinstance(m, T.Dropout):
        return [int(OpType.DROPOUT), m.p]
    if isinstance(m, T.Flatten):
        return [int(OpType.FLAT)]
    for cls, op in ((T.ReLU, OpType.RELU), (T.Sigmoid, OpType.SIGMOID), (T.Tanh, OpType.TANH), (T.ELU, OpType.ELU),
                    (T.Softmax, OpType.SOFTMAX)):
        if isinstance(m, cls):
            return [int(op)]
    raise ValueError(f"unsupported module {type(m).__name__}")


def _function_line(node):
    f = node.target
    name = getattr(f, "__name__", str(f))
    if f in (operator.add, torch.add) or name in ("add", "__add__"):
        return [int(OpType.ADD)]
    if f in (operator.sub, torch.sub) or name in ("sub", "__sub__"):
        return [int(OpType.SUBTRACT)]
    if f in (operator.mul, torch.mul) or name in ("mul", "__mul__"):
        return [int(OpType.MULTIPLY)]
    if f is torch.cat or name == "cat":
        dim = node.kwargs.get("dim", node.args[1] if len(node.args) > 1 else 0)
        return [int(OpType.CONCAT), dim]
    if name == "flatten":
        return [int(OpType.FLAT)]
    if name == "relu":
        return [int(OpType.RELU)]
    if name == "sigmoid":
        return [int(OpType.SIGMOID)]
    if name == "tanh":
        return [int(OpType.TANH)]
    if name == "softmax":
        return [int(OpType.SOFTMAX)]
    raise ValueError(f"unsupported function {name}")


def torch_to_flexflow(model: torch.nn.Module, filename: str):
    traced = torch.fx.symbolic_trace(model)
    mods = dict(model.named_modules())
    lines = []
    for node in traced.graph.nodes:
        if node.op == "placeholder":
            lines.append([node.name, "", int(OpType.INPUT)])
        elif node.op == "output":
            lines.append([node.name, ":".join(_args_names(node.args)) + ":", int(OpType.OUTPUT)])
        elif node.op == "call_module":
            lines.append([node.name, ":".join(_args_names(node.args)) + ":"] + _module_line(mods[node.target]))
        elif node.op in ("call_function", "call_method"):
            lines.append([node.name, ":".join(_args_names(node.args)) + ":"] + _function_line(node))
        elif node.op == "get_attr":
            continue
        else:
            raise ValueError(f"unhandled fx node {node.op}")
    with open(filename, "w") as f:
        for ln in lines:
            f.write(", ".join(str(x) for x in ln) + "\n")
    return lines
