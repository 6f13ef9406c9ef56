"""Offline torch -> ONNX exporter for the ONNX examples' ``*_pt.py`` scripts
(reference ``examples/python/onnx/*_pt.py`` call ``torch.onnx.export``, which needs the ``onnx``
package; it is not installed here).  The module is traced with ``torch.fx`` and each node is
written as an ONNX node with the built-in wire codec (:mod:`flexmi.onnx.proto`); weights become
initializers.  Covers the ops :class:`flexmi.onnx.ONNXModel` lowers: Linear (Gemm transB=1),
Conv2d, Max/AvgPool2d, BatchNorm2d, Dropout, Flatten, ReLU/Sigmoid/Tanh/ELU, Softmax, add/sub/mul,
cat."""
from __future__ import annotations

import operator

import numpy as np
import torch

from .proto import encode_model, encode_node


def _pair(v):
    return list(v) if isinstance(v, (tuple, list)) else [v, v]


def torch_to_onnx(module: torch.nn.Module, input_shapes, filename=None, input_names=None):
    """Export ``module`` (called with tensors of ``input_shapes``) to ONNX bytes; also written to
    ``filename`` when given.  Returns the bytes."""
    T = torch.nn
    if isinstance(input_shapes[0], int):
        input_shapes = [input_shapes]
    traced = torch.fx.symbolic_trace(module)
    mods = dict(module.named_modules())
    nodes, inits, inputs, outputs = [], {}, [], []
    shapes = {}
    ex = [torch.zeros(*s) for s in input_shapes]
    # shapes of every fx value, for the output value_info
    from torch.fx.passes.shape_prop import ShapeProp
    ShapeProp(traced).propagate(*ex)
    for n in traced.graph.nodes:
        meta = n.meta.get("tensor_meta")
        if meta is not None and hasattr(meta, "shape"):
            shapes[n.name] = list(meta.shape)
    names = list(input_names or [])
    ph = 0

    def arg(a):
        return a.name if isinstance(a, torch.fx.Node) else str(a)

    def add_init(name, t):
        inits[name] = t.detach().float().cpu().numpy()
        return name

    for n in traced.graph.nodes:
        if n.op == "placeholder":
            nm = names[ph] if ph < len(names) else n.name
            if nm != n.name:
                nodes.append(encode_node("Identity", [nm], [n.name]))
            inputs.append((nm, list(input_shapes[ph])))
            ph += 1
        elif n.op == "output":
            outs = n.args[0] if isinstance(n.args[0], (tuple, list)) else [n.args[0]]
            for o in outs:
                outputs.append((o.name, shapes.get(o.name, [])))
        elif n.op == "call_module":
            m = mods[n.target]
            x = arg(n.args[0])
            p = n.target.replace(".", "_")
            if isinstance(m, T.Linear):
                ins = [x, add_init(p + "_w", m.weight)] + ([add_init(p + "_b", m.bias)] if m.bias is not None else [])
                nodes.append(encode_node("Gemm", ins, [n.name], transB=1))
            elif isinstance(m, T.Conv2d):
                ins = [x, add_init(p + "_w", m.weight)] + ([add_init(p + "_b", m.bias)] if m.bias is not None else [])
                ph_, pw_ = _pair(m.padding)
                nodes.append(encode_node("Conv", ins, [n.name], kernel_shape=_pair(m.kernel_size),
                                         strides=_pair(m.stride), pads=[ph_, pw_, ph_, pw_], group=m.groups))
            elif isinstance(m, (T.MaxPool2d, T.AvgPool2d)):
                k, s, pd = _pair(m.kernel_size), _pair(m.stride or m.kernel_size), _pair(m.padding)
                nodes.append(encode_node("MaxPool" if isinstance(m, T.MaxPool2d) else "AveragePool", [x], [n.name],
                                         kernel_shape=k, strides=s, pads=[pd[0], pd[1], pd[0], pd[1]]))
            elif isinstance(m, T.BatchNorm2d):
                ins = [x, add_init(p + "_scale", m.weight), add_init(p + "_bias", m.bias),
                       add_init(p + "_mean", m.running_mean), add_init(p + "_var", m.running_var)]
                nodes.append(encode_node("BatchNormalization", ins, [n.name], epsilon=float(m.eps)))
            elif isinstance(m, T.Dropout):
                nodes.append(encode_node("Dropout", [x], [n.name]))
            elif isinstance(m, T.Flatten):
                nodes.append(encode_node("Flatten", [x], [n.name], axis=int(m.start_dim)))
            elif isinstance(m, T.Softmax):
                nodes.append(encode_node("Softmax", [x], [n.name], axis=int(m.dim if m.dim is not None else -1)))
            else:
                for cls, op in ((T.ReLU, "Relu"), (T.Sigmoid, "Sigmoid"), (T.Tanh, "Tanh"), (T.ELU, "Elu")):
                    if isinstance(m, cls):
                        nodes.append(encode_node(op, [x], [n.name]))
                        break
                else:
                    raise ValueError(f"torch_to_onnx: unsupported module {type(m).__name__}")
        elif n.op in ("call_function", "call_method"):
            f = n.target
            fname = getattr(f, "__name__", str(f))
            if f in (operator.add, torch.add) or fname in ("add", "__add__"):
                nodes.append(encode_node("Add", [arg(a) for a in n.args[:2]], [n.name]))
            elif f in (operator.sub, torch.sub) or fname in ("sub", "__sub__"):
                nodes.append(encode_node("Sub", [arg(a) for a in n.args[:2]], [n.name]))
            elif f in (operator.mul, torch.mul) or fname in ("mul", "__mul__"):
                nodes.append(encode_node("Mul", [arg(a) for a in n.args[:2]], [n.name]))
            elif f is torch.cat or fname == "cat":
                dim = n.kwargs.get("dim", n.args[1] if len(n.args) > 1 else 0)
                nodes.append(encode_node("Concat", [arg(a) for a in n.args[0]], [n.name], axis=int(dim)))
            elif fname == "flatten":
                nodes.append(encode_node("Flatten", [arg(n.args[0])], [n.name],
                                         axis=int(n.args[1] if len(n.args) > 1 else n.kwargs.get("start_dim", 1))))
            elif fname in ("relu", "sigmoid", "tanh"):
                nodes.append(encode_node(fname.capitalize(), [arg(n.args[0])], [n.name]))
            elif fname == "softmax":
                nodes.append(encode_node("Softmax", [arg(n.args[0])], [n.name], axis=int(n.kwargs.get("dim", -1))))
            else:
                raise ValueError(f"torch_to_onnx: unsupported function {fname}")
        elif n.op == "get_attr":
            raise ValueError("torch_to_onnx: get_attr nodes are not supported")
    blob = encode_model(nodes, inputs, outputs, inits)
    if filename:
        with open(filename, "wb") as f:
            f.write(blob)
    return blob


def weights_of(module: torch.nn.Module):
    return {k: v.detach().cpu().numpy() for k, v in module.state_dict().items() if isinstance(v, torch.Tensor)}


__all__ = ["torch_to_onnx", "weights_of", "np"]
