"""ONNX frontend (``python/flexflow/onnx/model.py:15-128``) on flexmi's own wire codec.

``ONNXModel(file).apply(ffmodel, {input_name: tensor})`` lowers the graph node by node
(``handle<OpType>``) and returns the graph output tensor; ``copy_weights(ffmodel)`` loads the
initializers (Conv / Gemm / BatchNormalization parameters) into the flexmi parameters after
``init_layers``.  Handlers: Add, Sub, Mul, AveragePool, GlobalAveragePool, BatchNormalization,
Concat, Conv, Dropout, Flatten, Gemm, MatMul (constant weight), MaxPool, Relu, Sigmoid, Tanh,
Elu, Softmax, Identity, Pad (pass-through, like the reference), Reshape (to 2-D).
"""
from __future__ import annotations

import logging

import numpy as np

from flexmi.core.types import ActiMode, PoolType

from .proto import decode_model


class ONNXModel:
    def __init__(self, filename_or_bytes):
        data = filename_or_bytes
        if isinstance(filename_or_bytes, str):
            with open(filename_or_bytes, "rb") as f:
                data = f.read()
        self.graph = decode_model(data)
        self.inits = self.graph["initializers"]
        self.inputs = {vi["name"]: vi for vi in self.graph["inputs"]}
        self.symbol_table = {}
        self.param_ops = []     # (op, {"weight": name, "bias": name, ...})

    # -- helpers -----------------------------------------------------------------------
    def _t(self, name):
        return self.symbol_table[name]

    def _attr(self, node, name, default=None):
        a = node["attrs"].get(name)
        if a is None:
            return default
        for k in ("ints", "floats", "i", "f", "s"):
            if k in a:
                return a[k]
        return default

    def _shape(self, name):
        if name in self.inits:
            return list(self.inits[name].shape)
        return self.inputs[name]["shape"]

    def _pool(self, ffmodel, node, kind):
        k = self._attr(node, "kernel_shape")
        p = self._attr(node, "pads", [0, 0, 0, 0])
        s = self._attr(node, "strides", [1, 1])
        return ffmodel.pool2d(self._t(node["input"][0]), k[0], k[1], s[0], s[1], p[0], p[1], kind)

    # -- handlers -----------------------------------------------------------------------
    def handleAdd(self, m, n):
        return m.add(self._t(n["input"][0]), self._t(n["input"][1]))

    def handleSub(self, m, n):
        return m.subtract(self._t(n["input"][0]), self._t(n["input"][1]))

    def handleMul(self, m, n):
        return m.multiply(self._t(n["input"][0]), self._t(n["input"][1]))

    def handleAveragePool(self, m, n):
        return self._pool(m, n, PoolType.POOL_AVG)

    def handleMaxPool(self, m, n):
        return self._pool(m, n, PoolType.POOL_MAX)

    def handleGlobalAveragePool(self, m, n):
        x = self._t(n["input"][0])
        return m.pool2d(x, x.dims[2], x.dims[3], 1, 1, 0, 0, PoolType.POOL_AVG)

    def handleBatchNormalization(self, m, n):
        out = m.batch_norm(self._t(n["input"][0]), False)
        self.param_ops.append((out.owner_op, {"scale": n["input"][1], "bias": n["input"][2]}))
        return out

    def handleConcat(self, m, n):
        return m.concat([self._t(i) for i in n["input"]], int(self._attr(n, "axis", 1)))

    def handleConv(self, m, n):
        w = n["input"][1]
        k = self._attr(n, "kernel_shape") or self._shape(w)[2:]
        p = self._attr(n, "pads", [0, 0, 0, 0])
        s = self._attr(n, "strides", [1, 1])
        g = int(self._attr(n, "group", 1))
        bias = len(n["input"]) > 2
        out = m.conv2d(self._t(n["input"][0]), self._shape(w)[0], k[0], k[1], s[0], s[1], p[0], p[1],
                       ActiMode.AC_MODE_NONE, bias, groups=g)
        self.param_ops.append((out.owner_op, {"weight": w, "bias": n["input"][2] if bias else None}))
        return out

    def handleDropout(self, m, n):
        return m.dropout(self._t(n["input"][0]), float(self._attr(n, "ratio", 0.5)), 0)

    def handleFlatten(self, m, n):
        x = self._t(n["input"][0])
        return x if len(x.dims) == 2 else m.flat(x)

    def handleReshape(self, m, n):
        x = self._t(n["input"][0])
        return x if len(x.dims) == 2 else m.flat(x)

    def handleGemm(self, m, n):
        w = n["input"][1]
        ws = self._shape(w)
        trans_b = int(self._attr(n, "transB", 0))
        out_dim = ws[0] if trans_b else ws[1]
        bias = len(n["input"]) > 2
        out = m.dense(self._t(n["input"][0]), out_dim, ActiMode.AC_MODE_NONE, bias)
        self.param_ops.append((out.owner_op, {"weight": w, "bias": n["input"][2] if bias else None,
                                              "transpose": not trans_b}))
        return out

    def handleMatMul(self, m, n):
        w = n["input"][1]
        out = m.dense(self._t(n["input"][0]), self._shape(w)[1], ActiMode.AC_MODE_NONE, False)
        self.param_ops.append((out.owner_op, {"weight": w, "bias": None, "transpose": True}))
        return out

    def handleRelu(self, m, n):
        return m.relu(self._t(n["input"][0]))

    def handleSigmoid(self, m, n):
        return m.sigmoid(self._t(n["input"][0]))

    def handleTanh(self, m, n):
        return m.tanh(self._t(n["input"][0]))

    def handleElu(self, m, n):
        return m.elu(self._t(n["input"][0]))

    def handleSoftmax(self, m, n):
        return m.softmax(self._t(n["input"][0]))

    def handleIdentity(self, m, n):
        return self._t(n["input"][0])

    def handlePad(self, m, n):
        logging.warning("ONNX Pad is passed through (reference behaviour)")
        return self._t(n["input"][0])

    # -- driver -------------------------------------------------------------------------
    def apply(self, ffmodel, input_dict):
        self.symbol_table = dict(input_dict)
        for n in self.graph["nodes"]:
            h = getattr(self, "handle" + n["op_type"], None)
            if h is None:
                raise ValueError(f"unsupported ONNX op {n['op_type']}")
            self.symbol_table[n["output"][0]] = h(ffmodel, n)
        return self.symbol_table[self.graph["outputs"][0]["name"]]

    def copy_weights(self, ffmodel):
        """Load the initializers of every lowered Conv/Gemm/MatMul/BatchNorm (after init_layers)."""
        for op, names in self.param_ops:
            if "scale" in names:
                op.weights[0].set_weights(ffmodel, self.inits[names["scale"]].astype(np.float32))
                op.weights[1].set_weights(ffmodel, self.inits[names["bias"]].astype(np.float32))
                continue
            w = self.inits[names["weight"]].astype(np.float32)
            if names.get("transpose"):
                w = w.T
            op.weights[0].set_weights(ffmodel, np.ascontiguousarray(w))
            if names.get("bias") is not None:
                op.weights[1].set_weights(ffmodel, self.inits[names["bias"]].astype(np.float32))
