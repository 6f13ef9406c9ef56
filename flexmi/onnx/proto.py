"""Minimal ONNX protobuf wire codec (no ``onnx`` package in the image).

Covers the subset of ``onnx.proto`` the frontend needs -- ModelProto.graph, GraphProto
{node, name, initializer, input, output}, NodeProto {input, output, name, op_type, attribute},
AttributeProto {name, f, i, s, t, floats, ints, type}, TensorProto {dims, data_type,
float_data, int64_data, name, raw_data}, ValueInfoProto {name, type.tensor_type.shape} -- with
the field numbers of the ONNX schema, so files written by ONNX exporters parse unchanged.
"""
from __future__ import annotations

import struct

import numpy as np

# TensorProto.DataType
FLOAT, INT32, INT64 = 1, 6, 7
# AttributeProto.AttributeType
A_FLOAT, A_INT, A_STRING, A_TENSOR, A_FLOATS, A_INTS = 1, 2, 3, 4, 6, 7


# ------------------------------------------------------------------ wire primitives
def _varint(buf, pos):
    out = shift = 0
    while True:
        b = buf[pos]
        pos += 1
        out |= (b & 0x7F) << shift
        if b < 0x80:
            return out, pos
        shift += 7


def _fields(buf):
    pos, n = 0, len(buf)
    while pos < n:
        key, pos = _varint(buf, pos)
        fn, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _varint(buf, pos)
        elif wt == 1:
            v = buf[pos:pos + 8]
            pos += 8
        elif wt == 2:
            ln, pos = _varint(buf, pos)
            v = buf[pos:pos + ln]
            pos += ln
        elif wt == 5:
            v = buf[pos:pos + 4]
            pos += 4
        else:
            raise ValueError(f"unsupported wire type {wt}")
        yield fn, wt, v


def _signed(v):
    return v - (1 << 64) if v >= (1 << 63) else v


def _packed_varints(b):
    out, pos = [], 0
    while pos < len(b):
        v, pos = _varint(b, pos)
        out.append(_signed(v))
    return out


# ------------------------------------------------------------------ decode
def decode_tensor(b):
    t = {"dims": [], "data_type": FLOAT, "name": "", "float_data": [], "int64_data": [], "raw": None}
    for fn, wt, v in _fields(b):
        if fn == 1:
            t["dims"] += _packed_varints(v) if wt == 2 else [_signed(v)]
        elif fn == 2:
            t["data_type"] = v
        elif fn == 4:
            t["float_data"] += list(struct.unpack(f"<{len(v) // 4}f", v)) if wt == 2 else [struct.unpack("<f", v)[0]]
        elif fn == 7:
            t["int64_data"] += _packed_varints(v) if wt == 2 else [_signed(v)]
        elif fn == 8:
            t["name"] = v.decode()
        elif fn == 9:
            t["raw"] = bytes(v)
    return t


def tensor_to_numpy(t):
    dt = {FLOAT: np.float32, INT32: np.int32, INT64: np.int64}[t["data_type"]]
    if t["raw"] is not None:
        a = np.frombuffer(t["raw"], dtype=dt).copy()
    elif t["data_type"] == FLOAT:
        a = np.asarray(t["float_data"], np.float32)
    else:
        a = np.asarray(t["int64_data"], dt)
    return a.reshape(t["dims"]) if t["dims"] else a


def _decode_attr(b):
    a = {"name": "", "type": 0}
    ints, floats = [], []
    for fn, wt, v in _fields(b):
        if fn == 1:
            a["name"] = v.decode()
        elif fn == 2:
            a["f"] = struct.unpack("<f", v)[0]
        elif fn == 3:
            a["i"] = _signed(v)
        elif fn == 4:
            a["s"] = bytes(v)
        elif fn == 5:
            a["t"] = decode_tensor(v)
        elif fn == 7:
            floats += list(struct.unpack(f"<{len(v) // 4}f", v)) if wt == 2 else [struct.unpack("<f", v)[0]]
        elif fn == 8:
            ints += _packed_varints(v) if wt == 2 else [_signed(v)]
        elif fn == 20:
            a["type"] = v
    if ints:
        a["ints"] = ints
    if floats:
        a["floats"] = floats
    return a


def _decode_node(b):
    n = {"input": [], "output": [], "name": "", "op_type": "", "attrs": {}}
    for fn, wt, v in _fields(b):
        if fn == 1:
            n["input"].append(v.decode())
        elif fn == 2:
            n["output"].append(v.decode())
        elif fn == 3:
            n["name"] = v.decode()
        elif fn == 4:
            n["op_type"] = v.decode()
        elif fn == 5:
            a = _decode_attr(v)
            n["attrs"][a["name"]] = a
    return n


def _decode_value_info(b):
    vi = {"name": "", "shape": []}
    for fn, wt, v in _fields(b):
        if fn == 1:
            vi["name"] = v.decode()
        elif fn == 2:                       # TypeProto
            for f2, _, v2 in _fields(v):
                if f2 == 1:                 # tensor_type
                    for f3, _, v3 in _fields(v2):
                        if f3 == 2:         # shape
                            for f4, _, v4 in _fields(v3):
                                if f4 == 1:  # dim
                                    val = None
                                    for f5, _, v5 in _fields(v4):
                                        if f5 == 1:
                                            val = _signed(v5)
                                    vi["shape"].append(val)
    return vi


def decode_model(data: bytes):
    graph = None
    opset = None
    for fn, wt, v in _fields(data):
        if fn == 7:
            graph = v
        elif fn == 8:
            for f2, _, v2 in _fields(v):
                if f2 == 2:
                    opset = v2
    if graph is None:
        raise ValueError("no graph in ONNX model")
    g = {"nodes": [], "name": "", "initializers": {}, "inputs": [], "outputs": [], "opset": opset}
    for fn, wt, v in _fields(graph):
        if fn == 1:
            g["nodes"].append(_decode_node(v))
        elif fn == 2:
            g["name"] = v.decode()
        elif fn == 5:
            t = decode_tensor(v)
            g["initializers"][t["name"]] = tensor_to_numpy(t)
        elif fn == 11:
            g["inputs"].append(_decode_value_info(v))
        elif fn == 12:
            g["outputs"].append(_decode_value_info(v))
    return g


# ------------------------------------------------------------------ encode (tests / export)
def _enc_varint(v):
    if v < 0:
        v += 1 << 64
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(fn, wt):
    return _enc_varint((fn << 3) | wt)


def _ld(fn, payload: bytes):
    return _key(fn, 2) + _enc_varint(len(payload)) + payload


def _vi(fn, v):
    return _key(fn, 0) + _enc_varint(int(v))


def encode_tensor(name, arr):
    arr = np.ascontiguousarray(arr)
    dt = {np.dtype(np.float32): FLOAT, np.dtype(np.int32): INT32, np.dtype(np.int64): INT64}[arr.dtype]
    b = b"".join(_vi(1, d) for d in arr.shape) + _vi(2, dt) + _ld(8, name.encode()) + _ld(9, arr.tobytes())
    return b


def _encode_attr(name, val):
    b = _ld(1, name.encode())
    if isinstance(val, float):
        b += _key(2, 5) + struct.pack("<f", val) + _vi(20, A_FLOAT)
    elif isinstance(val, int):
        b += _vi(3, val) + _vi(20, A_INT)
    elif isinstance(val, (bytes, str)):
        b += _ld(4, val.encode() if isinstance(val, str) else val) + _vi(20, A_STRING)
    elif isinstance(val, (list, tuple)) and all(isinstance(x, int) for x in val):
        b += b"".join(_vi(8, x) for x in val) + _vi(20, A_INTS)
    elif isinstance(val, (list, tuple)):
        b += b"".join(_key(7, 5) + struct.pack("<f", float(x)) for x in val) + _vi(20, A_FLOATS)
    else:
        raise TypeError(val)
    return b


def encode_node(op_type, inputs, outputs, name="", **attrs):
    b = b"".join(_ld(1, i.encode()) for i in inputs) + b"".join(_ld(2, o.encode()) for o in outputs)
    b += _ld(3, name.encode()) + _ld(4, op_type.encode())
    b += b"".join(_ld(5, _encode_attr(k, v)) for k, v in attrs.items())
    return b


def _encode_vi(name, shape):
    dims = b"".join(_ld(1, _vi(1, d)) for d in shape)
    tt = _vi(1, FLOAT) + _ld(2, dims)
    return _ld(1, name.encode()) + _ld(2, _ld(1, tt))


def encode_model(nodes, inputs, outputs, initializers, name="graph", opset=13):
    """nodes: encoded NodeProto bytes; inputs/outputs: [(name, shape)]; initializers {name: array}."""
    g = b"".join(_ld(1, n) for n in nodes) + _ld(2, name.encode())
    g += b"".join(_ld(5, encode_tensor(k, v)) for k, v in initializers.items())
    g += b"".join(_ld(11, _encode_vi(n, s)) for n, s in inputs)
    g += b"".join(_ld(12, _encode_vi(n, s)) for n, s in outputs)
    return _vi(1, 7) + _ld(7, g) + _ld(8, _vi(2, opset))
