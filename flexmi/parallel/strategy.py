"""Strategy files: the reference's protobuf format (``src/runtime/strategy.proto:1-23``).

``message Op {required string name=1; required DeviceType device_type=2; repeated int32 dims=3;
repeated int32 device_ids=4; repeated MemoryType memory_types=5}``, ``message Strategy
{repeated Op ops=1}`` (proto2, package FFProtoBuf).  Reader/writer semantics follow
``src/runtime/strategy.cc:96-172``.  The codec is native C++ (``csrc/runtime/strategy_pb.cc``,
a hand-rolled proto2 varint codec -- no protoc in the image) exposed through ``flexmi._native``;
the pure-Python codec below is kept as an independent cross-check.

Keys: the reference keyed configs by ``std::hash(op_name)`` (``strategy.cc:23-26``) and then
could not match the shipped DLRM files' op names (caveat C2).  flexmi keys by op name and also
resolves the reference's conventional names (``embedding<i>``, ``linear``, ``concat``,
``mse_loss``, ...) onto the ops of a graph (:func:`resolve_reference_names`).
"""
from __future__ import annotations

from typing import Dict

from .layout import ParallelConfig


# ---------------------------------------------------------------------- python codec
def _varint(n):
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf, i):
    shift = 0
    val = 0
    while True:
        b = buf[i]
        i += 1
        val |= (b & 0x7F) << shift
        if not b & 0x80:
            return val, i
        shift += 7


def _signed32(v):
    v &= (1 << 64) - 1
    if v >= 1 << 63:
        v -= 1 << 64
    return v


def encode_py(strategies: Dict[str, ParallelConfig]) -> bytes:
    out = bytearray()
    for name in sorted(strategies):
        pc = strategies[name]
        op = bytearray()
        nb = name.encode()
        op += b"\x0a" + _varint(len(nb)) + nb
        op += b"\x10" + _varint(pc.device_type)
        for d in pc.dims:
            op += b"\x18" + _varint(d)
        n = pc.num_parts()
        for d in pc.device_ids[:n]:
            op += b"\x20" + _varint(d)
        for m in pc.memory_types:
            op += b"\x28" + _varint(m)
        out += b"\x0a" + _varint(len(op)) + bytes(op)
    return bytes(out)


def _decode_op(buf):
    i = 0
    name, dt, dims, ids, mem = "", 0, [], [], []
    while i < len(buf):
        key, i = _read_varint(buf, i)
        field, wt = key >> 3, key & 7
        if wt == 2:
            ln, i = _read_varint(buf, i)
            chunk = buf[i:i + ln]
            i += ln
            if field == 1:
                name = chunk.decode()
            elif field in (3, 4, 5):  # packed repeated
                j = 0
                while j < len(chunk):
                    v, j = _read_varint(chunk, j)
                    [None, None, None, dims, ids, mem][field].append(_signed32(v))
        elif wt == 0:
            v, i = _read_varint(buf, i)
            if field == 2:
                dt = v
            elif field == 3:
                dims.append(_signed32(v))
            elif field == 4:
                ids.append(_signed32(v))
            elif field == 5:
                mem.append(_signed32(v))
        elif wt == 5:
            i += 4
        elif wt == 1:
            i += 8
        else:
            raise ValueError(f"bad wire type {wt}")
    return name, ParallelConfig(dims, ids, dt, mem)


def decode_py(data: bytes) -> Dict[str, ParallelConfig]:
    out = {}
    i = 0
    while i < len(data):
        key, i = _read_varint(data, i)
        field, wt = key >> 3, key & 7
        assert wt == 2 and field == 1, f"unexpected field {field}/{wt}"
        ln, i = _read_varint(data, i)
        name, pc = _decode_op(data[i:i + ln])
        i += ln
        assert name not in out, f"duplicate op {name} in strategy file"
        out[name] = pc
    return out


# ---------------------------------------------------------------------- public API
def _native():
    try:
        from flexmi import _native
        return _native
    except ImportError:
        return None


def load_strategies_from_file(path) -> Dict[str, ParallelConfig]:
    nat = _native()
    if nat is not None:
        ops = nat.load_strategy(str(path))
        return {name: ParallelConfig(list(dims), list(ids), dt, list(mem)) for name, dt, dims, ids, mem in ops}
    with open(path, "rb") as f:
        return decode_py(f.read())


def save_strategies_to_file(path, strategies: Dict[str, ParallelConfig]):
    nat = _native()
    if nat is not None:
        items = [(n, pc.device_type, list(pc.dims), list(pc.device_ids[:pc.num_parts()]), list(pc.memory_types))
                 for n, pc in sorted(strategies.items())]
        return nat.save_strategy(str(path), items)
    with open(path, "wb") as f:
        f.write(encode_py(strategies))
    return True


def resolve_reference_names(model, strategies: Dict[str, ParallelConfig]) -> Dict[str, ParallelConfig]:
    """Map the reference's conventional names onto this graph's op names (caveat C2):
    ``embedding<i>`` -> i-th Embedding op, ``linear``/``concat``/``mse_loss`` -> every op of that
    type (configs whose dims rank mismatches are skipped)."""
    from flexmi.core.types import OperatorType
    out = {}
    by_type = {}
    for op in model.layers:
        by_type.setdefault(op.op_type, []).append(op)
    embs = by_type.get(OperatorType.OP_EMBEDDING, [])
    for name, pc in strategies.items():
        matched = [op for op in model.layers if op.name == name]
        if name.startswith("embedding") and name[9:].isdigit():
            k = int(name[9:])
            matched = [embs[k]] if k < len(embs) else []
        elif name == "linear":
            matched = by_type.get(OperatorType.OP_LINEAR, [])
        elif name == "concat":
            matched = by_type.get(OperatorType.OP_CONCAT, [])
        elif name in ("batch_matmul",):
            matched = by_type.get(OperatorType.OP_BATCHMATMUL, [])
        elif name in ("transpose",):
            matched = by_type.get(OperatorType.OP_TRANSPOSE, [])
        for op in matched:
            if pc.nDims == op.out_ndims:
                out[op.name] = pc
    return out
