"""HDF5 datasets without libhdf5/h5py: the native reader (``csrc/runtime/hdf5_lite.cc``) locates
each dataset's contiguous data, which is then memory-mapped with numpy (zero-copy, the OS pages
in only the batches that are read).  Used for the DLRM ``--dataset`` files that the reference's
``examples/cpp/DLRM/preprocess_hdf.py`` writes (X_int float32 [N,13], X_cat int64 [N,26],
y float32 [N]) and read by ``dlrm.cc:284-330`` / ``:425-483`` with libhdf5.

:func:`write_h5` writes the same structure h5py produces with its default (earliest) format:
superblock v0, a symbol-table root group (v1 B-tree + local heap + symbol table node), v1 object
headers and contiguous little-endian datasets.  h5py is not installed in this image, so files
written by real h5py are parity-unpinned; the reader also accepts superblock v2/v3 files with
compact link groups.
"""
from __future__ import annotations

import struct
from typing import Dict

import numpy as np

UNDEF = 0xFFFFFFFFFFFFFFFF


def list_datasets(path):
    """{name: (dtype str, shape tuple, byte offset, nbytes)} of every dataset in the file."""
    from flexmi import _native
    return {n: (dt, tuple(sh), off, nb) for n, dt, sh, off, nb in _native.h5_datasets(path)}


def open_h5(path) -> Dict[str, np.ndarray]:
    """Memory-map every dataset of an HDF5 file as a read-only numpy array."""
    out = {}
    for name, (dt, shape, off, nb) in list_datasets(path).items():
        if off < 0:
            out[name] = np.zeros(shape, dtype=np.dtype(dt))
            continue
        out[name] = np.memmap(path, dtype=np.dtype(dt), mode="r", offset=off, shape=shape)
    return out


def _pad8(b):
    return b + b"\0" * (-len(b) % 8)


def _dtype_msg(a):
    dt = a.dtype
    if dt.byteorder == ">":
        raise ValueError("big-endian arrays are not supported")
    if dt.kind in "iu":
        bits0 = 0x08 if dt.kind == "i" else 0x00
        return struct.pack("<BBBBI", 0x10 | 0, bits0, 0, 0, dt.itemsize) + struct.pack("<HH", 0, 8 * dt.itemsize)
    if dt.kind == "f":
        if dt.itemsize == 4:
            props = struct.pack("<HHBBBBI", 0, 32, 23, 8, 0, 23, 127)
            sign = 31
        else:
            props = struct.pack("<HHBBBBI", 0, 64, 52, 11, 0, 52, 1023)
            sign = 63
        return struct.pack("<BBBBI", 0x10 | 1, 0x20, sign, 0, dt.itemsize) + props
    raise ValueError(f"unsupported dtype {dt}")


def _obj_header(msgs):
    body = b""
    for mtype, data in msgs:
        data = _pad8(data)
        body += struct.pack("<HHB3x", mtype, len(data), 0) + data
    return struct.pack("<BBHII", 1, 0, len(msgs), 1, len(body)) + b"\0" * 4 + body


def write_h5(path, arrays: Dict[str, np.ndarray]):
    """Write ``{name: array}`` as contiguous datasets in the root group (h5py default layout)."""
    names = sorted(arrays)
    arrays = {n: np.ascontiguousarray(arrays[n]) for n in names}
    # local heap data: "" at 0, then the names (8-byte aligned)
    heap_data = b"\0" * 8
    name_off = {}
    for n in names:
        name_off[n] = len(heap_data)
        heap_data += _pad8(n.encode() + b"\0")
    SB = 96
    root_oh = SB
    root_oh_bytes = _obj_header([(0x11, b"\0" * 16)])       # patched below
    heap = root_oh + len(root_oh_bytes)
    heap_hdr_len = 32
    heap_data_addr = heap + heap_hdr_len
    btree = heap_data_addr + len(heap_data)
    btree_len = 24 + 8 + 8 + 8
    snod = btree + btree_len
    snod_len = 8 + 40 * len(names)
    pos = snod + snod_len
    ohdrs = {}
    oh_bytes = {}
    for n in names:
        a = arrays[n]
        space = struct.pack("<BBBB4x", 1, a.ndim, 0, 0) + b"".join(struct.pack("<Q", d) for d in a.shape)
        layout_stub = struct.pack("<BBQQ", 3, 1, 0, a.nbytes)
        ob = _obj_header([(0x01, space), (0x03, _dtype_msg(a)), (0x08, layout_stub)])
        ohdrs[n] = pos
        oh_bytes[n] = (space, ob)
        pos += len(ob)
    data_addr = {}
    for n in names:
        pos = (pos + 511) // 512 * 512
        data_addr[n] = pos
        pos += arrays[n].nbytes
    eof = pos
    with open(path, "wb") as f:
        sb = b"\x89HDF\r\n\x1a\n" + struct.pack("<BBBBBBBB", 0, 0, 0, 0, 0, 8, 8, 0)
        sb += struct.pack("<HHI", 4, 16, 0)
        sb += struct.pack("<QQQQ", 0, UNDEF, eof, UNDEF)
        sb += struct.pack("<QQII", 0, root_oh, 1, 0) + struct.pack("<QQ", btree, heap)
        assert len(sb) == SB
        f.write(sb)
        f.write(_obj_header([(0x11, struct.pack("<QQ", btree, heap))]))
        f.write(b"HEAP" + struct.pack("<B3xQQQ", 0, len(heap_data), UNDEF, heap_data_addr))
        f.write(heap_data)
        last = name_off[names[-1]] if names else 0
        f.write(b"TREE" + struct.pack("<BBHQQ", 0, 0, 1, UNDEF, UNDEF) + struct.pack("<QQQ", 0, snod, last))
        f.write(b"SNOD" + struct.pack("<BBH", 1, 0, len(names)))
        for n in names:
            f.write(struct.pack("<QQII", name_off[n], ohdrs[n], 0, 0) + b"\0" * 16)
        for n in names:
            a = arrays[n]
            space, _ = oh_bytes[n]
            layout = struct.pack("<BBQQ", 3, 1, data_addr[n], a.nbytes)
            ob = _obj_header([(0x01, space), (0x03, _dtype_msg(a)), (0x08, layout)])
            assert f.tell() == ohdrs[n]
            f.write(ob)
        for n in names:
            f.seek(data_addr[n])
            f.write(arrays[n].tobytes())
        f.truncate(eof)
