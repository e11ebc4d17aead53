"""Host staging of XDR values into the device layout, and back.

The Python counterpart of include/xdrpp_gpu.hh's stager/unstager: values
of an XdrType (xdr_types.py) become n native records of the plan's stride
plus a byte heap (xdrg_bytes_ref payloads and xvector/pointer element
arrays), the layout xdrg_encode reads; a decode's native records and heap
read back as values.

Values: int for int/unsigned/hyper/enums, float for float/double, bool,
bytes for opaque/string, list for arrays and vectors, None or the value
for a pointer, dict {field: value} for a struct, (discriminant, arm value)
for a union (arm value None for a void arm).
"""
from __future__ import annotations

import struct

import numpy as np

from .xdr_types import (Bool, Enum, OpaqueArray, Pointer, Struct, Union, Void, XArray, XdrType,
                        XVector, _Scalar, _VarBytes, _align_up)

__all__ = ["stage", "unstage"]

_FMT = {"int": "<i", "unsigned": "<I", "hyper": "<q", "unsigned hyper": "<Q", "float": "<f",
        "double": "<d"}


def _arm(u: Union, disc: int):
    for cases, _, t in u.arms:
        if disc in cases:
            return t
    if u.default is not None:
        return u.default[1]
    raise ValueError(f"{u.name}: no arm for discriminant {disc}")


class _Heap:
    def __init__(self) -> None:
        self.buf = bytearray()

    def alloc(self, n: int, align: int) -> int:
        off = _align_up(len(self.buf), align)
        self.buf.extend(bytes(off + n - len(self.buf)))
        return off


def _put(t: XdrType, buf: bytearray, off: int, v, heap: _Heap) -> None:
    if t is Bool:
        buf[off] = 1 if v else 0
    elif isinstance(t, _Scalar):
        struct.pack_into(_FMT[t.name], buf, off, v)
    elif isinstance(t, Enum):
        struct.pack_into("<i", buf, off, v)
    elif isinstance(t, OpaqueArray):
        if len(v) != t.n:
            raise ValueError(f"opaque[{t.n}] given {len(v)} bytes")
        buf[off:off + t.n] = v
    elif isinstance(t, _VarBytes):
        h = heap.alloc(len(v), 1)
        heap.buf[h:h + len(v)] = v
        struct.pack_into("<QII", buf, off, h, len(v), 0)
    elif isinstance(t, XArray):
        step = _align_up(t.elem.size, t.elem.align)
        for i, e in enumerate(v):
            _put(t.elem, buf, off + i * step, e, heap)
    elif isinstance(t, XVector):
        items = ([] if v is None else [v]) if isinstance(t, Pointer) else list(v)
        arr = heap.alloc(len(items) * t.stride, 8)
        struct.pack_into("<QII", buf, off, arr, len(items), 0)
        for i, e in enumerate(items):  # the heap may grow: write through heap.buf
            _put(t.elem, heap.buf, arr + i * t.stride, e, heap)
    elif isinstance(t, Struct):
        for fname, ft in t.fields:
            _put(ft, buf, off + t.offsets[fname], v[fname], heap)
    elif isinstance(t, Union):
        disc, val = v
        struct.pack_into("<i" if disc < 0x80000000 else "<I", buf, off, disc)
        arm = _arm(t, disc)
        if arm is not Void:
            _put(arm, buf, off + t.arms_off, val, heap)
    elif t is Void:
        pass
    else:
        raise TypeError(f"cannot stage {t!r}")


def stage(t: XdrType, values) -> tuple[np.ndarray, np.ndarray]:
    """(native uint8 [n * stride], heap uint8) of `values`."""
    stride = _align_up(t.size, t.align)
    native = bytearray(len(values) * stride)
    heap = _Heap()
    for i, v in enumerate(values):
        _put(t, native, i * stride, v, heap)
    return np.frombuffer(bytes(native), dtype=np.uint8).copy(), \
        np.frombuffer(bytes(heap.buf), dtype=np.uint8).copy()


def _get(t: XdrType, buf, off: int, heap):
    if t is Bool:
        return bool(buf[off])
    if isinstance(t, _Scalar):
        return struct.unpack_from(_FMT[t.name], buf, off)[0]
    if isinstance(t, Enum):
        return struct.unpack_from("<i", buf, off)[0]
    if isinstance(t, OpaqueArray):
        return bytes(buf[off:off + t.n])
    if isinstance(t, _VarBytes):
        h, n, _ = struct.unpack_from("<QII", buf, off)
        return bytes(heap[h:h + n])
    if isinstance(t, XArray):
        step = _align_up(t.elem.size, t.elem.align)
        return [_get(t.elem, buf, off + i * step, heap) for i in range(t.n)]
    if isinstance(t, XVector):
        arr, n, _ = struct.unpack_from("<QII", buf, off)
        items = [_get(t.elem, heap, arr + i * t.stride, heap) for i in range(n)]
        return (items[0] if items else None) if isinstance(t, Pointer) else items
    if isinstance(t, Struct):
        return {fname: _get(ft, buf, off + t.offsets[fname], heap) for fname, ft in t.fields}
    if isinstance(t, Union):
        disc = struct.unpack_from("<i", buf, off)[0]
        arm = _arm(t, disc)
        return (disc, None if arm is Void else _get(arm, buf, off + t.arms_off, heap))
    if t is Void:
        return None
    raise TypeError(f"cannot unstage {t!r}")


def unstage(t: XdrType, native, heap, n: int) -> list:
    """The n values of decoded (or staged) native records and their heap."""
    stride = _align_up(t.size, t.align)
    nat = bytes(np.asarray(native, dtype=np.uint8))
    hp = b"" if heap is None else bytes(np.asarray(heap, dtype=np.uint8))
    return [_get(t, nat, i * stride, hp) for i in range(n)]
