"""ctypes bridge to the C restatement oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE: used only by tests/, __graft_entry__.smoke() (as the
checker) and bench.py's cpu_baseline leg.  Builds the oracle with gcc on
first use if it is missing (gcc exists on the GPU box too).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "_build", "liboracle.so")
REF_BIN = os.path.join(ORACLE_DIR, "_ref", "ref_golden")

_lib = None


SOURCES = [os.path.join(ORACLE_DIR, "xdr_oracle.c"), os.path.join(ORACLE_DIR, "cpu_bench.c")]


def build() -> None:
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.check_call(["gcc", "-O3", "-fPIC", "-shared", "-std=gnu11", "-pthread", "-o", LIB] + SOURCES)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB) or any(os.path.getmtime(LIB) < os.path.getmtime(f) for f in SOURCES):
            build()
        L = C.CDLL(LIB)
        vp, u64, u32 = C.c_void_p, C.c_uint64, C.c_uint32
        L.xdro_encode.argtypes = [vp, u32, vp, u32, vp, u64, vp, u64, vp, u64, vp, u32,
                                  C.POINTER(u64), C.POINTER(u32), C.POINTER(u64)]
        L.xdro_decode.argtypes = [vp, u32, vp, u32, vp, u64, vp, u64, vp, vp, u32,
                                  C.POINTER(u64), C.POINTER(u32)]
        L.xdro_sizes.argtypes = [vp, u32, vp, u32, vp, u64, vp, u64, vp, C.POINTER(u64), C.POINTER(u32)]
        L.xdro_depths.argtypes = L.xdro_sizes.argtypes
        L.xdro_encode_msgs.argtypes = L.xdro_encode.argtypes
        L.xdro_decode_msgs.argtypes = L.xdro_decode.argtypes
        L.xdro_index_msgs.argtypes = [vp, u64, u32, u64, vp, C.POINTER(u64), C.POINTER(u64)]
        L.xdro_decode_heap_size.argtypes = [vp, u32, u64]
        L.xdro_decode_heap_size.restype = u64
        _lib = L
    return _lib


def _p(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class OracleError(Exception):
    def __init__(self, code: int, record: int, op: int):
        super().__init__(f"oracle error code={code} record={record} op={op}")
        self.code, self.record, self.op = code, record, op


def _heap(heap):
    return np.zeros(1, dtype=np.uint8) if heap is None or heap.size == 0 else heap


def sizes(plan, native: np.ndarray, n: int, heap: np.ndarray | None = None) -> np.ndarray:
    """xdr_size of every record (uint32 [n]) or raises OracleError."""
    out = np.zeros(max(n, 1), dtype=np.uint32)
    er, eo = C.c_uint64(0), C.c_uint32(0)
    h = _heap(heap)
    rc = lib().xdro_sizes(_p(plan.ops), len(plan.ops), _p(plan.table), plan.stride, _p(native), n,
                          _p(h), 0 if heap is None else heap.size, _p(out), C.byref(er), C.byref(eo))
    if rc:
        raise OracleError(rc, er.value, eo.value)
    return out[:n]


def encode(plan, native: np.ndarray, n: int, heap: np.ndarray | None = None,
           stack_limit: int = 0xFFFFFFFF, cap: int | None = None):
    """Returns (xdr bytes, offsets[n+1]) or raises OracleError."""
    if heap is None or heap.size == 0:
        heap = np.zeros(1, dtype=np.uint8)
    sizes = np.zeros(max(n, 1), dtype=np.uint32)
    er, eo = C.c_uint64(0), C.c_uint32(0)
    if cap is None:
        rc = lib().xdro_sizes(_p(plan.ops), len(plan.ops), _p(plan.table), plan.stride,
                              _p(native), n, _p(heap), heap.size, _p(sizes), C.byref(er), C.byref(eo))
        cap = int(sizes[:n].astype(np.uint64).sum()) if rc == 0 else 1 << 20
    out = np.zeros(max(cap, 4), dtype=np.uint8)
    offs = np.zeros(n + 1, dtype=np.uint64)
    tot = C.c_uint64(0)
    rc = lib().xdro_encode(_p(plan.ops), len(plan.ops), _p(plan.table), plan.stride,
                           _p(native), n, _p(heap), heap.size, _p(out), cap, _p(offs),
                           stack_limit, C.byref(er), C.byref(eo), C.byref(tot))
    if rc:
        raise OracleError(rc, er.value, eo.value)
    return out[:tot.value], offs


def decode(plan, xdr: np.ndarray, n: int, offsets: np.ndarray | None = None,
           stack_limit: int = 0xFFFFFFFF):
    """Returns (native, heap) or raises OracleError.  heap = the stream
    verbatim, then (plans with xvector/pointer fields) the element area."""
    native = np.zeros(max(n, 1) * plan.stride, dtype=np.uint8)
    hsize = int(lib().xdro_decode_heap_size(_p(plan.ops), len(plan.ops), xdr.size))
    heap = np.zeros(max(hsize, 4), dtype=np.uint8)
    er, eo = C.c_uint64(0), C.c_uint32(0)
    x = xdr if xdr.size else np.zeros(4, dtype=np.uint8)
    rc = lib().xdro_decode(_p(plan.ops), len(plan.ops), _p(plan.table), plan.stride,
                           _p(x), xdr.size, _p(offsets), n, _p(native), _p(heap),
                           stack_limit, C.byref(er), C.byref(eo))
    if rc:
        raise OracleError(rc, er.value, eo.value)
    return native[:n * plan.stride], heap[:hsize]


# ------------------------------------------------- record-marked messages
def encode_msgs(plan, native: np.ndarray, n: int, heap: np.ndarray | None = None,
                stack_limit: int = 0xFFFFFFFF, cap: int | None = None):
    """xdr_to_msg of every record, back to back: (stream, offsets[n+1])."""
    if heap is None or heap.size == 0:
        heap = np.zeros(1, dtype=np.uint8)
    er, eo = C.c_uint64(0), C.c_uint32(0)
    if cap is None:
        sizes = np.zeros(max(n, 1), dtype=np.uint32)
        rc = lib().xdro_sizes(_p(plan.ops), len(plan.ops), _p(plan.table), plan.stride,
                              _p(native), n, _p(heap), heap.size, _p(sizes), C.byref(er), C.byref(eo))
        cap = int(sizes[:n].astype(np.uint64).sum()) + 4 * n if rc == 0 else 1 << 20
    out = np.zeros(max(cap, 4), dtype=np.uint8)
    offs = np.zeros(n + 1, dtype=np.uint64)
    tot = C.c_uint64(0)
    rc = lib().xdro_encode_msgs(_p(plan.ops), len(plan.ops), _p(plan.table), plan.stride,
                                _p(native), n, _p(heap), heap.size, _p(out), cap, _p(offs),
                                stack_limit, C.byref(er), C.byref(eo), C.byref(tot))
    if rc:
        raise OracleError(rc, er.value, eo.value)
    return out[:tot.value], offs


def decode_msgs(plan, stream: np.ndarray, n: int, offsets: np.ndarray,
                stack_limit: int = 0xFFFFFFFF):
    """xdr_from_msg of every indexed message: (native, heap)."""
    native = np.zeros(max(n, 1) * plan.stride, dtype=np.uint8)
    hsize = int(lib().xdro_decode_heap_size(_p(plan.ops), len(plan.ops), stream.size))
    heap = np.zeros(max(hsize, 4), dtype=np.uint8)
    er, eo = C.c_uint64(0), C.c_uint32(0)
    x = stream if stream.size else np.zeros(4, dtype=np.uint8)
    offs = np.ascontiguousarray(offsets, dtype=np.uint64)
    rc = lib().xdro_decode_msgs(_p(plan.ops), len(plan.ops), _p(plan.table), plan.stride,
                                _p(x), stream.size, _p(offs), n, _p(native), _p(heap),
                                stack_limit, C.byref(er), C.byref(eo))
    if rc:
        raise OracleError(rc, er.value, eo.value)
    return native[:n * plan.stride], heap[:hsize]


def index_msgs(stream: np.ndarray, max_msg_len: int, max_msgs: int | None = None):
    """read_message framing over the stream: (rc, count, offsets[:count+1])."""
    if max_msgs is None:
        max_msgs = stream.size // 4
    offs = np.zeros(max_msgs + 1, dtype=np.uint64)
    cnt, erec = C.c_uint64(0), C.c_uint64(0)
    x = stream if stream.size else np.zeros(4, dtype=np.uint8)
    rc = lib().xdro_index_msgs(_p(x), stream.size, max_msg_len, max_msgs, _p(offs),
                               C.byref(cnt), C.byref(erec))
    return rc, int(cnt.value), offs[:cnt.value + 1]


# ------------------------------------------------------------ RPC headers
def _rpc_lib():
    L = lib()
    if not getattr(L, "_rpc_bound", False):
        vp, u64, u32 = C.c_void_p, C.c_uint64, C.c_uint32
        L.xdro_rpc_headers.argtypes = [vp, u64, vp, u64, vp, u32, vp, C.c_int, vp]
        L.xdro_rpc_replies.argtypes = [vp, u64, vp, u64, vp, C.POINTER(u64), C.POINTER(u64)]
        L._rpc_bound = True
    return L


def rpc_headers(stream: np.ndarray, offsets: np.ndarray, procs: np.ndarray | None,
                client: bool = False, xids: np.ndarray | None = None) -> np.ndarray:
    """xdrg_rpc_hdr records (numpy structured, xdrpp_amd.rpc.HDR_DTYPE)."""
    from xdrpp_amd.rpc import HDR_DTYPE
    n = offsets.size - 1
    out = np.zeros(max(n, 1), dtype=HDR_DTYPE)
    s = np.ascontiguousarray(stream, dtype=np.uint8)
    o = np.ascontiguousarray(offsets, dtype=np.uint64)
    p = None if procs is None else np.ascontiguousarray(procs, dtype=np.uint32)
    x = None if xids is None else np.ascontiguousarray(xids, dtype=np.uint32)
    _rpc_lib().xdro_rpc_headers(_p(s), s.size, _p(o), n, _p(p), 0 if p is None else p.size // 4,
                                _p(x), int(client), _p(out))
    return out[:n]


def rpc_replies(hdrs: np.ndarray, cap: int | None = None):
    """(reply stream, offsets[n+1], error code, failing record)."""
    n = hdrs.size
    cap = 36 * n if cap is None else cap
    out = np.zeros(max(cap, 4), dtype=np.uint8)
    offs = np.zeros(n + 1, dtype=np.uint64)
    tot, er = C.c_uint64(0), C.c_uint64(0)
    h = np.ascontiguousarray(hdrs)
    rc = _rpc_lib().xdro_rpc_replies(_p(h), n, _p(out), cap, _p(offs), C.byref(tot), C.byref(er))
    return out[:min(tot.value, cap)], offs, rc, er.value


def index_records(plan, xdr: np.ndarray, n: int, maxlen: int):
    """xdro_index_records: (offsets[n+1], count, error code, error record)."""
    L = lib()
    vp, u64, u32 = C.c_void_p, C.c_uint64, C.c_uint32
    L.xdro_index_records.argtypes = [vp, u32, vp, vp, u64, u64, u32, vp, C.POINTER(u64), C.POINTER(u64)]
    offs = np.zeros(n + 1, dtype=np.uint64)
    cnt, er = C.c_uint64(0), C.c_uint64(0)
    x = xdr if xdr.size else np.zeros(4, dtype=np.uint8)
    rc = L.xdro_index_records(_p(plan.ops), len(plan.ops), _p(plan.table), _p(x), xdr.size, n, maxlen,
                              _p(offs), C.byref(cnt), C.byref(er))
    return offs, cnt.value, rc, er.value


def depths(plan, native: np.ndarray, n: int, heap: np.ndarray | None = None) -> np.ndarray:
    """depth_checker per record (xdro_depths); raises OracleError."""
    out = np.zeros(max(n, 1), dtype=np.uint32)
    er, eo = C.c_uint64(0), C.c_uint32(0)
    h = _heap(heap)
    rc = lib().xdro_depths(_p(plan.ops), len(plan.ops), _p(plan.table), plan.stride, _p(native), n,
                           _p(h), 0 if heap is None else heap.size, _p(out), C.byref(er), C.byref(eo))
    if rc:
        raise OracleError(rc, er.value, eo.value)
    return out[:n]
