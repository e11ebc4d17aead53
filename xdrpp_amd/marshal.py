"""Batched xdr_to_opaque / xdr_from_opaque on MI355X through the C ABI.

Host-side mirror of the reference entry points (xdrpp/marshal.h:252-306):

    xdr_to_opaque(r0, ..., rn-1)      -> to_opaque_batch(plan, native, heap)
    xdr_from_opaque(bytes, r0, ...)   -> from_opaque_batch(plan, xdr, n, offsets)

with the reference's exception classes and what() strings
(xdrpp/types.h:57-99).  Buffers are torch CUDA(HIP) tensors; torch is only
plumbing for device memory and streams — every byte is produced by the HIP
kernels in libxdrgpu.so.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np
import torch

from . import _abi as A
from .xdr_types import CompiledPlan, XdrType, compile_plan


# ---------------------------------------------------------------- exceptions
class XdrRuntimeError(RuntimeError):
    """xdr::xdr_runtime_error (types.h:59-61).  ``record``: index of the
    failing record in the batch; ``op``: plan op index (None: record level)."""

    def __init__(self, what: str, record: int | None = None, op: int | None = None,
                 code: int = 0):
        super().__init__(what)
        self.what, self.record, self.op, self.code = what, record, op, code


class XdrOverflow(XdrRuntimeError):  # types.h:64-66
    pass


class XdrStackOverflow(XdrRuntimeError):  # types.h:69-71
    pass


class XdrBadMessageSize(XdrRuntimeError):  # types.h:74-76
    pass


class XdrBadDiscriminant(XdrRuntimeError):  # types.h:79-81
    pass


class XdrShouldBeZero(XdrRuntimeError):  # types.h:84-86
    pass


class XdrInvariantFailed(XdrRuntimeError):  # types.h:89-91
    pass


_EXC = {1: XdrOverflow, 2: XdrStackOverflow, 3: XdrBadMessageSize, 4: XdrBadDiscriminant,
        5: XdrShouldBeZero, 6: XdrInvariantFailed}


# ---------------------------------------------------------------------- plan
class Plan:
    """A compiled, device-resident plan for one XDR type (xdrg_plan_create).
    ``options``: launch options of this plan (xdrg_plan_set_option; names
    in _abi.PLAN_OPTIONS), e.g. {"var_encode_kernel": 1}."""

    def __init__(self, t: XdrType | CompiledPlan, options: dict | None = None):
        self.cp = t if isinstance(t, CompiledPlan) else compile_plan(t)
        L = A.lib()
        ops = self.cp.ops
        table = self.cp.table if self.cp.table.size else None
        h = C.c_void_p()
        A.check(L.xdrg_plan_create(
            ops.ctypes.data_as(C.POINTER(A.XdrgOp)), len(ops),
            None if table is None else table.ctypes.data_as(C.POINTER(C.c_uint32)),
            0 if table is None else table.size, self.cp.stride, C.byref(h)), "xdrg_plan_create")
        self.handle = h
        for k, v in (options or {}).items():
            A.check(L.xdrg_plan_set_option(h, A.PLAN_OPTIONS[k], int(v)), f"xdrg_plan_set_option({k})")
        info = A.XdrgPlanInfo()
        A.check(L.xdrg_plan_get_info(h, C.byref(info)), "xdrg_plan_get_info")
        self.path = info.path
        self.fixed_size = info.fixed_size or None
        self.stride = info.native_stride
        self.max_depth = info.max_depth
        self.has_checks = bool(info.has_checks)
        self.max_record_bytes = int(info.max_record_bytes)
        self.group_records = int(info.group_records)

    @property
    def is_fixed(self) -> bool:
        return self.path != A.PATH_VAR

    def decode_heap_bytes(self, xdr_len: int) -> int:
        """Heap capacity decode needs (xdrg_decode_heap_size): the stream
        verbatim, plus the element area of xvector/pointer fields."""
        return int(A.lib().xdrg_decode_heap_size(self.handle, xdr_len))

    def workspace_bytes(self, n: int) -> int:
        return int(A.lib().xdrg_workspace_size(self.handle, n))

    def close(self) -> None:
        if getattr(self, "handle", None):
            A.lib().xdrg_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# -------------------------------------------------------------------- status
class Status:
    """Device-resident xdrg_status (16 bytes), born initialised: first_error
    all ones (no error), total 0 -- what xdrg_status_init writes -- so a raw
    launch whose caller skipped init() cannot read allocator garbage as an
    error."""

    def __init__(self, device: torch.device):
        self.buf = torch.tensor([-1, 0], dtype=torch.int64, device=device)

    @property
    def ptr(self) -> int:
        return self.buf.data_ptr()

    def init(self, stream: int) -> None:
        A.check(A.lib().xdrg_status_init(self.ptr, stream), "xdrg_status_init")

    def read(self, stream: int) -> A.XdrgError:
        e = A.XdrgError()
        A.check(A.lib().xdrg_status_read(self.ptr, stream, C.byref(e)), "xdrg_status_read")
        return e


def error_from(plan: Plan, e: A.XdrgError) -> XdrRuntimeError | None:
    if e.code == 0:
        return None
    what = A.lib().xdrg_error_message(e.code).decode()
    op = None if e.op == 0xFFFFFFFF else int(e.op)
    if e.code == A.ERR_BAD_DISCRIMINANT and op is not None:
        what = plan.cp.bad_discriminant_message(op)
    cls = _EXC.get(A.lib().xdrg_error_exception(e.code), XdrRuntimeError)
    return cls(what, int(e.record), op, int(e.code))


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None or t.numel() == 0 else t.data_ptr()


@dataclass
class EncodeResult:
    xdr: torch.Tensor            # uint8, exactly the encoded bytes
    offsets: torch.Tensor | None  # uint64-as-int64 [n+1] record offsets (var plans)


class Marshaler:
    """Reusable encode/decode launcher for one plan: owns the status block
    and the var-plan workspace so repeated calls allocate nothing."""

    def __init__(self, plan: Plan, device: torch.device | str = "cuda"):
        self.plan = plan
        self.device = torch.device(device)
        self.status = Status(self.device)
        self._ws = torch.empty(0, dtype=torch.uint8, device=self.device)

    def _workspace(self, n: int) -> torch.Tensor:
        need = self.plan.workspace_bytes(n)
        if self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        return self._ws

    def _deep(self, n: int) -> tuple[int | None, int]:
        """(pointer, bytes) of the deep-pass workspace decode, serial_sizes and
        record_depths take (xdrg_deep_workspace_size: none for most plans)."""
        need = int(A.lib().xdrg_deep_workspace_size(self.plan.handle, n))
        if not need:
            return None, 0
        return self._workspace(n).data_ptr(), need  # (xdrg_workspace_size holds it)

    # ---- raw launches (no sync, no status handling) -----------------------
    def launch_encode(self, native, n, out, heap=None, offsets=None, stack_limit=A.DEFAULT_STACK_LIMIT,
                      stream=None):
        ws = self._workspace(n) if not self.plan.is_fixed else None
        A.check(A.lib().xdrg_encode(
            self.plan.handle, _ptr(native), n, _ptr(heap), 0 if heap is None else heap.numel(),
            _ptr(out), out.numel(), _ptr(offsets), stack_limit, _ptr(ws),
            0 if ws is None else ws.numel(), self.status.ptr,
            _stream() if stream is None else stream), "xdrg_encode")

    def launch_decode(self, xdr, n, native_out, offsets=None, heap_out=None,
                      stack_limit=A.DEFAULT_STACK_LIMIT, stream=None):
        dw, dn = self._deep(n)
        A.check(A.lib().xdrg_decode(
            self.plan.handle, _ptr(xdr), xdr.numel(), _ptr(offsets), n, _ptr(native_out),
            _ptr(heap_out), 0 if heap_out is None else heap_out.numel(), stack_limit, dw, dn,
            self.status.ptr, _stream() if stream is None else stream), "xdrg_decode")

    def launch_encode_msgs(self, native, n, out, offsets, heap=None,
                           stack_limit=A.DEFAULT_STACK_LIMIT, stream=None):
        ws = self._workspace(n)
        A.check(A.lib().xdrg_encode_msgs(
            self.plan.handle, _ptr(native), n, _ptr(heap), 0 if heap is None else heap.numel(),
            _ptr(out), out.numel(), _ptr(offsets), stack_limit, _ptr(ws), ws.numel(),
            self.status.ptr, _stream() if stream is None else stream), "xdrg_encode_msgs")

    def launch_decode_msgs(self, stream_bytes, n, native_out, offsets, heap_out=None,
                           stack_limit=A.DEFAULT_STACK_LIMIT, stream=None):
        dw, dn = self._deep(n)
        A.check(A.lib().xdrg_decode_msgs(
            self.plan.handle, _ptr(stream_bytes), stream_bytes.numel(), _ptr(offsets), n,
            _ptr(native_out), _ptr(heap_out), 0 if heap_out is None else heap_out.numel(),
            stack_limit, dw, dn, self.status.ptr, _stream() if stream is None else stream),
            "xdrg_decode_msgs")

    def check(self, stream=None) -> A.XdrgError:
        e = self.status.read(_stream() if stream is None else stream)
        err = error_from(self.plan, e)
        if err is not None:
            raise err
        return e

    # ---- reference-shaped API --------------------------------------------
    def serial_sizes(self, native, n, stack_limit=A.DEFAULT_STACK_LIMIT, heap=None) -> torch.Tensor:
        """xdr_size of every record (xdrpp/types.h:240-244)."""
        sizes = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        s = _stream()
        self.status.init(s)
        dw, dn = self._deep(n)
        A.check(A.lib().xdrg_serial_sizes(self.plan.handle, _ptr(native), n, _ptr(heap),
                                          0 if heap is None else heap.numel(), _ptr(sizes),
                                          stack_limit, dw, dn, self.status.ptr, s), "xdrg_serial_sizes")
        self.check(s)
        return sizes[:n]

    def record_depths(self, native, n, heap=None) -> torch.Tensor:
        """Deepest class/container level of every record's walk
        (depth_checker, xdrpp/depth_checker.h:10-79); int32 [n]."""
        d = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        s = _stream()
        self.status.init(s)
        dw, dn = self._deep(n)
        A.check(A.lib().xdrg_record_depths(self.plan.handle, _ptr(native), n, _ptr(heap),
                                           0 if heap is None else heap.numel(), _ptr(d), dw, dn,
                                           self.status.ptr, s), "xdrg_record_depths")
        self.check(s)
        return d[:n]

    def check_xdr_depth(self, native, n, depth_limit: int, heap=None) -> torch.Tensor:
        """xdr::check_xdr_depth(r_i, depth_limit) for every record
        (xdrpp/depth_checker.h:72-79): bool [n]."""
        return self.record_depths(native, n, heap) <= depth_limit

    def encode(self, native: torch.Tensor, n: int, heap: torch.Tensor | None = None,
               stack_limit: int = A.DEFAULT_STACK_LIMIT, capacity: int | None = None) -> EncodeResult:
        """= xdr_to_opaque(r0, ..., rn-1) (marshal.h:264-272)."""
        s = _stream()
        if self.plan.is_fixed:
            cap = n * self.plan.fixed_size if capacity is None else capacity
            out = torch.empty(max(cap, 4), dtype=torch.uint8, device=self.device)[:cap]
            self.status.init(s)
            self.launch_encode(native, n, out, stack_limit=stack_limit, stream=s)
            self.check(s)
            return EncodeResult(out, None)
        offsets = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        if capacity is None:  # one size pass: the output is sized from it
            return self._encode_two_halves(native, n, heap, offsets, stack_limit, msgs=0)
        out = torch.empty(max(capacity, 4), dtype=torch.uint8, device=self.device)
        self.status.init(s)
        self.launch_encode(native, n, out, heap=heap, offsets=offsets, stack_limit=stack_limit,
                           stream=s)
        e = self.check(s)
        return EncodeResult(out[:e.total_bytes], offsets)

    def _encode_two_halves(self, native, n, heap, offsets, stack_limit, msgs: int) -> EncodeResult:
        """xdr_to_opaque's own order (marshal.h:264-272): xdrg_encode_sizes
        (xdr_argpack_size) into the workspace, the output allocated from its
        total, then xdrg_encode_sized over the same sizes: one size pass."""
        s = _stream()
        L = A.lib()
        ws = self._workspace(n)
        hl = 0 if heap is None else heap.numel()
        self.status.init(s)
        A.check(L.xdrg_encode_sizes(self.plan.handle, _ptr(native), n, _ptr(heap), hl, stack_limit, msgs,
                                    _ptr(ws), ws.numel(), self.status.ptr, s), "xdrg_encode_sizes")
        total = int(self.check(s).total_bytes)
        out = torch.empty(max(total, 4), dtype=torch.uint8, device=self.device)
        A.check(L.xdrg_encode_sized(self.plan.handle, _ptr(native), n, _ptr(heap), hl, _ptr(out), total,
                                    _ptr(offsets), stack_limit, msgs, _ptr(ws), ws.numel(), self.status.ptr, s),
                "xdrg_encode_sized")
        e = self.check(s)
        return EncodeResult(out[:e.total_bytes], offsets)

    def index_records(self, xdr: torch.Tensor, n: int, max_rec_len: int | None = None) -> torch.Tensor:
        """Record index of n records concatenated in `xdr`, on the device
        (xdrg_index_records): int64 offsets[n + 1] for decode.  max_rec_len
        (default: the plan's largest record, at most XDRG_MAX_MSG): records
        longer than the index window (XDRG_INDEX_MAX_MSG) or nested deeper
        than its frames are walked on the device between list-ranking
        windows; with max_rec_len at most the window, such a record raises
        XdrRuntimeError (XDRG_ERR_INDEX_LONG)."""
        if max_rec_len is None:
            max_rec_len = max(min(self.plan.max_record_bytes, A.MAX_MSG), 16)
        L = A.lib()
        total = xdr.numel()
        ws = torch.empty(max(L.xdrg_index_workspace_size(total, max_rec_len), 16), dtype=torch.uint8,
                         device=self.device)
        offs = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        cnt = torch.empty(1, dtype=torch.int64, device=self.device)
        s = _stream()
        self.status.init(s)
        A.check(L.xdrg_index_records(self.plan.handle, _ptr(xdr), total, n, max_rec_len, _ptr(offs),
                                     cnt.data_ptr(), _ptr(ws), ws.numel(), self.status.ptr, s),
                "xdrg_index_records")
        self.check(s)
        return offs

    def decode(self, xdr: torch.Tensor, n: int, offsets: torch.Tensor | None = None,
               stack_limit: int = A.DEFAULT_STACK_LIMIT):
        """= xdr_from_opaque(bytes, r0, ..., rn-1) (marshal.h:299-306).
        Var plans without `offsets` index the records on the device first
        (index_records: records of any length and nesting).  Returns (native
        uint8 tensor [n*stride], heap uint8 tensor or None)."""
        if offsets is None and not self.plan.is_fixed:
            try:
                offsets = self.index_records(xdr, n)
            except XdrRuntimeError as e:
                # a record nested past the window parse's frames, or longer
                # than the plan's bound: the whole-stream walk has neither
                # bound, and the decode reports that record's own error
                if e.code != A.ERR_INDEX_LONG:
                    raise
                offsets = self.index_records(xdr, n, A.MAX_MSG)
        s = _stream()
        native = torch.zeros(max(n, 1) * self.plan.stride, dtype=torch.uint8, device=self.device)
        heap = None
        hsize = 0
        if not self.plan.is_fixed:
            hsize = self.plan.decode_heap_bytes(xdr.numel())
            heap = torch.zeros(max(hsize, 4), dtype=torch.uint8, device=self.device)
        self.status.init(s)
        self.launch_decode(xdr, n, native, offsets=offsets, heap_out=heap,
                           stack_limit=stack_limit, stream=s)
        self.check(s)
        return native[:n * self.plan.stride], (None if heap is None else heap[:hsize])


    # ---- record-marked messages (message_t, RFC 5531) -----------------------
    def message_sizes(self, native, n, stack_limit=A.DEFAULT_STACK_LIMIT, heap=None) -> torch.Tensor:
        """raw_size() of xdr_to_msg(r) per record: 4 + xdr_size(r)."""
        return self.serial_sizes(native, n, stack_limit, heap) + 4

    def encode_msgs(self, native: torch.Tensor, n: int, heap: torch.Tensor | None = None,
                    stack_limit: int = A.DEFAULT_STACK_LIMIT,
                    capacity: int | None = None) -> EncodeResult:
        """Message r = xdr_to_msg(record r) (marshal.h:252-260), back to back:
        a 4-byte mark BE(size | 0x80000000) then the record's bytes.
        offsets[r] = message r's mark, offsets[n] = total."""
        s = _stream()
        offsets = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        if capacity is None:
            if not self.plan.is_fixed:  # one size pass: the output is sized from it
                return self._encode_two_halves(native, n, heap, offsets, stack_limit, msgs=1)
            capacity = n * (self.plan.fixed_size + 4)
        out = torch.empty(max(capacity, 4), dtype=torch.uint8, device=self.device)
        self.status.init(s)
        self.launch_encode_msgs(native, n, out, offsets, heap=heap, stack_limit=stack_limit, stream=s)
        e = self.check(s)
        return EncodeResult(out[:e.total_bytes], offsets)

    def decode_msgs(self, stream_bytes: torch.Tensor, n: int | None = None,
                    offsets: torch.Tensor | None = None, max_msg_len: int | None = None,
                    stack_limit: int = A.DEFAULT_STACK_LIMIT):
        """xdr_from_msg(m_r, r) for every message of the stream
        (marshal.h:278-284).  Without `offsets` the record index comes from
        the marks (index_messages, on the device; the message bound
        defaults to msg_sock's, msgsock.h:29).  Returns (native, heap)."""
        if offsets is None:
            if max_msg_len is None:
                max_msg_len = A.MSG_SOCK_MAXMSGLEN
            offsets = index_messages(stream_bytes, max_msg_len)
        if n is None:
            n = offsets.numel() - 1
        s = _stream()
        native = torch.zeros(max(n, 1) * self.plan.stride, dtype=torch.uint8, device=self.device)
        heap = None  # fixed plans: the decoded records point into no heap
        if not self.plan.is_fixed:
            hsize = self.plan.decode_heap_bytes(stream_bytes.numel())
            heap = torch.zeros(max(hsize, 4), dtype=torch.uint8, device=self.device)[:hsize]
        self.status.init(s)
        self.launch_decode_msgs(stream_bytes, n, native, offsets, heap_out=heap,
                                stack_limit=stack_limit, stream=s)
        self.check(s)
        return native[:n * self.plan.stride], heap


def host_index_records(cp, xdr: np.ndarray, n: int) -> np.ndarray:
    """The record boundaries xdr_from_opaque's walk finds in n records
    concatenated in `xdr` (marshal.h:299-306), walked on the host: lengths,
    counts and discriminants only.  Where the bytes run out, a length or
    count passes its bound, or a discriminant is bad, record k gets [off[k], len) and the rest
    [len, len), so the decode reports the reference's error for record k;
    trailing bytes leave off[n] < len.  The fallback of decode() for the
    streams the device index hands back (include/xdrpp_gpu.hh
    index_records is the C++ layer's); uint64 [n + 1]."""
    ops, table = cp.ops, cp.table
    L = int(xdr.size)
    buf = np.ascontiguousarray(xdr, dtype=np.uint8).tobytes()

    def word(p):
        return int.from_bytes(buf[p:p + 4], "big")

    def elem_wire(e):
        k = int(e["kind"])
        return 8 if k == A.OP_U64 else ((int(e["arg0"]) + 3) & ~3) if k == A.OP_OPAQUE else 4

    def enum_ok(o, v):  # xdr_traits<enum>::valid (the plan's value table)
        if not int(o["flags"]) & A.F_VALIDATE:
            return True
        t = int(o["arg0"])
        return any(int(table[t + i]) == v for i in range(int(o["arg1"])))

    def skip(p):  # one record from p: the end, or None
        stack = []  # [elements left, VECTOR pc]
        pc = 0
        while True:
            o = ops[pc]
            k = int(o["kind"])
            if k == A.OP_END:
                if not stack:
                    return p
                if stack[-1][0]:
                    stack[-1][0] -= 1
                    pc = int(ops[stack[-1][1]]["arg4"])
                    if p > L:
                        return None
                else:
                    pc = stack.pop()[1] + 1
                continue
            if k == A.OP_JUMP:
                pc = int(o["arg0"])
                continue
            if k == A.OP_U64:
                p += 8
            elif k == A.OP_OPAQUE:
                p += (int(o["arg0"]) + 3) & ~3
            elif k in (A.OP_VAROPAQUE, A.OP_STRING):
                if p + 4 > L:
                    return None
                v = word(p)
                if v > int(o["arg0"]):  # past its bound: the chain ends here (rx_len)
                    return None
                p += 4 + ((v + 3) & ~3)
            elif k == A.OP_VECTOR:
                if p + 4 > L:
                    return None
                cnt = word(p)
                if cnt > int(o["arg0"]):
                    return None
                p += 4
                if int(o["flags"]) & A.F_SUB:
                    if cnt:
                        if p > L:
                            return None
                        stack.append([cnt - 1, pc])
                        pc = int(o["arg4"])
                    else:
                        pc += 1
                    continue
                nb = int(o["arg2"])
                p += cnt * sum(elem_wire(ops[pc + j]) for j in range(1, nb + 1))
                pc += 1 + nb
                continue
            elif k == A.OP_UNION:
                if p + 4 > L:
                    return None
                d = word(p)
                p += 4
                if not enum_ok(o, d):
                    return None
                tgt = None
                for c in range(int(o["arg3"])):
                    if int(table[int(o["arg2"]) + 2 * c]) == d:
                        tgt = int(table[int(o["arg2"]) + 2 * c + 1])
                        break
                if tgt is None and int(o["flags"]) & A.F_DEFAULT:
                    tgt = int(o["arg4"])
                if tgt is None:
                    return None
                pc = tgt
                continue
            elif k == A.OP_ENUM:
                if p + 4 > L or not enum_ok(o, word(p)):
                    return None
                p += 4
            else:
                p += 4
            pc += 1

    off = np.full(n + 1, L, dtype=np.uint64)
    p = 0
    for r in range(n):
        off[r] = min(p, L)
        q = skip(p)
        if q is None or q > L:
            return off
        p = q
    off[n] = p
    return off


class _IndexErrorPlan:
    """error_from() needs only the bad-discriminant messages of a plan;
    framing errors have none."""

    class cp:  # noqa: N801
        @staticmethod
        def bad_discriminant_message(op):
            return "bad value of discriminant"


def index_messages(stream_bytes: torch.Tensor, max_msg_len: int = A.MSG_SOCK_MAXMSGLEN,
                   max_msgs: int | None = None) -> torch.Tensor:
    """Record index of a stream of record-marked messages, on the device
    (xdrg_index_msgs): the framing read_message / msg_sock::input apply
    (srpc.cc:29-55, msgsock.cc:38-119), messages up to max_msg_len (msg_sock's
    1 MiB by default; any length up to 2^31 - 1).  Returns int64
    offsets[count + 1] (mark of each message, then the end); raises
    XdrBadMessageSize with the reference's what() on a framing error."""
    dev = stream_bytes.device
    L = A.lib()
    total = stream_bytes.numel()
    if max_msgs is None:
        max_msgs = total // 4
    ws_n = L.xdrg_index_workspace_size(total, max_msg_len)
    ws = torch.empty(max(ws_n, 16), dtype=torch.uint8, device=dev)
    offs = torch.empty(max_msgs + 1, dtype=torch.int64, device=dev)
    cnt = torch.empty(1, dtype=torch.int64, device=dev)
    st = Status(dev)
    s = _stream()
    st.init(s)
    A.check(L.xdrg_index_msgs(_ptr(stream_bytes), total, max_msg_len, max_msgs, _ptr(offs),
                              cnt.data_ptr(), _ptr(ws), ws.numel(), st.ptr, s), "xdrg_index_msgs")
    e = st.read(s)
    err = error_from(_IndexErrorPlan, e)
    if err is not None:
        raise err
    return offs[:int(cnt.item()) + 1]


def to_msg_batch(plan: Plan, native: torch.Tensor, n: int, heap: torch.Tensor | None = None,
                 **kw) -> EncodeResult:
    """xdr_to_msg of every record, messages back to back (marshal.h:252-260)."""
    return Marshaler(plan, native.device).encode_msgs(native, n, heap, **kw)


def from_msg_batch(plan: Plan, stream_bytes: torch.Tensor, n: int | None = None,
                   offsets: torch.Tensor | None = None, **kw):
    """xdr_from_msg of every message of the stream (marshal.h:278-284)."""
    return Marshaler(plan, stream_bytes.device).decode_msgs(stream_bytes, n, offsets, **kw)


def to_opaque_batch(plan: Plan, native: torch.Tensor, n: int, heap: torch.Tensor | None = None,
                    **kw) -> EncodeResult:
    return Marshaler(plan, native.device).encode(native, n, heap, **kw)


def from_opaque_batch(plan: Plan, xdr: torch.Tensor, n: int, offsets: torch.Tensor | None = None,
                      **kw):
    return Marshaler(plan, xdr.device).decode(xdr, n, offsets, **kw)


def swap32(x: torch.Tensor) -> torch.Tensor:
    """Device swap32 over an int32 tensor (xdrpp/endian.h:56-60)."""
    out = torch.empty_like(x)
    A.check(A.lib().xdrg_swap32(_ptr(x), _ptr(out), x.numel(), _stream()), "xdrg_swap32")
    return out


def swap64(x: torch.Tensor) -> torch.Tensor:
    """Device swap64 over an int64 tensor (xdrpp/endian.h:62-68)."""
    out = torch.empty_like(x)
    A.check(A.lib().xdrg_swap64(_ptr(x), _ptr(out), x.numel(), _stream()), "xdrg_swap64")
    return out
