"""RPC header batches on MI355X through the C ABI.

Host-side mirror of the reference's RPC message handling, batched:

    rpc_server_base::dispatch (xdrpp/server.cc:78-117)
    + srpc_service::process proc switch (srpc.h:121-128)   -> dispatch()
    check_call_hdr (rpc_msg.cc:115-131) + xid test
      of synchronous_client_base::invoke (srpc.h:61-66)     -> check_replies()
    rpc_accepted_error_msg / rpc_prog_mismatch_msg /
      rpc_auth_error_msg / rpc_rpc_mismatch_msg (server.cc:8-67)
                                                            -> error_replies()
    xdr_to_msg(rpc_success_hdr(xid), res) (srpc.h:152)      -> success_reply_type()
                                                               + Marshaler.encode_msgs

Each header decodes to one 64-byte xdrg_rpc_hdr (HDR_DTYPE below).  The
exceptions a client raises for a reply (xdr_call_error with the
rpc_call_stat message, exception.h:25-57, rpc_msg.cc:8-109) come from
raise_for_reply().  Every byte is produced by the HIP kernels of
libxdrgpu.so (xdrpp_amd/csrc/rpc.hip).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _abi as A
from .marshal import Status, XdrRuntimeError, _EXC, _ptr, _stream
from .xdr_types import Struct, UInt, XdrType

HDR_DTYPE = np.dtype([("xid", "<u4"), ("action", "<u2"), ("err", "u1"), ("mtype", "u1"),
                      ("w", "<u4", (8,)), ("cred_len", "<u4"), ("verf_len", "<u4"),
                      ("body_off", "<u8"), ("end", "<u8")])
assert HDR_DTYPE.itemsize == A.RPC_HDR_BYTES
PROC_DTYPE = np.dtype([("prog", "<u4"), ("vers", "<u4"), ("proc", "<u4"), ("flags", "<u4")])

# ------------------------------------------------------------ call errors
# rpc_errmsg(accept_stat) / rpc_errmsg(auth_stat), xdrpp/rpc_msg.cc:8-64
_ACCEPT_MSG = {0: "RPC executed successfully", 1: "remote hasn't exported program",
               2: "remote can't support version #", 3: "program can't support procedure",
               4: "procedure can't decode params", 5: "RPC system error"}
_AUTH_MSG = {0: "success", 1: "bad credential (seal broken)", 2: "client must begin new session",
             3: "bad verifier (seal broken)", 4: "verifier expired or replayed",
             5: "rejected for security reasons", 6: "bogus response verifier",
             7: "reason unknown", 8: "kerberos generic error", 9: "time of credential expired",
             10: "problem with ticket file", 11: "can't decode authenticator",
             12: "wrong net address in ticket", 13: "no credentials for user",
             14: "problem with context"}


def rpc_errmsg_accept(stat: int) -> str:
    return _ACCEPT_MSG.get(int(stat), "unknown accept_stat error")


def rpc_errmsg_auth(stat: int) -> str:
    return _AUTH_MSG.get(int(stat), "auth_stat error")


class XdrCallError(XdrRuntimeError):
    """xdr_call_error (xdrpp/exception.h:53-57): the server refused the call.
    ``kind`` is the rpc_call_stat type ("accept", "auth", "rpcvers")."""

    def __init__(self, what: str, kind: str, stat: int | None, record: int | None = None):
        super().__init__(what, record)
        self.kind, self.stat = kind, stat


def raise_for_reply(h, record: int | None = None) -> None:
    """What synchronous_client_base::invoke raises for a reply header
    (srpc.h:61-66; check_call_hdr, rpc_msg.cc:115-131); returns for OK."""
    a = int(h["action"])
    if a == A.RPCR_OK:
        return
    if a == A.RPCR_ACCEPT_STAT:
        s = int(h["w"][A.RPC_W_STAT])
        raise XdrCallError(rpc_errmsg_accept(s), "accept", s, record)
    if a == A.RPCR_AUTH_STAT:
        s = int(h["w"][A.RPC_W_WHY])
        raise XdrCallError(rpc_errmsg_auth(s), "auth", s, record)
    if a == A.RPCR_RPCVERS_MISMATCH:  # rpc_call_stat::message, rpc_msg.cc:90-91
        raise XdrCallError("server reported rpcvers field with wrong value", "rpcvers", None, record)
    if a == A.RPCR_NOT_REPLY:
        raise XdrRuntimeError("call received when reply expected", record)
    if a == A.RPCR_BAD_XID:
        raise XdrRuntimeError("synchronous_client: unexpected xid", record)
    code = int(h["err"])
    what = A.lib().xdrg_error_message(code).decode()
    if code == A.ERR_BAD_DISCRIMINANT:  # xdrc's union names (gen_hh.cc:479-481)
        what = ("bad value of mtype in _body_t", "bad value of stat in reply_body",
                "bad value of stat in rejected_reply")[int(h["w"][0])]
    raise _EXC.get(A.lib().xdrg_error_exception(code), XdrRuntimeError)(what, record, None, code)


# --------------------------------------------------------------- registry
def proc_table(services: dict[int, dict[int, list[int]]]) -> np.ndarray:
    """The sorted (prog, vers, proc, flags) table xdrg_rpc_dispatch takes,
    from {prog: {vers: [proc, ...]}} (rpc_server_base::servers_,
    server.h:218-219; an empty proc list registers the interface only)."""
    rows = []
    for prog, vs in services.items():
        for vers, procs in vs.items():
            if procs:
                rows += [(prog, vers, p, 0) for p in sorted(set(procs))]
            else:
                rows.append((prog, vers, 0, A.RPC_PROC_IFACE_ONLY))
    t = np.array(sorted(rows), dtype=np.uint32).reshape(-1, 4)
    if len(t) > A.RPC_MAX_PROCS:
        raise ValueError(f"at most {A.RPC_MAX_PROCS} registered procedures")
    return t


def _check_table(t: np.ndarray) -> None:
    t = np.asarray(t, dtype=np.uint32).reshape(-1, 4)
    keys = [tuple(r[:3]) for r in t]
    if keys != sorted(keys) or len(set(keys)) != len(keys):
        raise ValueError("procedure table must be sorted by (prog, vers, proc) with no duplicates")


# ---------------------------------------------------------------- batches
def hdrs_numpy(hdrs: torch.Tensor) -> np.ndarray:
    """Device xdrg_rpc_hdr array -> numpy structured array (copies)."""
    return hdrs.cpu().numpy().view(HDR_DTYPE).reshape(-1)


def dispatch(stream_bytes: torch.Tensor, offsets: torch.Tensor, procs) -> torch.Tensor:
    """Decode and route every message's rpc_msg header (xdrg_rpc_dispatch).
    offsets: int64 [n+1] message marks (index_messages).  procs: the
    registered procedure table (proc_table()), numpy or a device tensor.
    Returns a uint8 device tensor of n * 64 bytes (xdrg_rpc_hdr records)."""
    dev = stream_bytes.device
    if isinstance(procs, np.ndarray):
        _check_table(procs)
        procs = torch.from_numpy(np.ascontiguousarray(procs, dtype=np.uint32).view(np.int32)).to(dev)
    n = offsets.numel() - 1
    out = torch.empty(max(n, 1) * A.RPC_HDR_BYTES, dtype=torch.uint8, device=dev)
    A.check(A.lib().xdrg_rpc_dispatch(_ptr(stream_bytes), stream_bytes.numel(), _ptr(offsets), n,
                                      _ptr(procs), procs.numel() // 4, _ptr(out), _stream()),
            "xdrg_rpc_dispatch")
    return out[:n * A.RPC_HDR_BYTES]


def check_replies(stream_bytes: torch.Tensor, offsets: torch.Tensor,
                  xids: torch.Tensor | None = None) -> torch.Tensor:
    """Decode every reply header and classify it as the client does
    (xdrg_rpc_check_replies); xids: int32 [n] expected xids or None."""
    dev = stream_bytes.device
    n = offsets.numel() - 1
    out = torch.empty(max(n, 1) * A.RPC_HDR_BYTES, dtype=torch.uint8, device=dev)
    A.check(A.lib().xdrg_rpc_check_replies(_ptr(stream_bytes), stream_bytes.numel(), _ptr(offsets),
                                           n, _ptr(xids), _ptr(out), _stream()),
            "xdrg_rpc_check_replies")
    return out[:n * A.RPC_HDR_BYTES]


class ReplyWriter:
    """Reusable xdrg_rpc_replies launcher (owns status + workspace)."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.status = Status(self.device)
        self._ws = torch.empty(0, dtype=torch.uint8, device=self.device)

    def launch(self, hdrs: torch.Tensor, out: torch.Tensor, offsets: torch.Tensor, stream=None):
        n = hdrs.numel() // A.RPC_HDR_BYTES
        need = A.lib().xdrg_rpc_replies_workspace_size(n)
        if self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        s = _stream() if stream is None else stream
        A.check(A.lib().xdrg_rpc_replies(_ptr(hdrs), n, _ptr(out), out.numel(), _ptr(offsets),
                                         _ptr(self._ws), self._ws.numel(), self.status.ptr, s),
                "xdrg_rpc_replies")

    def __call__(self, hdrs: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        n = hdrs.numel() // A.RPC_HDR_BYTES
        out = torch.empty(max(36 * n, 4), dtype=torch.uint8, device=self.device)
        offs = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        s = _stream()
        self.status.init(s)
        self.launch(hdrs, out, offs, s)
        e = self.status.read(s)
        if e.code:
            raise XdrRuntimeError(A.lib().xdrg_error_message(e.code).decode(), int(e.record),
                                  None, int(e.code))
        return out[:int(e.total_bytes)], offs


def error_replies(hdrs: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """The error replies of a dispatched batch as record-marked messages in
    message order (server.cc:8-67); returns (stream, offsets[n+1]) where
    header i's reply is stream[offsets[i]:offsets[i+1]] (empty if none)."""
    return ReplyWriter(hdrs.device)(hdrs)


def success_reply_type(res: XdrType, name: str = "rpc_success_reply") -> Struct:
    """The record xdr_to_msg(rpc_success_hdr(xid), res) marshals
    (server.h:27-49 + the argument pack of marshal.h:252-260): xid, REPLY,
    MSG_ACCEPTED, AUTH_NONE, an empty verf body, SUCCESS, then res.  The
    constant words are staged fields (mtype=1, the rest 0)."""
    return Struct(name, [("xid", UInt), ("mtype", UInt), ("stat", UInt), ("flavor", UInt),
                         ("body", UInt), ("accept", UInt), ("res", res)])
