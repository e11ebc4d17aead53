"""The benchmark schemas, written with the xdrc-mirror descriptors.

  numerics  tests/xdrtest.x:98-107 (44 wire bytes, 56-byte C++ struct)
  rec128    SURVEY.md §8: int a0..a7; unsigned hyper u0..u5; double d0..d5
            (128 wire bytes = 128-byte C++ struct, identity layout)
  recvar    SURVEY.md §8(d) config 3: unsigned hyper id; int kind;
            opaque blob<256>; string name<64>; double score
  rpc_msg   xdrpp/rpc_msg.x:5-140 (nested discriminated unions)
  containers of variable-size elements and a recursive type, from
  tests/xdrtest.x: containertest, containertest1 (:129-137), hasbytes
  (:94-96), test_recursive (:29-33), nested_cereal_adapter_calls (:172-176)
  rp__list  xdrpp/rpcb_prot.x:24-37, a linked list of rpcb entries

The union/type names match what xdrc generates, so bad-discriminant
messages equal the reference's ("bad value of mtype in _body_t", ...).
"""
from __future__ import annotations

from .xdr_types import (Bool, Double, Enum, Float, Hyper, Int, Opaque, OpaqueArray, Pointer, String,
                        Struct, UHyper, UInt, Union, Void, XArray, XVector)

# ------------------------------------------------------------- numerics
_COLOR_TAGS = {"RED": 0, "REDDER": 1, "REDDEST": 2}
other_color = Enum("other_color", _COLOR_TAGS)


def _numerics(color: Enum) -> Struct:
    return Struct("numerics", [
        ("b", Bool), ("i1", Int), ("i2", UInt), ("i3", Hyper), ("i4", UHyper),
        ("f1", Float), ("f2", Double), ("e1", color),
    ])


numerics = _numerics(other_color)
# tests/validate.cc:18-20: namespace-wide xdr_validate_enum opt-in
numerics_validated = _numerics(Enum("other_color", _COLOR_TAGS, validate=True))

# --------------------------------------------------------------- rec128
rec128 = Struct("rec128", [(f"a{i}", Int) for i in range(8)]
                + [(f"u{i}", UHyper) for i in range(6)]
                + [(f"d{i}", Double) for i in range(6)])

# --------------------------------------------------------------- recvar
recvar = Struct("recvar", [
    ("id", UHyper), ("kind", Int), ("blob", Opaque(256)), ("name", String(64)), ("score", Double),
])

# -------------------------------------------------------------- rpc_msg
auth_flavor = Enum("auth_flavor", {"AUTH_NONE": 0, "AUTH_SYS": 1, "AUTH_SHORT": 2,
                                   "AUTH_DH": 3, "RPCSEC_GSS": 6})
msg_type = Enum("msg_type", {"CALL": 0, "REPLY": 1})
reply_stat = Enum("reply_stat", {"MSG_ACCEPTED": 0, "MSG_DENIED": 1})
accept_stat = Enum("accept_stat", {"SUCCESS": 0, "PROG_UNAVAIL": 1, "PROG_MISMATCH": 2,
                                   "PROC_UNAVAIL": 3, "GARBAGE_ARGS": 4, "SYSTEM_ERR": 5})
reject_stat = Enum("reject_stat", {"RPC_MISMATCH": 0, "AUTH_ERROR": 1})
auth_stat = Enum("auth_stat", {f"S{i}": i for i in range(15)})

opaque_auth = Struct("opaque_auth", [("flavor", auth_flavor), ("body", Opaque(400))])
call_body = Struct("call_body", [
    ("rpcvers", UInt), ("prog", UInt), ("vers", UInt), ("proc", UInt),
    ("cred", opaque_auth), ("verf", opaque_auth),
])
mismatch_info = Struct("mismatch_info", [("low", UInt), ("high", UInt)])
reply_data = Union("_reply_data_t", "stat", accept_stat, [
    ([0], "results", OpaqueArray(0)),        # SUCCESS
    ([2], "mismatch_info", mismatch_info),   # PROG_MISMATCH
], default=("", Void))
accepted_reply = Struct("accepted_reply", [("verf", opaque_auth), ("reply_data", reply_data)])
rejected_reply = Union("rejected_reply", "stat", reject_stat, [
    ([0], "mismatch_info", mismatch_info),   # RPC_MISMATCH
    ([1], "rj_why", auth_stat),              # AUTH_ERROR
])
reply_body = Union("reply_body", "stat", reply_stat, [
    ([0], "areply", accepted_reply),
    ([1], "rreply", rejected_reply),
])
rpc_body = Union("_body_t", "mtype", msg_type, [
    ([0], "cbody", call_body),
    ([1], "rbody", reply_body),
])
rpc_msg = Struct("rpc_msg", [("xid", UInt), ("body", rpc_body)])

# --------------------------------------------------------------- vecrec
# Counted and optional containers of fixed-size elements (xvector<T>,
# pointer<T>; xdrpp/types.h:365-414, 476-512, 591-665):
#   struct vpair { hyper h; bool b; };
#   struct vecrec { unsigned id; int vals<16>; mismatch_info *opt;
#                   vpair pairs<8>; bool flag; };
vpair = Struct("vpair", [("h", Hyper), ("b", Bool)])
vecrec = Struct("vecrec", [("id", UInt), ("vals", XVector(Int, 16)), ("opt", Pointer(mismatch_info)),
                           ("pairs", XVector(vpair, 8)), ("flag", Bool)])

# --------------------------------------- tests/xdrtest.x: element subroutines
fix_4 = Struct("fix_4", [("i", Int)])
fix_12 = Struct("fix_12", [("i", Int), ("d", Double)])
u_4_12 = Union("u_4_12", "which", Int, [([4], "f4", fix_4), ([12], "f12", fix_12)])
containertest = Struct("containertest", [("uvec", XVector(u_4_12)), ("sarr", XArray(String(), 2))])
containertest1 = Struct("containertest1", [("uvec", XVector(u_4_12, 2)), ("sarr", XArray(String(), 2))])
xbytes = Struct("bytes", [("s", String(16)), ("fixed", OpaqueArray(16)), ("variable", Opaque(16))])
hasbytes = Struct("hasbytes", [("the_bytes", XVector(xbytes))])
test_recursive = Struct("test_recursive")
test_recursive.define([("elem", String()), ("next", Pointer(test_recursive)),
                       ("nextvec", XVector(test_recursive))])
string32 = String(32)  # typedef string string32<32>: one element subroutine for both containers
nested_cereal_adapter_calls = Struct("nested_cereal_adapter_calls", [
    ("strptr", Pointer(string32)), ("strvec", XVector(string32)), ("strarr", XArray(string32, 2))])
CONTAINERS = {"containertest": containertest, "containertest1": containertest1, "hasbytes": hasbytes,
              "test_recursive": test_recursive, "nested_cereal_adapter_calls": nested_cereal_adapter_calls}

# ------------------------------------------ xdrpp/rpcb_prot.x: linked lists
# The RPCBPROC_DUMP reply list (rpcb_prot.x:24-37): nested one pointer per
# entry, as deep as the list is long.
rpcb = Struct("rpcb", [("r_prog", UInt), ("r_vers", UInt), ("r_netid", String()), ("r_addr", String()),
                       ("r_owner", String())])
rp__list = Struct("rp__list")
rp__list.define([("rpcb_map", rpcb), ("rpcb_next", Pointer(rp__list))])

ALL = {"numerics": numerics, "rec128": rec128, "recvar": recvar, "rpc": rpc_msg, "vecrec": vecrec,
       "containertest": containertest, "rp_list": rp__list}
