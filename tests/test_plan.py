"""CPU: host-side plan logic through the C ABI (plan compile, validation,
path selection, workspace sizing, error strings).  Plan creation is
host-only (device tables are uploaded by a plan's first launch), so none of
this needs a GPU."""
import ctypes as C

import numpy as np
import pytest

from xdrpp_amd import _abi as A
from xdrpp_amd import marshal as M
from xdrpp_amd import schemas as S
from xdrpp_amd import xdr_types as T


def create(ops: np.ndarray, table: np.ndarray | None, stride: int) -> tuple[int, C.c_void_p]:
    L = A.lib()
    h = C.c_void_p()
    tab = None if table is None or table.size == 0 else table.ctypes.data_as(C.POINTER(C.c_uint32))
    rc = L.xdrg_plan_create(ops.ctypes.data_as(C.POINTER(A.XdrgOp)), len(ops), tab,
                            0 if tab is None else table.size, stride, C.byref(h))
    return rc, h


def ops_of(*rows) -> np.ndarray:
    a = np.zeros(len(rows), dtype=T.OP_DTYPE)
    for i, r in enumerate(rows):
        d = dict(kind=0, flags=0, depth=1, noff=0, arg0=0, arg1=0, arg2=0, arg3=0, arg4=0, name=0)
        d.update(r)
        a[i] = tuple(d[k] for k in T.OP_DTYPE.names)
    return a


END = dict(kind=A.OP_END, depth=0)


# ------------------------------------------------------------- schemas
@pytest.mark.parametrize("name,path,fixed,stride,depth", [
    ("numerics", A.PATH_FIXED_LDS, 44, 56, 1),
    ("rec128", A.PATH_FIXED_REG, 128, 128, 1),
    ("recvar", A.PATH_VAR, None, 56, 1),
    ("rpc", A.PATH_VAR, None, 80, 6),
])
def test_plan_info(name, path, fixed, stride, depth):
    p = M.Plan(S.ALL[name])
    assert (p.path, p.fixed_size, p.stride, p.max_depth) == (path, fixed, stride, depth)
    assert p.is_fixed == (fixed is not None)
    info = A.XdrgPlanInfo()
    assert A.lib().xdrg_plan_get_info(p.handle, C.byref(info)) == 0
    assert info.nops == len(p.cp.ops)
    # var plans validate on decode (bounds, pads, discriminants)
    assert bool(info.has_checks) == (fixed is None)


def test_validated_enum_plan_has_checks():
    assert M.Plan(S.numerics_validated).has_checks
    assert not M.Plan(S.numerics).has_checks


def test_workspace_size():
    fixed = M.Plan(S.rec128)
    # fixed plans: encode needs none, encode_msgs (interpreter path) does
    assert fixed.workspace_bytes(1 << 20) >= 4 * (1 << 20)
    var = M.Plan(S.recvar)
    w = [var.workspace_bytes(n) for n in (1, 1000, 1 << 20, 1 << 24)]
    assert all(x > 0 for x in w) and w == sorted(w)
    assert w[2] >= 4 * (1 << 20)  # at least one u32 size per record


def test_c_layout_of_schemas():
    """Python layouts follow the C ABI of the xdrc structs (natural
    alignment); the staged layouts are pinned byte-for-byte against the
    reference generator by tests/test_oracle.py."""
    assert S.rec128.size == 128
    o = S.recvar.offsets
    assert o["id"] == 0 and o["kind"] == 8 and o["blob"] == 16 and o["name"] == 32 and o["score"] == 48
    st = T.Struct("s", [("b", T.Bool), ("h", T.Hyper), ("i", T.Int)])
    assert st.offsets == {"b": 0, "h": 8, "i": 16} and st.size == 24


def test_union_messages_follow_the_reference():
    """bad value of <tag> in <union> (xdrc/gen_hh.cc union save/load)."""
    cp = T.compile_plan(S.rpc_msg)
    msgs = set(cp.messages.values())
    assert {"bad value of mtype in _body_t", "bad value of stat in reply_body",
            "bad value of stat in rejected_reply"} <= msgs


# ----------------------------------------------------------- validation
def test_valid_minimal_plan():
    rc, h = create(ops_of(dict(kind=A.OP_U32), END), None, 4)
    assert rc == 0
    A.lib().xdrg_plan_destroy(h)


@pytest.mark.parametrize("label,ops,table,stride,want", [
    ("no ops", [], None, 4, -1),
    ("no END", [dict(kind=A.OP_U32)], None, 4, -1),
    ("bad kind", [dict(kind=77), END], None, 4, -1),
    ("field past stride", [dict(kind=A.OP_U64, noff=4), END], None, 8, -1),
    ("misaligned u32", [dict(kind=A.OP_U32, noff=2), END], None, 8, -1),
    ("backward jump", [dict(kind=A.OP_U32), dict(kind=A.OP_JUMP, arg0=0), END], None, 4, -1),
    ("jump past end", [dict(kind=A.OP_U32), dict(kind=A.OP_JUMP, arg0=9), END], None, 4, -1),
    ("enum table out of range", [dict(kind=A.OP_ENUM, flags=A.F_VALIDATE, arg0=0, arg1=4), END],
     np.array([1, 2], dtype=np.uint32), 4, -1),
    ("union case out of range", [dict(kind=A.OP_UNION, arg0=0, arg1=0, arg2=0, arg3=2), END],
     np.array([0, 1], dtype=np.uint32), 4, -1),
    ("union target backwards", [dict(kind=A.OP_UNION, arg0=0, arg1=0, arg2=0, arg3=1), END],
     np.array([0, 0], dtype=np.uint32), 4, -1),
    ("stride not multiple of 4", [dict(kind=A.OP_BOOL), END], None, 2, -3),
])
def test_invalid_plans_rejected(label, ops, table, stride, want):
    rc, h = create(ops_of(*ops) if ops else np.zeros(1, dtype=T.OP_DTYPE)[:0], table, stride)
    assert rc == want, label
    assert not h.value


def test_unvalidated_enum_does_not_read_the_table():
    """Without F_VALIDATE the enum value list is never read (the reference
    validates enums only on request, types.h:157-173), so it is not bounds-checked."""
    rc, h = create(ops_of(dict(kind=A.OP_ENUM, arg0=0, arg1=4), END), None, 4)
    assert rc == 0
    A.lib().xdrg_plan_destroy(h)


def test_null_arguments():
    L = A.lib()
    h = C.c_void_p()
    assert L.xdrg_plan_create(None, 1, None, 0, 4, C.byref(h)) == -1
    assert L.xdrg_plan_get_info(None, None) == -1
    L.xdrg_plan_destroy(None)  # no-op


# --------------------------------------------------------- error strings
REFERENCE_WHAT = {  # xdrpp what() strings, by data error code
    A.ERR_OVERFLOW_GET: "insufficient buffer space in xdr_generic_get",  # marshal.h:160-170
    A.ERR_OVERFLOW_PUT: "insufficient buffer space in xdr_generic_put",  # marshal.h:104-108
    A.ERR_XVECTOR_BOUND: "xvector overflow",                              # types.h:515-524
    A.ERR_XSTRING_BOUND: "xstring overflow",                              # types.h:530-587
    A.ERR_NONZERO_PAD: "Non-zero padding bytes encountered",              # marshal.cc:43-57
    A.ERR_INVALID_ENUM: "Invalid enum value",                             # types.h:157-173
    A.ERR_STACK_PUT: "stack overflow in xdr_generic_put",                 # marshal.h:131-136
    A.ERR_STACK_GET: "stack overflow in xdr_generic_get",                 # marshal.h:198-205
    A.ERR_SIZE_NOT_MULT4: "xdr_generic_get: message size not multiple of 4",  # marshal.h:155-160
    A.ERR_TRAILING: "unmarshaling did not consume whole message",         # marshal.h:207-210
}
REFERENCE_CLASS = {
    A.ERR_OVERFLOW_GET: M.XdrOverflow, A.ERR_OVERFLOW_PUT: M.XdrOverflow,
    A.ERR_XVECTOR_BOUND: M.XdrOverflow, A.ERR_XSTRING_BOUND: M.XdrOverflow,
    A.ERR_NONZERO_PAD: M.XdrShouldBeZero, A.ERR_BAD_DISCRIMINANT: M.XdrBadDiscriminant,
    A.ERR_INVALID_ENUM: M.XdrInvariantFailed, A.ERR_STACK_PUT: M.XdrStackOverflow,
    A.ERR_STACK_GET: M.XdrStackOverflow, A.ERR_SIZE_NOT_MULT4: M.XdrBadMessageSize,
    A.ERR_TRAILING: M.XdrBadMessageSize,
}


@pytest.mark.parametrize("code", sorted(REFERENCE_CLASS))
def test_error_mapping(code):
    plan = M.Plan(S.rpc_msg)
    e = A.XdrgError(code=code, exc=0, record=7, op=0xFFFFFFFF, rsv=0, total_bytes=0)
    exc = M.error_from(plan, e)
    assert type(exc) is REFERENCE_CLASS[code]
    assert isinstance(exc, M.XdrRuntimeError) and exc.record == 7 and exc.op is None
    if code in REFERENCE_WHAT:
        assert str(exc) == REFERENCE_WHAT[code]


def test_bad_discriminant_message_names_the_union():
    plan = M.Plan(S.rpc_msg)
    union_ops = [i for i, o in enumerate(plan.cp.ops) if o["kind"] == A.OP_UNION]
    assert union_ops
    e = A.XdrgError(code=A.ERR_BAD_DISCRIMINANT, exc=0, record=3, op=union_ops[0], rsv=0,
                    total_bytes=0)
    exc = M.error_from(plan, e)
    assert str(exc) == "bad value of mtype in _body_t" and exc.op == union_ops[0]


def test_no_error():
    plan = M.Plan(S.rec128)
    assert M.error_from(plan, A.XdrgError()) is None
