"""XDR type descriptors mirroring the types xdrc emits (xdrpp/types.h).

Each descriptor knows
  * its *staged native layout* (size / alignment), which for fixed-size
    types is exactly the C++ struct layout xdrc generates (natural
    alignment, bool = 1 byte), and for variable-length bytes is an
    xdrg_bytes_ref {u64 off; u32 len; u32 rsv} into a heap;
  * how to append itself to a flat plan: the wire-ordered walk that
    xdr_traits<T>::save performs (xdrc/gen_hh.cc:233-243 structs,
    :649-660 unions; xdrpp/types.h:374-379 containers).

| descriptor        | reference type                         | file:line              |
|-------------------|----------------------------------------|------------------------|
| Int / UInt        | int32_t / uint32_t                     | types.h:310-317        |
| Hyper / UHyper    | int64_t / uint64_t                     | types.h:318-321        |
| Float / Double    | float / double (bit patterns)          | types.h:323-345        |
| Bool              | bool (decode: nonzero -> true)         | types.h:335-349        |
| Enum              | xdrc enum (int32), opt-in validation   | gen_hh.cc:271-305, types.h:157-173 |
| OpaqueArray(n)    | opaque_array<N>  (opaque x[N])         | types.h:455-470        |
| Opaque(max)       | opaque_vec<N>    (opaque x<N>)         | types.h:515-524        |
| String(max)       | xstring<N>       (string x<N>)         | types.h:530-587        |
| XArray(t, n)      | xarray<T,N>      (T x[N])              | types.h:424-452        |
| XVector(t, max)   | xvector<T,N>     (T x<N>)              | types.h:365-414,476-512|
| Pointer(t)        | pointer<T>       (T *x)                | types.h:591-665        |
| Struct            | xdrc struct + xdr_struct_base          | types.h:676-730, gen_hh.cc:212-250 |
| Union             | xdrc union                             | gen_hh.cc:368-675      |

Containers of fixed-size elements put the element's ops inline after the
VECTOR op; containers of any other element type (strings, structs with
bytes fields, unions, containers, the enclosing type itself) give the
element a subroutine (XDRG_F_SUB): its ops follow the record's END, emitted
once per element type.  A recursive type is declared first and given its
fields afterwards (``Struct(name)`` then ``.define(fields)``), as the
reference's test_recursive (tests/xdrtest.x:29-33) refers to itself.
"""
from __future__ import annotations

import numpy as np

from . import _abi as A

__all__ = [
    "XdrType", "Int", "UInt", "Hyper", "UHyper", "Float", "Double", "Bool", "Enum",
    "OpaqueArray", "Opaque", "String", "XArray", "XVector", "Pointer", "Struct", "Union", "Void",
    "CompiledPlan",
    "compile_plan", "OP_DTYPE",
]

OP_DTYPE = np.dtype([
    ("kind", "u1"), ("flags", "u1"), ("depth", "<u2"), ("noff", "<u4"), ("arg0", "<u4"),
    ("arg1", "<u4"), ("arg2", "<u4"), ("arg3", "<u4"), ("arg4", "<u4"), ("name", "<u4"),
])
assert OP_DTYPE.itemsize == 32


def _align_up(x: int, a: int) -> int:
    return (x + a - 1) // a * a


class _Ctx:
    """Plan under construction."""

    def __init__(self) -> None:
        self.ops: list[list[int]] = []  # [kind, flags, depth, noff, a0..a4, name]
        self.table: list[int] = []
        self.names: list[str] = []      # name id -> dotted field path
        self.messages: dict[int, str] = {}  # op index -> bad-discriminant what()
        self.subs: dict[int, list] = {}     # id(element type) -> [type, path, entry pc, VECTOR ops]
        self.pending: list[int] = []        # element types whose bodies are still to emit

    def sub(self, t: "XdrType", path: str, vec_op: int) -> None:
        """VECTOR op `vec_op` walks elements of `t` through t's subroutine."""
        e = self.subs.get(id(t))
        if e is None:
            e = self.subs[id(t)] = [t, path, None, []]
            self.pending.append(id(t))
        e[3].append(vec_op)

    def emit_subs(self) -> None:
        """Element subroutines after the record's END, each ending with END;
        a body may enter further (or its own) subroutines."""
        while self.pending:
            e = self.subs[self.pending.pop(0)]
            t, path = e[0], e[1]
            e[2] = len(self.ops)
            t.emit(self, 0, 0, path)  # element-relative offsets and depths
            self.emit(A.OP_END, 0, 0, "<end>")
        for t, _, entry, vecs in self.subs.values():
            for v in vecs:
                self.ops[v][8] = entry  # arg4

    def name(self, path: str) -> int:
        self.names.append(path)
        return len(self.names) - 1

    def emit(self, kind, noff, depth, path, flags=0, a0=0, a1=0, a2=0, a3=0, a4=0) -> int:
        self.ops.append([kind, flags, depth, noff, a0, a1, a2, a3, a4, self.name(path)])
        return len(self.ops) - 1

    def add_table(self, values) -> int:
        idx = len(self.table)
        self.table.extend(int(v) & 0xFFFFFFFF for v in values)
        return idx


class XdrType:
    size: int = 0
    align: int = 1
    fixed_wire: int | None = None  # xdr_traits<T>::fixed_size, None if variable
    is_class = False               # counts one stack level (struct/union)

    def emit(self, ctx: _Ctx, noff: int, depth: int, path: str) -> None:
        raise NotImplementedError


class _Scalar(XdrType):
    def __init__(self, name, kind, size, wire):
        self.name, self.kind, self.size, self.align, self.fixed_wire = name, kind, size, size, wire

    def emit(self, ctx, noff, depth, path):
        ctx.emit(self.kind, noff, depth, path)

    def __repr__(self):
        return self.name


Int = _Scalar("int", A.OP_U32, 4, 4)
UInt = _Scalar("unsigned", A.OP_U32, 4, 4)
Float = _Scalar("float", A.OP_U32, 4, 4)
Hyper = _Scalar("hyper", A.OP_U64, 8, 8)
UHyper = _Scalar("unsigned hyper", A.OP_U64, 8, 8)
Double = _Scalar("double", A.OP_U64, 8, 8)
Bool = _Scalar("bool", A.OP_BOOL, 1, 4)


class Enum(XdrType):
    """xdrc enum: an int32 on the wire.  ``validate=True`` mirrors declaring
    xdr_validate_enum for it (types.h:157-173): decode rejects values that
    are not tags with xdr_invariant_failed("Invalid enum value")."""

    size = align = 4
    fixed_wire = 4

    def __init__(self, name: str, tags: dict, validate: bool = False):
        self.name, self.tags, self.validate = name, dict(tags), validate

    def emit(self, ctx, noff, depth, path):
        if self.validate:
            vals = sorted(set(self.tags.values()))
            ctx.emit(A.OP_ENUM, noff, depth, path, A.F_VALIDATE, ctx.add_table(vals), len(vals))
        else:
            ctx.emit(A.OP_ENUM, noff, depth, path)

    def __repr__(self):
        return f"enum {self.name}"


class OpaqueArray(XdrType):
    """opaque x[N]: N bytes, padded to 4 on the wire, no length word."""

    def __init__(self, n: int):
        self.n, self.size, self.align = n, n, 1
        self.fixed_wire = (n + 3) & ~3

    def emit(self, ctx, noff, depth, path):
        ctx.emit(A.OP_OPAQUE, noff, depth, path, 0, self.n)


class _VarBytes(XdrType):
    size, align = 16, 8  # xdrg_bytes_ref
    fixed_wire = None
    kind = A.OP_VAROPAQUE

    def __init__(self, max_len: int = A.XDR_MAX_LEN):
        self.max_len = max_len

    def emit(self, ctx, noff, depth, path):
        ctx.emit(self.kind, noff, depth, path, 0, self.max_len)


class Opaque(_VarBytes):
    """opaque x<N> (opaque_vec<N>)."""
    kind = A.OP_VAROPAQUE


class String(_VarBytes):
    """string x<N> (xstring<N>)."""
    kind = A.OP_STRING


class XArray(XdrType):
    """T x[N] for non-byte T (xarray<T,N>, a container: one stack level)."""

    def __init__(self, elem: XdrType, n: int):
        self.elem, self.n = elem, n
        self.align = elem.align
        self.size = _align_up(elem.size, elem.align) * n
        self.fixed_wire = None if elem.fixed_wire is None else elem.fixed_wire * n

    def emit(self, ctx, noff, depth, path):
        step = _align_up(self.elem.size, self.elem.align)
        for i in range(self.n):
            self.elem.emit(ctx, noff + i * step, depth + 1, f"{path}[{i}]")


class XVector(XdrType):
    """T x<N> for non-byte T (xvector<T,N>): a container level, then a u32
    count and the elements.  Staged as xdrg_bytes_ref {heap offset, count}
    of an element array (stride = T's aligned size).  Fixed-size T: the
    element's ops follow the VECTOR op inline (arg2 of them); any other T:
    the element's subroutine (XDRG_F_SUB, arg4 = its pc)."""

    size, align = 16, 8
    fixed_wire = None
    pointer = False

    def __init__(self, elem: XdrType, max_len: int = A.XDR_MAX_LEN):
        self.elem, self.max_len = elem, max_len

    @property
    def stride(self) -> int:  # read late: the element may be a type still being defined
        return _align_up(self.elem.size, self.elem.align)

    def emit(self, ctx, noff, depth, path):
        d = depth + 1  # container level (marshal.h:129-136)
        flags = A.F_POINTER if self.pointer else 0
        if self.elem.fixed_wire is None:
            upc = ctx.emit(A.OP_VECTOR, noff, d, path, flags | A.F_SUB, self.max_len, self.stride)
            ctx.sub(self.elem, f"{path}[]", upc)
            return
        upc = ctx.emit(A.OP_VECTOR, noff, d, path, flags, self.max_len, self.stride)
        start = len(ctx.ops)
        self.elem.emit(ctx, 0, d, f"{path}[]")  # element-relative offsets
        ctx.ops[upc][6] = len(ctx.ops) - start  # arg2 = number of element ops


class Pointer(XVector):
    """T *x (xdr::pointer<T>): a vector of at most one element."""

    pointer = True

    def __init__(self, elem: XdrType):
        super().__init__(elem, 1)


class Struct(XdrType):
    is_class = True

    def __init__(self, name: str, fields: list | None = None):
        self.name = name
        self.fields = []
        self.size, self.align, self.fixed_wire, self.offsets = 0, 1, None, {}
        if fields is not None:
            self.define(fields)

    def define(self, fields: list) -> "Struct":
        """Give a declared struct its fields (a recursive type refers to
        itself through a container, whose staged size does not depend on
        the element's)."""
        self.fields = list(fields)
        off, al = 0, 1
        self.offsets = {}
        for fname, ft in self.fields:
            off = _align_up(off, ft.align)
            self.offsets[fname] = off
            off += ft.size
            al = max(al, ft.align)
        self.align = al
        self.size = _align_up(max(off, 1), al) if self.fields else 1
        fw = [ft.fixed_wire for _, ft in self.fields]
        self.fixed_wire = None if any(w is None for w in fw) else sum(fw)
        return self

    def emit(self, ctx, noff, depth, path):
        d = depth + 1  # xdr_generic_put/get operator() on a class, marshal.h:129-136
        for fname, ft in self.fields:
            ft.emit(ctx, noff + self.offsets[fname], d, f"{path}.{fname}" if path else fname)

    def offset_of(self, dotted: str) -> int:
        t, off = self, 0
        for part in dotted.split("."):
            if isinstance(t, Struct):
                off += t.offsets[part]
                t = dict(t.fields)[part]
            elif isinstance(t, Union):
                arm = t.arm_by_name(part)
                off += t.arms_off
                t = arm
            else:
                raise KeyError(dotted)
        return off

    def __repr__(self):
        return f"struct {self.name}"


class _VoidT(XdrType):
    size, align, fixed_wire = 0, 1, 0

    def emit(self, ctx, noff, depth, path):
        pass


Void = _VoidT()


class Union(XdrType):
    """xdrc union: discriminant (int32 native, u32 on the wire) followed by the
    selected arm.  Native staged layout = C struct {int32 tag; union {arms}}.

    ``arms``: list of (case_values, field_name, type) with type=Void for a
    void arm; ``default``: (field_name, type) or None (no default arm, so an
    unknown discriminant throws xdr_bad_discriminant).  ``tag_type`` may be an
    Enum with validate=True (the discriminant is then validated first, as
    archive(ar, which) does for an opt-in enum)."""

    is_class = True
    fixed_wire = None

    def __init__(self, name: str, tag_name: str, tag_type: XdrType, arms: list, default=None):
        self.name, self.tag_name, self.tag_type = name, tag_name, tag_type
        self.arms = [(list(c), f, t) for c, f, t in arms]
        self.default = default
        arm_types = [t for _, _, t in self.arms] + ([default[1]] if default else [])
        arm_align = max([4] + [t.align for t in arm_types])
        self.arms_off = _align_up(4, arm_align)
        arm_size = max([0] + [t.size for t in arm_types])
        self.align = arm_align
        self.size = _align_up(self.arms_off + arm_size, arm_align)

    def arm_by_name(self, fname):
        for _, f, t in self.arms:
            if f == fname:
                return t
        if self.default and self.default[0] == fname:
            return self.default[1]
        raise KeyError(fname)

    def message(self) -> str:
        return f"bad value of {self.tag_name} in {self.name}"  # gen_hh.cc:479-481

    def emit(self, ctx, noff, depth, path):
        d = depth + 1
        flags, a0, a1 = 0, 0, 0
        if isinstance(self.tag_type, Enum) and self.tag_type.validate:
            vals = sorted(set(self.tag_type.tags.values()))
            flags, a0, a1 = A.F_VALIDATE, ctx.add_table(vals), len(vals)
        upc = ctx.emit(A.OP_UNION, noff, d, f"{path}.{self.tag_name}" if path else self.tag_name,
                       flags, a0, a1)
        ctx.messages[upc] = self.message()
        targets, jumps = [], []  # (case, pc or None for void)
        arm_base = noff + self.arms_off
        for cases, fname, t in self.arms:
            if t is Void:
                targets.extend((c, None) for c in cases)
                continue
            pc = len(ctx.ops)
            t.emit(ctx, arm_base, d, f"{path}.{fname}" if path else fname)
            jumps.append(ctx.emit(A.OP_JUMP, 0, d, "<jump>"))
            targets.extend((c, pc) for c in cases)
        default_pc = None
        if self.default is not None:
            fname, t = self.default
            if t is Void:
                default_pc = -1
            else:
                default_pc = len(ctx.ops)
                t.emit(ctx, arm_base, d, f"{path}.{fname}" if path else fname)
                jumps.append(ctx.emit(A.OP_JUMP, 0, d, "<jump>"))
        end = len(ctx.ops)
        for j in jumps:
            ctx.ops[j][4] = end
        case_tab = []
        for c, pc in targets:
            case_tab += [int(c) & 0xFFFFFFFF, end if pc is None else pc]
        op = ctx.ops[upc]
        op[6] = ctx.add_table(case_tab)  # arg2
        op[7] = len(targets)              # arg3
        if default_pc is not None:
            op[1] |= A.F_DEFAULT
            op[8] = end if default_pc == -1 else default_pc

    def __repr__(self):
        return f"union {self.name}"


class CompiledPlan:
    """Host-side result of compiling a type: the op array and table exactly as
    passed to xdrg_plan_create, plus names for error messages."""

    def __init__(self, root: XdrType, ops: np.ndarray, table: np.ndarray, names, messages):
        self.root = root
        self.ops = ops
        self.table = table
        self.names = names
        self.messages = messages
        self.stride = _align_up(root.size, root.align)
        self.fixed_size = root.fixed_wire

    @property
    def is_var(self) -> bool:
        """Variable-length wire records (opaque<>/string<>/unions)."""
        return self.fixed_size is None

    def bad_discriminant_message(self, op: int) -> str:
        return self.messages.get(op, "bad value of discriminant")


def compile_plan(root: XdrType) -> CompiledPlan:
    """Flatten ``root`` (normally a Struct or Union) into plan ops."""
    ctx = _Ctx()
    if isinstance(root, (Struct, Union)):
        ctx.subs[id(root)] = [root, "", 0, []]  # the record's own ops serve as its subroutine
        root.emit(ctx, 0, 0, "")
    else:
        # a bare scalar/bytes record: one field, no class level
        root.emit(ctx, 0, 0, "value")
    ctx.emit(A.OP_END, 0, 0, "<end>")
    ctx.emit_subs()
    ops = np.zeros(len(ctx.ops), dtype=OP_DTYPE)
    for i, o in enumerate(ctx.ops):
        ops[i] = tuple(o)
    table = np.array(ctx.table, dtype=np.uint32)
    return CompiledPlan(root, ops, table, ctx.names, ctx.messages)
