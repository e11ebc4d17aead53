"""Containers of variable-size elements and recursive types (element
subroutines, XDRG_F_SUB): tests/xdrtest.x's containertest, containertest1,
hasbytes, test_recursive and nested_cereal_adapter_calls.

Golden vectors: tests/golden/containers.json, written by
oracle/ref_containers.cc (`make -C oracle containers`) -- the REAL
reference marshaler over genuine xdrc output of tests/xdrtest.x.  Per
record: the value, xdr_to_opaque of it, check_xdr_depth's smallest limit,
and the smallest marshaling_stack_limit for xdr_to_opaque / xdr_from_opaque.

CPU: the C restatement (oracle/) against the vectors; GPU: the frame-walk
kernels (xdrpp_amd/csrc/sub_kernels.h) against both.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLD, ROOT

from xdrpp_amd import _abi as A
from xdrpp_amd import objects as OB
from xdrpp_amd import schemas as S
from xdrpp_amd.xdr_types import (OpaqueArray, Pointer, Struct, Union, Void, XArray, XVector,
                                 _VarBytes, compile_plan)
import oracle_bridge as O

REF = "/root/reference"
NAMES = list(S.CONTAINERS)


@pytest.fixture(scope="module")
def gold():
    with open(os.path.join(GOLD, "containers.json")) as f:
        return json.load(f)


def from_json(t, j):
    """A value of the fixture's JSON convention as objects.py holds it."""
    if isinstance(t, (_VarBytes, OpaqueArray)):
        return bytes.fromhex(j)
    if isinstance(t, Pointer):
        return None if j is None else from_json(t.elem, j)
    if isinstance(t, (XVector, XArray)):
        return [from_json(t.elem, e) for e in j]
    if isinstance(t, Struct):
        return {f: from_json(ft, j[f]) for f, ft in t.fields}
    if isinstance(t, Union):
        arm = OB._arm(t, j[0])
        return (j[0], None if arm is Void else from_json(arm, j[1]))
    return j


def batch(gold, name):
    recs = gold["types"][name]["records"]
    t = S.CONTAINERS[name]
    vals = [from_json(t, r["value"]) for r in recs]
    wire = [bytes.fromhex(r["xdr"]) for r in recs]
    offs = np.zeros(len(recs) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(w) for w in wire])
    return t, vals, wire, offs, recs


# ------------------------------------------------------------------ CPU
@pytest.mark.skipif(not os.path.exists(f"{REF}/tests/xdrtest.x"), reason="reference tree absent")
@pytest.mark.parametrize("name", NAMES)
def test_schemas_equal_xdrtest_x(name):
    import xdrc_front as xdrc
    from test_xdrc import same_plan
    sp = xdrc.load_file(f"{REF}/tests/xdrtest.x")
    assert same_plan(sp.plan(name), compile_plan(S.CONTAINERS[name]))


def test_plan_layout():
    cp = compile_plan(S.test_recursive)
    vec = [o for o in cp.ops if o["kind"] == A.OP_VECTOR]
    assert [int(o["arg4"]) for o in vec] == [0, 0]  # the record's own ops are its element's
    assert all(o["flags"] & A.F_SUB for o in vec)
    cp = compile_plan(S.hasbytes)
    ends = [i for i, o in enumerate(cp.ops) if o["kind"] == A.OP_END]
    assert len(ends) == 2 and cp.ops[0]["arg4"] == ends[0] + 1  # body after the record's END


@pytest.mark.parametrize("name", NAMES)
def test_oracle_matches_reference(gold, name):
    t, vals, wire, offs, recs = batch(gold, name)
    cp = compile_plan(t)
    n = len(vals)
    nat, heap = OB.stage(t, vals)
    x, o = O.encode(cp, nat, n, heap)
    assert bytes(x) == b"".join(wire)
    assert np.array_equal(o, offs)
    assert np.array_equal(O.depths(cp, nat, n, heap), [r["depth"] for r in recs])
    assert np.array_equal(O.sizes(cp, nat, n, heap), [len(w) for w in wire])
    nat2, heap2 = O.decode(cp, np.frombuffer(b"".join(wire), dtype=np.uint8), n, offs)
    assert OB.unstage(t, nat2, heap2, n) == vals


@pytest.mark.parametrize("name", NAMES)
def test_oracle_stack_limits(gold, name):
    """marshaling_stack_limit (marshal.h:21,34): the first record whose
    put (get) limit exceeds L fails with xdr_stack_overflow."""
    t, vals, wire, offs, recs = batch(gold, name)
    cp = compile_plan(t)
    n = len(vals)
    nat, heap = OB.stage(t, vals)
    x = np.frombuffer(b"".join(wire), dtype=np.uint8)
    for L in sorted({r["put_limit"] for r in recs}):
        if L == 0:
            continue
        first = next(i for i, r in enumerate(recs) if r["put_limit"] > L - 1)
        with pytest.raises(O.OracleError) as e:
            O.encode(cp, nat, n, heap, stack_limit=L - 1)
        assert (e.value.code, e.value.record) == (A.ERR_STACK_PUT, first)
        first = next(i for i, r in enumerate(recs) if r["get_limit"] > L - 1)
        with pytest.raises(O.OracleError) as e:
            O.decode(cp, x, n, offs, stack_limit=L - 1)
        assert (e.value.code, e.value.record) == (A.ERR_STACK_GET, first)


def test_oracle_containertest1_overflow(gold):
    """tests/marshal.cc:568-572: 4 uvec elements read as uvec<2>."""
    k = gold["kat"][0]
    x = np.frombuffer(bytes.fromhex(k["xdr"]), dtype=np.uint8)
    with pytest.raises(O.OracleError) as e:
        O.decode(compile_plan(S.containertest1), x, 1, np.array([0, x.size], dtype=np.uint64))
    assert e.value.code == A.ERR_XVECTOR_BOUND and k["what"] == "xvector overflow"


def chain(depth: int):
    """test_recursive nested `depth` levels through `next`."""
    v = None
    for d in reversed(range(depth)):
        v = {"elem": f"n{d}".encode(), "next": v, "nextvec": []}
    return v


def test_oracle_no_frame_bound():
    """Element subroutines nest as deep as the data goes (types.h:591-665):
    only marshaling_stack_limit raises xdr_stack_overflow (marshal.h:131-132,
    :200-201).  Chains just past the device's private frames and well past
    them round-trip; the reference's own chains are in test_deep.py."""
    cp = compile_plan(S.test_recursive)
    vals = [chain(A.SUB_FRAMES + 1), chain(A.SUB_FRAMES + 2), chain(A.SUB_FRAMES + 60)]
    nat, heap = OB.stage(S.test_recursive, vals)
    x, offs = O.encode(cp, nat, 3, heap)
    nat2, heap2 = O.decode(cp, x, 3, offs)
    assert OB.unstage(S.test_recursive, nat2, heap2, 3) == vals
    # the stack budget of a chain of k nodes is 2k: the third record fails
    with pytest.raises(O.OracleError) as e:
        O.encode(cp, nat, 3, heap, stack_limit=2 * (A.SUB_FRAMES + 2))
    assert (e.value.code, e.value.record) == (A.ERR_STACK_PUT, 2)
    with pytest.raises(O.OracleError) as e:
        O.decode(cp, x, 3, offs, stack_limit=2 * (A.SUB_FRAMES + 2))
    assert (e.value.code, e.value.record) == (A.ERR_STACK_GET, 2)


@pytest.mark.parametrize("n", [1, 64, 200])
def test_oracle_packed_element_areas(n):
    """Fixed-element containers pack per group of 64 records (xdr_oracle.c
    rec_ebytes; include/xdrgpu.h xdrg_decode_heap_size): the arrays follow
    each other, 8-aligned, in record and field order from align8(ebase +
    F * off[64g]), inside the group's F-sized area, and the values are
    unchanged (the native records round-trip through the encoder)."""
    from xdrpp_amd import workloads as W
    cp = compile_plan(S.vecrec)
    nat, heap = W.GENERATORS["vecrec"](n)
    x, offs = O.encode(cp, nat, n, heap)
    dn, dh = O.decode(cp, x, n, offs)
    assert np.array_equal(O.encode(cp, dn, n, dh)[0], x)
    vec = [int(o["noff"]) for o in cp.ops if o["kind"] == A.OP_VECTOR]
    strides = [int(o["arg1"]) for o in cp.ops if o["kind"] == A.OP_VECTOR]
    ebase = (x.size + 15) & ~15
    F = (dh.size - ebase) // x.size
    recs = dn.reshape(n, cp.stride)
    for g in range(0, n, 64):
        cur = (ebase + F * int(offs[g]) + 7) & ~7
        end = ebase + F * int(offs[min(g + 64, n)])
        for r in range(g, min(g + 64, n)):
            for no, st in zip(vec, strides):
                off = int(recs[r, no:no + 8].view(np.uint64)[0])
                cnt = int(recs[r, no + 8:no + 12].view(np.uint32)[0])
                assert off == cur
                cur = (cur + cnt * st + 7) & ~7
        assert cur <= end


@pytest.mark.parametrize("n", [1, 64, 200])
def test_oracle_packed_subroutine_areas(n):
    """Element-subroutine containers of a non-recursive plan (containertest's
    u_4_12 uvec<>) pack the same way: each record's uvec array follows the
    one before it, 8-aligned, from align8(ebase + F * off[64g]); a
    recursive plan (test_recursive) keeps per-record areas."""
    from xdrpp_amd import workloads as W
    cp = compile_plan(S.containertest)
    nat, heap = W.GENERATORS["containertest"](n)
    x, offs = O.encode(cp, nat, n, heap)
    dn, dh = O.decode(cp, x, n, offs)
    assert np.array_equal(O.encode(cp, dn, n, dh)[0], x)
    no = S.containertest.offsets["uvec"]
    st = S.u_4_12.size
    ebase = (x.size + 15) & ~15
    F = (dh.size - ebase) // x.size
    recs = dn.reshape(n, cp.stride)
    for g in range(0, n, 64):
        cur = (ebase + F * int(offs[g]) + 7) & ~7
        end = ebase + F * int(offs[min(g + 64, n)])
        for r in range(g, min(g + 64, n)):
            off = int(recs[r, no:no + 8].view(np.uint64)[0])
            cnt = int(recs[r, no + 8:no + 12].view(np.uint32)[0])
            assert off == cur
            cur = (cur + cnt * st + 7) & ~7
        assert cur <= end


@pytest.mark.skipif(not os.path.exists(f"{REF}/xdrpp/marshal.cc"), reason="reference tree absent")
def test_fixture_regenerates(tmp_path):
    """containers.json is what the reference produces today (empty diff)."""
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "_ref/ref_containers"], check=True)
    out = tmp_path / "c.json"
    subprocess.run([os.path.join(ROOT, "oracle", "_ref", "ref_containers"), str(out)], check=True)
    assert out.read_bytes() == open(os.path.join(GOLD, "containers.json"), "rb").read()


# ------------------------------------------------------------------ GPU
def _dev(a, dev):
    import torch
    return torch.from_numpy(np.array(a)).to(dev)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_matches_reference(gold, dev, name):
    from xdrpp_amd import marshal as M
    t, vals, wire, offs, recs = batch(gold, name)
    n = len(vals)
    mar = M.Marshaler(M.Plan(t), dev)
    nat, heap = OB.stage(t, vals)
    dn, dh = _dev(nat, dev), _dev(heap, dev)
    r = mar.encode(dn, n, dh)
    assert bytes(r.xdr.cpu().numpy()) == b"".join(wire)
    assert np.array_equal(r.offsets.cpu().numpy().astype(np.uint64), offs)
    assert np.array_equal(mar.serial_sizes(dn, n, heap=dh).cpu().numpy(), [len(w) for w in wire])
    assert np.array_equal(mar.record_depths(dn, n, dh).cpu().numpy(), [r_["depth"] for r_ in recs])
    x = np.frombuffer(b"".join(wire), dtype=np.uint8)
    nat2, heap2 = mar.decode(_dev(x, dev), n, _dev(offs.astype(np.int64), dev))
    assert OB.unstage(t, nat2.cpu().numpy(), heap2.cpu().numpy(), n) == vals
    # the decoded native records equal the oracle's byte for byte
    onat, oheap = O.decode(compile_plan(t), x, n, offs)
    assert np.array_equal(nat2.cpu().numpy(), onat)
    assert np.array_equal(heap2.cpu().numpy(), oheap)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_messages(gold, dev, name):
    """xdr_to_msg / xdr_from_msg of every record through the frame walk."""
    from xdrpp_amd import marshal as M
    t, vals, wire, offs, recs = batch(gold, name)
    n = len(vals)
    mar = M.Marshaler(M.Plan(t), dev)
    nat, heap = OB.stage(t, vals)
    r = mar.encode_msgs(_dev(nat, dev), n, _dev(heap, dev))
    want = b"".join(((len(w) | 0x80000000).to_bytes(4, "big") + w) for w in wire)
    assert bytes(r.xdr.cpu().numpy()) == want
    nat2, heap2 = mar.decode_msgs(r.xdr)
    assert OB.unstage(t, nat2.cpu().numpy(), heap2.cpu().numpy(), n) == vals


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_stack_limits(gold, dev, name):
    from xdrpp_amd import marshal as M
    t, vals, wire, offs, recs = batch(gold, name)
    n = len(vals)
    mar = M.Marshaler(M.Plan(t), dev)
    nat, heap = OB.stage(t, vals)
    dn, dh = _dev(nat, dev), _dev(heap, dev)
    dx, do = _dev(np.frombuffer(b"".join(wire), dtype=np.uint8), dev), _dev(offs.astype(np.int64), dev)
    for L in sorted({r["put_limit"] for r in recs}):
        if L == 0:
            continue
        first = next(i for i, r in enumerate(recs) if r["put_limit"] > L - 1)
        with pytest.raises(M.XdrStackOverflow) as e:
            mar.encode(dn, n, dh, stack_limit=L - 1, capacity=int(offs[-1]))
        assert e.value.record == first and e.value.what == gold["stack_what"]["put"]
        first = next(i for i, r in enumerate(recs) if r["get_limit"] > L - 1)
        with pytest.raises(M.XdrStackOverflow) as e:
            mar.decode(dx, n, do, stack_limit=L - 1)
        assert e.value.record == first and e.value.what == gold["stack_what"]["get"]


@pytest.mark.gpu
def test_gpu_containertest1_overflow(gold, dev):
    from xdrpp_amd import marshal as M
    k = gold["kat"][0]
    x = np.frombuffer(bytes.fromhex(k["xdr"]), dtype=np.uint8)
    mar = M.Marshaler(M.Plan(S.containertest1), dev)
    with pytest.raises(M.XdrOverflow) as e:
        mar.decode(_dev(x, dev), 1, _dev(np.array([0, x.size], dtype=np.int64), dev))
    assert e.value.what == k["what"] and e.value.record == 0


@pytest.mark.gpu
def test_gpu_no_frame_bound(dev):
    """Past the private frames the deep passes walk the record: same bytes
    and decode as the oracle, and only the stack limit fails it."""
    from xdrpp_amd import marshal as M
    cp = compile_plan(S.test_recursive)
    mar = M.Marshaler(M.Plan(S.test_recursive), dev)
    vals = [chain(A.SUB_FRAMES + 1), chain(3), chain(A.SUB_FRAMES + 2), chain(A.SUB_FRAMES + 60)]
    nat, heap = OB.stage(S.test_recursive, vals)
    dn, dh = _dev(nat, dev), _dev(heap, dev)
    r = mar.encode(dn, 4, dh)
    x, offs = O.encode(cp, nat, 4, heap)
    assert bytes(r.xdr.cpu().numpy()) == bytes(x)
    assert np.array_equal(mar.record_depths(dn, 4, dh).cpu().numpy(), O.depths(cp, nat, 4, heap))
    nat2, heap2 = mar.decode(r.xdr, 4, r.offsets)
    assert OB.unstage(S.test_recursive, nat2.cpu().numpy(), heap2.cpu().numpy(), 4) == vals
    L = 2 * (A.SUB_FRAMES + 2)
    with pytest.raises(O.OracleError) as want:
        O.encode(cp, nat, 4, heap, stack_limit=L)
    with pytest.raises(M.XdrStackOverflow) as e:
        mar.encode(dn, 4, dh, stack_limit=L)
    assert (e.value.record, e.value.op) == (want.value.record, want.value.op) == (3, want.value.op)
    with pytest.raises(O.OracleError) as want:
        O.decode(cp, x, 4, offs, stack_limit=L)
    with pytest.raises(M.XdrStackOverflow) as e:
        mar.decode(r.xdr, 4, r.offsets, stack_limit=L)
    assert (e.value.record, e.value.op) == (want.value.record, want.value.op)


@pytest.mark.gpu
def test_gpu_random_recursive_batch(dev):
    """A larger seeded batch of trees against the oracle: bytes, offsets,
    sizes, depths, and the decode round trip."""
    from xdrpp_amd import marshal as M
    rng = np.random.default_rng(0xA8)

    def tree(d):
        return {"elem": rng.integers(0, 256, rng.integers(0, 20), dtype=np.uint8).tobytes(),
                "next": tree(d - 1) if d and rng.random() < 0.5 else None,
                "nextvec": [tree(d - 1) for _ in range(rng.integers(0, 3))] if d else []}

    vals = [tree(int(rng.integers(0, 6))) for _ in range(4000)]
    t, cp = S.test_recursive, compile_plan(S.test_recursive)
    n = len(vals)
    nat, heap = OB.stage(t, vals)
    mar = M.Marshaler(M.Plan(t), dev)
    dn, dh = _dev(nat, dev), _dev(heap, dev)
    r = mar.encode(dn, n, dh)
    x, offs = O.encode(cp, nat, n, heap)
    assert bytes(r.xdr.cpu().numpy()) == bytes(x)
    assert np.array_equal(r.offsets.cpu().numpy().astype(np.uint64), offs)
    assert np.array_equal(mar.record_depths(dn, n, dh).cpu().numpy(), O.depths(cp, nat, n, heap))
    nat2, heap2 = mar.decode(r.xdr, n, r.offsets)
    onat, oheap = O.decode(cp, x, n, offs)
    assert np.array_equal(nat2.cpu().numpy(), onat) and np.array_equal(heap2.cpu().numpy(), oheap)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES + ["vecrec"])
@pytest.mark.parametrize("seed", range(8))
def test_gpu_malformed_streams(gold, dev, name, seed):
    """Damaged container streams: flipped bytes, forged element counts and
    a truncated last record.  The device reports the oracle's error (code,
    record, op) and writes nothing past the decoded heap it was given
    (guard bytes after it stay intact)."""
    import torch
    from xdrpp_amd import marshal as M
    from xdrpp_amd import workloads as W
    if name == "vecrec":
        t = S.vecrec
        nat, heap = W.GENERATORS["vecrec"](64)
        x, offs = O.encode(compile_plan(t), nat, 64, heap)
        x = bytes(x)
    else:
        t, vals, wire, offs, recs = batch(gold, name)
        x = b"".join(wire)
    cp = compile_plan(t)
    n = len(offs) - 1
    x = np.frombuffer(x, dtype=np.uint8).copy()
    offs = offs.astype(np.uint64).copy()
    rng = np.random.default_rng(7000 + seed)
    mode = seed % 3
    if mode == 0:  # flipped bytes
        for _ in range(4):
            x[int(rng.integers(0, x.size))] = np.uint8(rng.integers(0, 256))
    elif mode == 1:  # a forged count or length: a big value in a random word
        w = int(rng.integers(0, x.size // 4))
        x[4 * w:4 * w + 4] = np.frombuffer(int(rng.integers(2, 1 << 20)).to_bytes(4, "big"), dtype=np.uint8)
    else:  # the last record cut short, a forged count in it
        a, b = int(offs[n - 1]), int(offs[n])
        if b - a >= 8:
            w = a // 4 + int(rng.integers(0, (b - a) // 4))
            x[4 * w:4 * w + 4] = np.frombuffer(int(rng.integers(2, 64)).to_bytes(4, "big"), dtype=np.uint8)
            cut = 4 * int(rng.integers(1, (b - a) // 4))
            x = x[:b - cut].copy()
            offs[n] = b - cut
    want = _oracle_err(lambda: O.decode(cp, x, n, offs))
    mar = M.Marshaler(M.Plan(t), dev)
    hsize = mar.plan.decode_heap_bytes(x.size)
    guard = 4096
    heap = torch.full((hsize + guard,), 0xA5, dtype=torch.uint8, device=dev)
    native = torch.zeros(n * mar.plan.stride + guard, dtype=torch.uint8, device=dev)
    native[n * mar.plan.stride:] = 0xA5
    s = torch.cuda.current_stream().cuda_stream
    mar.status.init(s)
    mar.launch_decode(_dev(x, dev), n, native[:n * mar.plan.stride], offsets=_dev(offs.view(np.int64), dev),
                      heap_out=heap[:hsize], stream=s)
    got = _gpu_err(lambda: mar.check(s))
    assert got == want
    assert bool((heap[hsize:] == 0xA5).all()), "decode wrote past its heap"
    assert bool((native[n * mar.plan.stride:] == 0xA5).all()), "decode wrote past its records"


def _oracle_err(fn):
    try:
        fn()
    except O.OracleError as e:
        return (e.code, e.record, e.op)
    return None


def _gpu_err(fn):
    from xdrpp_amd import marshal as M
    try:
        fn()
    except M.XdrRuntimeError as e:
        return (e.code, e.record, 0xFFFFFFFF if e.op is None else e.op)
    return None
