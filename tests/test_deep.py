"""Deeply nested element subroutines: linked lists through pointer<T>.

tests/xdrtest.x's test_recursive (`test_recursive *next`, :29-33) and
rpcbind's RPCBPROC_DUMP reply list rp__list (xdrpp/rpcb_prot.x:24-37)
nest one element frame per node.  The reference recurses through them on
its call stack (xdrpp/types.h:591-665, marshal.h:129-136, :198-205),
bounded only by marshaling_stack_limit.  The device keeps XDRG_SUB_FRAMES
frames per record in registers and walks deeper records again in its
deep passes (xdrpp_amd/csrc/sub_kernels.h); only XDRG_MAX_FRAMES, far past
the depth at which the reference's own recursion crashes, is a limit of
its own.

Golden vectors: tests/golden/deep.json, written by oracle/ref_deep.cc
(`make -C oracle deep`) -- the REAL reference marshaler over genuine xdrc
output.  Chains are staged and read back iteratively here (no recursion
in Python, whose limit a 3000-node chain would pass).
"""
import json
import os
import struct

import numpy as np
import pytest

from conftest import GOLD, ROOT

from xdrpp_amd import _abi as A
from xdrpp_amd import objects as OB
from xdrpp_amd import schemas as S
from xdrpp_amd.xdr_types import compile_plan
import oracle_bridge as O

REF = "/root/reference"
LINK = {"test_recursive": "next", "rp__list": "rpcb_next"}


@pytest.fixture(scope="module")
def gold():
    with open(os.path.join(GOLD, "deep.json")) as f:
        return json.load(f)


def node_value(name, j):
    """One chain node's non-link fields as objects.py holds them."""
    if name == "test_recursive":
        return {"elem": bytes.fromhex(j), "nextvec": []}
    prog, vers, netid, addr, owner = j
    return {"rpcb_map": {"r_prog": prog, "r_vers": vers, "r_netid": bytes.fromhex(netid),
                         "r_addr": bytes.fromhex(addr), "r_owner": bytes.fromhex(owner)}}


def stage_chains(name, chains):
    """Native records + heap of records that are linked lists (lists of
    node values), built iteratively: node i+1 is the single element of node
    i's link pointer."""
    t = S.CONTAINERS.get(name) or getattr(S, name)
    link = LINK[name]
    stride = OB._align_up(t.size, t.align)
    native = bytearray(len(chains) * stride)
    heap = OB._Heap()
    for r, nodes in enumerate(chains):
        buf, off = native, r * stride
        for i, node in enumerate(nodes):
            for fname, ft in t.fields:
                if fname != link:
                    OB._put(ft, buf, off + t.offsets[fname], node[fname], heap)
            nxt = i + 1 < len(nodes)
            arr = heap.alloc(stride if nxt else 0, 8)
            struct.pack_into("<QII", buf, off + t.offsets[link], arr, 1 if nxt else 0, 0)
            buf, off = heap.buf, arr
    return np.frombuffer(bytes(native), dtype=np.uint8).copy(), np.frombuffer(bytes(heap.buf), dtype=np.uint8).copy()


def unstage_chains(name, native, heap, n):
    """The node lists of n decoded list records (iterative walk)."""
    t = S.CONTAINERS.get(name) or getattr(S, name)
    link = LINK[name]
    stride = OB._align_up(t.size, t.align)
    nat, hp = bytes(np.asarray(native, dtype=np.uint8)), bytes(np.asarray(heap, dtype=np.uint8))
    out = []
    for r in range(n):
        buf, off, nodes = nat, r * stride, []
        while True:
            nodes.append({f: OB._get(ft, buf, off + t.offsets[f], hp) for f, ft in t.fields if f != link})
            arr, cnt, _ = struct.unpack_from("<QII", buf, off + t.offsets[link])
            if not cnt:
                break
            buf, off = hp, arr
        out.append(nodes)
    return out


def chains_of(gold, name):
    recs = gold[name]
    chains = [[node_value(name, j) for j in r["nodes"]] for r in recs]
    wire = [bytes.fromhex(r["xdr"]) for r in recs]
    offs = np.zeros(len(recs) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(w) for w in wire])
    return chains, wire, offs, recs


TYPES = ["test_recursive", "rp__list"]


def plan_of(name):
    return compile_plan(S.CONTAINERS.get(name) or getattr(S, name))


# ------------------------------------------------------------------ CPU
@pytest.mark.skipif(not os.path.exists(f"{REF}/xdrpp/rpcb_prot.x"), reason="reference tree absent")
def test_rp_list_schema_equals_rpcb_prot_x():
    import xdrc_front as xdrc
    from test_xdrc import same_plan
    sp = xdrc.load_file(f"{REF}/xdrpp/rpcb_prot.x")
    assert same_plan(sp.plan("rp__list"), compile_plan(S.rp__list))


@pytest.mark.parametrize("name", TYPES)
def test_oracle_matches_reference(gold, name):
    """The C restatement (no nesting bound but the stack limit) reproduces
    the reference's bytes, sizes, depths and decodes of every chain."""
    chains, wire, offs, recs = chains_of(gold, name)
    cp, n = plan_of(name), len(chains)
    nat, heap = stage_chains(name, chains)
    x, o = O.encode(cp, nat, n, heap)
    assert bytes(x) == b"".join(wire)
    assert np.array_equal(o, offs)
    assert np.array_equal(O.sizes(cp, nat, n, heap), [len(w) for w in wire])
    assert np.array_equal(O.depths(cp, nat, n, heap), [r["depth"] for r in recs])
    nat2, heap2 = O.decode(cp, np.frombuffer(b"".join(wire), dtype=np.uint8), n, offs)
    assert unstage_chains(name, nat2, heap2, n) == chains


@pytest.mark.parametrize("name", TYPES)
def test_oracle_stack_limits(gold, name):
    """Only marshaling_stack_limit stops a deep record (marshal.h:131-132,
    :200-201): the first record whose limit exceeds L fails."""
    chains, wire, offs, recs = chains_of(gold, name)
    cp, n = plan_of(name), len(chains)
    nat, heap = stage_chains(name, chains)
    x = np.frombuffer(b"".join(wire), dtype=np.uint8)
    for L in sorted({r["put_limit"] for r in recs})[-3:]:
        first = next(i for i, r in enumerate(recs) if r["put_limit"] > L - 1)
        with pytest.raises(O.OracleError) as e:
            O.encode(cp, nat, n, heap, stack_limit=L - 1)
        assert (e.value.code, e.value.record) == (A.ERR_STACK_PUT, first)
        first = next(i for i, r in enumerate(recs) if r["get_limit"] > L - 1)
        with pytest.raises(O.OracleError) as e:
            O.decode(cp, x, n, offs, stack_limit=L - 1)
        assert (e.value.code, e.value.record) == (A.ERR_STACK_GET, first)


@pytest.mark.skipif(not os.path.exists(f"{REF}/xdrpp/marshal.cc"), reason="reference tree absent")
def test_fixture_regenerates(tmp_path):
    """deep.json is what the reference produces today (empty diff)."""
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "_ref/ref_deep"], check=True)
    out = tmp_path / "d.json"
    subprocess.run([os.path.join(ROOT, "oracle", "_ref", "ref_deep"), str(out)], check=True)
    assert out.read_bytes() == open(os.path.join(GOLD, "deep.json"), "rb").read()


def chain_stream(depth):
    """xdr_to_opaque of a test_recursive chain of `depth` nodes with empty
    elems: depth x (elem len 0, pointer flag) then depth x (nextvec count 0),
    with the last flag 0."""
    w = np.zeros(3 * depth, dtype=">u4")
    w[1:2 * depth:2] = 1
    w[2 * depth - 1] = 0
    return w.view(np.uint8).copy()


# ------------------------------------------------------------------ GPU
def _dev(a, dev):
    import torch
    return torch.from_numpy(np.array(a)).to(dev)


@pytest.mark.gpu
@pytest.mark.parametrize("spec", [1, 0])
@pytest.mark.parametrize("name", TYPES)
def test_gpu_matches_reference(gold, dev, name, spec):
    """Every chain, 1 to 3000 nodes: bytes, offsets, sizes, depths and the
    decode, through the main pass and both deep passes -- on the plan's
    generated frame walks (spec 1, codegen.cpp frame_walk_source) and on the
    interpreter (spec 0)."""
    import ctypes as C
    from xdrpp_amd import marshal as M
    chains, wire, offs, recs = chains_of(gold, name)
    cp, n = plan_of(name), len(chains)
    plan = M.Plan(S.CONTAINERS.get(name) or getattr(S, name), {"specialize": spec})
    mar = M.Marshaler(plan, dev)
    nat, heap = stage_chains(name, chains)
    dn, dh = _dev(nat, dev), _dev(heap, dev)
    r = mar.encode(dn, n, dh)
    assert bytes(r.xdr.cpu().numpy()) == b"".join(wire)
    assert np.array_equal(r.offsets.cpu().numpy().astype(np.uint64), offs)
    assert np.array_equal(mar.serial_sizes(dn, n, heap=dh).cpu().numpy(), [len(w) for w in wire])
    assert np.array_equal(mar.record_depths(dn, n, dh).cpu().numpy(), [r_["depth"] for r_ in recs])
    x = np.frombuffer(b"".join(wire), dtype=np.uint8)
    nat2, heap2 = mar.decode(_dev(x, dev), n, _dev(offs.astype(np.int64), dev))
    assert unstage_chains(name, nat2.cpu().numpy(), heap2.cpu().numpy(), n) == chains
    onat, oheap = O.decode(cp, x, n, offs)
    assert np.array_equal(nat2.cpu().numpy(), onat)
    assert np.array_equal(heap2.cpu().numpy(), oheap)
    # record-marked messages take the same walks
    m = mar.encode_msgs(dn, n, dh)
    assert bytes(m.xdr.cpu().numpy()) == b"".join((len(w) | 0x80000000).to_bytes(4, "big") + w for w in wire)
    nat3, heap3 = mar.decode_msgs(m.xdr)
    assert unstage_chains(name, nat3.cpu().numpy(), heap3.cpu().numpy(), n) == chains
    info = A.XdrgPlanInfo()
    A.check(A.lib().xdrg_plan_get_info(plan.handle, C.byref(info)), "xdrg_plan_get_info")
    assert info.specialized == spec


@pytest.mark.gpu
def test_gpu_stack_limits(gold, dev):
    """marshaling_stack_limit is the only limit the reference's data meets:
    xdr_stack_overflow at the first record past it, whichever pass walks it."""
    from xdrpp_amd import marshal as M
    chains, wire, offs, recs = chains_of(gold, "test_recursive")
    n = len(chains)
    mar = M.Marshaler(M.Plan(S.test_recursive), dev)
    nat, heap = stage_chains("test_recursive", chains)
    dn, dh = _dev(nat, dev), _dev(heap, dev)
    dx, do = _dev(np.frombuffer(b"".join(wire), dtype=np.uint8), dev), _dev(offs.astype(np.int64), dev)
    for L in (60, 66, 2000, 2049, 2052, 6000):
        first = next((i for i, r in enumerate(recs) if r["put_limit"] > L), None)
        if first is None:
            assert bytes(mar.encode(dn, n, dh, stack_limit=L).xdr.cpu().numpy()) == b"".join(wire)
            continue
        with pytest.raises(M.XdrStackOverflow) as e:
            mar.encode(dn, n, dh, stack_limit=L, capacity=int(offs[-1]))
        assert e.value.record == first
        with pytest.raises(M.XdrStackOverflow) as e:
            mar.decode(dx, n, do, stack_limit=L)
        assert e.value.record == next(i for i, r in enumerate(recs) if r["get_limit"] > L)


@pytest.mark.gpu
def test_gpu_many_deep_records(gold, dev):
    """Hundreds of deep records at once (deep pass A's lanes, the lists)
    against the oracle, mixed with shallow ones."""
    from xdrpp_amd import marshal as M
    chains, wire, offs, recs = chains_of(gold, "test_recursive")
    pick = [0, 4, 5, 7, 8, 1, 11, 2]
    many = [chains[pick[i % len(pick)]] for i in range(400)]
    n, cp = len(many), plan_of("test_recursive")
    nat, heap = stage_chains("test_recursive", many)
    mar = M.Marshaler(M.Plan(S.test_recursive), dev)
    r = mar.encode(_dev(nat, dev), n, _dev(heap, dev))
    x, o = O.encode(cp, nat, n, heap)
    assert bytes(r.xdr.cpu().numpy()) == bytes(x)
    nat2, heap2 = mar.decode(r.xdr, n, r.offsets)
    onat, oheap = O.decode(cp, x, n, o)
    assert np.array_equal(nat2.cpu().numpy(), onat) and np.array_equal(heap2.cpu().numpy(), oheap)


@pytest.mark.gpu
def test_gpu_max_frames(dev):
    """XDRG_MAX_FRAMES: the device's own limit, past the reference's crash
    depth.  A chain that needs one frame more fails with xdr_stack_overflow
    at the `next` pointer that would open it, on encode (a cyclic staged heap
    too: it would never end) and on decode; one frame less passes."""
    from xdrpp_amd import marshal as M
    mar = M.Marshaler(M.Plan(S.test_recursive), dev)
    ok, bad = A.MAX_FRAMES + 1, A.MAX_FRAMES + 2  # nodes = frames + 1
    xs = [chain_stream(ok), chain_stream(bad)]
    for x, fails in zip(xs, (False, True)):
        offs = np.array([0, x.size], dtype=np.int64)
        if fails:
            with pytest.raises(M.XdrStackOverflow) as e:
                mar.decode(_dev(x, dev), 1, _dev(offs, dev))
            assert (e.value.record, e.value.op) == (0, 1)
        else:
            nat, heap = mar.decode(_dev(x, dev), 1, _dev(offs, dev))
            r = mar.encode(nat, 1, heap)
            assert np.array_equal(r.xdr.cpu().numpy(), x)
    # a node whose `next` is itself: the walk ends at the frame limit
    t = S.test_recursive
    nat = np.zeros(OB._align_up(t.size, t.align), dtype=np.uint8)
    struct.pack_into("<QII", nat, t.offsets["next"], 0, 1, 0)
    struct.pack_into("<QII", nat, t.offsets["nextvec"], 0, 0, 0)
    heap = nat.copy()  # element 0 of the pointer is the record's own image
    with pytest.raises(M.XdrStackOverflow) as e:
        mar.encode(_dev(nat, dev), 1, _dev(heap, dev))
    assert (e.value.record, e.value.op) == (0, 1)


@pytest.mark.gpu
@pytest.mark.parametrize("spec", [1, 0])
def test_gpu_tail_cycle_ends(dev, spec):
    """A linked list walks in one frame (its tail containers replace their
    frames, sub_kernels.h sub_tail), so a staged rp__list node whose
    rpcb_next is itself never runs out of frames: the walk still ends, at
    XDRG_MAX_FRAMES open frames counted with the replaced ones, with
    xdr_stack_overflow at rpcb_next (as a test_recursive chain through `next`
    does, test_gpu_max_frames) -- in the main pass, in well under a second."""
    import time
    from xdrpp_amd import marshal as M
    t = S.rp__list
    plan = M.Plan(t, {"specialize": spec})
    vpc = int(np.nonzero((plan.cp.ops["kind"] == A.OP_VECTOR))[0][-1])
    nat = np.zeros(t.size, dtype=np.uint8)
    struct.pack_into("<QII", nat, t.offsets["rpcb_next"], 0, 1, 0)  # element 0: the image itself
    heap = nat.copy()
    mar = M.Marshaler(plan, dev)
    t0 = time.perf_counter()
    with pytest.raises(M.XdrStackOverflow) as e:
        mar.encode(_dev(nat, dev), 1, _dev(heap, dev))
    assert (e.value.record, e.value.op) == (0, vpc)
    assert time.perf_counter() - t0 < 30


def chain_lists(lens):
    """rp__list records of the given node counts (node i of list r: r_prog
    100000 + i, strings of a few letters)."""
    return [[node_value("rp__list", [100000 + i, (r + i) % 5, "61" * ((i + r) % 9), "62" * ((3 * i + r) % 25),
                                     "63" * ((5 * i) % 13)]) for i in range(k)] for r, k in enumerate(lens)]


@pytest.mark.gpu
@pytest.mark.parametrize("spec", [1, 0])
def test_gpu_chain_log(dev, spec):
    """The chain log (sub_kernels.h "Chains"): the size walk logs a record's
    first tail chain past kChainT (32) replacements, the encode's main pass
    jumps over it and the node pass writes it, one lane a node.  Lists of 1
    to 700 nodes around the threshold encode to the restatement's bytes; a
    capacity that ends inside a logged chain, and stack limits that end
    inside one, fail at the restatement's record and op (those records are
    walked whole: the node pass writes only records that cannot fail)."""
    from xdrpp_amd import marshal as M
    lens = [1, 31, 32, 33, 34, 35, 2, 64, 200, 3, 33, 700, 5, 100]
    chains = chain_lists(lens)
    n, cp = len(chains), plan_of("rp__list")
    mar = M.Marshaler(M.Plan(S.rp__list, {"specialize": spec}), dev)
    nat, heap = stage_chains("rp__list", chains)
    dn, dh = _dev(nat, dev), _dev(heap, dev)
    want, woffs = O.encode(cp, nat, n, heap)
    r = mar.encode(dn, n, dh)
    assert np.array_equal(r.xdr.cpu().numpy(), want)
    assert np.array_equal(r.offsets.cpu().numpy().astype(np.uint64), woffs)
    # a capacity inside the 700-node list's chain (record 11), past its 40th node
    k = lens.index(700)
    cap = int(woffs[k]) + 40 * 60
    with pytest.raises(O.OracleError) as oe:
        O.encode(cp, nat, n, heap, cap=cap)
    with pytest.raises(M.XdrOverflow) as e:
        mar.encode(dn, n, dh, capacity=cap)
    assert (e.value.record, e.value.op) == (oe.value.record, oe.value.op)
    for L in (40, 150, 650):
        with pytest.raises(O.OracleError) as oe:
            O.encode(cp, nat, n, heap, stack_limit=L)
        with pytest.raises(M.XdrStackOverflow) as e:
            mar.encode(dn, n, dh, stack_limit=L, capacity=int(woffs[-1]))
        assert (e.value.record, e.value.op) == (oe.value.record, oe.value.op)
    # the decode of the same bytes
    nat2, heap2 = mar.decode(_dev(want, dev), n, _dev(woffs.astype(np.int64), dev))
    assert unstage_chains("rp__list", nat2.cpu().numpy(), heap2.cpu().numpy(), n) == chains


@pytest.mark.gpu
@pytest.mark.parametrize("spec", [1, 0])
def test_gpu_wave_pass(dev, spec):
    """The decode's wave pass (sub_kernels.h "Long records"): records of 4
    KiB or more are walked by a whole wave from LDS blocks of the stream.
    Lists of 1 to 1000 nodes on both sides of the threshold (and of the 8 KiB
    block) decode to the restatement's native records and heap bit for bit,
    mixed with test_recursive chains too deep for the wave's frames (deep
    pass A takes them).  Damaged long records -- a string length past the
    record, a bad count, a stack limit inside the list, a record cut short --
    fail at the restatement's record, op and code."""
    from xdrpp_amd import marshal as M
    lens = [1, 700, 3, 60, 64, 69, 70, 140, 141, 200, 2, 1000, 5, 130]
    chains = chain_lists(lens)
    n, cp = len(chains), plan_of("rp__list")
    mar = M.Marshaler(M.Plan(S.rp__list, {"specialize": spec}), dev)
    nat, heap = stage_chains("rp__list", chains)
    x, offs = O.encode(cp, nat, n, heap)
    sizes = np.diff(offs.astype(np.int64))
    assert (sizes >= 4096).sum() >= 6 and (sizes < 4096).sum() >= 6 and (sizes > 8192).sum() >= 3
    dx, do = _dev(x, dev), _dev(offs.astype(np.int64), dev)
    nat2, heap2 = mar.decode(dx, n, do)
    onat, oheap = O.decode(cp, x, n, offs)
    assert np.array_equal(nat2.cpu().numpy(), onat) and np.array_equal(heap2.cpu().numpy(), oheap)
    assert unstage_chains("rp__list", nat2.cpu().numpy(), heap2.cpu().numpy(), n) == chains

    def same_error(xb, ob, **kw):
        with pytest.raises(O.OracleError) as oe:
            O.decode(cp, xb, n, ob, **kw)
        with pytest.raises(M.XdrRuntimeError) as e:
            mar.decode(_dev(xb, dev), n, _dev(ob.astype(np.int64), dev), **kw)
        assert (e.value.record, e.value.op, e.value.code) == (oe.value.record, oe.value.op, oe.value.code)

    k = lens.index(1000)
    base = int(offs[k])
    for at, word in ((base + 40 * 60, 0x7FFF0000), (base + 4000, 0x00000005), (base + 9000, 0xFFFFFFFF),
                     (base + 20000, 0x00000002)):
        xb = x.copy()
        xb[at & ~3:(at & ~3) + 4] = np.frombuffer(word.to_bytes(4, "big"), np.uint8)
        try:
            on, oh = O.decode(cp, xb, n, offs)
        except O.OracleError:
            same_error(xb, offs)
        else:  # (the word fell in a payload)
            gn, gh = mar.decode(_dev(xb, dev), n, do)
            assert np.array_equal(gn.cpu().numpy(), on) and np.array_equal(gh.cpu().numpy(), oh)
    # one byte flipped across the list (pads, lengths, counts, values), in
    # and past the list decode's batches of 64 nodes and 8 KiB blocks
    for at in range(base + 3, int(offs[k + 1]), 1531):
        xb = x.copy()
        xb[at] ^= 0x5A
        try:
            on, oh = O.decode(cp, xb, n, offs)
        except O.OracleError:
            same_error(xb, offs)
        else:
            gn, gh = mar.decode(_dev(xb, dev), n, do)
            assert np.array_equal(gn.cpu().numpy(), on) and np.array_equal(gh.cpu().numpy(), oh), at
    for L in (40, 150, 650):
        same_error(x, offs, stack_limit=L)
    cut = offs.copy()
    cut[k + 1:] -= 8  # record k loses its last two words, the rest shift
    same_error(x[:int(cut[-1])].copy(), cut)
    # deep test_recursive chains (not tail containers: a frame a node) past the threshold
    tr = plan_of("test_recursive")
    mt = M.Marshaler(M.Plan(S.test_recursive, {"specialize": spec}), dev)
    parts = [chain_stream(d) for d in (3, 400, 9, 1200, 2)]
    xo = np.concatenate(parts)
    oo = np.zeros(len(parts) + 1, dtype=np.uint64)
    oo[1:] = np.cumsum([p.size for p in parts])
    a, ha = mt.decode(_dev(xo, dev), len(parts), _dev(oo.astype(np.int64), dev))
    ta, tha = O.decode(tr, xo, len(parts), oo)
    assert np.array_equal(a.cpu().numpy(), ta) and np.array_equal(ha.cpu().numpy(), tha)


def big_node_chains(lens, fields=1100):
    """A recursive plan of more than 1,024 ops: 1,100 unsigned
    fields (or `fields`), a string and `bignode *next` per node, and records
    of the given node counts, staged iteratively."""
    from xdrpp_amd.xdr_types import Pointer, String, Struct, UInt
    t = Struct("bignode")
    t.define([(f"f{i}", UInt) for i in range(fields)] + [("name", String()), ("next", Pointer(t))])
    stride = OB._align_up(t.size, t.align)
    native, heap = bytearray(len(lens) * stride), OB._Heap()
    for r, k in enumerate(lens):
        buf, off = native, r * stride
        for i in range(k):
            for j in range(fields):
                struct.pack_into("<I", buf, off + t.offsets[f"f{j}"], (r * 7919 + i * 104729 + j) & 0xFFFFFFFF)
            OB._put(t.fields[fields][1], buf, off + t.offsets["name"], b"n" * ((r + i) % 11), heap)
            nxt = i + 1 < k
            arr = heap.alloc(stride if nxt else 0, 8)
            struct.pack_into("<QII", buf, off + t.offsets["next"], arr, 1 if nxt else 0, 0)
            buf, off = heap.buf, arr
    return t, np.frombuffer(bytes(native), np.uint8).copy(), np.frombuffer(bytes(heap.buf), np.uint8).copy()


@pytest.mark.gpu
def test_gpu_recursive_plan_past_the_wave_lds(dev):
    """The decode's wave pass and its windows take 32 KiB of LDS beside the
    plan's ops (32 bytes an op): a recursive plan of more than about 1,000
    ops leaves no room for them, and its long records (4.4 KiB a node) are
    walked by the main pass instead -- the same natives and heap as the
    restatement, where the launch used to fail."""
    from xdrpp_amd import marshal as M
    lens = [1, 3, 2, 5, 1, 4]
    t, nat, heap = big_node_chains(lens)
    cp = compile_plan(t)
    assert len(cp.ops) > 1024
    n = len(lens)
    x, offs = O.encode(cp, nat, n, heap)
    assert int(np.diff(offs.astype(np.int64)).min()) >= 4096  # every record is a long one
    mar = M.Marshaler(M.Plan(t, {"specialize": 0}), dev)
    nat2, heap2 = mar.decode(_dev(x, dev), n, _dev(offs.astype(np.int64), dev))
    onat, oheap = O.decode(cp, x, n, offs)
    assert np.array_equal(nat2.cpu().numpy(), onat) and np.array_equal(heap2.cpu().numpy(), oheap)


@pytest.mark.gpu
@pytest.mark.parametrize("fields", [300, 600])
def test_gpu_list_decode_wide_nodes(dev, fields):
    """The wave pass's list decode (sub_kernels.h list_decode) on lists of
    wide nodes (1.2 / 2.4 KiB): with 300 fields the ops leave LDS for the
    node candidates; with 600 they do not, and the lengths are walked
    scalar.  Natives and heap as the restatement's, and a flipped byte in
    each long record decodes or fails exactly as it does."""
    from xdrpp_amd import marshal as M
    lens = [1, 3, 2, 5, 1, 4, 9]
    t, nat, heap = big_node_chains(lens, fields)
    cp = compile_plan(t)
    n = len(lens)
    x, offs = O.encode(cp, nat, n, heap)
    mar = M.Marshaler(M.Plan(t, {"specialize": 0}), dev)
    do = _dev(offs.astype(np.int64), dev)
    nat2, heap2 = mar.decode(_dev(x, dev), n, do)
    onat, oheap = O.decode(cp, x, n, offs)
    assert np.array_equal(nat2.cpu().numpy(), onat) and np.array_equal(heap2.cpu().numpy(), oheap)
    for r in range(n):
        if offs[r + 1] - offs[r] < 4096:
            continue
        # a value byte inside, and the last node's count made 2
        for at, v in ((int(offs[r]) + int(0.61 * (offs[r + 1] - offs[r])) | 3, None), (int(offs[r + 1]) - 1, 2)):
            xb = x.copy()
            xb[at] = xb[at] ^ 0x21 if v is None else v
            try:
                on, oh = O.decode(cp, xb, n, offs)
            except O.OracleError as oe:
                with pytest.raises(M.XdrRuntimeError) as e:
                    mar.decode(_dev(xb, dev), n, do)
                assert (e.value.record, e.value.op, e.value.code) == (oe.record, oe.op, oe.code)
            else:
                gn, gh = mar.decode(_dev(xb, dev), n, do)
                assert np.array_equal(gn.cpu().numpy(), on) and np.array_equal(gh.cpu().numpy(), oh), r


@pytest.mark.parametrize("name", TYPES)
def test_host_index_records(gold, name):
    """decode()'s host fallback finds the same record boundaries as the
    encoder (the device index hands streams of records nested deeper than
    its frames, or longer than its window, back to it)."""
    from xdrpp_amd import marshal as M
    chains, wire, offs, recs = chains_of(gold, name)
    x = np.frombuffer(b"".join(wire), dtype=np.uint8)
    got = M.host_index_records(plan_of(name), x, len(chains))
    assert np.array_equal(got, offs)
    # a stream cut short: the record it runs out in gets [off, len), the rest [len, len)
    cut = x[:int(offs[1]) + 8]
    got = M.host_index_records(plan_of(name), cut, len(chains))
    assert list(got[:2]) == list(offs[:2]) and (got[2:] == cut.size).all()


@pytest.mark.parametrize("name", TYPES)
def test_host_index_records_damaged(gold, name):
    """Damaged streams: a word of some record overwritten with a large
    length/count, a bad discriminant or a small value.  The host fallback
    stops the chain where the restatement's index (xdro_index_records, no
    window) does -- a length or count past its bound ends it as the device's
    rx_len does -- and gives the same [off[k], len) tail."""
    from xdrpp_amd import marshal as M
    chains, wire, offs, recs = chains_of(gold, name)
    x0 = np.frombuffer(b"".join(wire), dtype=np.uint8).copy()
    n = len(chains)
    cp = plan_of(name)
    rng = np.random.default_rng(11)
    for t in range(60):
        x = x0.copy()
        w = int(rng.integers(0, x.size // 4)) * 4
        x[w:w + 4] = np.frombuffer(int(rng.choice([0xFFFFFFF0, 0x7FFF, 0x10001, 3, 1, 0])).to_bytes(4, "big"),
                                   np.uint8)
        want, _, rc, er = O.index_records(cp, x, n, 0xFFFFFFFF)
        got = M.host_index_records(cp, x, n)
        if rc == A.ERR_INDEX_LONG:  # nested past the device's frames: the
            # restatement stops at that record, the host walks on
            assert np.array_equal(got[:er + 1], want[:er + 1]), (t, w)
        else:
            assert rc == 0 and np.array_equal(got, want), (t, w)


@pytest.mark.gpu
@pytest.mark.parametrize("name", TYPES)
def test_gpu_decode_without_offsets(gold, dev, name):
    """decode() with no record index: the device index hands these chains
    back (INDEX_LONG), the host walk indexes them, the decode matches."""
    from xdrpp_amd import marshal as M
    chains, wire, offs, recs = chains_of(gold, name)
    n = len(chains)
    mar = M.Marshaler(M.Plan(S.CONTAINERS.get(name) or getattr(S, name)), dev)
    x = _dev(np.frombuffer(b"".join(wire), dtype=np.uint8), dev)
    a, ha = mar.decode(x, n, _dev(offs.astype(np.int64), dev))
    b, hb = mar.decode(x, n)
    assert np.array_equal(a.cpu().numpy(), b.cpu().numpy()) and np.array_equal(ha.cpu().numpy(), hb.cpu().numpy())


@pytest.mark.gpu
def test_gpu_deep_two_streams_and_capture(gold, dev):
    """The deep passes' lists and frame slabs live in each caller's workspace
    (xdrg_deep_workspace_size): two marshalers encode and decode deep chains
    on two streams at once, each with its own workspace (no allocation, lock
    or host wait inside the calls); then an encode and a decode of the deep
    plan captured into a graph replay three times to the reference's bytes,
    through the generated frame walks and the interpreter.  (The main pass
    keeps its frames in registers: with frames in private memory the second
    replay faulted under ROCm's graph packet capture, profiles/r05a-b.)"""
    import torch
    from xdrpp_amd import marshal as M
    chains, wire, offs, recs = chains_of(gold, "test_recursive")
    pick = [0, 4, 5, 7, 8, 1, 11, 2]
    many = [chains[pick[i % len(pick)]] for i in range(300)]
    n, cp = len(many), plan_of("test_recursive")
    nat, heap = stage_chains("test_recursive", many)
    x, o = O.encode(cp, nat, n, heap)
    onat, oheap = O.decode(cp, x, n, o)
    plan = M.Plan(S.test_recursive)
    assert A.lib().xdrg_deep_workspace_size(plan.handle, n) > 0
    dn, dh = _dev(nat, dev), _dev(heap, dev)
    mars = [M.Marshaler(plan, dev) for _ in range(2)]
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    outs = [torch.empty(x.size, dtype=torch.uint8, device=dev) for _ in range(2)]
    offsets = [torch.empty(n + 1, dtype=torch.int64, device=dev) for _ in range(2)]
    backs = [torch.zeros(n * plan.stride, dtype=torch.uint8, device=dev) for _ in range(2)]
    hcap = plan.decode_heap_bytes(x.size)
    houts = [torch.zeros(hcap, dtype=torch.uint8, device=dev) for _ in range(2)]
    torch.cuda.synchronize()
    for _ in range(3):
        for k in range(2):
            s = streams[k].cuda_stream
            mars[k].status.init(s)
            mars[k].launch_encode(dn, n, outs[k], heap=dh, offsets=offsets[k], stream=s)
            mars[k].launch_decode(outs[k], n, backs[k], offsets=offsets[k], heap_out=houts[k], stream=s)
        for k in range(2):
            assert mars[k].check(streams[k].cuda_stream).code == 0
            assert bytes(outs[k].cpu().numpy()) == bytes(x)
            assert np.array_equal(backs[k].cpu().numpy(), onat)
            assert np.array_equal(houts[k].cpu().numpy(), oheap)
    for spec in (1, 0):
        mar = M.Marshaler(M.Plan(S.test_recursive, {"specialize": spec}), dev)
        cap_s = torch.cuda.Stream(dev)
        out, back, hout = outs[0], backs[0], houts[0]
        mar.status.init(cap_s.cuda_stream)
        mar.launch_encode(dn, n, out, heap=dh, offsets=offsets[0], stream=cap_s.cuda_stream)  # warm (tables, kernels)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=cap_s):
            mar.launch_encode(dn, n, out, heap=dh, offsets=offsets[0], stream=cap_s.cuda_stream)
            mar.launch_decode(out, n, back, offsets=offsets[0], heap_out=hout, stream=cap_s.cuda_stream)
        for _ in range(3):
            out.zero_()
            back.zero_()
            hout.zero_()
            mar.status.init(torch.cuda.current_stream().cuda_stream)
            g.replay()
            torch.cuda.synchronize()
            assert mar.check(cap_s.cuda_stream).code == 0
            assert bytes(out.cpu().numpy()) == bytes(x), spec
            assert np.array_equal(back.cpu().numpy(), onat), spec
            assert np.array_equal(hout.cpu().numpy(), oheap), spec
        del g
    torch.cuda.synchronize()
