"""The device record index of concatenated var records (xdrg_index_records):
the record boundaries xdr_from_opaque walks (xdrpp/marshal.h:299-306).

CPU: the C restatement (oracle/xdr_oracle.c xdro_index_records) against
the reference's own record offsets (golden fixtures written by the real
xdr_put, oracle/ref_golden.cc; containers.json from genuine xdrc output).
GPU: both device paths -- the speculative chain walk and the list ranking
it falls back to -- against the restatement: goldens, full-size encoded
batches (offsets of the encode == the index of its output, and the walk
must hold those itself), streams whose payloads hold records, and damaged
streams (bad lengths and discriminants, truncation, extra records, trailing
garbage, a record past the index window).
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLD, golden

from xdrpp_amd import _abi as A
from xdrpp_amd import schemas as S
from xdrpp_amd.xdr_types import compile_plan
import oracle_bridge as O

VAR = ["recvar", "rpc", "vecrec"]


def window(cp):
    return min(int(max(cp_max(cp), 16)), A.INDEX_MAX_MSG)


def cp_max(cp):
    from xdrpp_amd import marshal as M
    return M.Plan(cp).max_record_bytes


def gold_stream(name):
    n = 1024
    return golden(name, n, "xdr"), golden(name, n, "offsets", np.uint64), n


def containers_stream(name):
    with open(os.path.join(GOLD, "containers.json")) as f:
        recs = json.load(f)["types"][name]["records"]
    wire = [bytes.fromhex(r["xdr"]) for r in recs]
    offs = np.zeros(len(wire) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(w) for w in wire])
    return np.frombuffer(b"".join(wire), dtype=np.uint8).copy(), offs, len(wire)


def damaged(x, offs, n, seed):
    """(label, stream, n) cases around a good stream of n records."""
    rng = np.random.default_rng(seed)
    out = [("good", x, n), ("fewer", x[:int(offs[n // 2])], n), ("more", x, n // 2),
           ("cut", x[:int(offs[n // 3]) + 4], n), ("trailing", np.concatenate([x, np.full(8, 0xff, np.uint8)]), n)]
    for t in range(4):
        y = x.copy()
        r = int(rng.integers(0, n))
        w = int(offs[r]) // 4 + int(rng.integers(0, max(1, (int(offs[r + 1]) - int(offs[r])) // 4)))
        y[4 * w:4 * w + 4] = np.frombuffer(rng.integers(0, 2**32, 1, dtype=np.uint64).astype(">u4").tobytes(),
                                           dtype=np.uint8)
        out.append((f"word{t}", y, n))
    return out


# ------------------------------------------------------------------ CPU
@pytest.mark.parametrize("name", VAR)
def test_oracle_index_matches_reference(name):
    x, offs, n = gold_stream(name)
    cp = compile_plan(S.ALL[name])
    got, cnt, rc, _ = O.index_records(cp, x, n, window(cp))
    assert rc == 0 and cnt == n and np.array_equal(got, offs)


@pytest.mark.parametrize("name", list(S.CONTAINERS))
def test_oracle_index_matches_reference_containers(name):
    x, offs, n = containers_stream(name)
    cp = compile_plan(S.CONTAINERS[name])
    got, cnt, rc, _ = O.index_records(cp, x, n, A.INDEX_MAX_MSG)
    assert rc == 0 and cnt == n and np.array_equal(got, offs)


def test_oracle_index_semantics():
    x, offs, n = gold_stream("recvar")
    cp = compile_plan(S.recvar)
    W = window(cp)
    got, cnt, rc, _ = O.index_records(cp, x[:int(offs[10])], n, W)  # 10 records, then the end
    assert rc == 0 and cnt == 10 and np.array_equal(got[:11], offs[:11]) and (got[11:] == offs[10]).all()
    got, cnt, rc, _ = O.index_records(cp, x, 5, W)  # more records than asked for
    assert rc == 0 and cnt == 2**64 - 1 and np.array_equal(got, offs[:6])
    y = x.copy()
    y[int(offs[7]) + 12:int(offs[7]) + 16] = 0xff  # record 7's blob length: past its bound
    got, cnt, rc, _ = O.index_records(cp, y, n, W)
    assert rc == 0 and cnt == 7 and np.array_equal(got[:8], offs[:8]) and (got[8:] == x.size).all()
    got, cnt, rc, er = O.index_records(cp, x, n, 64)  # a window shorter than the records
    assert rc == A.ERR_INDEX_LONG and er == 0
    # a ragged stream whose last payload's padding overhangs its end: the
    # unpadded bound test passes and the stream ends there (the record count
    # is n, offsets[n] past len), read nowhere past the stream
    cp = compile_plan(S.rpc_msg)
    x, offs, n = gold_stream("rpc")
    for c in (1, 2):
        got, cnt, rc, _ = O.index_records(cp, x[:int(offs[n]) - c].copy(), n, window(cp))
        assert rc == 0 and cnt == n and got[n] == offs[n], c


# ------------------------------------------------------------------ GPU
def _dev(a, dev):
    import torch
    return torch.from_numpy(np.array(a)).to(dev)


def _gpu_index(mar, x, n, maxlen, dev, ws_tail=False):
    """(offsets, count, error) of the device index (+ the workspace's last
    256 bytes: the fast path's flag)."""
    import torch
    from xdrpp_amd import marshal as M
    L = A.lib()
    dx = _dev(x if x.size else np.zeros(4, np.uint8), dev)
    ws = torch.empty(max(L.xdrg_index_workspace_size(x.size, maxlen), 16), dtype=torch.uint8, device=dev)
    offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    cnt = torch.empty(1, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    mar.status.init(s)
    A.check(L.xdrg_index_records(mar.plan.handle, dx.data_ptr(), x.size, n, maxlen, offs.data_ptr(),
                                 cnt.data_ptr(), ws.data_ptr(), ws.numel(), mar.status.ptr, s),
            "xdrg_index_records")
    e = M.error_from(mar.plan, mar.status.read(s))
    res = offs.cpu().numpy().view(np.uint64), int(cnt.cpu().numpy().view(np.uint64)[0]), e
    if not ws_tail:
        return res
    # the fast path's flag: the last 256 bytes of the index layout (past the
    # window, rx_windows' continuation and frames follow it)
    w0 = L.xdrg_index_workspace_size(x.size, min(maxlen, A.INDEX_MAX_MSG)) if x.size else 0
    return res + (ws[max(w0, 256) - 256:max(w0, 256)].cpu().numpy(),)


@pytest.mark.gpu
@pytest.mark.parametrize("spec", [1, 0], ids=["generated", "interpreted"])
@pytest.mark.parametrize("name", VAR + list(S.CONTAINERS))
def test_gpu_index_matches_oracle(dev, name, spec):
    """Both record-start parses of the segment pass -- the plan's generated
    plan_rx and the interpreted rx_len -- against the C restatement, on
    damaged streams."""
    from xdrpp_amd import marshal as M
    t = S.ALL.get(name) or S.CONTAINERS[name]
    cp = compile_plan(t)
    x, offs, n = gold_stream(name) if name in VAR else containers_stream(name)
    mar = M.Marshaler(M.Plan(cp, {"specialize": spec}), dev)
    W = window(cp)
    for label, y, k in damaged(x, offs, n, 7):
        want, wcnt, wrc, wer = O.index_records(cp, y, k, W)
        got, gcnt, err = _gpu_index(mar, y, k, W, dev)
        assert np.array_equal(got, want), label
        assert gcnt == wcnt, label
        assert (err.code if err else 0) == wrc, label


def _recvar_bytes(rid, kind, blob, name, score):
    """One recvar record on the wire (oracle/x/bench.x), written by hand."""
    pad = lambda b: b + b"\0" * (-len(b) % 4)
    return (rid.to_bytes(8, "big") + kind.to_bytes(4, "big", signed=True) + len(blob).to_bytes(4, "big") +
            pad(blob) + len(name).to_bytes(4, "big") + pad(name) + score.to_bytes(8, "big"))


def nested_recvar_stream(n, seed):
    """recvar records whose blobs hold encoded recvar records (one or two):
    word positions inside a payload that parse as record chains, which the
    speculative walk may take as its guess."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        k = int(rng.integers(0, 4))
        if k == 0:
            blob = bytes(rng.integers(0, 256, int(rng.integers(0, 257)), dtype=np.uint8))
        else:
            inner = b"".join(_recvar_bytes(int(rng.integers(0, 2**40)), int(rng.integers(-9, 9)),
                                           bytes(int(rng.integers(0, 40))), b"in", 7) for _ in range(k))
            blob = inner[:256]
        name = bytes(rng.integers(97, 123, int(rng.integers(0, 65)), dtype=np.uint8))
        out.append(_recvar_bytes(i, int(rng.integers(-5, 5)), blob, name, int(rng.integers(0, 2**63))))
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(w) for w in out])
    return np.frombuffer(b"".join(out), dtype=np.uint8).copy(), offs, n


def tiled(x, offs, n, reps):
    """reps copies of a stream of n records: a stream of reps * n records."""
    L = int(offs[n])
    o = np.concatenate([offs[:n] + np.uint64(r * L) for r in range(reps)] + [np.array([reps * L], np.uint64)])
    return np.tile(x[:L], reps), o, reps * n


def _fast_flag(ws_tail):
    return int(ws_tail[:4].view(np.uint32)[0])


@pytest.mark.gpu
@pytest.mark.parametrize("spec", [1, 0], ids=["generated", "interpreted"])
@pytest.mark.parametrize("name", VAR + list(S.CONTAINERS) + ["nested_recvar"])
def test_gpu_index_fast_path(dev, name, spec):
    """The speculative walk and the list ranking on the same streams, both
    against the C restatement: streams long enough for the walk (>= 4
    segments), good and damaged at many places, and in every case the same
    offsets, count and error.  On the good streams the walk must hold the
    index itself (its flag), or it would only be tested as a pass-through."""
    import torch
    from xdrpp_amd import marshal as M
    if name == "nested_recvar":
        cp = compile_plan(S.recvar)
        x, offs, n = nested_recvar_stream(1500, 3)
    else:
        cp = compile_plan(S.ALL.get(name) or S.CONTAINERS[name])
        x, offs, n = gold_stream(name) if name in VAR else containers_stream(name)
    want0, _, _, _ = O.index_records(cp, x, n, A.INDEX_MAX_MSG)
    assert np.array_equal(want0, offs)
    reps = max(1, -(-(1 << 18) // int(offs[n])))  # >= 256 KiB
    x, offs, n = tiled(x, offs, n, reps)
    W = window(cp)
    cases = damaged(x, offs, n, 11) + damaged(x, offs, n, 12)[5:]
    for fast in (1, 2, 0):  # host-gated walk, asynchronous walk, list ranking alone
        mar = M.Marshaler(M.Plan(cp, {"specialize": spec, "index_fast": fast}), dev)
        for label, y, k in cases:
            want, wcnt, wrc, wer = O.index_records(cp, y, k, W)
            got, gcnt, err, tail = _gpu_index(mar, y, k, W, dev, ws_tail=True)
            assert np.array_equal(got, want), (fast, label)
            assert gcnt == wcnt, (fast, label)
            assert (err.code if err else 0) == wrc, (fast, label)
            if err:
                assert err.record == wer, (fast, label)
            # the walk must hold good streams of types whose payloads do not
            # parse as records (test_recursive's elements are records, and a
            # chain entering one need not rejoin the record chain: it may
            # take the list ranking, which the offsets above check)
            # (the walk runs the plan's generated parse: with the interpreted
            # one the list ranking serves, and the flag is not written)
            if fast and spec and label == "good" and name not in ("nested_recvar", "test_recursive"):
                assert _fast_flag(tail) == 1, label


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["recvar", "rpc", "containertest"])
def test_gpu_index_odd_bounds(dev, name):
    """Bounds that are not whole words from a record start: an odd maxlen
    (payloads are bound-tested unpadded, as the decode does, so a record may
    end up to 3 bytes past the window) and a stream cut to a ragged length.
    The walk's staged parse sends such records to global memory
    (index_kernels.h rx_lds::clamp); both device paths against the C
    restatement."""
    from xdrpp_amd import marshal as M
    cp = compile_plan(S.ALL.get(name) or S.CONTAINERS[name])
    x, offs, n = gold_stream(name) if name in VAR else containers_stream(name)
    reps = max(1, -(-(1 << 17) // int(offs[n])))
    x, offs, n = tiled(x, offs, n, reps)
    W = window(cp)
    sizes = np.diff(offs.astype(np.int64))
    cases = [(f"maxlen{m}", x, n, m) for m in (W - 1, W - 3, int(np.median(sizes)) + 1, int(np.median(sizes)) + 2)]
    cases += [(f"ragged{c}", x[:int(offs[n]) - c], n, W) for c in (1, 2, 3)]
    cases += [(f"ragged_mid{c}", x[:int(offs[n // 2]) + c], n, W) for c in (1, 2, 3)]
    for fast in (1, 0):
        mar = M.Marshaler(M.Plan(cp, {"specialize": 1, "index_fast": fast}), dev)
        for label, y, k, m in cases:
            want, wcnt, wrc, wer = O.index_records(cp, y, k, m)
            got, gcnt, err = _gpu_index(mar, y, k, m, dev)
            assert np.array_equal(got, want), (fast, label)
            assert gcnt == wcnt, (fast, label)
            assert (err.code if err else 0) == wrc, (fast, label)
            if err:
                assert err.record == wer, (fast, label)


@pytest.mark.gpu
def test_gpu_index_long_record(dev):
    from xdrpp_amd import marshal as M
    x, offs, n = gold_stream("recvar")
    cp = compile_plan(S.recvar)
    mar = M.Marshaler(M.Plan(cp), dev)
    got, cnt, err = _gpu_index(mar, x, n, 64, dev)
    want, wcnt, wrc, wer = O.index_records(cp, x, n, 64)
    assert err is not None and err.code == A.ERR_INDEX_LONG == wrc and err.record == wer
    assert np.array_equal(got, want) and cnt == wcnt


BIGREC = None


def bigrec_type():
    """struct bigrec { unsigned hyper id; opaque blob<1048576>; string name<64>; }:
    records from 20 bytes to past the index window."""
    global BIGREC
    if BIGREC is None:
        from xdrpp_amd.xdr_types import Opaque, String, Struct, UHyper
        BIGREC = Struct("bigrec", [("id", UHyper), ("blob", Opaque(1 << 20)), ("name", String(64))])
    return BIGREC


def long_records_stream(n, seed, every=29):
    """bigrec records on the wire, mostly short (blob < 200 B), every
    `every`-th (on average) with a 16-80 KiB blob: longer than one index
    window (XDRG_INDEX_MAX_MSG), runs of them back to back as well."""
    rng = np.random.default_rng(seed)
    pad = lambda b: b + b"\0" * (-len(b) % 4)  # noqa: E731
    out = []
    for i in range(n):
        long_ = rng.integers(0, every) == 0 or (i % 500 in (7, 8, 9))
        blen = int(rng.integers(16 << 10, 80 << 10)) if long_ else int(rng.integers(0, 200))
        blob = bytes(rng.integers(0, 256, blen, dtype=np.uint8))
        name = bytes(rng.integers(97, 123, int(rng.integers(0, 65)), dtype=np.uint8))
        out.append(int(i).to_bytes(8, "big") + len(blob).to_bytes(4, "big") + pad(blob)
                   + len(name).to_bytes(4, "big") + pad(name))
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(w) for w in out])
    return np.frombuffer(b"".join(out), dtype=np.uint8).copy(), offs, n


@pytest.mark.gpu
@pytest.mark.parametrize("spec", [1, 0], ids=["generated", "interpreted"])
def test_gpu_index_records_past_the_window(dev, spec):
    """Records longer than the index window, on the device (rx_windows:
    k_rx_long walks them, list-ranking windows index the rest): the same
    offsets, count and error as the sequential walk of the restatement
    (xdro_index_records with max_rec_len past one window), on good and
    damaged streams; and decode() without offsets uses it (no host walk)."""
    import torch
    from xdrpp_amd import marshal as M
    t = bigrec_type()
    cp = compile_plan(t)
    x, offs, n = long_records_stream(3000, 5)
    assert int(np.diff(offs.astype(np.int64)).max()) > A.INDEX_MAX_MSG
    want0, c0, rc0, _ = O.index_records(cp, x, n, A.MAX_MSG)
    assert rc0 == 0 and np.array_equal(want0, offs)
    mar = M.Marshaler(M.Plan(cp, {"specialize": spec}), dev)
    for label, y, k in damaged(x, offs, n, 21) + damaged(x, offs, n, 22)[5:]:
        want, wcnt, wrc, wer = O.index_records(cp, y, k, A.MAX_MSG)
        got, gcnt, err, tail = _gpu_index(mar, y, k, A.MAX_MSG, dev, ws_tail=True)
        assert np.array_equal(got, want), label
        assert gcnt == wcnt, label
        assert (err.code if err else 0) == wrc, label
        if label == "good" and spec:  # the walk over the whole stream held it (its waves parsed the long records)
            assert _fast_flag(tail) == 1
    # a window-sized max_rec_len still hands such a stream back (INDEX_LONG)
    got, gcnt, err = _gpu_index(mar, x, n, A.INDEX_MAX_MSG, dev)
    want, wcnt, wrc, wer = O.index_records(cp, x, n, A.INDEX_MAX_MSG)
    assert err is not None and err.code == A.ERR_INDEX_LONG == wrc and err.record == wer
    dx = _dev(x, dev)
    assert torch.equal(mar.index_records(dx, n).cpu(), torch.from_numpy(offs.view(np.int64)))
    a, ha = mar.decode(dx, n, _dev(offs.view(np.int64), dev))
    b, hb = mar.decode(dx, n)
    assert torch.equal(a, b) and torch.equal(ha, hb)


@pytest.mark.gpu
def test_gpu_index_rp_list_full_size(dev, manifest):
    """1M rpcbind rp__list records (xdrpp/rpcb_prot.x:32-37), 16 of them
    500-node lists nested 500 deep and longer than the index window: the
    device index of the encode's output is the encode's offsets, and the
    encoded bytes are the reference's (manifest hash)."""
    import hashlib
    import torch
    from xdrpp_amd import marshal as M
    from xdrpp_amd import workloads as W
    n = 1 << 20
    nat, heap = W.rp_list(n)
    mar = M.Marshaler(M.Plan(S.ALL["rp_list"]), dev)
    r = mar.encode(_dev(nat, dev), n, _dev(heap, dev))
    h = manifest["hashes"].get(f"rp_list_{n}")
    if h:
        assert hashlib.sha256(r.xdr.cpu().numpy().tobytes()).hexdigest() == h["xdr"]
    sizes = torch.diff(r.offsets)
    assert int(sizes.max()) > A.INDEX_MAX_MSG
    offs = mar.index_records(r.xdr, n)
    assert torch.equal(offs, r.offsets)
    # the speculative walk over the whole stream held it: the lists' generated
    # parse (codegen.cpp tail_list), the 500-node lists parsed by the walk's waves
    got, cnt, err, tail = _gpu_index(mar, r.xdr.cpu().numpy(), n, A.MAX_MSG, dev, ws_tail=True)
    assert err is None and cnt == n and np.array_equal(got, r.offsets.cpu().numpy().view(np.uint64))
    assert _fast_flag(tail) == 1


@pytest.mark.gpu
def test_gpu_index_rp_list_graph_capture(dev):
    """The index of rp__list records of any length captured into a graph:
    the walk over the whole stream runs asynchronously (no rounds, which
    wait on the host), and each replay indexes the stream, its two 500-node
    lists included."""
    import torch
    from xdrpp_amd import marshal as M
    from xdrpp_amd import workloads as W
    n = 1 << 17
    nat, heap = W.rp_list(n)
    mar = M.Marshaler(M.Plan(S.ALL["rp_list"]), dev)
    r = mar.encode(_dev(nat, dev), n, _dev(heap, dev))
    x = r.xdr
    L = A.lib()
    ws = torch.empty(L.xdrg_index_workspace_size(x.numel(), A.MAX_MSG), dtype=torch.uint8, device=dev)
    out = torch.full((n + 1,), -1, dtype=torch.int64, device=dev)
    cnt = torch.empty(1, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = torch.cuda.current_stream().cuda_stream
        A.check(L.xdrg_index_records(mar.plan.handle, x.data_ptr(), x.numel(), n, A.MAX_MSG, out.data_ptr(),
                                     cnt.data_ptr(), ws.data_ptr(), ws.numel(), mar.status.ptr, s), "index (capture)")
    for _ in range(3):
        out.fill_(-1)
        mar.status.init(torch.cuda.current_stream().cuda_stream)
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, r.offsets) and int(cnt.item()) == n
        assert mar.status.read(torch.cuda.current_stream().cuda_stream).code == 0


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["recvar", "rpc", "vecrec", "containertest"])
def test_gpu_index_full_size(dev, name):
    """1M records: the index of the encode's output is the encode's offsets
    (and the speculative walk held it: its flag), and decode without offsets
    (device index) equals decode with them."""
    import torch
    from xdrpp_amd import marshal as M
    from xdrpp_amd import workloads as W
    n = 1 << 20
    nat, heap = getattr(W, name)(n)
    nat, heap = _dev(nat, dev), _dev(heap, dev)
    mar = M.Marshaler(M.Plan(S.ALL[name]), dev)
    r = mar.encode(nat, n, heap)
    offs = mar.index_records(r.xdr, n)
    assert torch.equal(offs, r.offsets)
    L = A.lib()
    maxlen = min(mar.plan.max_record_bytes, A.INDEX_MAX_MSG)
    ws = torch.empty(L.xdrg_index_workspace_size(r.xdr.numel(), maxlen), dtype=torch.uint8, device=dev)
    o2 = torch.empty(n + 1, dtype=torch.int64, device=dev)
    cnt = torch.empty(1, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    mar.status.init(s)
    A.check(L.xdrg_index_records(mar.plan.handle, r.xdr.data_ptr(), r.xdr.numel(), n, maxlen, o2.data_ptr(),
                                 cnt.data_ptr(), ws.data_ptr(), ws.numel(), mar.status.ptr, s), "index")
    assert mar.status.read(s).code == 0
    assert torch.equal(o2, r.offsets) and int(cnt.item()) == n
    assert _fast_flag(ws[-256:].cpu().numpy()) == 1
    a, ha = mar.decode(r.xdr, n, r.offsets)
    b, hb = mar.decode(r.xdr, n)
    assert torch.equal(a, b) and torch.equal(ha, hb)


@pytest.mark.gpu
def test_gpu_index_graph_capture(dev):
    """xdrg_index_records captured into a graph (torch.cuda.graph over the
    call's stream): the walk cannot wait for its verdict there, so it stays
    asynchronous (the list ranking is captured too and skips itself), and a
    replay indexes the stream."""
    import torch
    from xdrpp_amd import marshal as M
    cp = compile_plan(S.recvar)
    x, offs, n = tiled(*gold_stream("recvar"), 4)
    mar = M.Marshaler(M.Plan(cp), dev)
    L = A.lib()
    maxlen = window(cp)
    dx = _dev(x, dev)
    ws = torch.empty(L.xdrg_index_workspace_size(x.size, maxlen), dtype=torch.uint8, device=dev)
    out = torch.full((n + 1,), -1, dtype=torch.int64, device=dev)
    cnt = torch.empty(1, dtype=torch.int64, device=dev)
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # warm: plan tables and kernels uploaded outside the capture
        mar.status.init(side.cuda_stream)
        A.check(L.xdrg_index_records(mar.plan.handle, dx.data_ptr(), x.size, n, maxlen, out.data_ptr(),
                                     cnt.data_ptr(), ws.data_ptr(), ws.numel(), mar.status.ptr, side.cuda_stream),
                "index (warm)")
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    out.fill_(-1)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = torch.cuda.current_stream().cuda_stream
        A.check(L.xdrg_index_records(mar.plan.handle, dx.data_ptr(), x.size, n, maxlen, out.data_ptr(),
                                     cnt.data_ptr(), ws.data_ptr(), ws.numel(), mar.status.ptr, s), "index (capture)")
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint64), offs) and int(cnt.item()) == n
    assert _fast_flag(ws[-256:].cpu().numpy()) == 1


def _nest_plan(depth):
    """n0 { int v; }, n_i { n_{i-1} *p; int x; }: bounded records (a
    pointer holds at most one element) nested depth - 1 element frames,
    past the window parse's XDRG_INDEX_FRAMES."""
    from xdrpp_amd.xdr_types import Int, Pointer, Struct
    t = Struct("n0", [("v", Int)])
    for i in range(1, depth + 1):
        t = Struct(f"n{i}", [("p", Pointer(t)), ("x", Int)])
    return t


def _nest_stream(depth, n, seed):
    rng = np.random.default_rng(seed)
    recs, offs = [], [0]
    for _ in range(n):
        d = int(rng.integers(0, depth + 1))  # levels holding their pointer
        w = []
        for lvl in range(depth, 0, -1):
            if depth - lvl < d:
                w.append(1)
            else:
                w.append(0)
                break
        else:
            w.append(int(rng.integers(0, 1 << 31)))  # n0.v
        w += [int(v) for v in rng.integers(0, 1 << 31, size=min(d, depth) + (0 if d >= depth else 1))]
        recs.append(np.array(w, dtype=">u4").tobytes())
        offs.append(offs[-1] + len(recs[-1]))
    return np.frombuffer(b"".join(recs), dtype=np.uint8).copy(), np.array(offs, dtype=np.int64)


@pytest.mark.gpu
def test_gpu_decode_without_offsets_nested_past_index_frames(dev):
    """A plan whose records fit the index window but nest past its
    XDRG_INDEX_FRAMES: decode() without offsets hands the INDEX_LONG of the
    window parse to the whole-stream walk, and decodes as with offsets."""
    import torch
    from xdrpp_amd import marshal as M
    depth = 24
    plan = M.Plan(compile_plan(_nest_plan(depth)))
    assert plan.max_record_bytes <= A.INDEX_MAX_MSG
    x, offs = _nest_stream(depth, 3000, 7)
    mar = M.Marshaler(plan, dev)
    xd = torch.from_numpy(x).to(dev)
    a, ha = mar.decode(xd, len(offs) - 1, torch.from_numpy(offs).to(dev))
    b, hb = mar.decode(xd, len(offs) - 1)
    assert torch.equal(a, b) and torch.equal(ha, hb)
    got = mar.index_records(xd, len(offs) - 1, A.MAX_MSG)
    assert np.array_equal(got.cpu().numpy(), offs)
