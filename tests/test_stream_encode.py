"""The walk-first encode of word-list plans (var_kernels.h var_encode_body,
PRE): xdrg_encode without a size pass or scan -- the record kernel's own
walk gives the sizes and each wave's base comes from a decoupled look-back
over the byte totals of the waves before it; and its sized half
(xdrg_encode_sized over xdrg_encode_sizes' scan, the sizes not read).

Checked against the C restatement (oracle/xdr_oracle.c, pinned to the real
reference's bytes by tests/test_oracle.py) on the same inputs: the bytes,
the record index and the total; heaps in record order, shuffled heaps with
gaps, heaps cut short (bytes past heap_len read 0), capacity and
bad-discriminant errors, record marks, and repeated 1M-record encodes (the
look-back under a full grid).  Reference path: xdr_to_opaque,
xdrpp/marshal.h:264-272 over xdr_generic_put :84-137.
"""
import hashlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from xdrpp_amd import _abi as A  # noqa: E402
from xdrpp_amd import marshal as M  # noqa: E402
from xdrpp_amd import schemas as S  # noqa: E402
from xdrpp_amd import workloads as W  # noqa: E402
import oracle_bridge as O  # noqa: E402

# plan options: the walk-first record kernel with no size pass (look-back),
# the default (size pass + scan + walk-first record kernel), and the record
# kernel that walks per window
MODES = {"stream": {"enc_stream": 1}, "walk_first": {}, "two_pass": {"enc_stream": 0}}
_plans = {}


def plan(name, mode):
    key = (name, mode)
    if key not in _plans:
        _plans[key] = M.Plan(S.ALL[name], MODES[mode])
    return _plans[key]


def to_dev(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def one_pass(mar, nat, n, heap, cap, dev, msgs=False):
    """xdrg_encode (msgs: xdrg_encode_msgs) into a buffer of `cap` bytes:
    (bytes up to the total, offsets, error or None)."""
    out = torch.full((max(cap, 4) + 64,), 0xEE, dtype=torch.uint8, device=dev)
    offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    mar.status.init(s)
    h = to_dev(heap, dev) if heap is not None and heap.size else None
    if msgs:
        mar.launch_encode_msgs(to_dev(nat, dev), n, out[:cap], offs, heap=h, stream=s)
    else:
        mar.launch_encode(to_dev(nat, dev), n, out[:cap], heap=h, offsets=offs, stream=s)
    e = mar.status.read(s)
    assert bool((out[cap:] == 0xEE).all()), "encode wrote past its capacity"
    err = None if e.code == 0 else (e.code, e.record, e.op)
    got = out[:e.total_bytes] if err is None else out[:cap]
    return got.cpu().numpy(), offs.cpu().numpy().view(np.uint64), err, e


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("name", ["recvar", "rpc"])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 4097, 70001])
def test_stream_matches_oracle(dev, mode, name, n):
    p = plan(name, mode)
    mar = M.Marshaler(p, dev)
    nat, heap = W.GENERATORS[name](n)
    want, woffs = O.encode(p.cp, nat, n, heap)
    got, offs, err, e = one_pass(mar, nat, n, heap, want.size, dev)
    assert err is None
    assert e.total_bytes == want.size
    assert np.array_equal(got, want)
    assert np.array_equal(offs, woffs)
    # the two halves (xdrg_encode_sizes, then xdrg_encode_sized)
    res = mar.encode(to_dev(nat, dev), n, to_dev(heap, dev))
    assert np.array_equal(res.xdr.cpu().numpy(), want)
    assert np.array_equal(res.offsets.cpu().numpy().view(np.uint64), woffs)


def _live_refs(name, rec):
    """Native offsets of the bytes refs a record's walk visits."""
    if name == "recvar":
        return [S.recvar.offsets["blob"], S.recvar.offsets["name"]]
    t = S.rpc_msg
    u32 = lambda o: int(rec[o:o + 4].view(np.uint32)[0])  # noqa: E731
    if u32(t.offset_of("body")) == 0:  # CALL
        return [t.offset_of("body.cbody.cred.body"), t.offset_of("body.cbody.verf.body")]
    if u32(t.offset_of("body.rbody")) == 0:  # MSG_ACCEPTED
        return [t.offset_of("body.rbody.areply.verf.body")]
    return []


def _shuffled_heap(name, n, seed):
    """The same records with each payload moved to a random place in a new
    heap, gaps between them: a wave's payloads span far more than its window."""
    p = plan(name, "stream")
    nat, heap = W.GENERATORS[name](n)
    rec = nat.reshape(n, p.stride).copy()
    rng = np.random.default_rng(seed)
    pieces = []
    for r in range(n):
        for off in _live_refs(name, rec[r]):
            src = int(rec[r, off:off + 8].view(np.uint64)[0])
            ln = int(rec[r, off + 8:off + 12].view(np.uint32)[0])
            pieces.append((r, off, heap[src:src + ln]))
    order = rng.permutation(len(pieces))
    out = bytearray()
    for i in order:
        r, off, b = pieces[i]
        out += rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8).tobytes()  # a gap
        rec[r, off:off + 8] = np.frombuffer(np.uint64(len(out)).tobytes(), np.uint8)
        out += b.tobytes()
    return rec.reshape(-1), np.frombuffer(bytes(out), np.uint8).copy()


@pytest.mark.parametrize("mode", ["stream"])
@pytest.mark.parametrize("name", ["recvar", "rpc"])
def test_stream_shuffled_heap(dev, mode, name):
    n = 3000
    nat, heap = _shuffled_heap(name, n, 7)
    p = plan(name, mode)
    want, woffs = O.encode(p.cp, nat, n, heap)
    got, offs, err, _ = one_pass(M.Marshaler(p, dev), nat, n, heap, want.size, dev)
    assert err is None and np.array_equal(got, want) and np.array_equal(offs, woffs)


@pytest.mark.parametrize("mode", ["stream"])
@pytest.mark.parametrize("cut", [1, 5, 16, 333])
def test_stream_heap_cut_short(dev, mode, cut):
    """Payloads that run past heap_len read 0 there (as every encode kernel
    does; the oracle is given the zeros explicitly)."""
    n = 500
    p = plan("recvar", mode)
    nat, heap = W.recvar(n)
    short = heap[:heap.size - cut].copy()
    want, woffs = O.encode(p.cp, nat, n, np.concatenate([short, np.zeros(cut + 64, np.uint8)]))
    got, offs, err, _ = one_pass(M.Marshaler(p, dev), nat, n, short, want.size, dev)
    assert err is None and np.array_equal(got, want) and np.array_equal(offs, woffs)


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("name", ["recvar", "rpc"])
@pytest.mark.parametrize("at", [0, 63, 64, 200, 2999])
def test_stream_capacity(dev, mode, name, at):
    """A buffer that ends inside record `at`: the reference's xdr_overflow at
    that record and op, nothing written past the capacity, and every record
    before it in place."""
    n = 3000
    p = plan(name, mode)
    nat, heap = W.GENERATORS[name](n)
    full, woffs = O.encode(p.cp, nat, n, heap)
    cap = int(woffs[at]) + 6
    with pytest.raises(O.OracleError) as oe:
        O.encode(p.cp, nat, n, heap, cap=cap)
    want = (oe.value.code, oe.value.record, oe.value.op)
    got, offs, err, e = one_pass(M.Marshaler(p, dev), nat, n, heap, cap, dev)
    assert err == want and want[1] == at
    assert np.array_equal(offs, woffs)
    # the records before the failing one are the reference's bytes
    assert np.array_equal(got[:int(woffs[at])], full[:int(woffs[at])])


@pytest.mark.parametrize("mode", list(MODES))
def test_stream_bad_discriminants(dev, mode):
    p = plan("rpc", mode)
    n = 5000
    nat, heap = W.rpc(n)
    rec = nat.reshape(n, p.stride).copy()
    off = S.rpc_msg.offset_of("body")
    for bad in (4321, 777, 778):
        rec[bad, off:off + 4] = np.frombuffer(np.uint32(9).tobytes(), np.uint8)
    with pytest.raises(O.OracleError) as oe:
        O.encode(p.cp, rec.reshape(-1), n, heap, cap=1 << 24)
    want = (oe.value.code, oe.value.record, oe.value.op)
    _, _, err, _ = one_pass(M.Marshaler(p, dev), rec.reshape(-1), n, heap, 1 << 24, dev)
    assert err == want and want[1] == 777


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("name", ["recvar", "rpc"])
def test_stream_messages(dev, mode, name):
    """xdrg_encode_msgs: each record's mark BE(size | 0x80000000) first
    (message_t::alloc, xdrpp/marshal.cc:15-31)."""
    n = 2049
    p = plan(name, mode)
    nat, heap = W.GENERATORS[name](n)
    want, woffs = O.encode_msgs(p.cp, nat, n, heap)
    got, offs, err, _ = one_pass(M.Marshaler(p, dev), nat, n, heap, want.size, dev, msgs=True)
    assert err is None and np.array_equal(got, want) and np.array_equal(offs, woffs)


@pytest.mark.parametrize("name", ["recvar", "rpc"])
def test_stream_full_grid_repeated(dev, manifest, name):
    """1M records five times in a row through the one-pass kernel (16,384
    waves looking back): the reference's sha256 every
    time."""
    n = 1 << 20
    p = plan(name, "stream")
    mar = M.Marshaler(p, dev)
    nat_np, heap_np = W.GENERATORS[name](n)
    nat, heap = to_dev(nat_np, dev), to_dev(heap_np, dev)
    h = manifest["hashes"][f"{name}_{n}"]
    out = torch.empty(int(h["xdr_bytes"]), dtype=torch.uint8, device=dev)
    offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(5):
        mar.status.init(s)
        mar.launch_encode(nat, n, out, heap=heap, offsets=offs, stream=s)
        e = mar.status.read(s)
        assert e.code == 0
        assert e.total_bytes == int(h["xdr_bytes"])
        assert hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest() == h["xdr"]
        out.fill_(0)


@pytest.mark.parametrize("mode", ["stream", "walk_first"])
def test_stream_large_wave_totals(dev, mode):
    """Waves whose byte totals run to megabytes: 65,536 records of 64-68 KiB
    blobs (about 4.2 MiB a wave, 4.4 GB over 1,024 waves) through the
    look-back (its block sums are split in 16-bit halves summed in u32 over
    up to 1,024 blocks a poll; a 24-bit split wrapped past 4 GiB a poll) and
    through the scan.  Every blob points into one 128 KiB heap, so the bytes
    are checked by property: the record index equals the running sum of the
    records' sizes, the total matches, and sampled records equal the
    restatement's encoding of the same record."""
    from xdrpp_amd.xdr_types import Opaque, Struct, UHyper
    t = Struct("bigblob", [("id", UHyper), ("blob", Opaque(1 << 20))])
    p = M.Plan(t, MODES[mode])
    n = 1 << 16
    rng = np.random.default_rng(5)
    heap = rng.integers(0, 256, 1 << 17, dtype=np.uint8)
    lens = (65536 + rng.integers(0, 4096, n)).astype(np.int64)
    nat = np.zeros((n, p.stride), dtype=np.uint8)
    nat[:, 0:8] = np.arange(n, dtype="<u8").view(np.uint8).reshape(n, 8)
    o = t.offsets["blob"]
    nat[:, o + 8:o + 12] = lens.astype("<u4").view(np.uint8).reshape(n, 4)
    sizes = 8 + 4 + ((lens + 3) & ~3)
    woffs = np.zeros(n + 1, dtype=np.uint64)
    woffs[1:] = np.cumsum(sizes)
    total = int(woffs[-1])
    assert total > (1 << 32)
    mar = M.Marshaler(p, dev)
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    dn, dh = to_dev(nat.reshape(-1), dev), to_dev(heap, dev)
    for _ in range(2):
        mar.status.init(s)
        mar.launch_encode(dn, n, out, heap=dh, offsets=offs, stream=s)
        e = mar.status.read(s)
        assert e.code == 0 and e.total_bytes == total
        assert np.array_equal(offs.cpu().numpy().view(np.uint64), woffs)
        for r in list(range(64)) + list(rng.integers(0, n, 40)) + [n - 1]:
            want, _ = O.encode(p.cp, nat[r].copy(), 1, heap)
            a = int(woffs[r])
            assert np.array_equal(out[a:a + want.size].cpu().numpy(), want), r
        out.fill_(0)
    del out


def test_fresh_status_reads_no_error(dev):
    """A Status that was never init()ed reads as 'no error' (it is born
    initialised), so a raw launch cannot report allocator garbage."""
    for _ in range(8):
        junk = torch.full((1 << 16,), 0x01, dtype=torch.uint8, device=dev)  # recycled by the allocator
        del junk
        st = M.Status(dev)
        e = st.read(torch.cuda.current_stream().cuda_stream)
        assert e.code == 0 and e.total_bytes == 0
